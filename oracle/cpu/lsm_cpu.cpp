// lsm_cpu.cpp -- TEST INFRASTRUCTURE ONLY: the C++/OpenMP CPU implementation of the ICP
// scan-matching path that SURVEY.md §8d names as the CPU baseline beside the GPU numbers.
//
// Only bench.py's cpu_baseline leg and tests/ load it (through oracle/cpu_ref.py); the product
// (lidar_slam_arvc_amd) never does. It restates, in f64 with an exact KD-tree, the same Open3D
// algorithms oracle/open3d_restated.py restates with NumPy/SciPy, and the tests check the two
// against each other:
//   filter_radius_height      keyframe.py:74-94
//   EstimateNormals(Hybrid)   keyframe.py:160-162 -> [O3D] KDTreeFlann::SearchHybrid,
//                             ComputeCovariance (raw f64 cumulants), FastEigen3x3
//   RegistrationICP           keyframe.py:246-252 -> [O3D] GetRegistrationResultAndCorrespondences,
//                             TransformationEstimationPointToPlane (Eigen LDLT, Rz*Ry*Rx) and
//                             PointToPoint (Umeyama without scaling; here Horn's quaternion form,
//                             the same proper rotation), convergence |dfit|, |drmse| < 1e-6
// C ABI, plain pointers; xyz arrays are row-major n x 3 f64.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace {

// nanoflann L2 metric for dim 3: ((dx^2 + dy^2) + dz^2), dx = q - p
inline double sqd(const double *q, const double *p) {
    const double dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
    return (dx * dx + dy * dy) + dz * dz;
}

// Static KD-tree: median split on the widest axis, leaves of <= LEAF points, a bounding box per
// node for pruning. Queries are exact; ties on d2 resolve to the lower point index.
struct KDTree {
    static constexpr int LEAF = 12;
    struct Node {
        double lo[3], hi[3];
        int32_t a, b, l, r;
    };
    const double *p = nullptr;
    std::vector<int32_t> idx;
    std::vector<Node> nodes;

    KDTree(const double *pts, int64_t n) : p(pts), idx(size_t(n)) {
        for (int64_t i = 0; i < n; ++i) idx[size_t(i)] = int32_t(i);
        nodes.reserve(size_t(2 * (n / LEAF + 1) + 1));
        if (n > 0) build(0, int32_t(n));
    }

    int32_t build(int32_t a, int32_t b) {
        const int32_t id = int32_t(nodes.size());
        nodes.emplace_back();
        Node nd;
        for (int d = 0; d < 3; ++d) {
            nd.lo[d] = INFINITY;
            nd.hi[d] = -INFINITY;
        }
        for (int32_t k = a; k < b; ++k) {
            const double *q = p + 3 * size_t(idx[size_t(k)]);
            for (int d = 0; d < 3; ++d) {
                nd.lo[d] = std::min(nd.lo[d], q[d]);
                nd.hi[d] = std::max(nd.hi[d], q[d]);
            }
        }
        nd.a = a;
        nd.b = b;
        nd.l = nd.r = -1;
        if (b - a > LEAF) {
            int dim = 0;
            for (int d = 1; d < 3; ++d)
                if (nd.hi[d] - nd.lo[d] > nd.hi[dim] - nd.lo[dim]) dim = d;
            const int32_t m = a + (b - a) / 2;
            std::nth_element(idx.begin() + a, idx.begin() + m, idx.begin() + b,
                             [&](int32_t u, int32_t v) {
                                 const double pu = p[3 * size_t(u) + dim], pv = p[3 * size_t(v) + dim];
                                 return pu < pv || (pu == pv && u < v);
                             });
            nd.l = build(a, m);
            nd.r = build(m, b);
        }
        nodes[size_t(id)] = nd;
        return id;
    }

    static double box_d2(const Node &nd, const double *q) {
        double s = 0.0;
        for (int d = 0; d < 3; ++d) {
            const double e = q[d] < nd.lo[d] ? nd.lo[d] - q[d] : (q[d] > nd.hi[d] ? q[d] - nd.hi[d] : 0.0);
            s += e * e;
        }
        return s;
    }

    // exact nearest neighbour with d2 < bound2 (bi = -1 when there is none)
    void nearest(const double *q, double bound2, int32_t &bi, double &bd2) const {
        bi = -1;
        bd2 = bound2;
        if (nodes.empty()) return;
        int32_t stack[128];
        double sd[128];
        int sp = 0;
        stack[sp] = 0;
        sd[sp++] = box_d2(nodes[0], q);
        while (sp > 0) {
            --sp;
            if (sd[sp] > bd2) continue;
            const Node &nd = nodes[size_t(stack[sp])];
            if (nd.l < 0) {
                for (int32_t k = nd.a; k < nd.b; ++k) {
                    const int32_t j = idx[size_t(k)];
                    const double d2 = sqd(q, p + 3 * size_t(j));
                    if (d2 < bd2 || (bi >= 0 && d2 == bd2 && j < bi)) {
                        bd2 = d2;
                        bi = j;
                    }
                }
                continue;
            }
            const double dl = box_d2(nodes[size_t(nd.l)], q), dr = box_d2(nodes[size_t(nd.r)], q);
            // the nearer child is popped first
            if (dl <= dr) {
                stack[sp] = nd.r; sd[sp++] = dr;
                stack[sp] = nd.l; sd[sp++] = dl;
            } else {
                stack[sp] = nd.l; sd[sp++] = dl;
                stack[sp] = nd.r; sd[sp++] = dr;
            }
        }
    }

    // SearchHybrid: the k nearest with d2 < r2, as (d2, index) ascending
    void hybrid(const double *q, int k, double r2, std::vector<std::pair<double, int32_t>> &out) const {
        out.clear();
        if (nodes.empty() || k <= 0) return;
        int32_t stack[128];
        double sd[128];
        int sp = 0;
        stack[sp] = 0;
        sd[sp++] = box_d2(nodes[0], q);
        auto bound_ok = [&](double d) {
            return d < r2 && (int(out.size()) < k || d <= out.front().first);
        };
        while (sp > 0) {
            --sp;
            if (!bound_ok(sd[sp])) continue;
            const Node &nd = nodes[size_t(stack[sp])];
            if (nd.l < 0) {
                for (int32_t t = nd.a; t < nd.b; ++t) {
                    const int32_t j = idx[size_t(t)];
                    const double d2 = sqd(q, p + 3 * size_t(j));
                    if (!(d2 < r2)) continue;
                    const std::pair<double, int32_t> e(d2, j);
                    if (int(out.size()) < k) {
                        out.push_back(e);
                        std::push_heap(out.begin(), out.end());
                    } else if (e < out.front()) {
                        std::pop_heap(out.begin(), out.end());
                        out.back() = e;
                        std::push_heap(out.begin(), out.end());
                    }
                }
                continue;
            }
            const double dl = box_d2(nodes[size_t(nd.l)], q), dr = box_d2(nodes[size_t(nd.r)], q);
            if (dl <= dr) {
                stack[sp] = nd.r; sd[sp++] = dr;
                stack[sp] = nd.l; sd[sp++] = dl;
            } else {
                stack[sp] = nd.l; sd[sp++] = dl;
                stack[sp] = nd.r; sd[sp++] = dr;
            }
        }
        std::sort_heap(out.begin(), out.end());
    }
};

// ---- FastEigen3x3 (Geometric Tools robust symmetric 3x3, as Open3D), smallest eigenvector ----
struct V3 {
    double x, y, z;
};
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V3 scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 divide(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }

struct Sym {
    double a00, a01, a02, a11, a12, a22;
    V3 mul(V3 v) const {
        return {(a00 * v.x + a01 * v.y) + a02 * v.z, (a01 * v.x + a11 * v.y) + a12 * v.z,
                (a02 * v.x + a12 * v.y) + a22 * v.z};
    }
};

V3 eigvec0(const Sym &A, double e) {
    const V3 r0 = {A.a00 - e, A.a01, A.a02}, r1 = {A.a01, A.a11 - e, A.a12}, r2 = {A.a02, A.a12, A.a22 - e};
    const V3 c01 = cross(r0, r1), c02 = cross(r0, r2), c12 = cross(r1, r2);
    const double d0 = dot(c01, c01), d1 = dot(c02, c02), d2 = dot(c12, c12);
    const bool pick1 = d1 > d0;
    const double best = pick1 ? d1 : d0;
    if (d2 > best) return divide(c12, std::sqrt(d2));
    return pick1 ? divide(c02, std::sqrt(d1)) : divide(c01, std::sqrt(d0));
}

V3 eigvec1(const Sym &A, V3 ev0, double e) {
    V3 U;
    if (std::fabs(ev0.x) > std::fabs(ev0.y)) {
        const double il = 1.0 / std::sqrt(ev0.x * ev0.x + ev0.z * ev0.z);
        U = {-ev0.z * il, 0.0, ev0.x * il};
    } else {
        const double il = 1.0 / std::sqrt(ev0.y * ev0.y + ev0.z * ev0.z);
        U = {0.0, ev0.z * il, -ev0.y * il};
    }
    const V3 V = cross(ev0, U);
    const V3 AU = A.mul(U), AV = A.mul(V);
    const double m00 = dot(U, AU) - e, m01 = dot(U, AV), m11 = dot(V, AV) - e;
    const double a00 = std::fabs(m00), a01 = std::fabs(m01), a11 = std::fabs(m11);
    if (a00 >= a11) {
        if (std::max(a00, a01) <= 0.0) return U;
        double r00, r01;
        if (a00 >= a01) {
            r01 = m01 / m00;
            r00 = 1.0 / std::sqrt(1.0 + r01 * r01);
            r01 *= r00;
        } else {
            r00 = m00 / m01;
            r01 = 1.0 / std::sqrt(1.0 + r00 * r00);
            r00 *= r01;
        }
        return sub(scale(U, r01), scale(V, r00));
    }
    if (std::max(a11, a01) <= 0.0) return U;
    double r11, r01;
    if (a11 >= a01) {
        r01 = m01 / m11;
        r11 = 1.0 / std::sqrt(1.0 + r01 * r01);
        r01 *= r11;
    } else {
        r11 = m11 / m01;
        r01 = 1.0 / std::sqrt(1.0 + r11 * r11);
        r11 *= r01;
    }
    return sub(scale(U, r11), scale(V, r01));
}

V3 fast_eigen3x3_min(const double C[6]) {   // C = a00 a01 a02 a11 a12 a22
    // Open3D divides by the (signed) largest coefficient
    double mc = C[0];
    mc = std::max(mc, C[1]);
    mc = std::max(mc, C[2]);
    mc = std::max(mc, C[3]);
    mc = std::max(mc, C[4]);
    mc = std::max(mc, C[5]);
    if (mc == 0.0) return {0.0, 0.0, 0.0};
    const Sym A = {C[0] / mc, C[1] / mc, C[2] / mc, C[3] / mc, C[4] / mc, C[5] / mc};
    const double norm = (A.a01 * A.a01 + A.a02 * A.a02) + A.a12 * A.a12;
    if (!(norm > 0.0)) {
        if (A.a00 < A.a11 && A.a00 < A.a22) return {1.0, 0.0, 0.0};
        if (A.a11 < A.a00 && A.a11 < A.a22) return {0.0, 1.0, 0.0};
        return {0.0, 0.0, 1.0};
    }
    const double q = ((A.a00 + A.a11) + A.a22) / 3.0;
    const double b00 = A.a00 - q, b11 = A.a11 - q, b22 = A.a22 - q;
    const double p = std::sqrt((((b00 * b00 + b11 * b11) + b22 * b22) + norm * 2.0) / 6.0);
    const double c00 = b11 * b22 - A.a12 * A.a12;
    const double c01 = A.a01 * b22 - A.a12 * A.a02;
    const double c02 = A.a01 * A.a12 - b11 * A.a02;
    const double det = ((b00 * c00 - A.a01 * c01) + A.a02 * c02) / (p * p * p);
    const double half = std::min(std::max(det * 0.5, -1.0), 1.0);
    const double ang = std::acos(half) / 3.0;
    const double beta2 = std::cos(ang) * 2.0;
    const double beta0 = std::cos(ang + 2.09439510239319549) * 2.0;
    const double beta1 = -(beta0 + beta2);
    const double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
    if (half >= 0.0) {
        const V3 v2 = eigvec0(A, e2);
        const V3 v1 = eigvec1(A, v2, e1);
        if (e2 < e0 && e2 < e1) return v2;
        if (e1 < e0 && e1 < e2) return v1;
        return cross(v1, v2);
    }
    const V3 v0 = eigvec0(A, e0);
    const V3 v1 = eigvec1(A, v0, e1);
    if (e0 < e1 && e0 < e2) return v0;
    if (e1 < e0 && e1 < e2) return v1;
    return cross(v0, v1);
}

// ---- registration ----
void transform(const double T[16], const double *in, double *out, int64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const double *a = in + 3 * i;
        double *o = out + 3 * i;
        const double x = a[0], y = a[1], z = a[2];
        o[0] = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
        o[1] = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
        o[2] = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
    }
}

void matmul4(const double A[16], const double B[16], double C[16]) {
    double R[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[4 * i + k] * B[4 * k + j];
            R[4 * i + j] = s;
        }
    std::memcpy(C, R, sizeof(R));
}

// correspondences: corr[i] = nearest target index or -1; returns (fitness, rmse) and the count
int64_t correspond(const KDTree &tree, const double *tgt, const double *src_t, int64_t ns,
                   double max_corr, int32_t *corr, double &fitness, double &rmse) {
    const double mc2 = max_corr * max_corr;
    int64_t cnt = 0;
    double s = 0.0;
#pragma omp parallel for schedule(dynamic, 512) reduction(+ : cnt, s)
    for (int64_t i = 0; i < ns; ++i) {
        int32_t bi;
        double bd2;
        tree.nearest(src_t + 3 * i, mc2, bi, bd2);
        corr[i] = bi;
        if (bi >= 0) {
            ++cnt;
            s += sqd(src_t + 3 * i, tgt + 3 * size_t(bi));
        }
    }
    fitness = cnt ? double(cnt) / double(ns) : 0.0;
    rmse = cnt ? std::sqrt(s / double(cnt)) : 0.0;
    return cnt;
}

// Eigen LDLT with diagonal pivoting and the pseudo-inverse of D (ldlt_solve in the NumPy oracle)
void ldlt_solve6(double A[6][6], const double b[6], double x[6]) {
    const int n = 6;
    int tr[6];
    for (int k = 0; k < n; ++k) {
        int j = k;
        for (int t = k + 1; t < n; ++t)
            if (std::fabs(A[t][t]) > std::fabs(A[j][j])) j = t;
        tr[k] = j;
        if (j != k) {
            for (int c = 0; c < n; ++c) std::swap(A[k][c], A[j][c]);
            for (int r = 0; r < n; ++r) std::swap(A[r][k], A[r][j]);
        }
        if (k > 0) {
            double t[6];
            for (int c = 0; c < k; ++c) t[c] = A[k][c] * A[c][c];
            double s = 0.0;
            for (int c = 0; c < k; ++c) s += A[k][c] * t[c];
            A[k][k] -= s;
            for (int r = k + 1; r < n; ++r) {
                double u = 0.0;
                for (int c = 0; c < k; ++c) u += A[r][c] * t[c];
                A[r][k] -= u;
            }
        }
        const double akk = A[k][k];
        if (k == 0 && akk == 0.0) {
            for (int i = 0; i < n; ++i) x[i] = 0.0;
            return;
        }
        if (k + 1 < n && akk != 0.0)
            for (int r = k + 1; r < n; ++r) A[r][k] /= akk;
    }
    for (int i = 0; i < n; ++i) x[i] = b[i];
    for (int k = 0; k < n; ++k) std::swap(x[k], x[tr[k]]);
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int c = 0; c < i; ++c) s += A[i][c] * x[c];
        x[i] -= s;
    }
    const double tiny = 2.2250738585072014e-308;
    for (int i = 0; i < n; ++i) x[i] = std::fabs(A[i][i]) > tiny ? x[i] / A[i][i] : 0.0;
    for (int i = n - 1; i >= 0; --i) {
        double s = 0.0;
        for (int r = i + 1; r < n; ++r) s += A[r][i] * x[r];
        x[i] -= s;
    }
    for (int k = n - 1; k >= 0; --k) std::swap(x[k], x[tr[k]]);
}

void vec6_to_mat4(const double x[6], double T[16]) {
    const double ca = std::cos(x[0]), sa = std::sin(x[0]), cb = std::cos(x[1]), sb = std::sin(x[1]),
                 cg = std::cos(x[2]), sg = std::sin(x[2]);
    const double Rx[9] = {1, 0, 0, 0, ca, -sa, 0, sa, ca};
    const double Ry[9] = {cb, 0, sb, 0, 1, 0, -sb, 0, cb};
    const double Rz[9] = {cg, -sg, 0, sg, cg, 0, 0, 0, 1};
    double RzRy[9], R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            RzRy[3 * i + j] = (Rz[3 * i] * Ry[j] + Rz[3 * i + 1] * Ry[3 + j]) + Rz[3 * i + 2] * Ry[6 + j];
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[3 * i + j] = (RzRy[3 * i] * Rx[j] + RzRy[3 * i + 1] * Rx[3 + j]) + RzRy[3 * i + 2] * Rx[6 + j];
    for (int i = 0; i < 16; ++i) T[i] = 0.0;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = R[3 * i + j];
        T[4 * i + 3] = x[3 + i];
    }
    T[15] = 1.0;
}

// P2Plane update: J = [p x n; n], r = (p - q) . n; x = LDLT(J^T J) \ -(J^T r)
void estimate_p2plane(const double *src_t, const double *tgt, const double *tn, const int32_t *corr,
                      int64_t ns, double T[16]) {
    const int nth = omp_get_max_threads();
    std::vector<double> part(size_t(nth) * 27, 0.0);
#pragma omp parallel
    {
        double *acc = part.data() + 27 * size_t(omp_get_thread_num());
#pragma omp for schedule(static)
        for (int64_t i = 0; i < ns; ++i) {
            const int32_t j = corr[i];
            if (j < 0) continue;
            const double *p = src_t + 3 * i, *q = tgt + 3 * size_t(j), *n = tn + 3 * size_t(j);
            const double r = ((p[0] - q[0]) * n[0] + (p[1] - q[1]) * n[1]) + (p[2] - q[2]) * n[2];
            const double J[6] = {p[1] * n[2] - p[2] * n[1], p[2] * n[0] - p[0] * n[2],
                                 p[0] * n[1] - p[1] * n[0], n[0], n[1], n[2]};
            int t = 0;
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) acc[t++] += J[a] * J[b];
            for (int a = 0; a < 6; ++a) acc[21 + a] += J[a] * r;
        }
    }
    double A[6][6], b[6], x[6];
    double s[27] = {0};
    for (int t = 0; t < nth; ++t)
        for (int c = 0; c < 27; ++c) s[c] += part[27 * size_t(t) + c];
    int t = 0;
    for (int a = 0; a < 6; ++a)
        for (int c = a; c < 6; ++c) A[a][c] = A[c][a] = s[t++];
    for (int a = 0; a < 6; ++a) b[a] = -s[21 + a];
    ldlt_solve6(A, b, x);
    vec6_to_mat4(x, T);
}

// symmetric 4x4 Jacobi eigen-decomposition: eigenvector of the largest eigenvalue
void jacobi4_max(double N[4][4], double v[4]) {
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int i = 0; i < 4; ++i)
            for (int j = i + 1; j < 4; ++j) off += N[i][j] * N[i][j];
        if (off < 1e-300) break;
        for (int p = 0; p < 4; ++p)
            for (int q = p + 1; q < 4; ++q) {
                if (N[p][q] == 0.0) continue;
                const double th = (N[q][q] - N[p][p]) / (2.0 * N[p][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; ++k) {
                    const double a = N[k][p], b = N[k][q];
                    N[k][p] = c * a - s * b;
                    N[k][q] = s * a + c * b;
                }
                for (int k = 0; k < 4; ++k) {
                    const double a = N[p][k], b = N[q][k];
                    N[p][k] = c * a - s * b;
                    N[q][k] = s * a + c * b;
                }
                for (int k = 0; k < 4; ++k) {
                    const double a = V[k][p], b = V[k][q];
                    V[k][p] = c * a - s * b;
                    V[k][q] = s * a + c * b;
                }
            }
    }
    int m = 0;
    for (int i = 1; i < 4; ++i)
        if (N[i][i] > N[m][m]) m = i;
    for (int k = 0; k < 4; ++k) v[k] = V[k][m];
}

// P2P update: the rotation/translation Umeyama (no scaling) gives, via Horn's quaternion
void estimate_p2p(const double *src_t, const double *tgt, const int32_t *corr, int64_t ns,
                  double T[16]) {
    double ms[3] = {0, 0, 0}, md[3] = {0, 0, 0};
    int64_t n = 0;
    for (int64_t i = 0; i < ns; ++i) {
        const int32_t j = corr[i];
        if (j < 0) continue;
        for (int d = 0; d < 3; ++d) {
            ms[d] += src_t[3 * i + d];
            md[d] += tgt[3 * size_t(j) + d];
        }
        ++n;
    }
    for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.0 : 0.0;
    if (n == 0) return;
    for (int d = 0; d < 3; ++d) {
        ms[d] /= double(n);
        md[d] /= double(n);
    }
    double S[3][3] = {{0}};   // S_ab = sum (s_a - ms_a)(d_b - md_b)
    for (int64_t i = 0; i < ns; ++i) {
        const int32_t j = corr[i];
        if (j < 0) continue;
        double a[3], b[3];
        for (int d = 0; d < 3; ++d) {
            a[d] = src_t[3 * i + d] - ms[d];
            b[d] = tgt[3 * size_t(j) + d] - md[d];
        }
        for (int u = 0; u < 3; ++u)
            for (int v = 0; v < 3; ++v) S[u][v] += a[u] * b[v];
    }
    double N[4][4] = {
        {S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0]},
        {S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2]},
        {S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1]},
        {S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]}};
    double qv[4];
    jacobi4_max(N, qv);
    const double w = qv[0], x = qv[1], y = qv[2], z = qv[3];
    const double R[9] = {w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y),
                         2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x),
                         2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z};
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = R[3 * i + j];
        T[4 * i + 3] = md[i] - ((R[3 * i] * ms[0] + R[3 * i + 1] * ms[1]) + R[3 * i + 2] * ms[2]);
    }
}

}   // namespace

extern "C" {

// threads for every later call (0: OpenMP's default)
void lsmcpu_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
}

// filter_radius_height (keyframe.py:74-94): strict r^2 in (rmin^2, rmax^2), z in (zmin, zmax),
// order-preserving; out (n x 3) may alias nothing. Returns the kept count.
int64_t lsmcpu_filter(const double *xyz, int64_t n, double rmin, double rmax, double zmin,
                      double zmax, double *out) {
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        const double r2 = x * x + y * y;
        if (r2 < rmax * rmax && r2 > rmin * rmin && z > zmin && z < zmax) {
            out[3 * m] = x;
            out[3 * m + 1] = y;
            out[3 * m + 2] = z;
            ++m;
        }
    }
    return m;
}

// VoxelDownSample (keyframe.py:150-151): origin min_bound - v/2, keys floor((p - o) / v), the
// per-voxel mean summed in point order; centroids (<= n x 3) in lexicographic key order (the
// NumPy oracle's order). Returns the voxel count, -1 for voxel_size <= 0, -2 when too small.
int64_t lsmcpu_voxel(const double *xyz, int64_t n, double v, double *out) {
    if (!(v > 0.0)) return -1;
    if (n == 0) return 0;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) {
            lo[d] = std::min(lo[d], xyz[3 * i + d]);
            hi[d] = std::max(hi[d], xyz[3 * i + d]);
        }
    double ext = 0.0;
    for (int d = 0; d < 3; ++d) {
        lo[d] -= v * 0.5;
        hi[d] += v * 0.5;
        ext = std::max(ext, hi[d] - lo[d]);
    }
    if (v * 2147483647.0 < ext) return -2;
    std::vector<int64_t> key(static_cast<size_t>(3 * n));
    for (int64_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) key[size_t(3 * i + d)] = int64_t(std::floor((xyz[3 * i + d] - lo[d]) / v));
    std::vector<int64_t> ord(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) ord[size_t(i)] = i;
    auto kless = [&](int64_t a, int64_t b) {
        for (int d = 0; d < 3; ++d)
            if (key[size_t(3 * a + d)] != key[size_t(3 * b + d)]) return key[size_t(3 * a + d)] < key[size_t(3 * b + d)];
        return false;
    };
    std::stable_sort(ord.begin(), ord.end(), kless);
    int64_t m = 0;
    for (int64_t s = 0; s < n;) {
        int64_t e = s + 1;
        while (e < n && !kless(ord[size_t(s)], ord[size_t(e)])) ++e;
        double acc[3] = {0.0, 0.0, 0.0};
        for (int64_t t = s; t < e; ++t)
            for (int d = 0; d < 3; ++d) acc[d] = acc[d] + xyz[3 * ord[size_t(t)] + d];
        for (int d = 0; d < 3; ++d) out[3 * m + d] = acc[d] / double(e - s);
        ++m;
        s = e;
    }
    return m;
}

// EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) on a cloud without normals:
// normals (n x 3), counts (nullable) = neighbourhood sizes. Returns 0.
int lsmcpu_normals(const double *xyz, int64_t n, double radius, int max_nn, double *normals,
                   int64_t *counts) {
    const KDTree tree(xyz, n);
    const double r2 = radius * radius;
#pragma omp parallel
    {
        std::vector<std::pair<double, int32_t>> nb;
        nb.reserve(size_t(max_nn > 0 ? max_nn : 1));
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < n; ++i) {
            tree.hybrid(xyz + 3 * i, max_nn, r2, nb);
            const int64_t c = int64_t(nb.size());
            if (counts) counts[i] = c;
            double C[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
            if (c >= 3) {
                // ComputeCovariance: raw cumulants in search order, / n, minus mu mu^T
                double s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (const auto &e : nb) {
                    const double *p = xyz + 3 * size_t(e.second);
                    s[0] += p[0];
                    s[1] += p[1];
                    s[2] += p[2];
                    s[3] += p[0] * p[0];
                    s[4] += p[0] * p[1];
                    s[5] += p[0] * p[2];
                    s[6] += p[1] * p[1];
                    s[7] += p[1] * p[2];
                    s[8] += p[2] * p[2];
                }
                // Eigen's `cumulants /= n` divides each cumulant (no reciprocal)
                const double dn = double(c);
                for (double &v : s) v /= dn;
                C[0] = s[3] - s[0] * s[0];
                C[1] = s[4] - s[0] * s[1];
                C[2] = s[5] - s[0] * s[2];
                C[3] = s[6] - s[1] * s[1];
                C[4] = s[7] - s[1] * s[2];
                C[5] = s[8] - s[2] * s[2];
            }
            V3 v = fast_eigen3x3_min(C);
            if (std::sqrt(dot(v, v)) == 0.0) v = {0.0, 0.0, 1.0};
            normals[3 * i] = v.x;
            normals[3 * i + 1] = v.y;
            normals[3 * i + 2] = v.z;
        }
    }
    return 0;
}

// RegistrationICP (method 0: point-to-point, 1: point-to-plane with target normals tn).
// T (16, row-major) holds the initial transform in and the result out; info[0..2] = fitness,
// inlier_rmse, correspondence count; iters = the update rounds run. corr (ns, nullable) = the
// final correspondences. Returns 0, or -1 on an invalid max_corr / missing normals (the two
// LogError cases of Open3D).
int lsmcpu_icp(const double *src, int64_t ns, const double *tgt, int64_t nt, const double *tn,
               double max_corr, int method, int max_iteration, double rel_fitness,
               double rel_rmse, double *T, double *info, int *iters, int32_t *corr_out) {
    if (!(max_corr > 0.0)) return -1;
    if (method == 1 && !tn) return -1;
    const KDTree tree(tgt, nt);
    std::vector<double> pcd(static_cast<size_t>(3 * ns));
    std::vector<int32_t> corr(static_cast<size_t>(ns));
    transform(T, src, pcd.data(), ns);
    double fit, rmse;
    int64_t cnt = correspond(tree, tgt, pcd.data(), ns, max_corr, corr.data(), fit, rmse);
    int it = 0;
    for (it = 1; it <= max_iteration; ++it) {
        double U[16];
        if (cnt == 0) {
            for (int i = 0; i < 16; ++i) U[i] = (i % 5 == 0) ? 1.0 : 0.0;
        } else if (method == 1) {
            estimate_p2plane(pcd.data(), tgt, tn, corr.data(), ns, U);
        } else {
            estimate_p2p(pcd.data(), tgt, corr.data(), ns, U);
        }
        matmul4(U, T, T);
        std::vector<double> nx(pcd.size());
        transform(U, pcd.data(), nx.data(), ns);
        pcd.swap(nx);
        const double pf = fit, pr = rmse;
        cnt = correspond(tree, tgt, pcd.data(), ns, max_corr, corr.data(), fit, rmse);
        if (std::fabs(pf - fit) < rel_fitness && std::fabs(pr - rmse) < rel_rmse) break;
    }
    if (it > max_iteration) it = max_iteration;
    info[0] = fit;
    info[1] = rmse;
    info[2] = double(cnt);
    *iters = it;
    if (corr_out) std::memcpy(corr_out, corr.data(), sizeof(int32_t) * size_t(ns));
    return 0;
}

}   // extern "C"
