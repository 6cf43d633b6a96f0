// fasteigen.h -- device f64 port of Open3D's FastEigen3x3 (Geometric Tools "Robust Eigensolver
// for 3x3 Symmetric Matrices"), used by PointCloud::EstimateNormals with
// fast_normal_computation = true (keyframe.py:160-162 -> [O3D] ComputeNormal).
// Returns the (unnormalised-sign) eigenvector of the smallest eigenvalue; the zero vector when
// the largest coefficient is 0. Branch structure follows the published algorithm exactly so the
// choice of eigenvector (and sign) matches the reference's on well-separated spectra.
#pragma once
#include <hip/hip_runtime.h>

struct d3 {
    double x, y, z;
};

__device__ __forceinline__ d3 d3_cross(d3 a, d3 b) {
#pragma clang fp contract(off)
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double d3_dot(d3 a, d3 b) {
#pragma clang fp contract(off)
    return (a.x * b.x + a.y * b.y) + a.z * b.z;
}

// Symmetric matrix kept as its 6 unique entries.
struct sym3 {
    double a00, a01, a02, a11, a12, a22;
};

__device__ __forceinline__ d3 fe_vec0(const sym3 &A, double e) {
#pragma clang fp contract(off)
    d3 r0 = {A.a00 - e, A.a01, A.a02};
    d3 r1 = {A.a01, A.a11 - e, A.a12};
    d3 r2 = {A.a02, A.a12, A.a22 - e};
    d3 c01 = d3_cross(r0, r1), c02 = d3_cross(r0, r2), c12 = d3_cross(r1, r2);
    double d0 = d3_dot(c01, c01), d1 = d3_dot(c02, c02), d2 = d3_dot(c12, c12);
    double dmax = d0;
    int which = 0;
    if (d1 > dmax) {
        dmax = d1;
        which = 1;
    }
    if (d2 > dmax) which = 2;
    if (which == 0) {
        double s = sqrt(d0);
        return {c01.x / s, c01.y / s, c01.z / s};
    }
    if (which == 1) {
        double s = sqrt(d1);
        return {c02.x / s, c02.y / s, c02.z / s};
    }
    double s = sqrt(d2);
    return {c12.x / s, c12.y / s, c12.z / s};
}

__device__ __forceinline__ d3 fe_vec1(const sym3 &A, d3 v0, double e) {
#pragma clang fp contract(off)
    d3 U;
    if (fabs(v0.x) > fabs(v0.y)) {
        double il = 1.0 / sqrt(v0.x * v0.x + v0.z * v0.z);
        U = {-v0.z * il, 0.0, v0.x * il};
    } else {
        double il = 1.0 / sqrt(v0.y * v0.y + v0.z * v0.z);
        U = {0.0, v0.z * il, -v0.y * il};
    }
    d3 V = d3_cross(v0, U);
    d3 AU = {(A.a00 * U.x + A.a01 * U.y) + A.a02 * U.z, (A.a01 * U.x + A.a11 * U.y) + A.a12 * U.z,
             (A.a02 * U.x + A.a12 * U.y) + A.a22 * U.z};
    d3 AV = {(A.a00 * V.x + A.a01 * V.y) + A.a02 * V.z, (A.a01 * V.x + A.a11 * V.y) + A.a12 * V.z,
             (A.a02 * V.x + A.a12 * V.y) + A.a22 * V.z};
    double m00 = d3_dot(U, AU) - e;
    double m01 = d3_dot(U, AV);
    double m11 = d3_dot(V, AV) - e;
    double b00 = fabs(m00), b01 = fabs(m01), b11 = fabs(m11);
    if (b00 >= b11) {
        if (fmax(b00, b01) > 0) {
            if (b00 >= b01) {
                m01 /= m00;
                m00 = 1.0 / sqrt(1.0 + m01 * m01);
                m01 *= m00;
            } else {
                m00 /= m01;
                m01 = 1.0 / sqrt(1.0 + m00 * m00);
                m00 *= m01;
            }
            return {m01 * U.x - m00 * V.x, m01 * U.y - m00 * V.y, m01 * U.z - m00 * V.z};
        }
        return U;
    }
    if (fmax(b11, b01) > 0) {
        if (b11 >= b01) {
            m01 /= m11;
            m11 = 1.0 / sqrt(1.0 + m01 * m01);
            m01 *= m11;
        } else {
            m11 /= m01;
            m01 = 1.0 / sqrt(1.0 + m11 * m11);
            m11 *= m01;
        }
        return {m11 * U.x - m01 * V.x, m11 * U.y - m01 * V.y, m11 * U.z - m01 * V.z};
    }
    return U;
}

__device__ inline d3 fast_eigen3x3_min(sym3 A) {
#pragma clang fp contract(off)
    double mc = fmax(fmax(fmax(A.a00, A.a01), fmax(A.a02, A.a11)), fmax(A.a12, A.a22));
    if (mc == 0.0) return {0.0, 0.0, 0.0};
    A.a00 /= mc;
    A.a01 /= mc;
    A.a02 /= mc;
    A.a11 /= mc;
    A.a12 /= mc;
    A.a22 /= mc;
    double norm = (A.a01 * A.a01 + A.a02 * A.a02) + A.a12 * A.a12;
    if (norm > 0) {
        double q = ((A.a00 + A.a11) + A.a22) / 3;
        double b00 = A.a00 - q, b11 = A.a11 - q, b22 = A.a22 - q;
        double p = sqrt((((b00 * b00 + b11 * b11) + b22 * b22) + norm * 2) / 6);
        double c00 = b11 * b22 - A.a12 * A.a12;
        double c01 = A.a01 * b22 - A.a12 * A.a02;
        double c02 = A.a01 * A.a12 - b11 * A.a02;
        double det = ((b00 * c00 - A.a01 * c01) + A.a02 * c02) / (p * p * p);
        double half = fmin(fmax(det * 0.5, -1.0), 1.0);
        double ang = acos(half) / 3.0;
        double beta2 = cos(ang) * 2;
        double beta0 = cos(ang + 2.09439510239319549) * 2;
        double beta1 = -(beta0 + beta2);
        double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
        if (half >= 0) {
            d3 v2 = fe_vec0(A, e2);
            if (e2 < e0 && e2 < e1) return v2;
            d3 v1 = fe_vec1(A, v2, e1);
            if (e1 < e0 && e1 < e2) return v1;
            return d3_cross(v1, v2);
        }
        d3 v0 = fe_vec0(A, e0);
        if (e0 < e1 && e0 < e2) return v0;
        d3 v1 = fe_vec1(A, v0, e1);
        if (e1 < e0 && e1 < e2) return v1;
        return d3_cross(v0, v1);
    }
    if (A.a00 < A.a11 && A.a00 < A.a22) return {1.0, 0.0, 0.0};
    if (A.a11 < A.a00 && A.a11 < A.a22) return {0.0, 1.0, 0.0};
    return {0.0, 0.0, 1.0};
}
