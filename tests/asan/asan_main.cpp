// Host sanitizer driver ("-fsanitize=address for the host lib"): the C++/OpenMP
// CPU implementation (oracle/cpu/lsm_cpu.cpp: filter, voxel, normals, ICP, their error cases)
// and the library's host-only SE(3) prefix (lidar_slam_arvc_amd/csrc/se3_host.cpp), built with
// -fsanitize=address,undefined by tests/asan/Makefile and run by tests/test_host.py. Exits 0 and
// prints "asan ok" when every call returns what it should; a sanitizer report aborts it.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

extern "C" {
void lsmcpu_set_threads(int n);
int64_t lsmcpu_filter(const double *xyz, int64_t n, double rmin, double rmax, double zmin,
                      double zmax, double *out);
int64_t lsmcpu_voxel(const double *xyz, int64_t n, double v, double *out);
int lsmcpu_normals(const double *xyz, int64_t n, double radius, int max_nn, double *normals,
                   int64_t *counts);
int lsmcpu_icp(const double *src, int64_t ns, const double *tgt, int64_t nt, const double *tn,
               double max_corr, int method, int max_iteration, double rel_fitness,
               double rel_rmse, double *T, double *info, int *iters, int32_t *corr_out);
int lsm_se3_prefix(const double *rel, int64_t n, double *out);
}

static int fails = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "check failed line %d: %s\n", __LINE__, #c); \
            ++fails;                                                   \
        }                                                              \
    } while (0)

// a ground patch with a wall and a pole, plus points the filter must drop (NaN, too near/far/low)
static std::vector<double> scene(uint64_t seed, int n) {
    std::vector<double> p;
    uint64_t s = seed;
    auto u = [&]() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return double(s >> 11) * (1.0 / 9007199254740992.0);
    };
    for (int i = 0; i < n; ++i) {
        const double a = u(), b = u();
        const int kind = i % 3;
        if (kind == 0) p.insert(p.end(), {2.0 + 4.0 * a, -2.0 + 4.0 * b, -0.69 + 0.01 * u()});
        else if (kind == 1) p.insert(p.end(), {5.0 + 0.01 * u(), -2.0 + 4.0 * a, -0.69 + 2.0 * b});
        else p.insert(p.end(), {3.0 + 0.1 * std::cos(6.283 * a), 1.0 + 0.1 * std::sin(6.283 * a), -0.69 + 3.0 * b});
    }
    p.insert(p.end(), {NAN, 0.0, 0.0, 0.1, 0.1, 0.0, 50.0, 0.0, 0.0, 3.0, 0.0, -5.0});
    return p;
}

int main() {
    lsmcpu_set_threads(2);
    const std::vector<double> raw = scene(7, 3000);
    const int64_t n_raw = int64_t(raw.size() / 3);
    std::vector<double> f(raw.size());
    const int64_t n = lsmcpu_filter(raw.data(), n_raw, 0.5, 35.0, -1.0, 50.0, f.data());
    CHECK(n == 3000);
    f.resize(size_t(3 * n));
    CHECK(lsmcpu_filter(raw.data(), 0, 0.5, 35.0, -1.0, 50.0, f.data()) == 0);

    std::vector<double> v(f.size());
    const int64_t nv = lsmcpu_voxel(f.data(), n, 0.2, v.data());
    CHECK(nv > 0 && nv < n);
    CHECK(lsmcpu_voxel(f.data(), n, 0.0, v.data()) == -1);
    CHECK(lsmcpu_voxel(f.data(), n, 1e-300, v.data()) == -2);

    std::vector<double> nr(f.size());
    std::vector<int64_t> cnt(static_cast<size_t>(n));
    for (int max_nn : {300, 30, 1}) {
        CHECK(lsmcpu_normals(f.data(), n, 0.3, max_nn, nr.data(), cnt.data()) == 0);
        for (int64_t i = 0; i < n; ++i) {
            const double l = std::sqrt(nr[3 * i] * nr[3 * i] + nr[3 * i + 1] * nr[3 * i + 1] +
                                       nr[3 * i + 2] * nr[3 * i + 2]);
            CHECK(std::fabs(l - 1.0) < 1e-9);
            CHECK(cnt[size_t(i)] <= max_nn);
        }
    }
    CHECK(lsmcpu_normals(f.data(), n, 0.3, 300, nr.data(), cnt.data()) == 0);

    // the source: the target moved by a small known motion
    std::vector<double> src(f.size());
    const double c = std::cos(0.02), s = std::sin(0.02);
    for (int64_t i = 0; i < n; ++i) {
        const double x = f[3 * i], y = f[3 * i + 1], z = f[3 * i + 2];
        src[3 * i] = c * x - s * y + 0.05;
        src[3 * i + 1] = s * x + c * y - 0.03;
        src[3 * i + 2] = z + 0.01;
    }
    std::vector<int32_t> corr(static_cast<size_t>(n));
    for (int method : {0, 1}) {
        double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}, info[3];
        int it = 0;
        CHECK(lsmcpu_icp(src.data(), n, f.data(), n, nr.data(), 10.0, method, 30, 1e-6, 1e-6, T,
                         info, &it, corr.data()) == 0);
        CHECK(it >= 1 && it <= 30 && info[0] > 0.99);
        CHECK(std::fabs(T[3] + 0.05 * c - 0.03 * s) < 0.02);   // recovers the inverse motion
    }
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}, info[3];
    int it = 0;
    CHECK(lsmcpu_icp(src.data(), n, f.data(), 0, nullptr, 10.0, 0, 30, 1e-6, 1e-6, T, info, &it,
                     nullptr) == 0);   // empty target: no correspondences, identity updates
    CHECK(info[0] == 0.0 && info[2] == 0.0);
    CHECK(lsmcpu_icp(src.data(), n, f.data(), n, nullptr, 10.0, 1, 30, 1e-6, 1e-6, T, info, &it,
                     nullptr) == -1);  // P2Plane without target normals
    CHECK(lsmcpu_icp(src.data(), n, f.data(), n, nr.data(), 0.0, 1, 30, 1e-6, 1e-6, T, info, &it,
                     nullptr) == -1);  // invalid max_correspondence_distance

    std::vector<double> rel(16 * 5), glob(16 * 6);
    for (int k = 0; k < 5; ++k)
        for (int i = 0; i < 16; ++i) rel[size_t(16 * k + i)] = (i % 5 == 0) ? 1.0 : (i == 3 ? 0.5 * k : 0.0);
    CHECK(lsm_se3_prefix(rel.data(), 5, glob.data()) == 0);
    CHECK(std::fabs(glob[16 * 5 + 3] - 5.0) < 1e-12);
    CHECK(lsm_se3_prefix(nullptr, 0, glob.data()) == 0 && glob[0] == 1.0);
    CHECK(lsm_se3_prefix(rel.data(), -1, glob.data()) != 0);
    CHECK(lsm_se3_prefix(nullptr, 3, glob.data()) != 0);

    if (fails) {
        std::fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    std::printf("asan ok\n");
    return 0;
}
