// se3_host.cpp -- host-only SE(3) helpers of liblidarsm (no HIP): the serial pose prefix product
// of compute_global_transformations (artelib/homogeneousmatrix.py:184-205). Kept apart from
// api.cpp so the sanitizer build (tests/asan/Makefile) compiles it with plain g++.
#include "../../include/lidarsm.h"

extern "C" int lsm_se3_prefix(const double *rel, int64_t n, double *out) {
    if (n < 0 || !out || (n > 0 && !rel)) return LSM_EINVAL;
    for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int64_t k = 0; k < n; ++k) {
        const double *A = out + 16 * k, *B = rel + 16 * k;
        double *C = out + 16 * (k + 1);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                C[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) +
                               A[4 * i + 3] * B[12 + j];
    }
    return LSM_OK;
}
