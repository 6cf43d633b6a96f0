// lsm_umeyama.h -- TransformationEstimationPointToPoint (with_scaling = false) on the device:
// the proper rotation maximising tr(R^T Sigma) (Umeyama / Kabsch) via Horn's quaternion, shared
// by the ICP solve (icp.hip) and the feature-RANSAC hypotheses (plane.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace lsm {

// Largest-eigenvalue eigenvector of a symmetric 4x4 (cyclic Jacobi).
__device__ inline void sym4_max_eigvec(double N[4][4], double v[4]) {
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 4; ++p)
            for (int q = p + 1; q < 4; ++q) off += N[p][q] * N[p][q];
        if (off < 1e-300) break;
        for (int p = 0; p < 4; ++p)
            for (int q = p + 1; q < 4; ++q) {
                if (N[p][q] == 0.0) continue;
                const double theta = (N[q][q] - N[p][p]) / (2.0 * N[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
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
    int best = 0;
    for (int k = 1; k < 4; ++k)
        if (N[k][k] > N[best][best]) best = k;
    for (int k = 0; k < 4; ++k) v[k] = V[k][best];
}

// Umeyama (with_scaling = false): the rotation maximising tr(R^T Sigma), via Horn's quaternion.
__device__ inline void umeyama_update(const double *tot, double D[16]) {
    const double n = tot[29];
    const double ms[3] = {tot[0] / n, tot[1] / n, tot[2] / n};
    const double mt[3] = {tot[3] / n, tot[4] / n, tot[5] / n};
    double H[3][3];  // H[a][b] = sum (s - ms)_a (t - mt)_b / n  (= Sigma^T)
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) H[a][b] = tot[6 + 3 * b + a] / n - mt[b] * ms[a];
    const double Sxx = H[0][0], Sxy = H[0][1], Sxz = H[0][2], Syx = H[1][0], Syy = H[1][1],
                 Syz = H[1][2], Szx = H[2][0], Szy = H[2][1], Szz = H[2][2];
    double N[4][4] = {{Sxx + Syy + Szz, Syz - Szy, Szx - Sxz, Sxy - Syx},
                      {Syz - Szy, Sxx - Syy - Szz, Sxy + Syx, Szx + Sxz},
                      {Szx - Sxz, Sxy + Syx, -Sxx + Syy - Szz, Syz + Szy},
                      {Sxy - Syx, Szx + Sxz, Syz + Szy, -Sxx - Syy + Szz}};
    double q[4];
    sym4_max_eigvec(N, q);
    const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double w = q[0] / qn, x = q[1] / qn, y = q[2] / qn, z = q[3] / qn;
    double R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w),     2 * (x * z + y * w),
                   2 * (x * y + z * w),     1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                   2 * (x * z - y * w),     2 * (y * z + x * w),     1 - 2 * (x * x + y * y)};
    for (int r = 0; r < 3; ++r) {
        D[4 * r + 0] = R[3 * r + 0];
        D[4 * r + 1] = R[3 * r + 1];
        D[4 * r + 2] = R[3 * r + 2];
        D[4 * r + 3] = mt[r] - (R[3 * r] * ms[0] + R[3 * r + 1] * ms[1] + R[3 * r + 2] * ms[2]);
    }
    D[12] = D[13] = D[14] = 0.0;
    D[15] = 1.0;
}


}  // namespace lsm
