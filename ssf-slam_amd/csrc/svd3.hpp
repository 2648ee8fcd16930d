// svd3.hpp -- 3x3 SVD by one-sided Jacobi in f64 (singular values descending, the LAPACK
// convention numpy's svd returns), shared by the Kabsch tail of k_mask_pose and the loop-closure
// ICP (Eigen::umeyama).  Same sweep as oracle/ssf_oracle.c orc_svd3.  Runs on one lane.
#pragma once
#include <hip/hip_runtime.h>

namespace ssf {

static __device__ __noinline__ void svd3(const double A[9], double U[9], double Sv[3], double Vt[9]) {
    double a[3][3], v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) a[i][j] = A[i * 3 + j];
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 3; ++i) { al += a[i][p] * a[i][p]; be += a[i][q] * a[i][q]; ga += a[i][p] * a[i][q]; }
                if (fabs(ga) <= 1e-300) continue;
                const double rel = fabs(ga) / sqrt(al * be);
                if (rel > off) off = rel;
                if (rel < 1e-17) continue;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 3; ++i) {
                    double x = a[i][p], y = a[i][q];
                    a[i][p] = c * x - s * y; a[i][q] = s * x + c * y;
                    x = v[i][p]; y = v[i][q];
                    v[i][p] = c * x - s * y; v[i][q] = s * x + c * y;
                }
            }
        if (off < 1e-16) break;
    }
    double sv[3];
    int ord[3] = {0, 1, 2};
    for (int j = 0; j < 3; ++j) sv[j] = sqrt(a[0][j] * a[0][j] + a[1][j] * a[1][j] + a[2][j] * a[2][j]);
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    double u[3][3];
    for (int k = 0; k < 3; ++k) {
        const int j = ord[k];
        Sv[k] = sv[j];
        for (int i = 0; i < 3; ++i) {
            u[i][k] = sv[j] > 0 ? a[i][j] / sv[j] : 0.0;
            Vt[k * 3 + i] = v[i][j];
        }
    }
    if (!(Sv[2] > 1e-12 * Sv[0])) {
        u[0][2] = u[1][0] * u[2][1] - u[2][0] * u[1][1];
        u[1][2] = u[2][0] * u[0][1] - u[0][0] * u[2][1];
        u[2][2] = u[0][0] * u[1][1] - u[1][0] * u[0][1];
        Vt[6] = Vt[1] * Vt[5] - Vt[2] * Vt[4];
        Vt[7] = Vt[2] * Vt[3] - Vt[0] * Vt[5];
        Vt[8] = Vt[0] * Vt[4] - Vt[1] * Vt[3];
    }
    for (int i = 0; i < 3; ++i) for (int k = 0; k < 3; ++k) U[i * 3 + k] = u[i][k];
}

}  // namespace ssf
