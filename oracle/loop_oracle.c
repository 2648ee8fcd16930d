/* loop_oracle.c -- CPU restatement of the mapOptmization loop-closure registration
 * (SURVEY.md §8(f) row 3): pcl::VoxelGrid<PointXYZI> and
 * pcl::IterativeClosestPoint<PointXYZI, PointXYZI> as src/mapOptmization.cpp:201-236 uses them
 * (leaf 0.1 m; max correspondence distance 50 m, 100 iterations, transformation epsilon 1e-6,
 * Euclidean fitness epsilon 1e-6, no RANSAC).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, the checker).  PCL is not on this filesystem, so the
 * restatement follows the published PCL 1.10 algorithms (VoxelGrid::applyFilter,
 * IterativeClosestPoint::computeTransformation, CorrespondenceEstimation::
 * determineCorrespondences, TransformationEstimationSVD with Eigen::umeyama,
 * DefaultConvergenceCriteria::hasConverged, Registration::getFitnessScore): PARITY UNPINNED
 * against the reference binary.  Stated deviations:
 *   - VoxelGrid sorts (voxel, point) pairs with std::sort (not stable): the float centroid sum
 *     order inside a voxel is implementation-defined there; here it is the input order.
 *   - KdTreeFLANN tie order: ties go to the lower target index.
 *   - umeyama in float with Eigen's vectorised reductions: here the means and the 3x3
 *     cross-covariance are accumulated in double in index order and the 3x3 SVD is f64 Jacobi;
 *     R and t are then rounded to float, as PCL's Matrix4f holds them.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ssf_oracle.h"

typedef struct { int64_t key; int64_t idx; } vg_pair;

static int vg_cmp(const void* a, const void* b) {
    const vg_pair* x = (const vg_pair*)a;
    const vg_pair* y = (const vg_pair*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.10 voxel_grid.hpp), downsample_all_data = true,
 * min_points_per_voxel = 0, no field filter; all input points finite. */
int64_t orc_voxel_grid(const float* xyzi, int64_t n, float leaf, float* out) {
    if (n <= 0) return 0;
    const float inv = 1.0f / leaf;                       /* inverse_leaf_size_ (Array4f) */
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = 0; i < n; ++i)                      /* getMinMax3D */
        for (int d = 0; d < 3; ++d) {
            const float v = xyzi[4 * i + d];
            if (v < mn[d]) mn[d] = v;
            if (v > mx[d]) mx[d] = v;
        }
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)INT32_MAX) {             /* "leaf size too small": input out */
        memcpy(out, xyzi, sizeof(float) * 4 * (size_t)n);
        return n;
    }
    int minb[3], maxb[3], divb[3], mul[3];
    for (int d = 0; d < 3; ++d) {
        minb[d] = (int)floorf(mn[d] * inv);
        maxb[d] = (int)floorf(mx[d] * inv);
        divb[d] = maxb[d] - minb[d] + 1;
    }
    mul[0] = 1; mul[1] = divb[0]; mul[2] = divb[0] * divb[1];
    vg_pair* pr = (vg_pair*)malloc(sizeof(vg_pair) * (size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        int64_t key = 0;
        for (int d = 0; d < 3; ++d) key += (int64_t)((int)floorf(xyzi[4 * i + d] * inv) - minb[d]) * mul[d];
        pr[i].key = key; pr[i].idx = i;
    }
    qsort(pr, (size_t)n, sizeof(vg_pair), vg_cmp);
    int64_t m = 0;
    for (int64_t a = 0; a < n;) {
        int64_t b = a;
        while (b < n && pr[b].key == pr[a].key) ++b;
        float c[4] = {0.f, 0.f, 0.f, 0.f};
        for (int64_t k = a; k < b; ++k)
            for (int f = 0; f < 4; ++f) c[f] += xyzi[4 * pr[k].idx + f];
        for (int f = 0; f < 4; ++f) out[4 * m + f] = c[f] / (float)(b - a);
        ++m;
        a = b;
    }
    free(pr);
    return m;
}

/* Eigen Matrix4f * point (pcl::transformPointCloud): x' = ((r00 x + r01 y) + r02 z) + t0 */
static void tf_point(const float T[16], const float* p, float* o) {
    for (int r = 0; r < 3; ++r) o[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}

/* A * B for row-major 4x4 float, Eigen lazy-product order ((a0 b0 + a1 b1) + a2 b2) + a3 b3 */
static void mat4_mul(const float A[16], const float B[16], float O[16]) {
    float t[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            t[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) + A[4 * i + 3] * B[12 + j];
    memcpy(O, t, sizeof(t));
}

/* exact 1-NN, FLANN L2_Simple float distance ((dx^2 + dy^2) + dz^2), ties to the lower index */
static int64_t nn1(const float* tgt, int64_t nt, const float* q, float* d2) {
    int64_t bi = -1;
    float bd = INFINITY;
    for (int64_t j = 0; j < nt; ++j) {
        const float dx = q[0] - tgt[4 * j], dy = q[1] - tgt[4 * j + 1], dz = q[2] - tgt[4 * j + 2];
        float d = dx * dx + dy * dy;
        d = d + dz * dz;
        if (d < bd) { bd = d; bi = j; }
    }
    *d2 = bd;
    return bi;
}

/* Eigen::umeyama(src, dst, false) on the correspondences: sigma = (dst - dm)(src - sm)^T / n,
 * R = U diag(1, 1, det(U)det(V) < 0 ? -1 : 1) V^T, t = dm - R sm. */
static void umeyama(const float* src, const float* tgt, const int64_t* qi, const int64_t* mi, int64_t c,
                    float T[16]) {
    double sm[3] = {0, 0, 0}, dm[3] = {0, 0, 0};
    for (int64_t k = 0; k < c; ++k)
        for (int d = 0; d < 3; ++d) { sm[d] += src[4 * qi[k] + d]; dm[d] += tgt[4 * mi[k] + d]; }
    for (int d = 0; d < 3; ++d) { sm[d] /= (double)c; dm[d] /= (double)c; }
    double H[9] = {0};
    for (int64_t k = 0; k < c; ++k) {
        double s[3], t[3];
        for (int d = 0; d < 3; ++d) { s[d] = src[4 * qi[k] + d] - sm[d]; t[d] = tgt[4 * mi[k] + d] - dm[d]; }
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) H[3 * r + q] += t[r] * s[q];
    }
    for (int k = 0; k < 9; ++k) H[k] /= (double)c;
    double U[9], S[3], Vt[9];
    orc_svd3(H, U, S, Vt);
    const double du = U[0] * (U[4] * U[8] - U[5] * U[7]) - U[1] * (U[3] * U[8] - U[5] * U[6]) + U[2] * (U[3] * U[7] - U[4] * U[6]);
    const double dv = Vt[0] * (Vt[4] * Vt[8] - Vt[5] * Vt[7]) - Vt[1] * (Vt[3] * Vt[8] - Vt[5] * Vt[6]) + Vt[2] * (Vt[3] * Vt[7] - Vt[4] * Vt[6]);
    const double s3 = du * dv < 0 ? -1.0 : 1.0;
    double R[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            R[3 * r + q] = U[3 * r] * Vt[q] + U[3 * r + 1] * Vt[3 + q] + s3 * U[3 * r + 2] * Vt[6 + q];
    memset(T, 0, sizeof(float) * 16);
    for (int r = 0; r < 3; ++r) {
        for (int q = 0; q < 3; ++q) T[4 * r + q] = (float)R[3 * r + q];
        T[4 * r + 3] = (float)(dm[r] - (R[3 * r] * sm[0] + R[3 * r + 1] * sm[1] + R[3 * r + 2] * sm[2]));
    }
    T[15] = 1.0f;
}

/* pcl::IterativeClosestPoint::computeTransformation + DefaultConvergenceCriteria (PCL 1.10)
 * + getFitnessScore(DBL_MAX).  src / tgt are n x 4 (x, y, z, intensity). */
int32_t orc_icp(const float* src, int64_t ns, const float* tgt, int64_t nt, const orc_icp_params* p,
                const float guess[16], orc_icp_result* r) {
    float* cur = (float*)malloc(sizeof(float) * 4 * (size_t)(ns > 0 ? ns : 1));
    int64_t* qi = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ns > 0 ? ns : 1));
    int64_t* mi = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ns > 0 ? ns : 1));
    float fin[16], inc[16];
    memcpy(fin, guess, sizeof(fin));
    for (int64_t i = 0; i < ns; ++i) { tf_point(guess, src + 4 * i, cur + 4 * i); cur[4 * i + 3] = src[4 * i + 3]; }
    const double max_d2 = (double)p->max_corr_dist * (double)p->max_corr_dist;
    const double rot_thr = 1.0 - p->trans_eps, trans_thr = p->trans_eps;
    double prev_mse = DBL_MAX;
    int32_t it = 0, converged = 0, state = ORC_ICP_NOT_CONVERGED, similar = 0;
    int64_t c = 0;
    while (1) {
        c = 0;
        double mse = 0.0;
        for (int64_t i = 0; i < ns; ++i) {                     /* determineCorrespondences */
            float d2;
            const int64_t j = nn1(tgt, nt, cur + 4 * i, &d2);
            if (j < 0 || (double)d2 > max_d2) continue;
            qi[c] = i; mi[c] = j; ++c;
            mse += (double)d2;
        }
        if (c < 3) { state = ORC_ICP_NO_CORRESPONDENCES; converged = 0; break; }
        umeyama(cur, tgt, qi, mi, c, inc);
        for (int64_t i = 0; i < ns; ++i) {                     /* transformCloud (in place) */
            float o[3];
            tf_point(inc, cur + 4 * i, o);
            cur[4 * i] = o[0]; cur[4 * i + 1] = o[1]; cur[4 * i + 2] = o[2];
        }
        mat4_mul(inc, fin, fin);
        ++it;
        /* DefaultConvergenceCriteria::hasConverged (max_iterations_similar_transforms_ = 0) */
        if (it >= p->max_iter) { state = ORC_ICP_ITERATIONS; converged = 1; break; }
        const double cos_a = 0.5 * ((double)inc[0] + (double)inc[5] + (double)inc[10] - 1.0);
        const double tr2 = (double)inc[3] * inc[3] + (double)inc[7] * inc[7] + (double)inc[11] * inc[11];
        if (cos_a >= rot_thr && tr2 <= trans_thr) { state = ORC_ICP_TRANSFORM; converged = 1; break; }
        mse /= (double)c;
        if (fabs(mse - prev_mse) < 1e-12) { state = ORC_ICP_ABS_MSE; converged = 1; break; }
        if (fabs(mse - prev_mse) / prev_mse < p->fit_eps) { state = ORC_ICP_REL_MSE; converged = 1; break; }
        (void)similar;
        prev_mse = mse;
    }
    /* getFitnessScore(): the ORIGINAL source through the final transform, mean 1-NN d2 */
    double fit = 0.0;
    int64_t nr = 0;
    for (int64_t i = 0; i < ns; ++i) {
        float q[3], d2;
        tf_point(fin, src + 4 * i, q);
        if (nn1(tgt, nt, q, &d2) >= 0) { fit += d2; ++nr; }
    }
    memcpy(r->T, fin, sizeof(fin));
    r->fitness = nr > 0 ? fit / (double)nr : DBL_MAX;
    r->converged = converged;
    r->iterations = it;
    r->state = state;
    r->n_corr = (int32_t)c;
    free(cur); free(qi); free(mi);
    return 0;
}
