/*
 * pn2_oracle.c -- CPU restatement of the point-set operators of the TFlow scene-flow network
 * (SURVEY.md §8(f) row 4).  TEST INFRASTRUCTURE ONLY: the checker for the HIP kernels in
 * ssf-slam_amd/csrc/pointnet2.hip; the product path never links it.
 *
 * The reference calls these operators through `lib.pointnet2_utils`, a CUDA extension that is
 * not vendored (scripts/ActiveSceneFlow/utils/utils.py:7).  This file restates the reference's
 * OWN torch versions of the same operators, which tests/golden/make_golden_pn2.py imports to
 * produce the golden vectors this oracle is pinned against (tests/test_oracle_pn2.py):
 *   orc_pn2_fps        utils/utils.py:68-89   farthest_point_sample
 *   orc_pn2_knn        utils/utils.py:92-108  knn_point (ties: lower index; topk leaves them open)
 *   orc_pn2_gather     utils/utils.py:48-65   index_points, on the [C, N] feature layout
 *   orc_pn2_interp3    utils/utils.py:658-663 weighted 3-NN sum
 *   orc_pn2_upsample   utils/soflow.py:1442-1470 UpsampleFlow.forward (soflow.py needs
 *                      torch_scatter, absent, so it is not imported: parity of the composition
 *                      is pinned through the golden script's restatement of :1454-1470 on top
 *                      of the imported knn_point / index_points)
 * One batch element per call; float arithmetic with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static float sq3(float dx, float dy, float dz) { return (dx * dx + dy * dy) + dz * dz; }

/* utils.py:68-89: centroid i = farthest; dist = sum((xyz - centroid)^2); distance = min;
 * farthest = argmax (first maximum).  temp: n floats of scratch. */
void orc_pn2_fps(const float* xyz, int64_t n, int32_t npoint, int32_t start, float* temp,
                 int32_t* out) {
    for (int64_t i = 0; i < n; ++i) temp[i] = 1e10f;                 /* :80 */
    int32_t far = start;
    for (int32_t it = 0; it < npoint; ++it) {
        out[it] = far;                                               /* :84 */
        const float cx = xyz[3 * far], cy = xyz[3 * far + 1], cz = xyz[3 * far + 2];
        float best = -1.0f;
        int32_t bi = 0;
        for (int64_t i = 0; i < n; ++i) {
            const float d = sq3(xyz[3 * i] - cx, xyz[3 * i + 1] - cy, xyz[3 * i + 2] - cz);
            if (d < temp[i]) temp[i] = d;                            /* :87-88 */
            if (temp[i] > best) { best = temp[i]; bi = (int32_t)i; } /* :89 first maximum */
        }
        far = bi;
    }
}

/* utils.py:92-108: k smallest squared distances of each query to the n reference points,
 * ascending (stable: equal distances keep index order), sqrt on output. */
void orc_pn2_knn(const float* query, int64_t s, const float* ref, int64_t n, int32_t k,
                 float* dist, int32_t* idx) {
    float bd[64];
    int32_t bi[64];
    for (int64_t q = 0; q < s; ++q) {
        const float qx = query[3 * q], qy = query[3 * q + 1], qz = query[3 * q + 2];
        int32_t cnt = 0;
        for (int64_t i = 0; i < n; ++i) {
            const float d = sq3(ref[3 * i] - qx, ref[3 * i + 1] - qy, ref[3 * i + 2] - qz);
            if (cnt == k && !(d < bd[k - 1])) continue;
            int32_t p = cnt < k ? cnt : k - 1;
            while (p > 0 && d < bd[p - 1]) { bd[p] = bd[p - 1]; bi[p] = bi[p - 1]; --p; }
            bd[p] = d; bi[p] = (int32_t)i;
            if (cnt < k) ++cnt;
        }
        for (int32_t j = 0; j < k; ++j) {
            dist[q * k + j] = j < cnt ? sqrtf(bd[j]) : 0.0f;
            idx[q * k + j] = j < cnt ? bi[j] : 0;
        }
    }
}

/* index_points on [C, N]: out[c, j] = feat[c, idx[j]] for g indices. */
void orc_pn2_gather(const float* feat, int32_t c, int64_t n, const int32_t* idx, int64_t g,
                    float* out) {
    for (int32_t ch = 0; ch < c; ++ch)
        for (int64_t j = 0; j < g; ++j) out[ch * g + j] = feat[ch * n + idx[j]];
}

/* utils.py:662-663: out[c, j] = (w0 f[i0] + w1 f[i1]) + w2 f[i2]. */
void orc_pn2_interp3(const float* feat, int32_t c, int64_t m, const int32_t* idx, const float* w,
                     int64_t n, float* out) {
    for (int32_t ch = 0; ch < c; ++ch)
        for (int64_t j = 0; j < n; ++j) {
            const float* F = feat + ch * m;
            out[ch * n + j] = (w[3 * j] * F[idx[3 * j]] + w[3 * j + 1] * F[idx[3 * j + 1]]) +
                              w[3 * j + 2] * F[idx[3 * j + 2]];
        }
}

/* soflow.py:1442-1470 for one batch element: xyz [3, n], sxyz [3, s], sfeat [c, s] -> out
 * [c, n].  k nearest sparse points per dense point (the knn above), dist = |sparse - xyz|
 * clamped at 1e-10, weights (1/d) / sum(1/d), weighted sum in neighbour order, clamp +-100. */
void orc_pn2_upsample(const float* xyz, int64_t n, const float* sxyz, int64_t s,
                      const float* sfeat, int32_t c, int32_t k, float* out) {
    float bd[64], w[64];
    int32_t bi[64];
    for (int64_t q = 0; q < n; ++q) {
        const float qx = xyz[q], qy = xyz[n + q], qz = xyz[2 * n + q];
        int32_t cnt = 0;
        for (int64_t i = 0; i < s; ++i) {
            const float d = sq3(sxyz[i] - qx, sxyz[s + i] - qy, sxyz[2 * s + i] - qz);
            if (cnt == k && !(d < bd[k - 1])) continue;
            int32_t p = cnt < k ? cnt : k - 1;
            while (p > 0 && d < bd[p - 1]) { bd[p] = bd[p - 1]; bi[p] = bi[p - 1]; --p; }
            bd[p] = d; bi[p] = (int32_t)i;
            if (cnt < k) ++cnt;
        }
        float norm = 0.0f;
        for (int32_t j = 0; j < cnt; ++j) {
            const int32_t i = bi[j];
            float d = sqrtf(sq3(sxyz[i] - qx, sxyz[s + i] - qy, sxyz[2 * s + i] - qz));
            if (!(d > 1e-10f)) d = 1e-10f;                           /* :1463 clamp */
            w[j] = 1.0f / d;
            norm = j == 0 ? w[j] : norm + w[j];                      /* :1464 */
        }
        for (int32_t j = 0; j < cnt; ++j) w[j] = w[j] / norm;        /* :1465 */
        for (int32_t ch = 0; ch < c; ++ch) {
            const float* F = sfeat + ch * s;
            float acc = 0.0f;
            for (int32_t j = 0; j < cnt; ++j) acc = j == 0 ? w[j] * F[bi[j]] : acc + w[j] * F[bi[j]];
            out[ch * n + q] = fminf(fmaxf(acc, -100.0f), 100.0f);    /* :1477 clamp */
        }
    }
}
