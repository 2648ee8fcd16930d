// kabsch_f32.hip -- slove_RT_by_SVD + Quaternion(matrix=R) on float32 arrays, the tail of the ASF
// block (scripts/ActiveSceneFlow/main_sju_occ_ros.py:273-284; slove_RT_by_SVD :455-473), on gfx950.
//
// The ASF node hands float32 network flow to the block, so numpy runs every line of the Kabsch in
// float32.  k_mask_pose computes its own tail in f64 (the reference's behaviour on
// float64 inputs); this kernel replaces it with the float32 arithmetic for callers that ask for it
// (ssf_kabsch_f32_batch), step by step as oracle/ssf_oracle.c orc_kabsch_f32 restates it:
//   target = points[bg] + move_gt[bg]   f32 add (:273)
//   src.mean(axis=0)                    numpy add.reduce over axis 0 of a C-ordered (n, 3) array:
//                                       row after row into the f32 accumulator, from the first
//                                       row; the count divide in f64, stored to f32 (_mean)
//   src - src_mean                      f32 (:461-462)
//   H = src.T @ dst                     sgemm (order unpinned): the exact f32 products summed in f64
//   svd, R = Vt.T @ U.T, det            f64 one-sided Jacobi (svd3.hpp), R rounded to f32
//   t = -R @ src_mean.T + dst_mean.T    the 3-term product rounded once to f32, then the f32 add
//   Quaternion(matrix=R)                allclose(dot(R, R^T), I) with the dot in f32, the trace
//                                       method's terms in f32, the 0.5 / sqrt(t) scale in f64
//
// One 256-thread work-group per frame.  The means are inherently serial (f32 rounding after every
// row), so the frame streams through LDS in 2048-point chunks (coalesced loads of the packed xyz)
// and lanes 0..5 of wave 0 walk each chunk in row order, one coordinate each; the H pass is an
// ordinary deterministic block reduction.  About 16 cycles per background row for the serial walk:
// ~60 us for the ASF's 8192-point frames; an opt-in tail, not on the LiDAR bench path.
#include "ssf_device.hpp"
#include "ssf_internal.hpp"
#include "svd3.hpp"

namespace ssf {

constexpr int kKT = 256;
constexpr int kKChunk = 2048;

__global__ __launch_bounds__(kKT) void k_kabsch_f32(const float* __restrict__ src,
                                                     const float* __restrict__ dst,
                                                     const float* __restrict__ flow,
                                                     const int64_t* __restrict__ off,
                                                     const uint8_t* __restrict__ mask,
                                                     int reflection, int keep_failures,
                                                     double* __restrict__ out_all) {
    __shared__ float tile[6][kKChunk];          // src x, y, z, dst x, y, z of one chunk (48 KB)
    __shared__ uint8_t keep[kKChunk];
    __shared__ double red[(kKT / 64) * 9];
    __shared__ float mean_s[6];
    __shared__ int cnt_s, skip_s;
    const int tid = threadIdx.x;
    const int f = blockIdx.x;
    const int64_t b = off[f], n = off[f + 1] - b;
    double* out = out_all + (size_t)f * SSF_POSE_OUT_STRIDE;
    if (tid == 0) {
        skip_s = 0;
        if (keep_failures) {    // after k_mask_pose: a failed fit (no labels) keeps its status
            const int st = (int)out[SSF_POSE_OUT_STATUS];
            skip_s = st == SSF_POSE_GMM_FAILED || st == SSF_POSE_SYNC_FAILED;
        } else {                // standalone: the fit fields are not this call's
            for (int i = 0; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
        }
    }
    __syncthreads();
    if (skip_s) return;

    // ---- the two means: serial f32 accumulation in row order (lanes 0..5 of wave 0) ----
    float acc = -0.0f;                          // -0 + v == v for every v: "start from row 0"
    int cnt = 0;
    const int col = tid < 6 ? tid : 0;
    for (int64_t c0 = 0; c0 < n; c0 += kKChunk) {
        const int m = (int)(n - c0 < kKChunk ? n - c0 : kKChunk);
        const int64_t base = 3 * (b + c0);
        for (int k = tid; k < 3 * m; k += kKT) {    // packed xyz: coalesced across the block
            const int j = k / 3, d = k - 3 * j;
            const float p = dst[base + k];
            tile[3 + d][j] = p;
            tile[d][j] = flow ? p + flow[base + k] : src[base + k];
        }
        for (int j = tid; j < m; j += kKT) keep[j] = mask ? mask[b + c0 + j] : (uint8_t)1;
        __syncthreads();
        if (tid < 6) {
            const float* cv = tile[col];
#pragma unroll 8
            for (int j = 0; j < m; ++j) {
                const float v = cv[j];
                const bool kj = keep[j] != 0;
                acc = kj ? acc + v : acc;
                cnt += kj ? 1 : 0;
            }
        }
        __syncthreads();
    }
    if (tid < 6) mean_s[tid] = (float)((double)acc / (double)(cnt > 0 ? cnt : 1));
    if (tid == 0) cnt_s = cnt;
    __syncthreads();
    const int nbg = cnt_s;
    float ms[3], md[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) { ms[d] = mean_s[d]; md[d] = mean_s[3 + d]; }

    // ---- H = (src - ms)^T (dst - md): exact f32 products, f64 sums --------------------------
    double h[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) h[k] = 0.0;
    for (int64_t j = tid; j < n; j += kKT) {
        if (mask && !mask[b + j]) continue;
        const int64_t i = 3 * (b + j);
        float a[3], c[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float p = dst[i + d];
            const float s = flow ? p + flow[i + d] : src[i + d];
            a[d] = s - ms[d];
            c[d] = p - md[d];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) h[r * 3 + q] += (double)a[r] * (double)c[q];
    }
    block_sum<9>(h, red);
    if (tid != 0) return;

    for (int i = 0; i < 7; ++i) out[i] = 0.0;
    for (int i = 0; i < 9; ++i) out[SSF_POSE_OUT_R + i] = 0.0;
    out[SSF_POSE_OUT_NBG] = (double)nbg;
    if (nbg == 0) { out[SSF_POSE_OUT_STATUS] = SSF_POSE_EMPTY; return; }
    double U[9], Sv[3], Vt[9], R[9];
    svd3(h, U, Sv, Vt);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int j = 0; j < 3; ++j) s += Vt[j * 3 + r] * U[c * 3 + j];
            R[r * 3 + c] = s;
        }
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    int status = 0;
    if (det < 0) {
        if (!reflection) status = SSF_POSE_REFLECTION;
        for (int j = 0; j < 3; ++j) Vt[6 + j] *= -1.0;
        if (reflection)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    double s = 0.0;
                    for (int j = 0; j < 3; ++j) s += Vt[j * 3 + r] * U[c * 3 + j];
                    R[r * 3 + c] = s;
                }
    }
    float R32[9], t32[3];
    for (int k = 0; k < 9; ++k) R32[k] = (float)R[k];
    for (int r = 0; r < 3; ++r) {
        const double dot = (double)R32[r * 3] * (double)ms[0] + (double)R32[r * 3 + 1] * (double)ms[1] +
                           (double)R32[r * 3 + 2] * (double)ms[2];
        t32[r] = (float)(-dot) + md[r];
    }
    for (int k = 0; k < 9; ++k) out[SSF_POSE_OUT_R + k] = (double)R32[k];
    for (int r = 0; r < 3; ++r) out[SSF_POSE_OUT_T + r] = (double)t32[r];
    if (status == 0) {
        bool orth = true;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const float s = (R32[i * 3] * R32[j * 3] + R32[i * 3 + 1] * R32[j * 3 + 1]) +
                                R32[i * 3 + 2] * R32[j * 3 + 2];
                const double e = (i == j) ? 1.0 : 0.0;
                if (!(fabs((double)s - e) <= 1e-8 + 1e-5 * fabs(e))) orth = false;
            }
        if (!orth) {
            status = SSF_POSE_NOT_ORTHOGONAL;
        } else {
            float m[3][3];
            for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) m[i][j] = R32[j * 3 + i];
            float tt, w, x, y, z;
            if (m[2][2] < 0) {
                if (m[0][0] > m[1][1]) {
                    tt = ((1.0f + m[0][0]) - m[1][1]) - m[2][2];
                    w = m[1][2] - m[2][1]; x = tt; y = m[0][1] + m[1][0]; z = m[2][0] + m[0][2];
                } else {
                    tt = ((1.0f - m[0][0]) + m[1][1]) - m[2][2];
                    w = m[2][0] - m[0][2]; x = m[0][1] + m[1][0]; y = tt; z = m[1][2] + m[2][1];
                }
            } else {
                if (m[0][0] < -m[1][1]) {
                    tt = ((1.0f - m[0][0]) - m[1][1]) + m[2][2];
                    w = m[0][1] - m[1][0]; x = m[2][0] + m[0][2]; y = m[1][2] + m[2][1]; z = tt;
                } else {
                    tt = ((1.0f + m[0][0]) + m[1][1]) + m[2][2];
                    w = tt; x = m[1][2] - m[2][1]; y = m[2][0] - m[0][2]; z = m[0][1] - m[1][0];
                }
            }
            const double fq = 0.5 / sqrt((double)tt);
            out[SSF_POSE_OUT_Q + 0] = (double)x * fq;
            out[SSF_POSE_OUT_Q + 1] = (double)y * fq;
            out[SSF_POSE_OUT_Q + 2] = (double)z * fq;
            out[SSF_POSE_OUT_Q + 3] = (double)w * fq;
        }
    }
    out[SSF_POSE_OUT_STATUS] = status;
}

hipError_t launch_kabsch_f32(hipStream_t s, int n_frames, const float* src, const float* dst,
                             const float* flow, const int64_t* frame_off, const uint8_t* mask,
                             int reflection, int keep_failures, double* out) {
    if (n_frames <= 0) return hipSuccess;
    kmark(s, "k_kabsch_f32");
    hipLaunchKernelGGL(k_kabsch_f32, dim3(n_frames), dim3(kKT), 0, s, src, dst, flow, frame_off, mask,
                       reflection, keep_failures, out);
    return hipGetLastError();
}

}  // namespace ssf
