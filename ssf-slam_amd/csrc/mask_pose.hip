// mask_pose.hip -- the dynamic-point mask + Kabsch pose block of
// scripts/PointCloudOdometry_noSeg.py:97-125 (and PointCloudOdometry.py:91-101) on gfx950.
//
// One work-group owns one frame and runs the WHOLE GaussianMixture(n_components=2).fit_predict
// on device (sklearn 1.7.2 semantics, f64 arithmetic on the f32 point / flow storage):
//   pass 0      X = [flow, xyz]: column means and variances (KMeans centering, tol)
//   k-means++   distances to the first centre (index chosen from the caller's RandomState
//               draw), in-order chunked prefix scan -> the two local-trial candidates, potentials
//   Lloyd       one streaming pass per iteration (labels, per-cluster sums, changed-label count)
//   GMM init    one-hot responsibilities -> shifted first/second moments -> 6x6 Cholesky
//   EM          ONE fused pass per iteration: E-step (log-prob difference of the two components,
//               responsibilities) and the M-step moment sums of the next parameters together
//   final       argmax labels + per-label Kabsch sums (src = pos + flow, dst = pos) in one pass,
//               background = majority label, 3x3 SVD (one-sided Jacobi, f64) on one lane,
//               R, t, pyquaternion trace-method q; then one pass writes the uint8 mask.
// The small dense algebra runs between passes: the two components' Cholesky / difference form on
// lanes 0 and 1 in registers (gmm_params2), the SVD and convergence tests on lane 0;
// no host round trip for the whole fit.  Every pass is a coalesced stream of 24 B/point.
#include "ssf_device.hpp"
#include "ssf_internal.hpp"
#include "svd3.hpp"

#include <float.h>
#include <type_traits>

namespace ssf {

#ifndef SSF_MASK_THREADS
#define SSF_MASK_THREADS 768
#endif
constexpr int kMaskThreads = SSF_MASK_THREADS;   // 12 waves: 3 per SIMD at <= 168 VGPRs

// Diagnostic build only (-DSSF_MASK_STAMPS, libssf_frontend_diag.so): lane 0 records the
// s_memtime cycle count at each phase boundary into the frame's unused out slots 26..31.
// The product library is compiled without it; no product output is computed from a stamp.
#ifdef SSF_MASK_STAMPS
#define SSF_STAMP(slot)                                                                   \
    do {                                                                                  \
        if (threadIdx.x == 0) {                                                           \
            const unsigned long long _t = __builtin_amdgcn_s_memtime();                   \
            out[26 + (slot)] = (double)(_t - stamp0);                                     \
        }                                                                                 \
    } while (0)
#else
#define SSF_STAMP(slot) do { } while (0)
#endif
constexpr int kNW = kMaskThreads / 64;
#ifndef SSF_LLOYD_DEEP
#define SSF_LLOYD_DEEP 2
#endif
constexpr int kLloydDeep = SSF_LLOYD_DEEP;   // points in flight per thread in the Lloyd passes
#ifndef SSF_KPP_DEEP
#define SSF_KPP_DEEP 2
#endif
constexpr int kKppBlocks = 4096;             // k-means++ block totals in LDS (frames up to ~262k points)
constexpr double kPi = 3.14159265358979323846;
#ifndef SSF_LLOYD_FULL_PASSES
#define SSF_LLOYD_FULL_PASSES 4
#endif
constexpr int kLloydFullPasses = SSF_LLOYD_FULL_PASSES;   // full Lloyd passes before skipping
#ifndef SSF_LLOYD_REFULL
#define SSF_LLOYD_REFULL 4
#endif
constexpr int kLloydRefull = SSF_LLOYD_REFULL;   // back to a full pass when > n / this relabel
#ifndef SSF_LLOYD_REC_DEEP
#define SSF_LLOYD_REC_DEEP 8
#endif
constexpr int kLloydRecDeep = SSF_LLOYD_REC_DEEP;         // 16-byte record loads in flight per lane
constexpr int kLQ = SSF_LLOYD_REC_DEEP * 128;   // a record trip: D loads of two records per lane
constexpr int kLloydMax = 300;               // sklearn KMeans max_iter (pass index fits 9 bits)

// packed upper-triangular index of a 6x6 matrix (row i <= col j)
SSF_DEV constexpr int up(int i, int j) { return i * 6 - (i * (i - 1)) / 2 + (j - i); }

// Everything lane 0 touches between passes lives here, in LDS: no private arrays, so the
// streaming passes keep the whole VGPR budget (1024 threads -> <= 128 VGPRs per lane).
struct MaskShared {
    double mean[6], tol;
    double tot[28];            // {N, sum(x-mean)[6], sum(x-mean)(x-mean)^T [21 packed]}
    double cen[12], csn[2], cenp[12], csnp[2];   // current / previous Lloyd centres
    double x0[6], ktot[16];    // pass-0 shift (point 0) and total Kabsch sums about it
    double mu[12], U[42], logdet[2], logw[2];  // U: packed upper precision Cholesky per component
    double Aq[21], bq[6], cq, C0;  // EM difference form: delta = a1 - a0 = v'A v + b'v + c (v = x - mean)
    double rand1, rand2;
    double lb;
    double C[36], L[36], Li[36];  // lane-0 scratch for the 6x6 algebra
    double sums[29];           // lane 0's copy of a pass's block sums (never a per-lane array)
    double lsum[14];           // running Lloyd cluster sums {n0, S0[6], n1, S1[6]} about mean
    double lhist[kLloydMax * 9];   // per labelling pass t: w = c1 - c0 [6], s = csn0 - csn1,
                                   // |c0| + |c1|, csn0 + csn1 (lloyd_skip_bounds)
    float lb1[512], lb2[512];   // this pass's drift bounds against pass r (9-bit index)
    int64_t c0, c1;
    double dg_cyc, dg_n, dg_lab, dg_wfull, dg_full1;   // diagnostic build only
#ifdef SSF_MASK_STAMPS
    double dg_e[3];            // EM pass: points + block sum, exchange, M-step (cycles, summed)
#endif
    double passes;             // algorithmic bytes / (24 B x n): 1 per full pass (see the Lloyd loop)
    int km_iter, em_iter, strict, converged, done, status, label0, bg, bg_pred, lfull;
    double hnk[2], hq[2], hpm[12];   // gmm_params2: per-component results of lanes 0 / 1
    int hrc[2];
};

// T: the storage type of pos / flow (float: LiDAR data; double: the f64 Python boundary).
template <class T>
SSF_DEV void load_x(const T* __restrict__ P, const T* __restrict__ Fl, int64_t i, double x[6]) {
    x[0] = (double)Fl[3 * i]; x[1] = (double)Fl[3 * i + 1]; x[2] = (double)Fl[3 * i + 2];
    x[3] = (double)P[3 * i];  x[4] = (double)P[3 * i + 1];  x[5] = (double)P[3 * i + 2];
}

// The E-step in difference form (gmm_params2).  With P_k = U_k U_k^T, v = x - s (s = S.mean) and
// m_k = mu_k - s, sklearn's weighted log-probabilities a_k = -0.5 (v - m_k)' P_k (v - m_k) + K_k,
// K_k = -3 log(2 pi) + logdet_k + logw_k, differ by the quadratic
//     delta = a1 - a0 = v' A v + b' v + c,   A = -0.5 (P1 - P0),  b = P1 m1 - P0 m0,
//     c = -0.5 (m1' P1 m1 - m0' P0 m0) + K1 - K0,
// which is all the per-point work needs: resp1 = sigmoid(delta), argmax = [delta > 0], and
// logsumexp(a0, a1) = a0 + max(delta, 0) + log1p(exp(-|delta|)).  The a0 part of the lower bound
// is summed over the frame from the pass-0 moments about s (S.tot = {N, M1, M2}):
//     sum_i a0_i = N K0 - 0.5 (tr(P0 M2) - 2 m0' P0 M1 + N m0' P0 m0).
// Aq is packed upper with the off-diagonal entries doubled (v'Av = sum_j v_j sum_{k>=j} Aq_jk v_k).

// ---- the M-step algebra on two lanes -------------------------------------------------------
// sklearn _estimate_gaussian_parameters + _compute_precision_cholesky + the difference form
// above, between passes: component k on lane k of wave 0 (both lanes run one instruction
// stream, so two components cost one) with every 6x6 quantity in registers (fully unrolled).
// Round 2 ran the same operations in the same order on lane 0 over LDS arrays, element by
// element (40-53 k cycles per EM pass); the outputs are bit-identical to that version on a
// 256-frame batch (every output double, every mask byte), and the launch is 4 % shorter.

// C (6x6, row-major) -> precision Cholesky, packed upper U, and its log det: scipy
// linalg.cholesky(lower) + solve_triangular(L, I).T as sklearn _compute_precision_cholesky.
SSF_DEV int prec_chol6_r(const double (&C)[36], double (&U)[21], double& logdet) {
    double L[36], Li[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) { L[k] = 0.0; Li[k] = 0.0; }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double s = C[j * 6 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
        ok = ok && (s > 0.0);
        L[j * 6 + j] = sqrt(s);
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double v = C[i * 6 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = v / L[j * 6 + j];
        }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c)
#pragma unroll
        for (int i = c; i < 6; ++i) {
            double v = (i == c) ? 1.0 : 0.0;
#pragma unroll
            for (int k = c; k < i; ++k) v -= L[i * 6 + k] * Li[k * 6 + c];
            Li[i * 6 + c] = v / L[i * 6 + i];
        }
    double ld = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 6; ++j) U[up(i, j)] = Li[j * 6 + i];
#pragma unroll
    for (int i = 0; i < 6; ++i) ld += log(Li[i * 6 + i]);
    logdet = ld;
    return ok ? 0 : -1;
}

// Lanes 0 and 1 of wave 0 (lane k: component k): the M-step and the difference form.  Returns, in lane 0,
// -1 when a covariance is not positive definite (the parameters are then left as they were).
__device__ __noinline__ int gmm_params2(MaskShared& S, const double* comp1, int init, int64_t n) {
    const int k = (int)(threadIdx.x & 1u);
    const double eps10 = 10.0 * DBL_EPSILON;
    double a[28];
#pragma unroll
    for (int i = 0; i < 28; ++i) a[i] = k == 1 ? comp1[i] : S.tot[i] - comp1[i];
    const double nk = a[0] + eps10;
    double d[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double mu = (a[0] * S.mean[i] + a[1 + i]) / nk;
        d[i] = mu - S.mean[i];
        S.hpm[6 * k + i] = mu;        // staged: S.mu is only updated when both components are valid
    }
    double C[36];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 6; ++j) {
            double v = a[7 + up(i, j)] - a[1 + i] * d[j] - d[i] * a[1 + j] + a[0] * d[i] * d[j];
            v = v / nk;
            C[i * 6 + j] = v; C[j * 6 + i] = v;
        }
#pragma unroll
    for (int i = 0; i < 6; ++i) C[i * 6 + i] += 1e-6;
    double U[21], ld;
    const int rc = prec_chol6_r(C, U, ld);
    // em_diff_form, per component: P_k = U_k U_k', m_k = mu_k - s (= d), P_k m_k, m_k' P_k m_k
    double P[36];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) {
            double v = 0.0;
#pragma unroll
            for (int j = c; j < 6; ++j) v += U[up(r, j)] * U[up(c, j)];
            P[r * 6 + c] = v; P[c * 6 + r] = v;
        }
    double q = 0.0, Pm[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) v += P[r * 6 + c] * d[c];
        Pm[r] = v;
        q += d[r] * v;
    }
    S.hnk[k] = nk; S.hq[k] = q; S.hrc[k] = rc;
    __builtin_amdgcn_wave_barrier();
    const bool ok = S.hrc[0] == 0 && S.hrc[1] == 0;
    if (ok) {                                   // both lanes: their component's parameters
#pragma unroll
        for (int i = 0; i < 6; ++i) S.mu[6 * k + i] = S.hpm[6 * k + i];
#pragma unroll
        for (int i = 0; i < 21; ++i) S.U[21 * k + i] = U[i];
        S.logdet[k] = ld;
        double* Pk = k ? S.L : S.C;             // P1 / P0 as em_diff_form keeps them
#pragma unroll
        for (int i = 0; i < 36; ++i) Pk[i] = P[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) S.hpm[6 * k + i] = Pm[i];
    }
    __builtin_amdgcn_wave_barrier();
    if (k != 0) return 0;
    if (!ok) return -1;
    // lane 0: weights, then the difference form from both components
    const double nk0 = S.hnk[0], nk1 = S.hnk[1];
    double w0, w1;
    if (init) { w0 = nk0 / (double)n; w1 = nk1 / (double)n; }
    else { const double sw = nk0 + nk1; w0 = nk0 / sw; w1 = nk1 / sw; }
    S.logw[0] = log(w0); S.logw[1] = log(w1);
    const double* P0 = S.C;
    const double* P1 = S.L;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const double A = -0.5 * (P1[r * 6 + c] - P0[r * 6 + c]);
            S.Aq[up(r, c)] = r == c ? A : 2.0 * A;
        }
        S.bq[r] = S.hpm[6 + r] - S.hpm[r];
    }
    S.cq = -0.5 * (S.hq[1] - S.hq[0]) + (S.logdet[1] + S.logw[1]) - (S.logdet[0] + S.logw[0]);
    const double N = S.tot[0];
    double tr = 0.0, lin = 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        lin += S.hpm[r] * S.tot[1 + r];
#pragma unroll
        for (int c = 0; c < 6; ++c) tr += P0[r * 6 + c] * S.tot[7 + (r <= c ? up(r, c) : up(c, r))];
    }
    const double K0 = -3.0 * log(2.0 * kPi) + S.logdet[0] + S.logw[0];
    S.C0 = N * K0 - 0.5 * (tr - 2.0 * lin + N * S.hq[0]);
    return 0;
}

typedef __attribute__((address_space(3))) const double LdsDouble;

// The LDS address of the E-step parameters laundered through a VGPR once per point: the compiler can neither
// hoist the 27 loop-invariant doubles into VGPRs nor has to rebuild each address in an SGPR
// (one VGPR base, immediate ds_read2 offsets).  The low 32 bits of a generic LDS pointer are
// its LDS offset.
SSF_DEV const LdsDouble* lds_laundered(const double* p) {
    uint32_t a = (uint32_t)(uintptr_t)p;
    asm volatile("" : "+v"(a));
    return (const LdsDouble*)(uintptr_t)a;
}

// delta = v'A v + b'v + c (em_diff_form) for two points at once: every Aq / bq read from LDS
// serves both.
template <class Ptr>
SSF_DEV void em_delta2(const double va[6], const double vb[6], Ptr Aq, Ptr bq, double cq,
                       double& da, double& db) {
    da = cq; db = cq;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double ta = bq[j], tb = ta;
#pragma unroll
        for (int k = j; k < 6; ++k) { const double a = Aq[up(j, k)]; ta += a * va[k]; tb += a * vb[k]; }
        da += va[j] * ta; db += vb[j] * tb;
    }
}

template <class Ptr>
SSF_DEV double em_delta1(const double v[6], Ptr Aq, Ptr bq, double cq) {
    double d = cq;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double t = bq[j];
#pragma unroll
        for (int k = j; k < 6; ++k) t += Aq[up(j, k)] * v[k];
        d += v[j] * t;
    }
    return d;
}

// Streams the frame's points through f(i, x): every thread keeps the NEXT point's loads in
// flight (as the raw six floats, converted when used) while it computes the current one.
template <class T>
SSF_DEV void load_raw(const T* __restrict__ P, const T* __restrict__ Fl, int64_t i, T r[6]) {
    r[0] = Fl[3 * i]; r[1] = Fl[3 * i + 1]; r[2] = Fl[3 * i + 2];
    r[3] = P[3 * i];  r[4] = P[3 * i + 1];  r[5] = P[3 * i + 2];
}

#ifndef SSF_EM_OFF32
#define SSF_EM_OFF32 1                           // EM / Lloyd loads: 32-bit byte offsets from the part's base (A/B: 0)
#endif
// three consecutive Ts at byte offset o (< 2^32) of a wave-uniform base: the global_load's SGPR
// base + 32-bit VGPR offset form, so the clamped index costs a min and a multiply per point
// instead of 64-bit compares, selects and address arithmetic
template <class Ts>
SSF_DEV void load3_off(const Ts* __restrict__ base, uint32_t o, Ts r[3]) {
    const Ts* p = reinterpret_cast<const Ts*>(reinterpret_cast<const char*>(base) + o);
    r[0] = p[0]; r[1] = p[1]; r[2] = p[2];
}
// Points [r0, r1) of the frame (the work-group's part, see Split).
template <class Ts, class Fn>
SSF_DEV void for_points(const Ts* __restrict__ P, const Ts* __restrict__ Fl, int64_t r0, int64_t r1, Fn&& fn) {
    const int64_t T = blockDim.x;
    int64_t i = r0 + threadIdx.x;
    if (i >= r1) return;
    Ts rn[6];
    load_raw(P, Fl, i, rn);
    for (; i < r1; i += T) {
        double x[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) x[d] = (double)rn[d];
        load_raw(P, Fl, min(i + T, r1 - 1), rn);    // unconditional (clamped): a counted wait
        fn(i, x);
    }
}

// A wave-uniform LDS value moved to SGPRs: the per-point loops keep their VGPRs for the point
// data and the accumulators (1024-thread work-groups leave 128 VGPRs per lane).
SSF_DEV double uni(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}

// Lloyd only: D points in flight per thread (a rolling register buffer of raw floats).  Each
// thread visits its points in the same order as for_points, so every sum is bit-identical.
// fn(i, x, val) runs for every slot of the last trip too (val = false past r1, x = the clamped
// last point): a store under a branch in a streaming loop made the compiler drain the prefetches
// at the join (the record-writing full pass took 411 k cycles against 264 k without records).
template <int D, class Ts, class Fn>
SSF_DEV void for_points_deep(const Ts* __restrict__ P, const Ts* __restrict__ Fl, int64_t r0, int64_t r1, Fn&& fn) {
#if SSF_EM_OFF32
    {   // frames of at most 2^32 / (3 sizeof(Ts)) points (mask_pose_batch rejects larger ones)
        if (r1 <= r0) return;                              // uniform (an empty part)
        const Ts* Pb = P + 3 * r0;
        const Ts* Fb = Fl + 3 * r0;
        const uint32_t n = (uint32_t)(r1 - r0), T = blockDim.x, last = n - 1;
        constexpr uint32_t S = 3 * sizeof(Ts);
        const uint32_t j0 = threadIdx.x;
        auto load = [&](uint32_t k, Ts r[6]) { load3_off(Fb, k * S, r); load3_off(Pb, k * S, r + 3); };
        Ts buf[D][6];
#pragma unroll
        for (int d = 0; d < D; ++d) load(min(j0 + d * T, last), buf[d]);
        for (uint32_t base = j0; base < n; base += D * T) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t j = base + d * T;
                double x[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) x[k] = (double)buf[d][k];
                load(min(j + D * T, last), buf[d]);
                fn(r0 + (int64_t)j, x, j < n);
            }
        }
    }
#else
    const int64_t T = blockDim.x;
    const int64_t i0 = r0 + threadIdx.x;
    if (r1 <= r0) return;                                  // uniform (an empty part)
    // loads are unconditional (indices clamped to the last point): the compiler can then count
    // them and wait with vmcnt(N) instead of draining every prefetch at a conditional join
    Ts buf[D][6];
#pragma unroll
    for (int d = 0; d < D; ++d) load_raw(P, Fl, min(i0 + d * T, r1 - 1), buf[d]);
    for (int64_t base = i0; base < r1; base += D * T) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int64_t i = base + d * T;
            double x[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) x[k] = (double)buf[d][k];
            load_raw(P, Fl, min(i + D * T, r1 - 1), buf[d]);
            fn(i, x, i < r1);   // every slot (no branch around the body's stores); val = 0 is weighted out
        }
    }
#endif
}

// EM: two points per step (i, i + T) so every parameter read serves both.  The second point of
// the last step may not exist (w1 = 0: computed on a duplicate, weighted out).  Loads clamped
// and unconditional, as in for_points.  SSF_EM_DEEP = 1 (default): the next step's pair in
// registers; 4: staged by LDS-DMA with the parameters in SGPRs, below -- +1.5 % on the mask
// alone (r6u) but not in the pipeline (r6za / r6zb: its 16 KiB more LDS keeps the other
// kernels off the mask's CUs; a one-point 2 KiB-slot form without the extra LDS was no faster).
// Two register pairs in flight, or the loop unrolled with swapping register sets, were 6 % / 4 %
// slower (the compiler waits for the loads right after issuing them, r6t / r6u).
#ifndef SSF_EM_DEEP
#define SSF_EM_DEEP 1
#endif
#ifndef SSF_LLOYD_LDS_HOIST
#define SSF_LLOYD_LDS_HOIST 0                    // Lloyd: the centres' bases laundered once per pass (A/B: 2.3x
#endif                                           // slower, the centres hoisted into VGPRs spill in the loops, r6zd)
#ifndef SSF_EM_LDS_HOIST
#define SSF_EM_LDS_HOIST 1                       // EM: the LDS parameter bases laundered once per pass (r6zc/r6zd)
#endif
#ifndef SSF_EM_SGPR
#define SSF_EM_SGPR (SSF_EM_DEEP == 4)           // E-step parameters as wave-uniform SGPR operands
#endif
template <class Ts, class Fn>
SSF_DEV void for_point_pairs(const Ts* __restrict__ P, const Ts* __restrict__ Fl, int64_t r0, int64_t r1, Fn&& fn) {
#if SSF_EM_OFF32
    {   // frames of at most 2^32 / (3 sizeof(Ts)) points (mask_pose_batch rejects larger ones)
        const Ts* Pb = P + 3 * r0;
        const Ts* Fb = Fl + 3 * r0;
        const uint32_t n = (uint32_t)(r1 - r0), T = blockDim.x, last = n - 1;
        constexpr uint32_t S = 3 * sizeof(Ts);
        uint32_t i = threadIdx.x;
        if (i >= n) return;
        Ts ra[6], rb[6];
        auto load = [&](uint32_t k, Ts r[6]) { load3_off(Fb, k * S, r); load3_off(Pb, k * S, r + 3); };
        load(i, ra);
        load(min(i + T, last), rb);
        for (; i < n; i += 2 * T) {
            double xa[6], xb[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) { xa[d] = (double)ra[d]; xb[d] = (double)rb[d]; }
            const double wb = (i + T < n) ? 1.0 : 0.0;
            load(min(i + 2 * T, last), ra);
            load(min(i + 3 * T, last), rb);
            fn(xa, xb, wb);
        }
    }
#else
    const int64_t T = blockDim.x;
    int64_t i = r0 + threadIdx.x;
    if (i >= r1) return;
    Ts ra[6], rb[6];
    load_raw(P, Fl, i, ra);
    load_raw(P, Fl, min(i + T, r1 - 1), rb);
    for (; i < r1; i += 2 * T) {
        double xa[6], xb[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) { xa[d] = (double)ra[d]; xb[d] = (double)rb[d]; }
        const double wb = (i + T < r1) ? 1.0 : 0.0;
        load_raw(P, Fl, min(i + 2 * T, r1 - 1), ra);
        load_raw(P, Fl, min(i + 3 * T, r1 - 1), rb);
        fn(xa, xb, wb);
    }
#endif
}

#if SSF_EM_DEEP == 4
// A/B (SSF_EM_DEEP = 4): the pair of the next step staged by LDS-DMA (global_load_lds_dwordx3: lane l's 12 bytes at
// base + 16 l, tools/probes/glds_x3_layout.hip) into a per-wave 4 KiB slot (k-means++'s bsum
// block, idle during EM), so the loads in flight hold no VGPRs and cannot be sunk to their use.
// Same per-thread point order, so the same sums.  The slot is read (lgkmcnt(0)) before the next
// DMA overwrites it; vmcnt(0) before the read.  hipcc drains every pending LDS-DMA before any
// LDS read it cannot prove disjoint, so the loop reads no other LDS: the E-step parameters come
// in SGPRs (SSF_EM_SGPR).
SSF_DEV void glds_x3(const float* g, float* lds_base) {
    __builtin_amdgcn_global_load_lds((const void*)g,
                                     (__attribute__((address_space(3))) void*)lds_base, 12, 0, 0);
}
template <class Fn>
SSF_DEV void for_point_pairs_glds(const float* __restrict__ P, const float* __restrict__ Fl,
                                  int64_t r0, int64_t r1, float* slot, Fn&& fn) {
    const int64_t T = blockDim.x;
    const int lane = threadIdx.x & 63;
    int64_t i = r0 + threadIdx.x;
    if (i >= r1) return;
    // a lane that has left the loop takes no part in a DMA and its 16 bytes of the slot are not
    // written (EXEC-masked); the others' land at base + 16 lane as before
    const int64_t last = r1 - 1;
    auto issue = [&](int64_t ia, int64_t ib) {
        ia = min(ia, last); ib = min(ib, last);
        glds_x3(Fl + 3 * ia, slot);
        glds_x3(P + 3 * ia, slot + 256);
        glds_x3(Fl + 3 * ib, slot + 512);
        glds_x3(P + 3 * ib, slot + 768);
    };
    issue(i, i + T);
    for (; i < r1; i += 2 * T) {
        __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0): this step's DMA has landed
        double xa[6], xb[6];
        const float* s = slot + 4 * lane;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            xa[d] = (double)s[d];       xa[3 + d] = (double)s[256 + d];
            xb[d] = (double)s[512 + d]; xb[3 + d] = (double)s[768 + d];
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): the slot is read
        const double wb = (i + T < r1) ? 1.0 : 0.0;
        issue(i + 2 * T, i + 3 * T);
        fn(xa, xb, wb);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);              // the last (clamped) DMA drained
}
#endif

// 1/d for d in [1, 2] (d = 1 + e, e in (0, 1]): v_rcp_f64 and two Newton steps, ~1 ulp,
// instead of the IEEE division sequence.
SSF_DEV double recip_1_2(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}

SSF_DEV double lse2(double a, double b) {  // scipy 1.15 logsumexp on two terms
    const double mx = a > b ? a : b;
    if (a == b) return log1p(0.0) + log(2.0) + mx;
    const double mn = a > b ? b : a;
    return log1p(exp(mn - mx)) + mx;
}

// Kabsch from shifted sums k[16] = {cnt, sum(s-cs)[3], sum(d-cd)[3], sum (s-cs)(d-cd)^T [9]}.
__device__ __noinline__ int kabsch_finish(const double* k, const double cs[3], const double cd[3], int reflection,
                          double* out) {
    const double n = k[0];
    if (!(n > 0.0)) return SSF_POSE_EMPTY;
    double es[3], ed[3], ms[3], md[3];
    for (int i = 0; i < 3; ++i) {
        es[i] = k[1 + i] / n; ed[i] = k[4 + i] / n;
        ms[i] = cs[i] + es[i]; md[i] = cd[i] + ed[i];
    }
    double H[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) H[r * 3 + c] = k[7 + r * 3 + c] - n * es[r] * ed[c];
    double U[9], Sv[3], Vt[9], R[9];
    svd3(H, U, Sv, Vt);
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
    double t[3];
    for (int r = 0; r < 3; ++r) t[r] = -(R[r * 3] * ms[0] + R[r * 3 + 1] * ms[1] + R[r * 3 + 2] * ms[2]) + md[r];
    // pyquaternion Quaternion(matrix=R): orthogonality check, trace method on m = R^T
    bool orth = true;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int kk = 0; kk < 3; ++kk) s += R[i * 3 + kk] * R[j * 3 + kk];
            const double e = (i == j) ? 1.0 : 0.0;
            if (!(fabs(s - e) <= 1e-8 + 1e-5 * fabs(e))) orth = false;
        }
    double q[4] = {0, 0, 0, 0};
    if (orth) {
        double m[3][3];
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) m[i][j] = R[j * 3 + i];
        double tt, w, x, y, z;
        if (m[2][2] < 0) {
            if (m[0][0] > m[1][1]) {
                tt = 1 + m[0][0] - m[1][1] - m[2][2];
                w = m[1][2] - m[2][1]; x = tt; y = m[0][1] + m[1][0]; z = m[2][0] + m[0][2];
            } else {
                tt = 1 - m[0][0] + m[1][1] - m[2][2];
                w = m[2][0] - m[0][2]; x = m[0][1] + m[1][0]; y = tt; z = m[1][2] + m[2][1];
            }
        } else {
            if (m[0][0] < -m[1][1]) {
                tt = 1 - m[0][0] - m[1][1] + m[2][2];
                w = m[0][1] - m[1][0]; x = m[2][0] + m[0][2]; y = m[1][2] + m[2][1]; z = tt;
            } else {
                tt = 1 + m[0][0] + m[1][1] + m[2][2];
                w = tt; x = m[1][2] - m[2][1]; y = m[2][0] - m[0][2]; z = m[0][1] - m[1][0];
            }
        }
        const double f = 0.5 / sqrt(tt);
        q[0] = x * f; q[1] = y * f; q[2] = z * f; q[3] = w * f;
    } else if (status == 0) {
        status = SSF_POSE_NOT_ORTHOGONAL;
    }
    for (int i = 0; i < 3; ++i) out[SSF_POSE_OUT_T + i] = t[i];
    for (int i = 0; i < 4; ++i) out[SSF_POSE_OUT_Q + i] = q[i];
    for (int i = 0; i < 9; ++i) out[SSF_POSE_OUT_R + i] = R[i];
    out[SSF_POSE_OUT_NBG] = n;
    return status;
}

// ---- one frame over G work-groups --------------------------------------------------------
// With G > 1 (small batches: G x frames fills the chip; see launch_mask_pose) every frame is
// cut into G contiguous parts of its points, one work-group each.  Each pass then sums over
// the work-group's part and the G partial sums are exchanged through global memory: every part
// stores its block totals write-through (sc1, relaxed agent-scope atomic stores) into its slot,
// drains them (s_waitcnt vmcnt(0)) and adds 1 to the frame's arrival counter; lane 0 polls the
// counter (relaxed agent loads, s_sleep) until all G parts of this exchange have arrived, and
// the totals are read back with sc1 loads and added in part order -- so every work-group of the
// frame holds the same bits and runs the same lane-0 algebra to the same decisions
// (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "Valid forms", row 1: one
// storing wave, one atomic-add signal, sc1 polls and sc1 loads, one work-group per CU).
// Every exchange of a launch has its OWN slot lines (slot = exchange index), never a line
// rewritten in the launch: an sc1 load bypasses the CU's L1 but is served by the reader XCD's
// L2 when that L2 already holds the line, and another XCD's sc1 store does not reach that copy.
// Measured on MI355X with a work-sharing variant of this kernel that re-read rewritten
// parameter lines across XCDs: 375-810 stale reads per 256-frame launch.  A
// line read here for the first time cannot be cached stale.
// Work-groups take (frame, part) tickets in order from a counter, so every partly started frame
// has its parts on resident work-groups and the ones it waits for are taken by the next
// work-group that becomes free (no wait on a work-group that cannot be dispatched).  A bounded
// spin turns a lost partner into status SSF_POSE_SYNC_FAILED, never a hang.
constexpr int kSlot = 32;                         // doubles per part and exchange
constexpr int kMaxSplit = kMaskMaxSplit;          // parts per frame at most (32)
constexpr uint32_t kSpinLimit = 1u << 24;         // x s_sleep 2 (~128 cycles): ~1 s
// exchanges per frame at most: pass 0, 3 in k-means++, one per Lloyd iteration (<= 300), the
// GMM init, one per EM iteration (<= 100), the final pass
constexpr int kMaxExchanges = 1 + 3 + 300 + 1 + 100 + 1;

struct Split {
    int G, g;                  // parts per frame, this work-group's part
    int64_t r0, r1;            // its points [r0, r1) of the frame
    double* part;              // the frame's slots [kMaxExchanges][G][kSlot]
    uint32_t* arrive;          // the frame's arrival counter (monotonic over its exchanges)
    uint32_t* fail;            // the frame's failure word: set by any part whose wait timed out
    uint32_t seq;              // exchanges done (uniform)
};

// The write-through form below matches a measured valid hand-off (MI355X_MICROARCH.md "Valid
// forms", row 1), which the guide marks as measured on gfx950 / ROCm 7.2, not an architectural
// guarantee.  So the exchange also carries the architectural pair: an agent-scope release fence
// before the arrival add and an agent-scope acquire after the poll (round 3).  Cost,
// same box A/B: configs[1] latency 0.554 -> 0.574 ms, configs[2] as written 4868 -> 4715
// frames/s (tools/gpu/r3i.sh); B = 256 runs G = 1 and never exchanges.  -DSSF_MASK_XCHG_FENCES=0
// drops the pair (A/B only).
#ifndef SSF_MASK_XCHG_FENCES
#define SSF_MASK_XCHG_FENCES 1
#endif

// lane 0: wait until the frame's arrival counter reaches `target` (relaxed sc1 polls with
// s_sleep back-off); false when a partner reported a timeout or the spin bound ran out
SSF_DEV bool wait_arrivals(const Split& X, uint32_t target) {
    uint32_t spins = 0;
    while (__hip_atomic_load(X.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit ||
            __hip_atomic_load(X.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
            return false;
    }
    return true;
}

template <int N, bool kMin = false>
SSF_DEV bool exchange(Split& X, double (&v)[N], double* tmp, int* okflag) {
    static_assert(N <= kSlot, "exchange: N <= kSlot");
    if (X.G == 1) return true;
    if (X.seq >= (uint32_t)kMaxExchanges) return false;   // cannot happen (iteration caps); never reuse a line
    double* slot = X.part + (size_t)X.seq * (size_t)X.G * kSlot;
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (threadIdx.x == (unsigned)k)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(slot + X.g * kSlot + k),
                               (unsigned long long)__double_as_longlong(v[k]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    X.seq += 1u;
    if (threadIdx.x < 64) {                        // wave 0 stored every value
        // drain the write-through stores before the signal (R1); the asm is also the compiler
        // barrier that keeps them above the add
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) {
#if SSF_MASK_XCHG_FENCES
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            __hip_atomic_fetch_add(X.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int ok = wait_arrivals(X, (uint32_t)X.G * X.seq) ? 1 : 0;
#if SSF_MASK_XCHG_FENCES
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            *okflag = ok;
        }
    }
    __syncthreads();
    // no instruction: keeps the compiler from moving the slot loads above the poll and the
    // barrier (the sc1 loads themselves stand in for the acquire: Guideline 16, Valid forms row 1)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!*okflag) return false;                    // uniform
    // every (part, value) on its own thread: one load latency for the G x N values (a loop over
    // the parts per value waited for G loads in a row); tmp holds kMaxSplit x kSlot doubles
    for (int t = threadIdx.x; t < X.G * N; t += blockDim.x) {
        const int gg = t / N, k = t - gg * N;
        tmp[kSlot + t] = __longlong_as_double((long long)__hip_atomic_load(
            reinterpret_cast<unsigned long long*>(slot + gg * kSlot + k), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)N) {
        double acc = kMin ? __builtin_inf() : 0.0;
        for (int gg = 0; gg < X.G; ++gg) {                 // part order: the same bits everywhere
            const double x = tmp[kSlot + gg * N + threadIdx.x];
            acc = kMin ? (x < acc ? x : acc) : acc + x;
        }
        tmp[threadIdx.x] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = tmp[k];
    __syncthreads();
    return true;
}

// One value per part; every part reads the G values in part order -> the sum over the parts
// before this one and the total (the k-means++ cumulative potential).  Same protocol as exchange.
SSF_DEV bool exchange_prefix(Split& X, double v, double* tmp, int* okflag, double& before, double& total) {
    if (X.seq >= (uint32_t)kMaxExchanges) return false;
    double* slot = X.part + (size_t)X.seq * (size_t)X.G * kSlot;
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(slot + X.g * kSlot),
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    X.seq += 1u;
    if (threadIdx.x < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) {
#if SSF_MASK_XCHG_FENCES
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            __hip_atomic_fetch_add(X.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int ok = wait_arrivals(X, (uint32_t)X.G * X.seq) ? 1 : 0;
#if SSF_MASK_XCHG_FENCES
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            *okflag = ok;
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!*okflag) return false;                    // uniform
    if (threadIdx.x < (unsigned)X.G)
        tmp[kSlot + threadIdx.x] = __longlong_as_double((long long)__hip_atomic_load(
            reinterpret_cast<unsigned long long*>(slot + threadIdx.x * kSlot), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0, t = 0.0;
        for (int gg = 0; gg < X.G; ++gg) {
            const double x = tmp[kSlot + gg];
            if (gg < X.g) b += x;
            t += x;
        }
        tmp[0] = b; tmp[1] = t;
    }
    __syncthreads();
    before = tmp[0];
    total = tmp[1];
    __syncthreads();
    return true;
}

SSF_DEV void accum_kabsch(double (&k)[16], const double* x, const double cs[3], const double cd[3]) {
    double s[3], d[3];
    for (int i = 0; i < 3; ++i) { d[i] = x[3 + i] - cd[i]; s[i] = (x[3 + i] + x[i]) - cs[i]; }
    k[0] += 1.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) { k[1 + i] += s[i]; k[4 + i] += d[i]; }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) k[7 + r * 3 + c] += s[r] * d[c];
}

template <class T>
__global__ __launch_bounds__(kMaskThreads) void k_mask_pose(
    const T* __restrict__ pts, const T* __restrict__ flow,
    const int64_t* __restrict__ frame_off, int mode, const uint8_t* __restrict__ mask_in,
    const double* __restrict__ draws, uint2* __restrict__ lloyd_rec, int reflection,
    uint8_t* __restrict__ bg_mask, double* __restrict__ out_all, int n_frames, int G,
    uint32_t* __restrict__ sync, double* __restrict__ parts, const int32_t* __restrict__ order,
    int tickets) {
    __shared__ MaskShared S;
    __shared__ double red[kNW * 32];
    __shared__ int ired[kNW];
    __shared__ unsigned long long cand_lds[2];
#if SSF_EM_DEEP == 4
    __shared__ __attribute__((aligned(16))) double bsum[kKppBlocks > kNW * 512 ? kKppBlocks : kNW * 512];  // + the EM's DMA slots
#else
    __shared__ double bsum[kKppBlocks];   // k-means++ per-64-point-block distance totals
#endif
    __shared__ uint32_t lq[kNW * kLQ];     // Lloyd skip passes: per-wave relabel entries of a trip
    __shared__ double xtmp[kSlot + kMaxSplit * kSlot];   // exchange totals + the gathered parts
    __shared__ int tk, okflag;
    const int tid = threadIdx.x;
    // G == 1 without tickets: work-group = frame.  Otherwise (frame, part) tickets in order (see
    // Split; with G == 1 a frame queue: a work-group takes the next frame when its frame is
    // done, so a slow frame holds one CU while the others drain the batch).  order (optional): the
    // k-th frame dispatched is order[k] (a permutation; results do not depend on it).
    for (int iter = 0;; ++iter) {
    int f, g = 0;
    if (G == 1 && !tickets) {
        if (iter > 0) break;
        f = blockIdx.x;
    } else {
        __syncthreads();                       // the previous frame's readers of S / tk are done
        if (tid == 0) tk = (int)atomicAdd(sync, 1u);
        __syncthreads();
        f = tk / G;
        g = tk - f * G;
        if (f >= n_frames) break;              // uniform: every wave leaves
    }
    if (order) {
        f = order[f];
        if ((unsigned)f >= (unsigned)n_frames) continue;   // uniform: not a frame (skipped)
    }
    [&]() {                                    // one frame part; `return` ends it
    const int64_t fb = frame_off[f], n = frame_off[f + 1] - fb;
    const T* P = pts + 3 * fb;
    const T* Fl = flow + 3 * fb;
    double* out = out_all + (int64_t)f * SSF_POSE_OUT_STRIDE;
    Split X;
    X.G = G; X.g = g;
    {
        const int64_t chunk = ((n + G - 1) / G + 127) / 128 * 128;   // parts start at even records
        X.r0 = min(n, (int64_t)g * chunk);
        X.r1 = min(n, X.r0 + chunk);
    }
    X.part = parts + (size_t)f * kMaxExchanges * (size_t)G * kSlot;
    X.arrive = sync + 4 + f;
    X.fail = sync + 4 + n_frames + f;
    X.seq = 0;
    const int64_t r0 = X.r0, r1 = X.r1;
    auto sync_failed = [&]() {                 // a partner never arrived: report, never hang
        if (tid == 0) {
            // every part reports, so part 0 never publishes a frame whose other parts stopped
            // before their share of the mask (the done round below)
            __hip_atomic_store(X.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (g == 0) {
                for (int i = 0; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
                out[SSF_POSE_OUT_STATUS] = SSF_POSE_SYNC_FAILED;
            }
        }
    };
    if (tid == 0) {
        S.passes = 0; S.status = 0; S.km_iter = 0; S.em_iter = 0; S.converged = 0;
        if (g == 0) for (int i = 26; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
    }
#ifdef SSF_MASK_STAMPS
    const unsigned long long stamp0 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();

    if (mode != SSF_MASK_GMM) {
        // background from the given / ground-truth mask; Kabsch sums shifted by point 0
        double cs[3] = {0, 0, 0}, cd[3] = {0, 0, 0};
        if (n > 0) {
            double x0[6];
            load_x(P, Fl, 0, x0);
            for (int i = 0; i < 3; ++i) { cd[i] = x0[3 + i]; cs[i] = x0[3 + i] + x0[i]; }
        }
        double k[16];
        for (int i = 0; i < 16; ++i) k[i] = 0.0;
        for (int64_t i = tid; i < n; i += blockDim.x) {
            const uint8_t mv = mask_in[fb + i];
            const bool bg = (mode == SSF_MASK_GT) ? (mv == 0) : (mv != 0);
            if (bg_mask) bg_mask[fb + i] = bg ? 1 : 0;
            if (!bg) continue;
            double x[6];
            load_x(P, Fl, i, x);
            accum_kabsch(k, x, cs, cd);
        }
        block_sum_rs<16>(k, red);
        if (tid == 0) {
            for (int i = 0; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
            for (int i = 0; i < 16; ++i) S.sums[i] = k[i];
            const int st = kabsch_finish(S.sums, cs, cd, reflection, out);
            out[SSF_POSE_OUT_STATUS] = st;
            out[SSF_POSE_OUT_BGLABEL] = -1;
            out[SSF_POSE_OUT_PASSES] = 1;
        }
        return;
    }

    if (n < 2) {
        if (tid == 0 && g == 0) {
            for (int i = 0; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
            out[SSF_POSE_OUT_STATUS] = SSF_POSE_GMM_FAILED;
        }
        return;
    }

    // ---- pass 0: column means, variances (KMeans tol) and the total first/second moments
    //      about point 0, converted by lane 0 to moments about the mean (the common shift of
    //      every later moment sum).
    {
        double x0[6];
        load_x(P, Fl, 0, x0);
        double a[27];
#pragma unroll
        for (int i = 0; i < 27; ++i) a[i] = 0.0;
        // two points in flight per thread (for_points_deep: the same per-thread order, so the
        // same sums); a slot past r1 adds zeros
        for_points_deep<kLloydDeep>(P, Fl, r0, r1, [&](int64_t, const double* x, bool val) {
            double v[6], vw[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) { v[d] = x[d] - x0[d]; vw[d] = val ? v[d] : 0.0; a[d] += vw[d]; }
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int c = r; c < 6; ++c) a[6 + up(r, c)] += vw[r] * v[c];
        });
        block_sum_rs<27>(a, red);
        if (!exchange<27>(X, a, xtmp, &okflag)) { sync_failed(); return; }
        if (tid == 0) {
            const double nn = (double)n;
            double m[6];
            double tol = 0.0;
            for (int d = 0; d < 6; ++d) { m[d] = a[d] / nn; S.mean[d] = x0[d] + m[d]; }
            S.tot[0] = nn;
            for (int d = 0; d < 6; ++d) S.tot[1 + d] = a[d] - nn * m[d];
            for (int r = 0; r < 6; ++r)
                for (int c = r; c < 6; ++c) S.tot[7 + up(r, c)] = a[6 + up(r, c)] - nn * m[r] * m[c];
            for (int d = 0; d < 6; ++d) tol += S.tot[7 + up(d, d)] / nn;
            S.tol = tol / 6.0 * 1e-4;
            // Kabsch sums over ALL points about (cs, cd) = (x0_p + x0_f, x0_p), from the raw
            // moments about x0: s - cs = v_f + v_p, d - cd = v_p  (v = x - x0; f = 0..2, p = 3..5)
            for (int d = 0; d < 6; ++d) S.x0[d] = x0[d];
            S.ktot[0] = nn;
            for (int r = 0; r < 3; ++r) { S.ktot[1 + r] = a[r] + a[3 + r]; S.ktot[4 + r] = a[3 + r]; }
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    const int fr = r, pr = 3 + r, pc = 3 + c;
                    const double sfp = a[6 + (fr <= pc ? up(fr, pc) : up(pc, fr))];
                    const double spp = a[6 + (pr <= pc ? up(pr, pc) : up(pc, pr))];
                    S.ktot[7 + r * 3 + c] = sfp + spp;
                }
            S.c0 = (int64_t)draws[3 * f];
            if (S.c0 < 0) S.c0 = 0;
            if (S.c0 >= n) S.c0 = n - 1;
            S.passes = 1;
        }
        __syncthreads();
    }
    SSF_STAMP(0);
    double mean[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) mean[d] = uni(S.mean[d]);

    // ---- k-means++ (sklearn _kmeans_plusplus, n_local_trials = 2)
    {
        double c0[6], cn0 = 0.0;
        {
            double x[6];
            load_x(P, Fl, S.c0, x);
            for (int d = 0; d < 6; ++d) { c0[d] = x[d] - mean[d]; cn0 += c0[d] * c0[d]; }
        }
        // distances to the first centre; each wave owns a contiguous segment so the
        // in-order cumulative sum needs only one block-level exchange of wave totals
        const int nw = blockDim.x >> 6, w = tid >> 6, lane = lane_id();
        const int64_t nloc = r1 - r0;
        const int64_t seg = (((nloc + nw - 1) / nw) + 63) / 64 * 64;
        const int64_t ws = r0 + (int64_t)w * seg, we = ws + seg < r1 ? ws + seg : r1;
        // D(i) = squared distance to the first centre; recomputed (same expression, same bits)
        // wherever it is needed instead of being stored
        auto dist0x = [&](const double* x) {
            double dt = 0.0, xs = 0.0;
#pragma unroll
            for (int d = 0; d < 6; ++d) { const double v = x[d] - mean[d]; dt += c0[d] * v; xs += v * v; }
            const double v = (-2.0 * dt + cn0) + xs;
            return v > 0.0 ? v : 0.0;
        };
        auto dist0 = [&](int64_t i) {
            double x[6];
            load_x(P, Fl, i, x);
            return dist0x(x);
        };
        // the wave's segment streamed with the next kKppDeep blocks' points in flight (raw floats,
        // loads clamped and unconditional): each block was one dependent load latency before.
        // Diag stamps, B = 256: k-means++ 0.75 -> 0.56 M cycles per frame at depth 2; depth 4
        // 0.58 (tools/gpu/r3y.sh, r3z.sh)
        constexpr int kKppDeep = SSF_KPP_DEEP;
        const int64_t wlast = we > ws ? we - 1 : ws;
        // per 64-point block: the in-block inclusive scan's total (lane 63) goes to LDS, so the
        // draw search below only re-scans the one block that holds the draw
        const int64_t spw = seg / 64;                            // blocks per wave segment
        const bool use_blocks = spw * nw <= kKppBlocks;          // uniform
        double wsum = 0.0;
        T kb[kKppDeep][6];
        if (ws < we) {
#pragma unroll
            for (int k = 0; k < kKppDeep; ++k) load_raw(P, Fl, min(ws + 64 * k + lane, wlast), kb[k]);
        }
        for (int64_t b0 = ws; b0 < we; b0 += 64 * kKppDeep)
#pragma unroll
        for (int k = 0; k < kKppDeep; ++k) {
            const int64_t b = b0 + 64 * k;
            if (b >= we) break;                                  // uniform
            const int64_t i = b + lane;
            double x[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) x[d] = (double)kb[k][d];
            load_raw(P, Fl, min(i + 64 * kKppDeep, wlast), kb[k]);
            const double d = i < we ? dist0x(x) : 0.0;
            wsum += d;
            if (use_blocks) {
                double v = d;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const double y = __shfl_up(v, o, 64);
                    if (lane >= o) v += y;
                }
                if (lane == 63) bsum[w * spw + (b - ws) / 64] = v;
            }
        }
        wsum = wave_sum(wsum);
        if (lane == 0) red[w] = wsum;
        if (tid == 0) { cand_lds[0] = (unsigned long long)n; cand_lds[1] = (unsigned long long)n; }
        __syncthreads();
        double pot = 0.0, carry = 0.0;
        for (int k = 0; k < nw; ++k) { if (k == w) carry = pot; pot += red[k]; }
        if (G > 1) {
            // the in-order cumulative sum runs over the parts in order: part g starts after the
            // potentials of parts 0..g-1 (one value per part; every part reads all G in order)
            double before = 0.0, total = 0.0;
            if (!exchange_prefix(X, pot, xtmp, &okflag, before, total)) { sync_failed(); return; }
            carry += before;
            pot = total;
        }
        if (tid == 0) {
            S.rand1 = draws[3 * f + 1] * pot;
            S.rand2 = draws[3 * f + 2] * pot;
            S.passes += 1;
        }
        const double r1 = draws[3 * f + 1] * pot, r2 = draws[3 * f + 2] * pot;
        // wave-local in-order inclusive scan of its segment; first index with cumsum >= rand.
        // A wave whose whole segment ends below both draws cannot hold either index and skips
        // the scan (1e-9 slack >> the scan's rounding); the others stop once both are found.
        const double wtot = red[w];
        bool f1 = carry + wtot < r1 * (1.0 - 1e-9), f2 = carry + wtot < r2 * (1.0 - 1e-9);
        if (use_blocks) {
            // walk the wave's block totals with the same carry arithmetic as the full scan
            // (carry + block total, then carry += total): the first block whose end reaches a
            // draw is the block the full scan would stop in; only that block is re-scanned
            int64_t blk1 = -1, blk2 = -1;
            double cb1 = 0.0, cb2 = 0.0;
            if (lane == 0 && !(f1 && f2)) {
                double cr = carry;
                for (int64_t k = 0; ws + 64 * k < we; ++k) {
                    const double tot = bsum[w * spw + k];
                    if (!f1 && blk1 < 0 && cr + tot >= r1) { blk1 = k; cb1 = cr; }
                    if (!f2 && blk2 < 0 && cr + tot >= r2) { blk2 = k; cb2 = cr; }
                    if ((f1 || blk1 >= 0) && (f2 || blk2 >= 0)) break;
                    cr += tot;
                }
            }
            blk1 = __shfl(blk1, 0, 64); blk2 = __shfl(blk2, 0, 64);
            cb1 = __shfl(cb1, 0, 64); cb2 = __shfl(cb2, 0, 64);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int64_t blk = j ? blk2 : blk1;
                if (blk < 0) continue;                           // wave-uniform
                const int64_t b = ws + 64 * blk;
                const int64_t i = b + lane;
                double v = i < we ? dist0(i) : 0.0;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const double y = __shfl_up(v, o, 64);
                    if (lane >= o) v += y;
                }
                const double incl = (j ? cb2 : cb1) + v;
                const uint64_t mm = __ballot(i < we && incl >= (j ? r2 : r1));
                if (mm && lane == 0) atomicMin(&cand_lds[j], (unsigned long long)(b + __ffsll((unsigned long long)mm) - 1));
            }
            f1 = f2 = true;                                      // skip the sequential scan
        }
        for (int64_t b = ws; b < we && !(f1 && f2); b += 64) {
            const int64_t i = b + lane;
            double v = i < we ? dist0(i) : 0.0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const double y = __shfl_up(v, o, 64);
                if (lane >= o) v += y;
            }
            const double incl = carry + v;
            const uint64_t m1 = __ballot(i < we && incl >= r1), m2 = __ballot(i < we && incl >= r2);
            if (!f1 && m1) { f1 = true; if (lane == 0) atomicMin(&cand_lds[0], (unsigned long long)(b + __ffsll((unsigned long long)m1) - 1)); }
            if (!f2 && m2) { f2 = true; if (lane == 0) atomicMin(&cand_lds[1], (unsigned long long)(b + __ffsll((unsigned long long)m2) - 1)); }
            carry += __shfl(v, 63, 64);
        }
        __syncthreads();
        double cmin[2] = {(double)cand_lds[0], (double)cand_lds[1]};   // < 2^53: exact
        if (!exchange<2, true>(X, cmin, xtmp, &okflag)) { sync_failed(); return; }
        const int64_t cand[2] = {cmin[0] < (double)n ? (int64_t)cmin[0] : n - 1,
                                 cmin[1] < (double)n ? (int64_t)cmin[1] : n - 1};
        double cc[2][6], ccn[2] = {0.0, 0.0};
        for (int j = 0; j < 2; ++j) {
            double x[6];
            load_x(P, Fl, cand[j], x);
            for (int d = 0; d < 6; ++d) { cc[j][d] = x[d] - mean[d]; ccn[j] += cc[j][d] * cc[j][d]; }
        }
        double cp[2] = {0.0, 0.0};
        if (ws < we) {
#pragma unroll
            for (int k = 0; k < kKppDeep; ++k) load_raw(P, Fl, min(ws + 64 * k + lane, wlast), kb[k]);
        }
        for (int64_t b0 = ws; b0 < we; b0 += 64 * kKppDeep)
#pragma unroll
        for (int k = 0; k < kKppDeep; ++k) {
            const int64_t b = b0 + 64 * k;
            if (b >= we) break;                                  // uniform
            const int64_t i = b + lane;
            double x[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) x[d] = (double)kb[k][d];
            load_raw(P, Fl, min(i + 64 * kKppDeep, wlast), kb[k]);
            if (i < we) {
                double xs = 0.0, dt0 = 0.0, dt1 = 0.0, dtc = 0.0;
#pragma unroll
                for (int d = 0; d < 6; ++d) {
                    const double v = x[d] - mean[d];
                    dtc += c0[d] * v; xs += v * v; dt0 += cc[0][d] * v; dt1 += cc[1][d] * v;
                }
                double di = (-2.0 * dtc + cn0) + xs;             // = dist0(i), bit for bit
                di = di > 0.0 ? di : 0.0;
                double v0 = (-2.0 * dt0 + ccn[0]) + xs, v1 = (-2.0 * dt1 + ccn[1]) + xs;
                v0 = v0 > 0.0 ? v0 : 0.0; v1 = v1 > 0.0 ? v1 : 0.0;
                cp[0] += v0 < di ? v0 : di;
                cp[1] += v1 < di ? v1 : di;
            }
        }
        block_sum<2>(cp, red);
        if (!exchange<2>(X, cp, xtmp, &okflag)) { sync_failed(); return; }
        if (tid == 0) {
            const int best = cp[1] < cp[0] ? 1 : 0;
            S.c1 = cand[best];
            for (int d = 0; d < 6; ++d) { S.cen[d] = c0[d]; S.cen[6 + d] = cc[best][d]; }
            for (int d = 0; d < 12; ++d) S.cenp[d] = 0.0;
            S.csnp[0] = S.csnp[1] = 0.0;
            S.passes += 2;
        }
        __syncthreads();
    }

    SSF_STAMP(1);
    // ---- Lloyd iterations (_kmeans_single_lloyd, max_iter 300) with exact label skipping.
    //      A point's label at pass t is the sign of g_t = D0 - D1 (D_k = -2 v.c_k + |c_k|^2, the
    //      expression the label is computed with).  In exact arithmetic g_t(v) = 2 v.w_t + s_t
    //      (w = c1 - c0, s = |c0|^2 - |c1|^2), so |g_t - g_r| <= 2|v| |w_t - w_r| + |s_t - s_r|.
    //      Every labelled point leaves an 8-byte record {|g_r| rounded down, |v| rounded up,
    //      pass r, label}; a later pass t re-reads the point's 24 bytes only when
    //          |g_r| <= B1(t, r) |v| + B2(t, r)
    //      (B1/B2: the drift bounds plus 1e-13-relative margins for the f64 rounding of both
    //      evaluations, >= 50x the dot-product error bound), i.e. whenever the sign could
    //      differ.  Skipped points keep their label, so the labels, the changed-label count and
    //      the strict-convergence decision are those of the full pass; the cluster sums are
    //      updated by the points that changed label.
    if (tid == 0) { S.strict = 0; S.done = 0; S.lfull = 1; S.dg_cyc = S.dg_n = S.dg_lab = S.dg_wfull = S.dg_full1 = 0.0; }
    // records at an even offset (16-byte aligned pairs) with at least one spare slot (index n)
    // after each frame: frame f at ((fb + 2 f + 1) & ~1); the buffer holds total + 2 F + 2
    // records, then total + 64 F 4-byte queue entries
    uint2* __restrict__ LR = lloyd_rec + ((fb + 2 * (int64_t)f + 1) & ~(int64_t)1);
    // the relabel queues follow the records: frame f's at fb + 64 f, n entries + 64 spare slots
    uint32_t* __restrict__ LQ =
        reinterpret_cast<uint32_t*>(lloyd_rec + frame_off[n_frames] + 2 * (int64_t)n_frames + 2) + fb +
        64 * (int64_t)f;
    for (int it = 0; it < kLloydMax; ++it) {
        if (tid == 0) {
            double* h = S.lhist + 9 * it;
            for (int k = 0; k < 2; ++k) {
                double sn = 0.0;
                for (int d = 0; d < 6; ++d) sn += S.cen[6 * k + d] * S.cen[6 * k + d];
                S.csn[k] = sn;
            }
            for (int d = 0; d < 6; ++d) h[d] = S.cen[6 + d] - S.cen[d];
            h[6] = S.csn[0] - S.csn[1];
            h[7] = sqrt(S.csn[0]) + sqrt(S.csn[1]);
            h[8] = S.csn[0] + S.csn[1];
        }
        __syncthreads();
        if (tid < it) {   // drift bounds of this pass against every earlier labelling pass
            const double* h = S.lhist + 9 * it;
            const double* g = S.lhist + 9 * tid;
            double dw = 0.0;
            for (int d = 0; d < 6; ++d) dw += (h[d] - g[d]) * (h[d] - g[d]);
            S.lb1[tid] = __double2float_ru(2.0 * sqrt(dw) + 2e-13 * (h[7] + g[7]));
            S.lb2[tid] = __double2float_ru(fabs(h[6] - g[6]) + 1e-13 * (h[8] + g[8]));
        }
        __syncthreads();
        // the centres are read from LDS (broadcast) at every point through a laundered base,
        // like the EM parameters: held in registers they spilled to scratch in these loops
        const double csn0 = uni(S.csn[0]), csn1 = uni(S.csn[1]);
        double acc[14];
#pragma unroll
        for (int k = 0; k < 14; ++k) acc[k] = 0.0;
        int changed = 0, nlab = 0;
        const bool full = S.lfull != 0;
#ifdef SSF_MASK_STAMPS
        const unsigned long long pass_t0 = __builtin_amdgcn_s_memtime();
#endif
        const bool wrec = it >= kLloydFullPasses - 1;   // a skip pass may follow this full pass
        // exact labelling of one point (the expression of every earlier version of this pass):
        // sums (full pass) or sum deltas (skip pass), changed count, new record
        // (val = 0: a pipeline slot with no point -- computed, weighted out, record written to
        // the frame's spare slot n)
#if SSF_LLOYD_LDS_HOIST
        const LdsDouble* cenL = lds_laundered(S.cen);   // once per pass (see SSF_EM_LDS_HOIST)
#endif
        auto label = [&](auto wrec_c, int64_t i, const double* x, int lp, bool val) {
#if SSF_LLOYD_LDS_HOIST
            const LdsDouble* cen = cenL;
#else
            const LdsDouble* cen = lds_laundered(S.cen);
#endif
            double v[6], dt0 = 0.0, dt1 = 0.0, vn = 0.0;
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                v[d] = x[d] - mean[d];
                dt0 += v[d] * cen[d]; dt1 += v[d] * cen[6 + d]; vn += v[d] * v[d];
            }
            const double D0 = -2.0 * dt0 + csn0, D1 = -2.0 * dt1 + csn1;
            const int l = D1 < D0 ? 1 : 0;
            double d1 = full ? (double)l : (double)(l - lp), d0 = full ? 1.0 - d1 : -d1;
            d1 = val ? d1 : 0.0; d0 = val ? d0 : 0.0;
            changed += val && (it == 0 || l != lp);
            acc[0] += d0; acc[7] += d1;
#pragma unroll
            for (int d = 0; d < 6; ++d) { acc[1 + d] += d0 * v[d]; acc[8 + d] += d1 * v[d]; }
            // |g| one f32 ulp below its nearest float (<= |g|); |v| from an f32 sqrt, 4 ulps up,
            // then up to the 2^-14-relative grid that leaves the low 9 bits for the pass index
            const uint32_t gb = __float_as_uint((float)fabs(D0 - D1));
            const uint32_t nvb = (__float_as_uint(__builtin_sqrtf((float)vn)) + 4u + 0x1FFu) & 0x7FFFFE00u;
            if constexpr (decltype(wrec_c)::value) LR[val ? i : n] = make_uint2(gb ? gb - 1u : 0u, nvb | (uint32_t)it | ((uint32_t)l << 31));
        };
        if (full) {
            // every point: a prefetched stream of [flow, xyz]; the previous label is recomputed
            // from the previous centres (the pass that wrote it used the same expression)
            const double cpn0 = uni(S.csnp[0]), cpn1 = uni(S.csnp[1]);
#if SSF_LLOYD_LDS_HOIST
            const LdsDouble* cenpL = lds_laundered(S.cenp);
#endif
            auto full_pass = [&](auto wrec_c) {
                for_points_deep<kLloydDeep>(P, Fl, r0, r1, [&](int64_t i, const double* x, bool val) {
#if SSF_LLOYD_LDS_HOIST
                    const LdsDouble* cenp = cenpL;
#else
                    const LdsDouble* cenp = lds_laundered(S.cenp);
#endif
                    double dp0 = 0.0, dp1 = 0.0;
#pragma unroll
                    for (int d = 0; d < 6; ++d) {
                        const double v = x[d] - mean[d];
                        dp0 += v * cenp[d]; dp1 += v * cenp[6 + d];
                    }
                    const int lp = (-2.0 * dp1 + cpn1) < (-2.0 * dp0 + cpn0) ? 1 : 0;
                    label(wrec_c, i, x, lp, val);
                });
            };
            if (wrec) full_pass(std::true_type{});    // two loop bodies: no branch per point
            else full_pass(std::false_type{});
            nlab = (int)((r1 - r0 - tid + blockDim.x - 1) / blockDim.x);
        } else {
            // skip pass, two streams per wave over its own segment.  (1) the records, 16 bytes
            // (two records) per lane per load, 8 loads in flight: the points whose sign could
            // change are appended (ballot compaction, label in bit 31) to the wave's queue in
            // global memory.  (2) the queue, 512 entries at a time: every entry load, then every
            // point gather, then the relabelling -- two round trips per 512 queued points.
            const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = lane_id();
            const int64_t seg = ((r1 - r0 + kNW - 1) / kNW + 127) / 128 * 128;
            const int64_t ws = r0 + (int64_t)w * seg, we = ws + seg < r1 ? ws + seg : r1;
            uint32_t* __restrict__ WQ = LQ + ws;        // capacity seg >= the wave's points
            const int64_t qspare = n - ws;               // LQ[n, n + 64): spare slots
            const uint4* __restrict__ LR4 = reinterpret_cast<const uint4*>(LR);
            const int64_t plast = (n - 1) >> 1;
            uint32_t* Q = lq + w * kLQ;                 // this trip's entries (<= D * 128)
            int qc = 0, nl = 0;                         // wave-uniform
            constexpr int D = kLloydRecDeep;
            uint4 buf[D];
#pragma unroll
            for (int d = 0; d < D; ++d) buf[d] = LR4[min((ws >> 1) + d * 64 + lane, plast)];
            for (int64_t base = ws; base < we; base += D * 128) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const int64_t b = base + d * 128;
                    const uint4 q = buf[d];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t gx = h ? q.z : q.x, gy = h ? q.w : q.y;
                        const int64_t i = b + 2 * lane + h;
                        const int tr = (int)(gy & 0x1FFu);
                        const float nv = __uint_as_float(gy & 0x7FFFFE00u);
                        const bool skip = __uint_as_float(gx) > __builtin_fmaf(S.lb1[tr], nv, S.lb2[tr]) * 1.00001f;
#ifdef SSF_LLOYD_EXP_NOQUEUE
                        const bool nd = (i < we) & !skip & (gx == 0x7FFFFFFFu);
#else
                        const bool nd = (i < we) & !skip;
#endif
                        const uint64_t m = __ballot(nd);
                        if (nd) Q[nl + __popcll(m & lanemask_lt())] = (uint32_t)i | (gy & 0x80000000u);
                        nl += __popcll(m);
                    }
                    // reloaded only after q is consumed: the load can reuse q's registers, so
                    // the loop-carried buffers need no copies (a copy waits for its load)
                    buf[d] = LR4[min(((b + D * 128) >> 1) + lane, plast)];
                }
                // the trip's queue entries leave LDS: two unconditional 64-entry stores (lanes
                // without an entry write the frame's spare slots), more only past 128 entries
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    WQ[h * 64 + lane < nl ? qc + h * 64 + lane : qspare + lane] = Q[h * 64 + lane];
                for (int k = 128; k < nl; k += 64)
                    if (k + lane < nl) WQ[qc + k + lane] = Q[k + lane];
                __builtin_amdgcn_wave_barrier();
                qc += nl;
                nl = 0;
            }
            __threadfence_block();   // the wave's queue stores are visible to its loads below
            for (int j0 = 0; j0 < qc; j0 += 512) {
                uint32_t e[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) e[k] = WQ[min(j0 + k * 64 + lane, qc - 1)];
                T px[8][6];
#pragma unroll
                for (int k = 0; k < 8; ++k) load_raw(P, Fl, (int64_t)(e[k] & 0x7FFFFFFFu), px[k]);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    double x[6];
#pragma unroll
                    for (int d = 0; d < 6; ++d) x[d] = (double)px[k][d];
                    const bool val = j0 + k * 64 + lane < qc;
                    label(std::true_type{}, (int64_t)(e[k] & 0x7FFFFFFFu), x, (int)(e[k] >> 31), val);
                    nlab += val ? 1 : 0;
                }
            }
        }
        block_sum_rs<14>(acc, red);
        changed = block_sum_scalar<int>(changed, ired);
        nlab = block_sum_scalar<int>(nlab, ired);
        if (G > 1) {
            double v[16];
#pragma unroll
            for (int k = 0; k < 14; ++k) v[k] = acc[k];
            v[14] = (double)changed; v[15] = (double)nlab;
            if (!exchange<16>(X, v, xtmp, &okflag)) { sync_failed(); return; }
#pragma unroll
            for (int k = 0; k < 14; ++k) acc[k] = v[k];
            changed = (int)v[14]; nlab = (int)v[15];
        }
        if (tid == 0) {
            // traffic accounting in 24-byte-per-point units: a full pass reads [flow, xyz] (+8 B
            // of records written when wrec); a skip pass reads 8 B of records per point and
            // 24 B per relabelled point, and writes (reads) 8 B of record + 4 (4) B of queue
            // per relabel
            S.passes += full ? 1.0 + (wrec ? 8.0 / 24.0 : 0.0)
                             : (8.0 * (double)n + 40.0 * (double)nlab) / (24.0 * (double)n);
            S.km_iter = it + 1;
            for (int k = 0; k < 14; ++k) S.lsum[k] = full ? acc[k] : S.lsum[k] + acc[k];
            // the first passes move the centres most (typically 35-45 % of the points would be
            // relabelled): full passes through it = 3, then skip passes while they relabel < 1/4
            S.lfull = full ? it < kLloydFullPasses - 1 : nlab * kLloydRefull > n;
#ifdef SSF_MASK_STAMPS
            // diagnostic: cycles and relabelled points of the skip passes (k_mask_pose stamps
            // build only; reported through the k-means++ centre slots, which it overwrites)
            if (!full) { S.dg_cyc += (double)(__builtin_amdgcn_s_memtime() - pass_t0); S.dg_n += 1.0; S.dg_lab += nlab; }
            else if (it == kLloydFullPasses - 1) S.dg_wfull = (double)(__builtin_amdgcn_s_memtime() - pass_t0);
            else if (it == 1) S.dg_full1 = (double)(__builtin_amdgcn_s_memtime() - pass_t0);
#endif
            for (int k = 0; k < 12; ++k) S.cenp[k] = S.cen[k];
            S.csnp[0] = S.csn[0]; S.csnp[1] = S.csn[1];
            double shift = 0.0;
            for (int k = 0; k < 2; ++k) {
                const double wgt = S.lsum[7 * k];
                double sh = 0.0;
                for (int d = 0; d < 6; ++d) {
                    const double nc = wgt > 0.0 ? S.lsum[7 * k + 1 + d] * (1.0 / wgt) : S.cen[6 * k + d];
                    const double df = nc - S.cen[6 * k + d];
                    sh += df * df;
                    S.cen[6 * k + d] = nc;
                }
                sh = sqrt(sh);
                shift += sh * sh;
            }
            if (changed == 0) { S.strict = 1; S.done = 1; }
            else if (shift <= S.tol) S.done = 1;
        }
        __syncthreads();
        if (S.done) break;
    }

    SSF_STAMP(2);
    // ---- GMM init from one-hot k-means labels: strict convergence keeps the labels of the last
    //      pass (centres S.cenp), otherwise sklearn relabels with the final centres (S.cen).
    //      Only cluster 1's moments are summed, cluster 0 = total - cluster 1.
    {
        double cen[12], csn0, csn1;
        if (S.strict) {
#pragma unroll
            for (int k = 0; k < 12; ++k) cen[k] = uni(S.cenp[k]);
            csn0 = S.csnp[0]; csn1 = S.csnp[1];
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) cen[k] = uni(S.cen[k]);
            csn0 = 0.0; csn1 = 0.0;
            for (int d = 0; d < 6; ++d) { csn0 += cen[d] * cen[d]; csn1 += cen[6 + d] * cen[6 + d]; }
        }
        double acc[28];
#pragma unroll
        for (int k = 0; k < 28; ++k) acc[k] = 0.0;
        for_points_deep<kLloydDeep>(P, Fl, r0, r1, [&](int64_t, const double* x, bool val) {
            double v[6], dt0 = 0.0, dt1 = 0.0;
#pragma unroll
            for (int d = 0; d < 6; ++d) { v[d] = x[d] - mean[d]; dt0 += v[d] * cen[d]; dt1 += v[d] * cen[6 + d]; }
            const int l = (-2.0 * dt1 + csn1) < (-2.0 * dt0 + csn0) ? 1 : 0;
            const double w1 = val ? (double)l : 0.0;
            acc[0] += w1;
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double wv = w1 * v[a];
                acc[1 + a] += wv;
#pragma unroll
                for (int b = a; b < 6; ++b) acc[7 + up(a, b)] += wv * v[b];
            }
        });
        block_sum_rs<28>(acc, red);
        if (!exchange<28>(X, acc, xtmp, &okflag)) { sync_failed(); return; }
        if (tid < 2) {                           // lanes 0 / 1: the two components
            if (tid == 0) {
                S.passes += 1;
                for (int k = 0; k < 28; ++k) S.sums[k] = acc[k];
            }
            const int rc = gmm_params2(S, S.sums, 1, n);
            if (tid == 0) {
                if (rc != 0) S.status = SSF_POSE_GMM_FAILED;
                S.lb = -__builtin_inf();
                S.done = 0;
            }
        }
        __syncthreads();
    }

    SSF_STAMP(3);
    // ---- EM: one fused pass per iteration -- E-step with the current parameters and the
    //      M-step moments of component 1 (component 0 = total - component 1), in the
    //      difference form of em_diff_form: per point only delta = a1 - a0 (27 FMAs instead of
    //      two 27-FMA Mahalanobis forms), e = exp(-|delta|), r1 = 1/(1+e) if delta > 0 else
    //      e/(1+e), and the lower bound's per-point part max(delta, 0) + log1p(e).
    for (int it = 1; it <= 100 && S.status == 0; ++it) {
        const double cq = uni(S.cq);
        double acc[29];
#pragma unroll
        for (int k = 0; k < 29; ++k) acc[k] = 0.0;
        // sum of log1p(e) over the thread's points = log of the product of (1 + e), kept as
        // mantissa * 2^pexp (frexp per point: the product never overflows, one log per thread)
        double prod = 1.0;
        int pexp = 0;
#ifdef SSF_MASK_STAMPS
        if (it == 1 && tid == 0) S.dg_e[0] = S.dg_e[1] = S.dg_e[2] = 0.0;
        const unsigned long long e_t0 = __builtin_amdgcn_s_memtime();
#endif
#if SSF_EM_SGPR
        // the 27 E-step parameters as wave-uniform SGPR operands, read
        // from LDS once per pass instead of once per point pair
        double Aqs[21], bqs[6];
#pragma unroll
        for (int k = 0; k < 21; ++k) Aqs[k] = uni(S.Aq[k]);
#pragma unroll
        for (int k = 0; k < 6; ++k) bqs[k] = uni(S.bq[k]);
#elif SSF_EM_LDS_HOIST
        // the laundered LDS bases outside the loop: two loop-invariant VGPRs.  Laundered per
        // pair, their constants were rematerialised every iteration into registers the
        // prefetched point loads had landed in, so the loads were copied away (and waited for)
        // right after they were issued
        const LdsDouble* AqL = lds_laundered(S.Aq);
        const LdsDouble* bqL = lds_laundered(S.bq);
#endif
#if SSF_EM_DEEP == 4
        auto em_pair = [&](const double* xa, const double* xb, double wb) {
#else
        for_point_pairs(P, Fl, r0, r1, [&](const double* xa, const double* xb, double wb) {
#endif
#if SSF_EM_SGPR
            const double* Aq = Aqs;
            const double* bq = bqs;
#elif SSF_EM_LDS_HOIST
            const LdsDouble* Aq = AqL;
            const LdsDouble* bq = bqL;
#else
            // Aq / bq are re-read from LDS once per PAIR of points (lds_laundered)
            const LdsDouble* Aq = lds_laundered(S.Aq);
            const LdsDouble* bq = lds_laundered(S.bq);
#endif
            double va[6], vb[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) { va[a] = xa[a] - mean[a]; vb[a] = xb[a] - mean[a]; }
            double dl[2];
            em_delta2(va, vb, Aq, bq, cq, dl[0], dl[1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const double* v = h ? vb : va;
                const double wgt = h ? wb : 1.0;
                const double e = exp(-fabs(dl[h]));
                const double d = 1.0 + e;
                acc[28] += wgt * (dl[h] > 0.0 ? dl[h] : 0.0);
                prod *= (h ? (wb > 0.0 ? d : 1.0) : d);
                pexp += __builtin_amdgcn_frexp_exp(prod);
                prod = __builtin_amdgcn_frexp_mant(prod);
                const double inv = recip_1_2(d);
                const double r = wgt * (dl[h] > 0.0 ? inv : e * inv);
                acc[0] += r;
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    const double rv = r * v[a];
                    acc[1 + a] += rv;
#pragma unroll
                    for (int b = a; b < 6; ++b) acc[7 + up(a, b)] += rv * v[b];
                }
            }
#if SSF_EM_DEEP == 4
        };
        if constexpr (sizeof(T) == 4)
            for_point_pairs_glds(P, Fl, r0, r1, reinterpret_cast<float*>(bsum) + (tid >> 6) * 1024, em_pair);
        else
            for_point_pairs(P, Fl, r0, r1, em_pair);
#else
        });
#endif
        acc[28] += log(prod) + (double)pexp * 0.69314718055994530942;
        block_sum_rs<29>(acc, red);
#ifdef SSF_MASK_STAMPS
        const unsigned long long e_t1 = __builtin_amdgcn_s_memtime();
#endif
        if (!exchange<29>(X, acc, xtmp, &okflag)) { sync_failed(); return; }
#ifdef SSF_MASK_STAMPS
        const unsigned long long e_t2 = __builtin_amdgcn_s_memtime();
#endif
        if (tid < 2) {                           // lanes 0 / 1: the two components
            double prev = 0.0;
            if (tid == 0) {
                S.passes += 1;
                S.em_iter = it;
                prev = S.lb;
                S.lb = (S.C0 + acc[28]) / (double)n;   // C0: the a0 part, from this E-step's parameters
                for (int k = 0; k < 29; ++k) S.sums[k] = acc[k];
            }
            const int rc = gmm_params2(S, S.sums, 0, n);
            if (tid == 0) {
                if (rc != 0) S.status = SSF_POSE_GMM_FAILED;
                if (fabs(S.lb - prev) < 1e-3) { S.converged = 1; S.done = 1; }
            }
        }
        __syncthreads();
#ifdef SSF_MASK_STAMPS
        if (tid == 0) {
            S.dg_e[0] += (double)(e_t1 - e_t0); S.dg_e[1] += (double)(e_t2 - e_t1);
            S.dg_e[2] += (double)(__builtin_amdgcn_s_memtime() - e_t2);
        }
#endif
        if (S.done) break;
    }

    SSF_STAMP(4);
    // ---- final E-step labels + label-1 Kabsch sums (label 0 = totals from pass 0 - label 1).
    //      The mask is written in the same pass against a predicted background label (the
    //      heavier component); the rare frame whose majority disagrees gets one flip pass.
    {
        const int pred = S.logw[1] > S.logw[0] ? 1 : 0;
        const double cq = uni(S.cq);
        double x0[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) x0[d] = uni(S.x0[d]);
        double k1[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) k1[i] = 0.0;
        if (tid == 0) S.label0 = 0;
        __syncthreads();
        for_points_deep<kLloydDeep>(P, Fl, r0, r1, [&](int64_t i, const double* x, bool val) {
            // Aq / bq are re-read from LDS (broadcast ds_reads) for every point (lds_laundered)
            const LdsDouble* Aq = lds_laundered(S.Aq);
            const LdsDouble* bq = lds_laundered(S.bq);
            double v[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) v[a] = x[a] - mean[a];
            const int l = em_delta1(v, Aq, bq, cq) > 0.0 ? 1 : 0;   // a1 > a0
            // a slot past r1 holds point r1 - 1 again: its byte is rewritten with the same value
            if (bg_mask) bg_mask[fb + (val ? i : r1 - 1)] = (uint8_t)(l == pred);
            if (i == 0) S.label0 = l;
            const double w1 = val ? (double)l : 0.0;
            double sv[3], dv[3];
#pragma unroll
            for (int r = 0; r < 3; ++r) { dv[r] = x[3 + r] - x0[3 + r]; sv[r] = dv[r] + (x[r] - x0[r]); }
            k1[0] += w1;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const double ws = w1 * sv[r];
                k1[1 + r] += ws;
                k1[4 + r] += w1 * dv[r];
#pragma unroll
                for (int c = 0; c < 3; ++c) k1[7 + r * 3 + c] += ws * dv[c];
            }
        });
        block_sum_rs<16>(k1, red);
        if (G > 1) {                             // + the label of point 0 (part 0 has it)
            double v[17];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = k1[k];
            v[16] = g == 0 ? (double)S.label0 : 0.0;
            if (!exchange<17>(X, v, xtmp, &okflag)) { sync_failed(); return; }
#pragma unroll
            for (int k = 0; k < 16; ++k) k1[k] = v[k];
            if (tid == 0) S.label0 = (int)v[16];
            __syncthreads();
        }
        if (tid == 0) {
            S.passes += 1;
            const double n1 = k1[0];
            int bg;
            if (n1 * 2.0 > (double)n) bg = 1;
            else if (n1 * 2.0 < (double)n) bg = 0;
            else bg = S.label0;                     // Counter.most_common tie -> first seen
            S.bg = bg;
            S.bg_pred = pred;
            if (g == 0) {                           // part 0 publishes the frame's pose
                for (int i = 0; i < 26; ++i) out[i] = 0.0;
                double* kb = S.sums;
                for (int i = 0; i < 16; ++i) kb[i] = bg ? k1[i] : S.ktot[i] - k1[i];
                const double cs[3] = {S.x0[3] + S.x0[0], S.x0[4] + S.x0[1], S.x0[5] + S.x0[2]};
                const double cd[3] = {S.x0[3], S.x0[4], S.x0[5]};
                int st = S.status;
                if (st == 0) st = kabsch_finish(kb, cs, cd, reflection, out);
                out[SSF_POSE_OUT_STATUS] = st;
                out[SSF_POSE_OUT_BGLABEL] = bg;
                out[SSF_POSE_OUT_NBG] = kb[0];
                out[SSF_POSE_OUT_KM_ITER] = S.km_iter;
                out[SSF_POSE_OUT_EM_ITER] = S.em_iter;
                out[SSF_POSE_OUT_CONVERGED] = S.converged;
                out[SSF_POSE_OUT_CENTER0] = (double)S.c0;
                out[SSF_POSE_OUT_CENTER1] = (double)S.c1;
#ifdef SSF_MASK_STAMPS
                out[SSF_POSE_OUT_CENTER0] = S.dg_n > 0.0 ? S.dg_cyc / S.dg_n : 0.0;
                out[SSF_POSE_OUT_CENTER1] = S.dg_n > 0.0 ? S.dg_lab / (S.dg_n * (double)n) : 0.0;
                out[SSF_POSE_OUT_CONVERGED] = S.dg_wfull;
                out[SSF_POSE_OUT_NBG] = S.dg_full1;
                // EM pass split: points + block sum, exchange, M-step (cycles per pass)
                for (int k = 0; k < 3; ++k) out[SSF_POSE_OUT_T + k] = S.em_iter > 0 ? S.dg_e[k] / S.em_iter : 0.0;
#endif
                out[SSF_POSE_OUT_LOWER_BOUND] = S.lb;
                out[SSF_POSE_OUT_PASSES] = S.passes;
            }
        }
        __syncthreads();
    }
    if (bg_mask && S.bg != S.bg_pred) {
        for (int64_t i = r0 + tid; i < r1; i += blockDim.x) bg_mask[fb + i] ^= 1;
    }
    if (G > 1) {
        // done round: part 0's success status stands only once every part has finished its
        // share of the mask (a part whose wait timed out returned early and set the failure word)
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(X.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            X.seq += 1u;
            if (g == 0 && !wait_arrivals(X, (uint32_t)G * X.seq)) {
                for (int i = 0; i < SSF_POSE_OUT_STRIDE; ++i) out[i] = 0.0;
                out[SSF_POSE_OUT_STATUS] = SSF_POSE_SYNC_FAILED;
            }
        }
    }
    SSF_STAMP(5);
    }();                                       // the frame part
    }                                          // tickets
}

template <class T>
static hipError_t launch_mask_pose_t(hipStream_t s, int n_frames, const T* pts, const T* flow,
                                     const int64_t* frame_off, int mode, const uint8_t* mask_in,
                                     const double* draws, uint2* lloyd_rec, int reflection,
                                     uint8_t* bg_mask, double* out, int G, int slots,
                                     uint32_t* sync, double* parts, const int32_t* order, int queue) {
    if (n_frames <= 0) return hipSuccess;
    if (mode != SSF_MASK_GMM || G < 1 || !sync || !parts) G = 1;
    if (G > kMaxSplit) G = kMaxSplit;
    int grid = n_frames;
    // the frame queue (G == 1): at most `queue` work-groups, each taking frame tickets in order
    const bool tickets = G > 1 || (queue > 0 && sync && queue < n_frames);
    if (tickets) {
        // zero the ticket and arrival counters (16-byte multiple, from the allocation start)
        const size_t zb = (mask_sync_bytes(n_frames) + 15) & ~(size_t)15;
        hipError_t e = hipMemsetAsync(sync, 0, zb, s);
        if (e != hipSuccess) return e;
        const int64_t want = (int64_t)n_frames * G;
        const int cap = G > 1 ? slots : queue;
        grid = (int)(cap > 0 && want > cap ? cap : want);
    }
    kmark(s, sizeof(T) == 8 ? "k_mask_pose_f64" : "k_mask_pose");
    hipLaunchKernelGGL(k_mask_pose<T>, dim3(grid), dim3(kMaskThreads), 0, s, pts, flow, frame_off,
                       mode, mask_in, draws, lloyd_rec, reflection, bg_mask, out, n_frames, G, sync,
                       parts, order, tickets ? 1 : 0);
    return hipGetLastError();
}

// One storage type per translation unit (mask_pose_f64.hip compiles this file again with
// SSF_MASK_F64_TU), so the float kernel's code generation does not depend on the f64 variant.
#ifndef SSF_MASK_F64_TU
int mask_pose_slots(int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_mask_pose<float>, kMaskThreads, 0) != hipSuccess) return 0;
    return cus * per;
}

// ticket words, then per frame its arrival counter and its failure word
size_t mask_sync_bytes(int n_frames) { return (size_t)(4 + 2 * n_frames) * sizeof(uint32_t); }
size_t mask_parts_bytes(int n_frames, int G) {
    return G > 1 ? (size_t)n_frames * kMaxExchanges * G * kSlot * sizeof(double) : 0;
}

hipError_t launch_mask_pose(hipStream_t s, int n_frames, const float* pts, const float* flow,
                            const int64_t* frame_off, int mode, const uint8_t* mask_in,
                            const double* draws, uint2* lloyd_rec, int reflection, uint8_t* bg_mask,
                            double* out, int G, int slots, uint32_t* sync, double* parts,
                            const int32_t* order, int queue) {
    return launch_mask_pose_t(s, n_frames, pts, flow, frame_off, mode, mask_in, draws, lloyd_rec,
                              reflection, bg_mask, out, G, slots, sync, parts, order, queue);
}

#else
hipError_t launch_mask_pose(hipStream_t s, int n_frames, const double* pts, const double* flow,
                            const int64_t* frame_off, int mode, const uint8_t* mask_in,
                            const double* draws, uint2* lloyd_rec, int reflection, uint8_t* bg_mask,
                            double* out, int G, int slots, uint32_t* sync, double* parts,
                            const int32_t* order, int queue) {
    return launch_mask_pose_t(s, n_frames, pts, flow, frame_off, mode, mask_in, draws, lloyd_rec,
                              reflection, bg_mask, out, G, slots, sync, parts, order, queue);
}

#endif

}  // namespace ssf
