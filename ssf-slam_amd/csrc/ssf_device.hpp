// ssf_device.hpp -- device helpers shared by the gfx950 front-end kernels.
//
// Built with -ffp-contract=off: every float/double expression below is evaluated exactly as
// written (no FMA contraction) so the float stages reproduce the reference's x86 (non-FMA)
// arithmetic bit for bit, and the CPU oracle (oracle/ssf_oracle.c) can check them bitwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SSF_DEV __device__ __forceinline__

namespace ssf {

constexpr int kWave = 64;

SSF_DEV int lane_id() { return __lane_id(); }
SSF_DEV uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

SSF_DEV double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

SSF_DEV int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Deterministic block sum of N doubles per thread.  lds must hold (blockDim/64)*N doubles.
// On return every thread holds the block totals in v[].  Summation order is fixed (butterfly
// within a wave, then waves in index order) so results are reproducible run to run.
template <int N>
SSF_DEV void block_sum(double (&v)[N], double* lds) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = wave_sum(v[k]);
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) lds[w * N + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        for (int i = 0; i < nw; ++i) s += lds[i * N + k];
        v[k] = s;
    }
    __syncthreads();
}

// Deterministic block sum of N <= 32 doubles per thread, reduce-scatter form: five butterfly
// steps halve the values each lane carries (32 shuffled doubles instead of 6 N), lane L ends
// with value L >> 1 summed over its 32-lane half, one more step completes the wave; lane pairs
// write their value to LDS, thread k < N adds the waves in index order, every thread reads the
// N totals.  lds must hold (blockDim/64) * N doubles.  Same fixed order on every run.
template <int N>
SSF_DEV void block_sum_rs(double (&v)[N], double* lds) {
    static_assert(N <= 32, "block_sum_rs: N <= 32");
    const int lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    double a[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = i < N ? v[i] : 0.0;
#pragma unroll
    for (int h = 16, bit = 32; h >= 1; h >>= 1, bit >>= 1) {
        const bool up = (lane & bit) != 0;
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const double keep = up ? a[h + i] : a[i];
            const double send = up ? a[i] : a[h + i];
            a[i] = keep + __shfl_xor(send, bit, kWave);
        }
    }
    a[0] += __shfl_xor(a[0], 1, kWave);
    const int idx = lane >> 1;
    if ((lane & 1) == 0 && idx < N) lds[w * N + idx] = a[0];
    __syncthreads();
    if (threadIdx.x < N) {
        double s = 0.0;
        for (int i = 0; i < nw; ++i) s += lds[i * N + threadIdx.x];
        lds[threadIdx.x] = s;                  // only this thread reads slot threadIdx.x
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = lds[k];
    __syncthreads();
}

// block_sum_rs with the first four butterfly steps as DPP lane permutes (VALU; a shuffle is an
// LDS-unit round trip, and with one wave per SIMD k_solve's evaluations wait on each one) and
// the LDS staging double-buffered: the partials go to one of two LDS halves, alternating per call
// (`parity`), so no trailing barrier protects them from the next call.  The steps pair lanes as
// row_mirror (i <-> 15 - i: bit 3), row_half_mirror (i <-> 7 - i: bit 2), quad_perm xor 2 and
// xor 1 -- each pairs lanes that hold the same value subset -- then xor 16 and xor 32 by
// shuffles; lane L ends with value idx = L3 L2 L1 L0 L4 (bits).  ONE_BARRIER: every thread adds
// the NW waves' partials of all N values itself (NW x N broadcast LDS reads, one barrier); else
// thread k < N adds value k's and all threads read the N totals (two barriers).  lds must hold
// 2 x (NW + 1) x N doubles.  Fixed order: the same bits on every run.
SSF_DEV double dpp_perm_f64(double v, int ctrl_id) {
    const uint64_t b = __double_as_longlong(v);
    int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
    switch (ctrl_id) {                                         // compile-time after unrolling
        case 0: lo = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xf, 0xf, false); break;
        case 1: lo = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xf, 0xf, false); break;
        case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xf, 0xf, false); break;
        default: lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xf, 0xf, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xf, 0xf, false); break;
    }
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

template <int N, int NW, bool DPP, bool ONE_BARRIER>
SSF_DEV void block_sum_db(double (&v)[N], double* lds, int parity) {
    static_assert(N <= 32, "block_sum_db: N <= 32");
    const int lane = lane_id(), w = threadIdx.x >> 6;
    double a[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = i < N ? v[i] : 0.0;
    constexpr int kBitDpp[5] = {8, 4, 2, 1, 16}, kBitShfl[5] = {32, 16, 8, 4, 2};
#pragma unroll
    for (int st = 0, h = 16; st < 5; ++st, h >>= 1) {
        const int bit = DPP ? kBitDpp[st] : kBitShfl[st];
        const bool up = (lane & bit) != 0;
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const double keep = up ? a[h + i] : a[i];
            const double send = up ? a[i] : a[h + i];
            a[i] = keep + ((DPP && st < 4) ? dpp_perm_f64(send, st) : __shfl_xor(send, bit, kWave));
        }
    }
    int idx;
    bool wr;
    if (DPP) {
        a[0] += __shfl_xor(a[0], 32, kWave);
        idx = (((lane >> 3) & 1) << 4) | (((lane >> 2) & 1) << 3) | (((lane >> 1) & 1) << 2) |
              ((lane & 1) << 1) | ((lane >> 4) & 1);
        wr = lane < 32;
    } else {
        a[0] += __shfl_xor(a[0], 1, kWave);
        idx = lane >> 1;
        wr = (lane & 1) == 0;
    }
    double* L = lds + parity * (NW + 1) * N;
    if (wr && idx < N) L[w * N + idx] = a[0];
    __syncthreads();
    if (ONE_BARRIER) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            double s = L[k];
#pragma unroll
            for (int i = 1; i < NW; ++i) s += L[i * N + k];
            v[k] = s;
        }
    } else {
        if (threadIdx.x < N) {
            double s = L[threadIdx.x];
#pragma unroll
            for (int i = 1; i < NW; ++i) s += L[i * N + threadIdx.x];
            L[NW * N + threadIdx.x] = s;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = L[NW * N + k];
    }
}

template <typename T>
SSF_DEV T block_sum_scalar(T x, T* lds) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    if (lane_id() == 0) lds[w] = x;
    __syncthreads();
    T s = 0;
    for (int i = 0; i < nw; ++i) s += lds[i];
    __syncthreads();
    return s;
}

// ---- quaternion helpers, Eigen / Ceres semantics (x, y, z, w storage) -----------------
// Eigen Quaterniond * Vector3d (_transformVector): uv = 2 (qv x v); v + w uv + qv x uv.
SSF_DEV void quat_rotate(const double q[4], const double v[3], double out[3]) {
    double uv0 = q[1] * v[2] - q[2] * v[1];
    double uv1 = q[2] * v[0] - q[0] * v[2];
    double uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 = uv0 + uv0; uv1 = uv1 + uv1; uv2 = uv2 + uv2;
    double c0 = q[1] * uv2 - q[2] * uv1;
    double c1 = q[2] * uv0 - q[0] * uv2;
    double c2 = q[0] * uv1 - q[1] * uv0;
    out[0] = (v[0] + q[3] * uv0) + c0;
    out[1] = (v[1] + q[3] * uv1) + c1;
    out[2] = (v[2] + q[3] * uv2) + c2;
}

// Eigen quaternion product a * b.
SSF_DEV void quat_mul(const double a[4], const double b[4], double o[4]) {
    double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

// ceres::EigenQuaternionParameterization::Plus.
SSF_DEV void quat_plus(const double q[4], const double d[3], double o[4]) {
    double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (nd > 0.0) {
        double s = sin(nd) / nd;
        double dq[4] = {s * d[0], s * d[1], s * d[2], cos(nd)};
        quat_mul(dq, q, o);
    } else {
        o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3];
    }
}

}  // namespace ssf
