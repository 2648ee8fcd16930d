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
