// Point-set operators of the TFlow scene-flow network for gfx950.
//
// The reference imports them as `lib.pointnet2_utils` (scripts/ActiveSceneFlow/utils/utils.py:7,
// utils/soflow.py:7), a CUDA extension that is not vendored in the repository.  Semantics follow
// the reference's own torch restatements of the same operators, which are what this build can
// pin (tests/golden/make_golden_pn2.py imports them):
//   furthest_point_sample  <- farthest_point_sample   utils/utils.py:68-89
//   knn / three_nn         <- knn_point               utils/utils.py:92-108
//   gather_operation       <- index_points            utils/utils.py:48-65  ([B,C,N] layout)
//   grouping_operation     <- index_points_group      utils/soflow.py:21-32 ([B,C,N] layout)
//   three_interpolate      <- the weighted 3-NN sum   utils/utils.py:658-663
//   upsample_flow (fused)  <- UpsampleFlow.forward    utils/soflow.py:1442-1470
//   group_relative (fused) <- the grouping block of PointNetSetAbstraction.forward, utils.py:228-234
//
// Kernels (DESIGN.md §5 has their measured rates): k_fps_pk / k_fps (one work-group per cloud,
// packed-f32 distances, DPP wave reductions), k_knn / k_knn_split (brute-force exact k-NN over
// LDS tiles; the split variant spreads one cloud's reference set over 8 waves), k_gather_lds /
// k_three_interp_lds (feature rows staged in LDS) with global fallbacks, k_upsample (fused).
//
// Layouts are the extension's: coordinates [B, N, 3] ("xyz_t"), features [B, C, N], indices
// int32.  Every entry point is stateless and asynchronous on the caller's stream.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "ssf_device.hpp"
#include "../../include/ssf_pointnet2.h"

namespace {

thread_local char g_err[256] = "";

int32_t fail(int32_t code, const char* msg) {
    std::snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}

int32_t hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return SSF_PN2_OK;
    std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return SSF_PN2_E_HIP;
}

// (distance, index) packed into one positive double: high word = f32 distance bits (>= 0, so
// its bit order is its numeric order), low word = index.  The f64 order of such keys is the
// lexicographic (distance, index) order, so ties go to the lower index, as a stable top-k over
// indices in ascending order returns them.
SSF_DEV double nn_key(float d, int id) { return __hiloint2double(__float_as_int(d), id); }
SSF_DEV float nn_dist(double k) { return __int_as_float(__double2hiint(k)); }
SSF_DEV int nn_index(double k) { return __double2loint(k); }

template <int K>
SSF_DEV void nn_insert(double (&kk)[K], double key) {
#pragma unroll
    for (int s = 0; s < K; ++s) {
        double hi;
        asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(kk[s]), "v"(key));
        asm("v_min_f64 %0, %0, %1" : "+v"(kk[s]) : "v"(key));
        key = hi;
    }
}

// torch.sum(-(p1 - p2) ** 2, -1) (utils.py:106) negated: ((dx^2 + dy^2) + dz^2) in f32, no FMA
// (the library is compiled with -ffp-contract=off).
SSF_DEV float sq3(float dx, float dy, float dz) { return (dx * dx + dy * dy) + dz * dz; }

// ------------------------------------------------------------------------------------------
// Furthest point sampling (utils.py:68-89), clouds of more than 8192 points (k_fps_pk below
// takes the smaller ones).  One work-group per cloud; PPT points per thread kept in registers
// (point t + j * kFpsThreads), with their running min distance.  Iteration i: every thread folds
// the last centroid into its distances and keeps its best (distance, lowest index); a wave
// reduction to a u64 key (distance bits : ~index) and a cross-wave pass over an LDS slot
// (double-buffered by iteration parity, so one barrier per iteration) give the next centroid,
// whose coordinates travel with the key.  torch.max returns the FIRST maximum, hence the lowest
// index on ties.  PPT == 0: distances live in global scratch (N > 16384).
constexpr int kFpsThreads = 512;
constexpr int kFpsWaves = kFpsThreads / 64;

struct FpsSlot {
    unsigned long long key;
    float x, y, z, pad;
};

template <int PPT>
__global__ __launch_bounds__(kFpsThreads) void k_fps(const float* __restrict__ xyz, int n,
                                                     int npoint, const int32_t* __restrict__ start,
                                                     float* __restrict__ temp,
                                                     int32_t* __restrict__ out) {
    __shared__ FpsSlot slot[2][kFpsWaves];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* P = xyz + (int64_t)b * n * 3;
    float* T = temp ? temp + (int64_t)b * n : nullptr;
    int32_t* O = out + (int64_t)b * npoint;
    float px[PPT > 0 ? PPT : 1], py[PPT > 0 ? PPT : 1], pz[PPT > 0 ? PPT : 1], pd[PPT > 0 ? PPT : 1];
    if constexpr (PPT > 0) {
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int i = tid + j * kFpsThreads;
            const int ic = i < n ? i : n - 1;
            px[j] = P[3 * ic]; py[j] = P[3 * ic + 1]; pz[j] = P[3 * ic + 2];
            pd[j] = i < n ? 1e10f : -1.0f;               // padding never wins (distances >= 0)
        }
    } else {
        for (int i = tid; i < n; i += kFpsThreads) T[i] = 1e10f;   // torch.ones * 1e10 (:80)
    }
    int far = start ? min(max(start[b], 0), n - 1) : 0;
    float cx = P[3 * far], cy = P[3 * far + 1], cz = P[3 * far + 2];
    for (int it = 0; it < npoint; ++it) {
        if (tid == 0) O[it] = far;                                   // centroids[:, i] (:84)
        if (it + 1 == npoint) break;
        float bd = -1.0f, bx = 0.f, by = 0.f, bz = 0.f;
        int bi = 0x7fffffff;
        if constexpr (PPT > 0) {
#pragma unroll
            for (int j = 0; j < PPT; ++j) {
                const float d = sq3(px[j] - cx, py[j] - cy, pz[j] - cz);     // :86
                pd[j] = d < pd[j] ? d : pd[j];                                // :87-88
                if (pd[j] > bd) { bd = pd[j]; bi = tid + j * kFpsThreads; bx = px[j]; by = py[j]; bz = pz[j]; }
            }
        } else {
            for (int i = tid; i < n; i += kFpsThreads) {
                const float x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
                const float d = sq3(x - cx, y - cy, z - cz);
                const float t = d < T[i] ? d : T[i];
                T[i] = t;
                if (t > bd) { bd = t; bi = i; bx = x; by = y; bz = z; }
            }
        }
        // wave (max distance, min index): two 32-bit DPP reductions, as in k_fps_pk below; the
        // one lane holding the winner writes it with its coordinates
        const unsigned dbits = bd >= 0.0f ? __float_as_uint(bd) : 0u;
        const unsigned wmax = __ockl_wfred_max_u32(dbits);
        const unsigned myidx = bd >= 0.0f ? (unsigned)bi : 0x7fffffffu;
        const unsigned widx = __ockl_wfred_min_u32(dbits == wmax ? myidx : 0x7fffffffu);
        const unsigned long long key = ((unsigned long long)wmax << 32) | (0x7fffffffu - widx);
        if (myidx == widx || (widx == 0x7fffffffu && lane == 0)) {
            slot[it & 1][w] = FpsSlot{key, bx, by, bz, 0.f};
        }
        __syncthreads();
        FpsSlot best = slot[it & 1][0];
#pragma unroll
        for (int k = 1; k < kFpsWaves; ++k) {
            const FpsSlot s = slot[it & 1][k];
            if (s.key > best.key) best = s;
        }
        far = 0x7fffffff - (int)(unsigned)(best.key & 0xffffffffu);          // :89
        cx = best.x; cy = best.y; cz = best.z;
    }
}

// Clouds of up to 8192 points: the same iteration with two points per packed-f32 operation
// (v_pk_add_f32 / v_pk_mul_f32 on the pairs (j, j + 1)), and only (distance, slot) tracked per
// thread -- the winner's coordinates are read back from an LDS copy of the cloud after the
// cross-wave pass instead of being carried through three selects per point.
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int kFpsLdsMax = 8192;

template <int PPT, int TPB>
__global__ __launch_bounds__(TPB) void k_fps_pk(const float* __restrict__ xyz, int n,
                                                        int npoint, const int32_t* __restrict__ start,
                                                        int32_t* __restrict__ out) {
    static_assert(PPT % 2 == 0 && PPT * TPB <= kFpsLdsMax, "PPT");
    __shared__ float sx[kFpsLdsMax], sy[kFpsLdsMax], sz[kFpsLdsMax];
    __shared__ unsigned long long slot[2][TPB / 64];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* P = xyz + (int64_t)b * n * 3;
    int32_t* O = out + (int64_t)b * npoint;
    f2v px[PPT / 2], py[PPT / 2], pz[PPT / 2];
    float pd[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int i = tid + j * TPB;
        const int ic = i < n ? i : n - 1;
        const float x = P[3 * ic], y = P[3 * ic + 1], z = P[3 * ic + 2];
        px[j / 2][j % 2] = x; py[j / 2][j % 2] = y; pz[j / 2][j % 2] = z;
        pd[j] = i < n ? 1e10f : -1.0f;                  // padding never wins (distances >= 0)
        if (i < n) { sx[i] = x; sy[i] = y; sz[i] = z; }
    }
    __syncthreads();
    int far = start ? min(max(start[b], 0), n - 1) : 0;
    float cx = sx[far], cy = sy[far], cz = sz[far];
    for (int it = 0; it < npoint; ++it) {
        if (tid == 0) O[it] = far;                                   // centroids[:, i] (:84)
        if (it + 1 == npoint) break;
        const f2v c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
        float bd = -1.0f;
        int bj = 0;
#pragma unroll
        for (int h = 0; h < PPT / 2; ++h) {
            const f2v dx = px[h] - c2x, dy = py[h] - c2y, dz = pz[h] - c2z;
            const f2v d = (dx * dx + dy * dy) + dz * dz;                       // :86
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int j = 2 * h + e;
                pd[j] = d[e] < pd[j] ? d[e] : pd[j];                           // :87-88
                if (pd[j] > bd) { bd = pd[j]; bj = j; }
            }
        }
        // wave (max distance, min index) in two 32-bit DPP reductions (OCKL wave reduce): the
        // distance bits first (distances >= 0, so their u32 order is their numeric order;
        // padding lanes enter as 0 with index 0x7fffffff), then the lowest index among the
        // lanes holding that maximum
        const unsigned dbits = bd >= 0.0f ? __float_as_uint(bd) : 0u;
        const unsigned wmax = __ockl_wfred_max_u32(dbits);
        const unsigned myidx = bd >= 0.0f ? (unsigned)(tid + bj * TPB) : 0x7fffffffu;
        const unsigned widx = __ockl_wfred_min_u32(dbits == wmax ? myidx : 0x7fffffffu);
        if (lane == 0) slot[it & 1][w] = ((unsigned long long)wmax << 32) | (0x7fffffffu - widx);
        __syncthreads();
        unsigned long long best = slot[it & 1][0];
#pragma unroll
        for (int k = 1; k < TPB / 64; ++k) {
            const unsigned long long s2 = slot[it & 1][k];
            best = s2 > best ? s2 : best;
        }
        far = 0x7fffffff - (int)(unsigned)(best & 0xffffffffu);             // :89
        cx = sx[far]; cy = sy[far]; cz = sz[far];
    }
}

// ------------------------------------------------------------------------------------------
// Exact k-NN (knn_point, utils.py:92-108): for each query of [B, S, 3], the k nearest points of
// [B, N, 3] by f32 squared distance, ascending, ties to the lower index; outputs sqrt(distance)
// (:108) and int32 indices.  One query per thread, reference points staged through LDS in
// 2048-point tiles (SoA: broadcast reads), a sorted list of KM packed keys per thread with a
// branch-free insertion behind a threshold test.  KM >= k; the first k entries are the result.
constexpr int kKnnThreads = 256;
constexpr int kKnnTile = 2048;

template <int KM, int TPB>
__global__ __launch_bounds__(TPB) void k_knn(const float* __restrict__ query, int s,
                                                     const float* __restrict__ ref, int n, int k,
                                                     float* __restrict__ dist,
                                                     int32_t* __restrict__ idx) {
    __shared__ __attribute__((aligned(8))) float tx[kKnnTile], ty[kKnnTile], tz[kKnnTile];
    const int b = blockIdx.y;
    const int q = blockIdx.x * TPB + threadIdx.x;
    const float* Q = query + (int64_t)b * s * 3;
    const float* R = ref + (int64_t)b * n * 3;
    const int qc = q < s ? q : s - 1;
    const float qx = Q[3 * qc], qy = Q[3 * qc + 1], qz = Q[3 * qc + 2];
    const f2v q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz};
    double kk[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) kk[j] = nn_key(__builtin_inff(), 0x7fffffff);
    for (int t0 = 0; t0 < n; t0 += kKnnTile) {
        const int nt = min(kKnnTile, n - t0);
        __syncthreads();
        for (int j = threadIdx.x; j < nt; j += TPB) {
            tx[j] = R[3 * (t0 + j)]; ty[j] = R[3 * (t0 + j) + 1]; tz[j] = R[3 * (t0 + j) + 2];
        }
        __syncthreads();
        int j = 0;
        for (; j + 1 < nt; j += 2) {            // two candidates per packed-f32 operation
            const f2v dx = *reinterpret_cast<const f2v*>(tx + j) - q2x;
            const f2v dy = *reinterpret_cast<const f2v*>(ty + j) - q2y;
            const f2v dz = *reinterpret_cast<const f2v*>(tz + j) - q2z;
            const f2v d = (dx * dx + dy * dy) + dz * dz;
            const double k0 = nn_key(d[0], t0 + j), k1 = nn_key(d[1], t0 + j + 1);
            if (k0 < kk[KM - 1]) nn_insert<KM>(kk, k0);
            if (k1 < kk[KM - 1]) nn_insert<KM>(kk, k1);
        }
        if (j < nt) {
            const double key = nn_key(sq3(tx[j] - qx, ty[j] - qy, tz[j] - qz), t0 + j);
            if (key < kk[KM - 1]) nn_insert<KM>(kk, key);
        }
    }
    if (q >= s) return;
    const int64_t o = ((int64_t)b * s + q) * k;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j < k) {
            const bool have = j < n;
            dist[o + j] = have ? __builtin_sqrtf(nn_dist(kk[j])) : 0.0f;
            idx[o + j] = have ? nn_index(kk[j]) : 0;
        }
    }
}

// Small batches (the live node runs one cloud): 64 queries per work-group and W waves that each
// scan 1/W of every LDS tile, then wave 0 merges the W sorted partial lists from LDS.  Keys
// order (distance, index) totally, so the merged list is exactly the sequential scan's.
template <int KM, int W>
__global__ __launch_bounds__(64 * W) void k_knn_split(const float* __restrict__ query, int s,
                                                      const float* __restrict__ ref, int n, int k,
                                                      float* __restrict__ dist,
                                                      int32_t* __restrict__ idx) {
    __shared__ __attribute__((aligned(8))) float tx[kKnnTile], ty[kKnnTile], tz[kKnnTile];
    __shared__ double part[W - 1][KM][64];
    const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q = blockIdx.x * 64 + lane;
    const float* Q = query + (int64_t)b * s * 3;
    const float* R = ref + (int64_t)b * n * 3;
    const int qc = q < s ? q : s - 1;
    const float qx = Q[3 * qc], qy = Q[3 * qc + 1], qz = Q[3 * qc + 2];
    const f2v q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz};
    double kk[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) kk[j] = nn_key(__builtin_inff(), 0x7fffffff);
    constexpr int kSlice = kKnnTile / W;                     // even: pairs never straddle slices
    for (int t0 = 0; t0 < n; t0 += kKnnTile) {
        const int nt = min(kKnnTile, n - t0);
        __syncthreads();
        for (int j = threadIdx.x; j < nt; j += 64 * W) {
            tx[j] = R[3 * (t0 + j)]; ty[j] = R[3 * (t0 + j) + 1]; tz[j] = R[3 * (t0 + j) + 2];
        }
        __syncthreads();
        const int j1 = min(nt, (w + 1) * kSlice);
        int j = w * kSlice;
        for (; j + 1 < j1; j += 2) {
            const f2v dx = *reinterpret_cast<const f2v*>(tx + j) - q2x;
            const f2v dy = *reinterpret_cast<const f2v*>(ty + j) - q2y;
            const f2v dz = *reinterpret_cast<const f2v*>(tz + j) - q2z;
            const f2v d = (dx * dx + dy * dy) + dz * dz;
            const double k0 = nn_key(d[0], t0 + j), k1 = nn_key(d[1], t0 + j + 1);
            if (k0 < kk[KM - 1]) nn_insert<KM>(kk, k0);
            if (k1 < kk[KM - 1]) nn_insert<KM>(kk, k1);
        }
        if (j < j1) {
            const double key = nn_key(sq3(tx[j] - qx, ty[j] - qy, tz[j] - qz), t0 + j);
            if (key < kk[KM - 1]) nn_insert<KM>(kk, key);
        }
    }
    if (w > 0) {
#pragma unroll
        for (int j = 0; j < KM; ++j) part[w - 1][j][lane] = kk[j];
    }
    __syncthreads();
    if (w != 0 || q >= s) return;
    for (int v = 0; v < W - 1; ++v) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const double key = part[v][j][lane];
            if (key < kk[KM - 1]) nn_insert<KM>(kk, key);
        }
    }
    const int64_t o = ((int64_t)b * s + q) * k;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        if (j < k) {
            const bool have = j < n;
            dist[o + j] = have ? __builtin_sqrtf(nn_dist(kk[j])) : 0.0f;
            idx[o + j] = have ? nn_index(kk[j]) : 0;
        }
    }
}

// ------------------------------------------------------------------------------------------
// gather_operation(features [B,C,N], idx [B,S]) -> [B,C,S] and grouping_operation(features
// [B,C,N], idx [B,S,K]) -> [B,C,S,K]: one thread per output element (coalesced stores, the
// gathered reads hit L2 for the small feature maps of the network; a 2-D grid, rows = (batch,
// channel), so no per-element 64-bit divide).  Both are the same gather
// with G = S or S*K indices per batch element.  An index outside [0, N) yields 0 and sets *bad.
__global__ __launch_bounds__(256) void k_gather(const float* __restrict__ feat, int c, int n,
                                                const int32_t* __restrict__ idx, int g,
                                                int64_t nbc, float* __restrict__ out,
                                                int32_t* __restrict__ bad) {
    // grid: x over the g outputs of a (batch, channel) row, y over the B * C rows (no divides)
    for (int64_t bc = blockIdx.y; bc < nbc; bc += gridDim.y) {
        const int32_t* I = idx + (bc / c) * g;
        const float* F = feat + bc * n;
        float* O = out + bc * g;
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < g; j += gridDim.x * blockDim.x) {
            const int i = I[j];
            float v = 0.0f;
            if ((unsigned)i < (unsigned)n) v = F[i];
            else *bad = 1;
            O[j] = v;
        }
    }
}

// LDS-staged variants for feature rows that fit: a work-group owns CH consecutive channels of
// one batch element, loads their rows (CH * n floats) into LDS with coalesced reads, then walks
// the index list once (coalesced) and answers every channel from LDS.  Random 4-byte gathers
// from L2 each cost a whole cache line of L2->L1 traffic (the bound of k_gather above); here
// HBM sees the feature map once, the indices C / CH times and the output once.
constexpr int kStageThreads = 1024;
constexpr int kStageFloats = 36864;        // 144 KiB of LDS

// Output rows go to channel out_c0 + (c0 + k) of an out_c-channel output; center (nullable,
// [B, c, g / kdiv]) is subtracted from every gathered value of its row (grouped xyz minus the
// centroid, utils.py:232).
__global__ __launch_bounds__(kStageThreads) void k_gather_lds(const float* __restrict__ feat, int c,
                                                              int n, const int32_t* __restrict__ idx,
                                                              int g, int ch, float* __restrict__ out,
                                                              int out_c, int out_c0,
                                                              const float* __restrict__ center, int kdiv,
                                                              int32_t* __restrict__ bad) {
    extern __shared__ float rows[];
    const int b = blockIdx.y, c0 = blockIdx.x * ch;
    const int nch = min(ch, c - c0);
    const float* F = feat + ((int64_t)b * c + c0) * n;
    for (int e = threadIdx.x; e < nch * n; e += kStageThreads) rows[e] = F[e];
    __syncthreads();
    const int32_t* I = idx + (int64_t)b * g;
    float* O = out + ((int64_t)b * out_c + out_c0 + c0) * g;
    const int gc = g / kdiv;
    const float* CT = center ? center + ((int64_t)b * c + c0) * gc : nullptr;
    for (int j = threadIdx.x; j < g; j += kStageThreads) {
        int i = I[j];
        if ((unsigned)i >= (unsigned)n) { *bad = 1; i = -1; }
        const int jc = j / kdiv;
        for (int k = 0; k < nch; ++k) {
            const float v = i >= 0 ? rows[k * n + i] : 0.0f;
            O[(int64_t)k * g + j] = CT ? v - CT[(int64_t)k * gc + jc] : v;
        }
    }
}

__global__ __launch_bounds__(kStageThreads) void k_three_interp_lds(
    const float* __restrict__ feat, int c, int m, const int32_t* __restrict__ idx,
    const float* __restrict__ w, int n, int ch, float* __restrict__ out, int32_t* __restrict__ bad) {
    extern __shared__ float rows[];
    const int b = blockIdx.y, c0 = blockIdx.x * ch;
    const int nch = min(ch, c - c0);
    const float* F = feat + ((int64_t)b * c + c0) * m;
    for (int e = threadIdx.x; e < nch * m; e += kStageThreads) rows[e] = F[e];
    __syncthreads();
    const int32_t* I = idx + (int64_t)b * n * 3;
    const float* W = w + (int64_t)b * n * 3;
    float* O = out + ((int64_t)b * c + c0) * n;
    for (int j = threadIdx.x; j < n; j += kStageThreads) {
        int i[3];
        float wt[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            i[t] = I[3 * j + t];
            wt[t] = W[3 * j + t];
            if ((unsigned)i[t] >= (unsigned)m) { *bad = 1; i[t] = -1; }
        }
        for (int k = 0; k < nch; ++k) {
            const float* R = rows + k * m;
            const float v0 = i[0] >= 0 ? R[i[0]] : 0.0f, v1 = i[1] >= 0 ? R[i[1]] : 0.0f,
                        v2 = i[2] >= 0 ? R[i[2]] : 0.0f;
            O[(int64_t)k * n + j] = (wt[0] * v0 + wt[1] * v1) + wt[2] * v2;
        }
    }
}

// three_interpolate (utils.py:662-663 with normalised weights): out[b,c,n] =
// w0 f[i0] + w1 f[i1] + w2 f[i2], summed in that order.
__global__ __launch_bounds__(256) void k_three_interp(const float* __restrict__ feat, int c, int m,
                                                      const int32_t* __restrict__ idx,
                                                      const float* __restrict__ w, int n,
                                                      int64_t nbc, float* __restrict__ out,
                                                      int32_t* __restrict__ bad) {
    for (int64_t bc = blockIdx.y; bc < nbc; bc += gridDim.y) {
        const int64_t b = bc / c;
        const int32_t* I = idx + b * n * 3;
        const float* W = w + b * n * 3;
        const float* F = feat + bc * m;
        float* O = out + bc * n;
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
            float acc = 0.0f;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int i = I[3 * j + t];
                float v = 0.0f;
                if ((unsigned)i < (unsigned)m) v = F[i];
                else *bad = 1;
                acc = t == 0 ? W[3 * j] * v : acc + W[3 * j + t] * v;
            }
            O[j] = acc;
        }
    }
}

// ------------------------------------------------------------------------------------------
// UpsampleFlow.forward (soflow.py:1442-1470), fused: per dense point the k nearest sparse
// points (three_nn for k = 3, knn otherwise: the same exact k-NN), their Euclidean distances
// clamped at 1e-10 (:1463), inverse-distance weights normalised by their sum (:1464-1465), the
// weighted sum of the sparse features (:1472-1473) clamped to [-100, 100] (:1477).  The sparse
// cloud (S <= 4096 points) is staged once in LDS; one dense point per thread; each thread keeps
// its k indices and weights and then streams the C channels (one coalesced store per channel).
constexpr int kUpThreads = 256;
constexpr int kUpMaxSparse = 4096;

template <int KM, int TPB>
__global__ __launch_bounds__(TPB) void k_upsample(const float* __restrict__ xyz, int n,
                                                         const float* __restrict__ sxyz, int s,
                                                         const float* __restrict__ sfeat, int c,
                                                         int k, float* __restrict__ out) {
    __shared__ __attribute__((aligned(8))) float tx[kUpMaxSparse], ty[kUpMaxSparse], tz[kUpMaxSparse];
    const int b = blockIdx.y;
    const int q = blockIdx.x * TPB + threadIdx.x;
    const float* X = xyz + (int64_t)b * 3 * n;       // [B, 3, N] (the module's input layout)
    const float* SX = sxyz + (int64_t)b * 3 * s;     // [B, 3, S]
    for (int j = threadIdx.x; j < s; j += TPB) {
        tx[j] = SX[j]; ty[j] = SX[s + j]; tz[j] = SX[2 * s + j];
    }
    __syncthreads();
    if (q >= n) return;
    const float qx = X[q], qy = X[n + q], qz = X[2 * n + q];
    double kk[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) kk[j] = nn_key(__builtin_inff(), 0x7fffffff);
    const f2v q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz};
    int j0 = 0;
    for (; j0 + 1 < s; j0 += 2) {
        const f2v dx = *reinterpret_cast<const f2v*>(tx + j0) - q2x;
        const f2v dy = *reinterpret_cast<const f2v*>(ty + j0) - q2y;
        const f2v dz = *reinterpret_cast<const f2v*>(tz + j0) - q2z;
        const f2v d = (dx * dx + dy * dy) + dz * dz;
        const double k0 = nn_key(d[0], j0), k1 = nn_key(d[1], j0 + 1);
        if (k0 < kk[KM - 1]) nn_insert<KM>(kk, k0);
        if (k1 < kk[KM - 1]) nn_insert<KM>(kk, k1);
    }
    if (j0 < s) {
        const double key = nn_key(sq3(tx[j0] - qx, ty[j0] - qy, tz[j0] - qz), j0);
        if (key < kk[KM - 1]) nn_insert<KM>(kk, key);
    }
    int id[KM];
    float wt[KM];
    float norm = 0.0f;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        id[j] = 0; wt[j] = 0.0f;
        if (j < k && j < s) {
            id[j] = nn_index(kk[j]);
            // grouped_xyz_norm = sparse[idx] - xyz (:1462); torch.norm over the 3 channels
            const float gx = tx[id[j]] - qx, gy = ty[id[j]] - qy, gz = tz[id[j]] - qz;
            float d = __builtin_sqrtf(sq3(gx, gy, gz));
            d = d > 1e-10f ? d : 1e-10f;
            wt[j] = 1.0f / d;
            norm = j == 0 ? wt[j] : norm + wt[j];
        }
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) wt[j] = wt[j] / norm;
    const float* SF = sfeat + (int64_t)b * c * s;
    float* O = out + (int64_t)b * c * n;
    for (int ch = 0; ch < c; ++ch) {
        const float* F = SF + (int64_t)ch * s;
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < KM; ++j)
            if (j < k && j < s) acc = j == 0 ? wt[j] * F[id[j]] : acc + wt[j] * F[id[j]];
        O[(int64_t)ch * n + q] = fminf(fmaxf(acc, -100.0f), 100.0f);
    }
}

// The LDS-staged kernels take up to 144 KiB of dynamic LDS (above the 64 KiB default limit).
hipError_t allow_stage_lds() {
    static hipError_t once = [] {
        hipError_t e = hipFuncSetAttribute((const void*)k_gather_lds,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kStageFloats * 4);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)k_three_interp_lds,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kStageFloats * 4);
        return e;
    }();
    return once;
}

// Channels per staging work-group: as many as fit in LDS, but few enough that the launch has
// about 512 work-groups (a single cloud with wide feature maps would otherwise run on a few CUs).
int stage_channels(int c, int b, int row) {
    const int fit = kStageFloats / row;
    const int want = (int)(((int64_t)c * b + 511) / 512);
    return max(1, min(c, min(fit, want)));
}

dim3 grid_rows(int64_t per_row, int64_t rows) {
    const int64_t gx = (per_row + 255) / 256;
    return dim3((unsigned)(gx < 4096 ? (gx > 0 ? gx : 1) : 4096), (unsigned)(rows < 65535 ? rows : 65535));
}

}  // namespace

// ------------------------------------------------------------------------------------------
extern "C" {

const char* ssf_pn2_last_error(void) { return g_err; }

int32_t ssf_pn2_furthest_point_sample(void* stream, int32_t b, int32_t n, int32_t npoint,
                                      const float* d_xyz, const int32_t* d_start, float* d_temp,
                                      int32_t* d_idx) {
    if (b < 0 || n <= 0 || npoint < 0 || !d_xyz || !d_idx) return fail(SSF_PN2_E_ARG, "fps: bad arguments");
    if (b == 0 || npoint == 0) return SSF_PN2_OK;
    hipStream_t s = (hipStream_t)stream;
    const int ppt = (n + kFpsThreads - 1) / kFpsThreads;
    if (n <= 4096) hipLaunchKernelGGL((k_fps_pk<16, 256>), dim3(b), dim3(256), 0, s, d_xyz, n, npoint, d_start, d_idx);
    else if (n <= 8192) hipLaunchKernelGGL((k_fps_pk<32, 256>), dim3(b), dim3(256), 0, s, d_xyz, n, npoint, d_start, d_idx);
    else if (ppt <= 32) hipLaunchKernelGGL(k_fps<32>, dim3(b), dim3(kFpsThreads), 0, s, d_xyz, n, npoint, d_start, nullptr, d_idx);
    else {
        if (!d_temp) return fail(SSF_PN2_E_ARG, "fps: n > 16384 needs d_temp (b * n floats)");
        hipLaunchKernelGGL(k_fps<0>, dim3(b), dim3(kFpsThreads), 0, s, d_xyz, n, npoint, d_start, d_temp, d_idx);
    }
    return hip_status(hipGetLastError(), "k_fps");
}

int32_t ssf_pn2_knn(void* stream, int32_t b, int32_t s_q, int32_t n, int32_t k,
                    const float* d_query, const float* d_ref, float* d_dist, int32_t* d_idx) {
    if (b < 0 || s_q < 0 || n <= 0 || k <= 0 || k > SSF_PN2_KNN_MAX || !d_query || !d_ref || !d_dist || !d_idx)
        return fail(SSF_PN2_E_ARG, "knn: bad arguments (need n > 0, 0 < k <= 32)");
    if (b == 0 || s_q == 0) return SSF_PN2_OK;
    if (b > 65535) return fail(SSF_PN2_E_ARG, "knn: b > 65535");
    hipStream_t st = (hipStream_t)stream;
    // small batches (the live node runs one cloud): the reference set is split over the waves
    // of a work-group (8 waves, 4 for k > 16) and the partial lists merged in LDS
    if ((int64_t)b * ((s_q + kKnnThreads - 1) / kKnnThreads) < 512) {
        const dim3 grid((s_q + 63) / 64, b);
        if (k <= 4) hipLaunchKernelGGL((k_knn_split<4, 8>), grid, dim3(512), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else if (k <= 8) hipLaunchKernelGGL((k_knn_split<8, 8>), grid, dim3(512), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else if (k <= 16) hipLaunchKernelGGL((k_knn_split<16, 8>), grid, dim3(512), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else hipLaunchKernelGGL((k_knn_split<32, 4>), grid, dim3(256), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
    } else {
        const dim3 grid((s_q + kKnnThreads - 1) / kKnnThreads, b);
        if (k <= 4) hipLaunchKernelGGL((k_knn<4, kKnnThreads>), grid, dim3(kKnnThreads), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else if (k <= 8) hipLaunchKernelGGL((k_knn<8, kKnnThreads>), grid, dim3(kKnnThreads), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else if (k <= 16) hipLaunchKernelGGL((k_knn<16, kKnnThreads>), grid, dim3(kKnnThreads), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
        else hipLaunchKernelGGL((k_knn<32, kKnnThreads>), grid, dim3(kKnnThreads), 0, st, d_query, s_q, d_ref, n, k, d_dist, d_idx);
    }
    return hip_status(hipGetLastError(), "k_knn");
}

int32_t ssf_pn2_three_nn(void* stream, int32_t b, int32_t n, int32_t m, const float* d_unknown,
                         const float* d_known, float* d_dist, int32_t* d_idx) {
    return ssf_pn2_knn(stream, b, n, m, 3, d_unknown, d_known, d_dist, d_idx);
}

int32_t ssf_pn2_gather(void* stream, int32_t b, int32_t c, int32_t n, int32_t g,
                       const float* d_feat, const int32_t* d_idx, float* d_out, int32_t* d_bad) {
    if (b < 0 || c < 0 || n <= 0 || g < 0 || !d_feat || !d_idx || !d_out || !d_bad)
        return fail(SSF_PN2_E_ARG, "gather: bad arguments");
    const int64_t total = (int64_t)b * c * g;
    if (total == 0) return SSF_PN2_OK;
    if (n <= kStageFloats && b <= 65535) {
        if (hipError_t e = allow_stage_lds(); e != hipSuccess) return hip_status(e, "gather: LDS limit");
        const int ch = stage_channels(c, b, n);
        hipLaunchKernelGGL(k_gather_lds, dim3((c + ch - 1) / ch, b), dim3(kStageThreads),
                           (size_t)ch * n * 4, (hipStream_t)stream, d_feat, c, n, d_idx, g, ch, d_out, c, 0,
                           (const float*)nullptr, 1, d_bad);
    } else {
        hipLaunchKernelGGL(k_gather, grid_rows(g, (int64_t)b * c), dim3(256), 0, (hipStream_t)stream, d_feat,
                           c, n, d_idx, g, (int64_t)b * c, d_out, d_bad);
    }
    return hip_status(hipGetLastError(), "k_gather");
}

int32_t ssf_pn2_group_relative(void* stream, int32_t b, int32_t n, int32_t s, int32_t k, int32_t c,
                               const float* d_xyz, const float* d_new_xyz, const float* d_feat,
                               const int32_t* d_idx, float* d_out, int32_t* d_bad) {
    if (b < 0 || n <= 0 || n > kStageFloats || s < 0 || k <= 0 || c < 0 || (c > 0 && !d_feat) ||
        !d_xyz || !d_new_xyz || !d_idx || !d_out || !d_bad)
        return fail(SSF_PN2_E_ARG, "group_relative: bad arguments (0 < n <= 36864)");
    if (b == 0 || s == 0) return SSF_PN2_OK;
    if (b > 65535) return fail(SSF_PN2_E_ARG, "group_relative: b > 65535");
    if (hipError_t e = allow_stage_lds(); e != hipSuccess) return hip_status(e, "group_relative: LDS limit");
    hipStream_t st = (hipStream_t)stream;
    const int g = s * k, oc = 3 + c;
    const int chx = stage_channels(3, b, n);
    hipLaunchKernelGGL(k_gather_lds, dim3((3 + chx - 1) / chx, b), dim3(kStageThreads), (size_t)chx * n * 4, st,
                       d_xyz, 3, n, d_idx, g, chx, d_out, oc, 0, d_new_xyz, k, d_bad);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return hip_status(e, "k_gather_lds (xyz)");
    if (c > 0) {
        const int ch = stage_channels(c, b, n);
        hipLaunchKernelGGL(k_gather_lds, dim3((c + ch - 1) / ch, b), dim3(kStageThreads), (size_t)ch * n * 4, st,
                           d_feat, c, n, d_idx, g, ch, d_out, oc, 3, (const float*)nullptr, 1, d_bad);
    }
    return hip_status(hipGetLastError(), "k_gather_lds (features)");
}

int32_t ssf_pn2_three_interpolate(void* stream, int32_t b, int32_t c, int32_t m, int32_t n,
                                  const float* d_feat, const int32_t* d_idx, const float* d_weight,
                                  float* d_out, int32_t* d_bad) {
    if (b < 0 || c < 0 || m <= 0 || n < 0 || !d_feat || !d_idx || !d_weight || !d_out || !d_bad)
        return fail(SSF_PN2_E_ARG, "three_interpolate: bad arguments");
    const int64_t total = (int64_t)b * c * n;
    if (total == 0) return SSF_PN2_OK;
    if (m <= kStageFloats && b <= 65535) {
        if (hipError_t e = allow_stage_lds(); e != hipSuccess) return hip_status(e, "three_interpolate: LDS limit");
        const int ch = stage_channels(c, b, m);
        hipLaunchKernelGGL(k_three_interp_lds, dim3((c + ch - 1) / ch, b), dim3(kStageThreads),
                           (size_t)ch * m * 4, (hipStream_t)stream, d_feat, c, m, d_idx, d_weight, n, ch,
                           d_out, d_bad);
    } else {
        hipLaunchKernelGGL(k_three_interp, grid_rows(n, (int64_t)b * c), dim3(256), 0, (hipStream_t)stream,
                           d_feat, c, m, d_idx, d_weight, n, (int64_t)b * c, d_out, d_bad);
    }
    return hip_status(hipGetLastError(), "k_three_interp");
}

int32_t ssf_pn2_upsample_flow(void* stream, int32_t b, int32_t n, int32_t s, int32_t c, int32_t k,
                              const float* d_xyz, const float* d_sparse_xyz,
                              const float* d_sparse_feat, float* d_out) {
    if (b < 0 || n < 0 || s <= 0 || s > SSF_PN2_UPSAMPLE_MAX_SPARSE || c < 0 || k <= 0 || k > 16 ||
        !d_xyz || !d_sparse_xyz || !d_sparse_feat || !d_out)
        return fail(SSF_PN2_E_ARG, "upsample_flow: bad arguments (0 < s <= 4096, 0 < k <= 16)");
    if (b == 0 || n == 0) return SSF_PN2_OK;
    if (b > 65535) return fail(SSF_PN2_E_ARG, "upsample_flow: b > 65535");
    hipStream_t st = (hipStream_t)stream;
    if ((int64_t)b * ((n + kUpThreads - 1) / kUpThreads) < 512) {
        const dim3 grid((n + 63) / 64, b);
        if (k <= 4) hipLaunchKernelGGL((k_upsample<4, 64>), grid, dim3(64), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
        else if (k <= 8) hipLaunchKernelGGL((k_upsample<8, 64>), grid, dim3(64), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
        else hipLaunchKernelGGL((k_upsample<16, 64>), grid, dim3(64), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
    } else {
        const dim3 grid((n + kUpThreads - 1) / kUpThreads, b);
        if (k <= 4) hipLaunchKernelGGL((k_upsample<4, kUpThreads>), grid, dim3(kUpThreads), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
        else if (k <= 8) hipLaunchKernelGGL((k_upsample<8, kUpThreads>), grid, dim3(kUpThreads), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
        else hipLaunchKernelGGL((k_upsample<16, kUpThreads>), grid, dim3(kUpThreads), 0, st, d_xyz, n, d_sparse_xyz, s, d_sparse_feat, c, k, d_out);
    }
    return hip_status(hipGetLastError(), "k_upsample");
}

}  // extern "C"
