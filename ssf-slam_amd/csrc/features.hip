// features.hip -- frameFeature::cloudHandler (src/frameFeature.cpp:35-139) on gfx950.
//
// Four kernels per batch of frames, all HBM-streaming:
//   k_bin_count   ring id per point (frameFeature.cpp:57-72) + per-chunk ring histogram
//   k_bin_scan    per-frame exclusive scans -> per-(chunk,row) bases and row offsets
//   k_bin_scatter stable per-row partition (:73-80): wave ballot "match" on the 6-bit row id
//                 gives each point its rank among same-row points of its wave; waves are
//                 ordered through LDS -> the reference's push_back order is reproduced exactly.
//                 intensity = indexInRow + row/100.0 (:77)
//   k_curv_select one work-group per (frame,row): the row is streamed through LDS in tiles with
//                 a 5-point halo, the 11-tap stencil (:84-107) is evaluated left to right in
//                 float, and wave 0 runs the greedy spacing rule (:110-123) with a 64-bit ballot
//                 of candidates per 64 points (jstart is wave-uniform).
//   k_compact     row-major concatenation of the selected points (framePlanePtr order).
#include "ssf_device.hpp"
#include "ssf_internal.hpp"

namespace ssf {

// frameFeature.cpp:57-72 (see oracle/ssf_oracle.c orc_ring_id for the precision choices).
SSF_DEV int ring_id(float x, float y, float z, int n_rows) {
    float r2 = x * x + y * y;
    float ratio = z / sqrtf(r2);
    float angle = (float)(atan((double)ratio) * 180.0 / 3.14159265358979323846);
    int id = -1;
    if (n_rows == 16) {
        id = (int)((double)((angle + 15.0f) / 2.0f) + 0.5);
    } else if (n_rows == 64) {
        if ((double)angle >= -8.83)
            id = (int)((2.0 - (double)angle) * 3.0 + 0.5);
        else
            id = n_rows / 2 + (int)((-8.83 - (double)angle) * 2.0 + 0.5);
    }
    return (id > -1 && id < n_rows) ? id : -1;
}

__global__ __launch_bounds__(256) void k_bin_count(const float* __restrict__ pts, int stride,
                                                   const int64_t* __restrict__ frame_off,
                                                   int n_rows, int n_chunks,
                                                   int8_t* __restrict__ rid,
                                                   int32_t* __restrict__ hist) {
    __shared__ int h[kMaxRows];
    const int f = blockIdx.y, c = blockIdx.x;
    if (threadIdx.x < kMaxRows) h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t b = frame_off[f], e = frame_off[f + 1];
    const int64_t s = b + (int64_t)c * kBinChunk;
    if (s < e) {
        const int64_t t = min(e, s + (int64_t)kBinChunk);
        for (int64_t i = s + threadIdx.x; i < t; i += blockDim.x) {
            const float* p = pts + i * stride;
            int id = ring_id(p[0], p[1], p[2], n_rows);
            rid[i] = (int8_t)id;
            if (id >= 0) atomicAdd(&h[id], 1);
        }
    }
    __syncthreads();
    if (threadIdx.x < n_rows) hist[((int64_t)f * n_chunks + c) * n_rows + threadIdx.x] = h[threadIdx.x];
}

// One wave per frame: thread r scans its row's chunk counts in chunk order.
__global__ __launch_bounds__(64) void k_bin_scan(int n_rows, int n_chunks, int32_t* __restrict__ hist,
                                                 int32_t* __restrict__ ring_off) {
    const int f = blockIdx.x, r = threadIdx.x;
    int run = 0;
    if (r < n_rows) {
        int32_t* hp = hist + (int64_t)f * n_chunks * n_rows + r;
        for (int c = 0; c < n_chunks; ++c) {
            int v = hp[(int64_t)c * n_rows];
            hp[(int64_t)c * n_rows] = run;
            run += v;
        }
    }
    // exclusive scan of row totals across the wave
    int incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(incl, o, 64);
        if (r >= o) incl += y;
    }
    int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    if (r < n_rows) ro[r] = incl - run;
    if (r == n_rows - 1) ro[n_rows] = incl;
}

__global__ __launch_bounds__(256) void k_bin_scatter(const float* __restrict__ pts, int stride,
                                                     const int64_t* __restrict__ frame_off,
                                                     int n_rows, int n_chunks,
                                                     const int8_t* __restrict__ rid,
                                                     const int32_t* __restrict__ chunk_base,
                                                     const int32_t* __restrict__ ring_off,
                                                     float4* __restrict__ out) {
    __shared__ int run[kMaxRows];
    __shared__ int wcnt[4][kMaxRows];
    const int f = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) return;  // uniform
    const int64_t t = min(e, s + (int64_t)kBinChunk);
    if (tid < kMaxRows) {
        run[tid] = 0;
        wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    }
    __syncthreads();
    const int32_t* cb = chunk_base + ((int64_t)f * n_chunks + c) * n_rows;
    const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    for (int64_t base = s; base < t; base += 256) {
        const int64_t i = base + tid;
        const int id = (i < t) ? (int)rid[i] : -1;
        uint64_t m = __ballot(id >= 0);
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {
            const bool on = (id >> bit) & 1;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const int rank = __popcll(m & lanemask_lt());
        if (id >= 0 && rank == 0) wcnt[w][id] = __popcll(m);
        __syncthreads();
        if (id >= 0) {
            int pre = run[id];
            for (int k = 0; k < w; ++k) pre += wcnt[k][id];
            const int idx_in_row = cb[id] + pre + rank;
            const float* p = pts + i * stride;
            float4 v;
            v.x = p[0]; v.y = p[1]; v.z = p[2];
            v.w = (float)((double)idx_in_row + (double)id / 100.0);
            out[fb + ro[id] + idx_in_row] = v;
        }
        __syncthreads();
        if (tid < kMaxRows) {
            run[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
            wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
        }
        __syncthreads();
    }
}

constexpr int kCurvTile = 2048;

SSF_DEV float stencil11(const float* a, int k) {  // a[k] is point j-5 ... a[k+10] is j+5
    float s = a[k] + a[k + 1];
    s = s + a[k + 2];
    s = s + a[k + 3];
    s = s + a[k + 4];
    s = s - 10.0f * a[k + 5];
    s = s + a[k + 6];
    s = s + a[k + 7];
    s = s + a[k + 8];
    s = s + a[k + 9];
    s = s + a[k + 10];
    return s;
}

__global__ __launch_bounds__(256) void k_curv_select(const int64_t* __restrict__ frame_off,
                                                     int n_rows, int row_start, int row_end,
                                                     float plane_min, int plane_span,
                                                     const int32_t* __restrict__ ring_off,
                                                     const float4* __restrict__ rxyzi,
                                                     float* __restrict__ curv,
                                                     int32_t* __restrict__ sel,
                                                     int32_t* __restrict__ sel_cnt) {
    __shared__ float sx[kCurvTile + 16], sy[kCurvTile + 16], sz[kCurvTile + 16];
    __shared__ float cv[kCurvTile];
    const int r = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    const int rs = ro[r], n_r = ro[r + 1] - rs;
    const int64_t base = frame_off[f] + rs;
    const bool in_rows = (r >= row_start) && (r < n_rows - row_end);
    if (!in_rows) {
        if (curv)
            for (int j = tid; j < n_r; j += blockDim.x) curv[base + j] = 0.0f;
        if (tid == 0) sel_cnt[(int64_t)f * n_rows + r] = 0;
        return;
    }
    int cnt = 0;     // wave-0 uniform
    int jstart = 0;  // wave-0 uniform
    for (int t0 = 0; t0 < n_r; t0 += kCurvTile) {
        for (int k = tid; k < kCurvTile + 10; k += blockDim.x) {
            const int j = t0 - 5 + k;
            if (j >= 0 && j < n_r) {
                const float4 v = rxyzi[base + j];
                sx[k] = v.x; sy[k] = v.y; sz[k] = v.z;
            }
        }
        __syncthreads();
        for (int k = tid; k < kCurvTile; k += blockDim.x) {
            const int j = t0 + k;
            if (j >= n_r) break;
            float v = 0.0f;
            if (j >= 5 && j < n_r - 5) {
                const float dx = stencil11(sx, k), dy = stencil11(sy, k), dz = stencil11(sz, k);
                v = dx * dx + dy * dy;
                v = v + dz * dz;
            }
            cv[k] = v;
            if (curv) curv[base + j] = v;
        }
        __syncthreads();
        if (tid < 64) {
            const int lim = min(kCurvTile, n_r - t0);
            for (int sub = 0; sub < lim; sub += 64) {
                const int k = sub + tid;
                const bool cand = (k < lim) && (cv[k] < plane_min);
                uint64_t m = __ballot(cand);
                const int j0 = t0 + sub;
                while (true) {
                    const int lo = jstart - j0;
                    if (lo >= 64) break;
                    if (lo > 0) m &= ~((1ull << lo) - 1ull);
                    if (!m) break;
                    const int l = __ffsll((unsigned long long)m) - 1;
                    const int jj = j0 + l;
                    if (tid == 0) sel[base + cnt] = jj;
                    cnt++;
                    jstart = jj + plane_span;
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) sel_cnt[(int64_t)f * n_rows + r] = cnt;
}

__global__ __launch_bounds__(256) void k_compact(const int64_t* __restrict__ frame_off, int n_rows,
                                                 const int32_t* __restrict__ ring_off,
                                                 const float4* __restrict__ rxyzi,
                                                 const int32_t* __restrict__ sel,
                                                 const int32_t* __restrict__ sel_cnt,
                                                 float4* __restrict__ plane,
                                                 int32_t* __restrict__ plane_count) {
    const int r = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const int32_t* sc = sel_cnt + (int64_t)f * n_rows;
    int pre = 0;
    for (int k = 0; k < r; ++k) pre += sc[k];  // <= 63 uniform loads
    const int n = sc[r];
    if (r == n_rows - 1 && tid == 0) plane_count[f] = pre + n;
    const int64_t fb = frame_off[f];
    const int64_t base = fb + ring_off[(int64_t)f * (n_rows + 1) + r];
    for (int k = tid; k < n; k += blockDim.x) plane[fb + pre + k] = rxyzi[base + sel[base + k]];
}

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, int8_t* rid, int32_t* hist, int32_t* ring_off,
                                 float4* ring_xyzi, float* curv, int32_t* sel, int32_t* sel_cnt,
                                 float4* plane, int32_t* plane_count) {
    const int R = cfg.n_rows;
    const int n_chunks = (int)((max_pts + kBinChunk - 1) / kBinChunk);
    if (n_frames <= 0) return hipSuccess;
    if (n_chunks > 0) {
        hipLaunchKernelGGL(k_bin_count, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, rid, hist);
    }
    hipLaunchKernelGGL(k_bin_scan, dim3(n_frames), dim3(64), 0, s, R, n_chunks, hist, ring_off);
    if (n_chunks > 0) {
        hipLaunchKernelGGL(k_bin_scatter, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, rid, hist, ring_off, ring_xyzi);
    }
    hipLaunchKernelGGL(k_curv_select, dim3(R, n_frames), dim3(256), 0, s, frame_off, R,
                       cfg.row_start, cfg.row_end, cfg.plane_min, cfg.plane_span, ring_off,
                       ring_xyzi, curv, sel, sel_cnt);
    hipLaunchKernelGGL(k_compact, dim3(R, n_frames), dim3(256), 0, s, frame_off, R, ring_off,
                       ring_xyzi, sel, sel_cnt, plane, plane_count);
    return hipGetLastError();
}

}  // namespace ssf
