// features.hip -- frameFeature::cloudHandler (src/frameFeature.cpp:35-139) on gfx950.
//
// Four kernels per batch of frames, all HBM-streaming:
//   k_bin_count   ring id per point (frameFeature.cpp:57-72) + per-chunk ring histogram
//   k_bin_scan    per-frame exclusive scans -> per-(chunk,row) bases and row offsets
//   k_bin_scatter stable per-row partition (:73-80): wave ballot "match" on the 6-bit row id
//                 gives each point its rank among same-row points; waves own contiguous
//                 quarters of the chunk and are prefixed in order -> the reference's push_back
//                 order exactly.  The chunk is regrouped by row in LDS and stored in contiguous
//                 per-row runs of packed xyz (12 B/pt: the ring order alone carries indexInRow,
//                 so intensity = indexInRow + row/100.0 (:77) is recomputed where it is needed)
//   k_curv_select one work-group per (frame,row): the row in one burst into an LDS tile, the
//                 11-tap stencil (:84-107) evaluated left to right in float, 8 centres per
//                 thread; the greedy spacing rule (:110-123) on one wave over candidate words;
//                 the selected points (with their encoded intensity) stored into per-row slots
//   k_compact     one work-group per frame: the per-row runs copied into the row-major plane
//                 cloud (framePlanePtr order).
#include "ssf_device.hpp"
#include "ssf_internal.hpp"

namespace ssf {

// frameFeature.cpp:57-72 (see oracle/ssf_oracle.c orc_ring_id for the precision choices).
SSF_DEV int ring_id_exact(float ratio, int n_rows) {
    float angle = (float)(atan((double)ratio) * 180.0 / 3.14159265358979323846);
    int id = -1;
    if (n_rows == 16) {
        id = (int)((double)((angle + 15.0f) / 2.0f) + 0.5);
    } else if (n_rows == 64) {
        if ((double)angle >= -8.83)
            id = (int)((double)(2.0f - angle) * 3.0 + 0.5);      // int - float: a float subtraction
        else
            id = n_rows / 2 + (int)((-8.83 - (double)angle) * 2.0 + 0.5);
    }
    return (id > -1 && id < n_rows) ? id : -1;
}

// The same id with a float atan (the f64 atan made k_bin_count f64-issue-bound).  The float
// angle is within ~3e-5 deg of the f64 expression's; whenever it lies within 1e-3 deg of a bin
// edge (or of the -8.83 switch, or is not finite) the exact f64 path decides, so the id is the
// exact path's for every input.
SSF_DEV int ring_id(float x, float y, float z, int n_rows) {
    float r2 = x * x + y * y;
    float ratio = z / sqrtf(r2);
    const float af = atanf(ratio) * 57.29577951308232f;
    double v;
    float margin;
    if (n_rows == 16) {
        v = (double)((af + 15.0f) / 2.0f) + 0.5;
        margin = 0.5e-3f;
    } else {
        const bool upper = (double)af >= -8.83;
        v = upper ? (double)(2.0f - af) * 3.0 + 0.5 : (-8.83 - (double)af) * 2.0 + 0.5;
        margin = upper ? 3e-3f : 2e-3f;
        if (!(fabsf(af + 8.83f) > 1e-3f)) margin = -1.0f;   // near the switch (or NaN): exact
    }
    const float edge = (float)fabs(v - rint(v));
    if (!(edge > margin)) return ring_id_exact(ratio, n_rows);
    int id = (n_rows == 16 || (double)af >= -8.83) ? (int)v : n_rows / 2 + (int)v;
    if (n_rows != 16 && n_rows != 64) id = -1;
    return (id > -1 && id < n_rows) ? id : -1;
}

// Each thread issues all of its kCountSteps point loads (clamped, unconditional) before the first ring
// id: one load latency per chunk instead of one per point.
constexpr int kCountSteps = kBinChunk / 256;

__global__ __launch_bounds__(256) void k_bin_count(const float* __restrict__ pts, int stride,
                                                   const int64_t* __restrict__ frame_off,
                                                   int n_rows, int n_chunks,
                                                   const uint8_t* __restrict__ keep,
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
        float px[kCountSteps], py[kCountSteps], pz[kCountSteps];
#pragma unroll
        for (int k = 0; k < kCountSteps; ++k) {
            const float* p = pts + min(s + threadIdx.x + 256 * k, t - 1) * stride;
            px[k] = p[0]; py[k] = p[1]; pz[k] = p[2];
        }
#pragma unroll
        for (int k = 0; k < kCountSteps; ++k) {
            const int64_t i = s + threadIdx.x + 256 * k;
            if (i < t) {
                const int id = (keep && !keep[i]) ? -1 : ring_id(px[k], py[k], pz[k], n_rows);
                rid[i] = (int8_t)id;
                if (id >= 0) atomicAdd(&h[id], 1);
            }
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
        // 16 counts loaded before any is rewritten: one memory latency per 16 chunks (a load
        // after a store to the same array otherwise waits for the previous chunk's round trip)
        int32_t* hp = hist + (int64_t)f * n_chunks * n_rows + r;
        for (int c0 = 0; c0 < n_chunks; c0 += 16) {
            int v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = hp[(int64_t)min(c0 + k, n_chunks - 1) * n_rows];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (c0 + k < n_chunks) {
                    hp[(int64_t)(c0 + k) * n_rows] = run;
                    run += v[k];
                }
            }
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

// Stable per-row partition of one kBinChunk-point chunk.  Wave w owns the chunk's points
// [kBinChunk/4 w, kBinChunk/4 (w + 1)) in steps of 64: a 7-ballot "match" on the 6-bit row id gives each
// point its rank among same-row lanes, and a wave-private running count per row (LDS, no
// barrier) turns that into its rank among the wave's same-row points.  One barrier later the
// per-wave counts are prefixed (waves in order, then rows), every point lands in a row-grouped
// LDS tile, and the tile leaves in contiguous per-row runs: coalesced 16-B stores instead of
// one scattered store per point (a LiDAR scan interleaves the rows point by point).
constexpr int kScatterSteps = kBinChunk / 256;   // points per thread

struct Xyz { float x, y, z; };                      // packed ring-ordered point (12 B)

__global__ __launch_bounds__(256) void k_bin_scatter(const float* __restrict__ pts, int stride,
                                                     const int64_t* __restrict__ frame_off,
                                                     int n_rows, int n_chunks,
                                                     const int8_t* __restrict__ rid,
                                                     const int32_t* __restrict__ chunk_base,
                                                     const int32_t* __restrict__ ring_off,
                                                     Xyz* __restrict__ out, float4* __restrict__ out4) {
    __shared__ float4 tile[kBinChunk];            // 16 B per point
    __shared__ uint8_t row_of[kBinChunk];
    __shared__ int wrun[4][kMaxRows];
    __shared__ int roff[kMaxRows + 1];            // chunk-local row offsets
    __shared__ int64_t rbase[kMaxRows];           // global index of row r's first chunk point - roff[r]
    __shared__ double rfrac[kMaxRows];            // id / 100.0, the f64 division done once per row
    const int f = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) return;  // uniform
    const int64_t t = min(e, s + (int64_t)kBinChunk);
    if (tid < kMaxRows) {
        wrun[0][tid] = wrun[1][tid] = wrun[2][tid] = wrun[3][tid] = 0;
        rfrac[tid] = (double)tid / 100.0;
    }
    __syncthreads();
    // all loads first (ids, then points at clamped indices, unconditionally): one wait for the
    // whole kScatterSteps-point batch instead of one load latency per step
    int idr[kScatterSteps];       // row id, then row id | rank-in-wave << 8
    float px[kScatterSteps], py[kScatterSteps], pz[kScatterSteps];
    const int64_t i0 = s + (kBinChunk / 4) * w + (tid & 63);
#pragma unroll
    for (int st = 0; st < kScatterSteps; ++st) {
        const int64_t i = i0 + 64 * st;
        idr[st] = (i < t) ? (int)rid[i] : -1;
    }
#pragma unroll
    for (int st = 0; st < kScatterSteps; ++st) {
        const float* p = pts + min(i0 + 64 * st, t - 1) * stride;
        px[st] = p[0]; py[st] = p[1]; pz[st] = p[2];
    }
#pragma unroll
    for (int st = 0; st < kScatterSteps; ++st) {
        const int id = idr[st];
        uint64_t m = __ballot(id >= 0);
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {
            const bool on = (id >> bit) & 1;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const int rin = __popcll(m & lanemask_lt());
        int rank = 0;
        if (id >= 0) {
            const int before = wrun[w][id];                  // read by every lane first,
            rank = before + rin;
            if (rin == 0) wrun[w][id] = before + __popcll(m);   // then the group leader adds
        }
        idr[st] = (id & 0xff) | (rank << 8);
    }
    __syncthreads();
    const int32_t* cb = chunk_base + ((int64_t)f * n_chunks + c) * n_rows;
    const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    if (tid < 64) {                                          // rows on the lanes of wave 0
        const int r = tid;
        int tot = 0;
        if (r < n_rows) {
            int acc = 0;
            for (int k = 0; k < 4; ++k) { const int v = wrun[k][r]; wrun[k][r] = acc; acc += v; }
            tot = acc;
        }
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (r >= o) incl += y;
        }
        if (r < n_rows) {
            roff[r] = incl - tot;
            rbase[r] = fb + ro[r] + cb[r] - (incl - tot);
        }
        if (r == 63) roff[kMaxRows] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kScatterSteps; ++st) {
        const int id = (int)(int8_t)(idr[st] & 0xff);
        if (id >= 0) {
            const int in_row = wrun[w][id] + (idr[st] >> 8);    // rank among the chunk's row-id points
            const int loc = roff[id] + in_row;
            float4 v;
            v.x = px[st]; v.y = py[st]; v.z = pz[st];
            // frameFeature.cpp:77, needed only by the debug ring-ordered cloud (out4 is uniform)
            v.w = out4 ? (float)((double)(cb[id] + in_row) + rfrac[id]) : 0.0f;
            tile[loc] = v;
            row_of[loc] = (uint8_t)id;
        }
    }
    __syncthreads();
    const int total = roff[kMaxRows];
    for (int k = tid; k < total; k += 256) {
        const float4 v = tile[k];
        const int64_t o = rbase[row_of[k]] + k;
        out[o] = Xyz{v.x, v.y, v.z};
        if (out4) out4[o] = v;                      // debug ring-ordered cloud (x, y, z, intensity)
    }
}

// One WORK-GROUP per (frame, row).  The row is requested in one burst of 2048-point tiles
// (each thread issues its 9 clamped 12-byte loads before the first use, as the binning kernels
// do) into an LDS tile of x | y | z float arrays with an 8-point halo on both sides.  Every
// thread then owns 8 consecutive centres: it reads the 24 points around them as six aligned
// ds_read_b128 per coordinate and evaluates the 11-tap sums (:84-107) left to right in float,
// exactly as the reference, one coordinate at a time (8 partial sums live, not 33 taps).  The
// planar candidates (value < planeMin, the value staying 0 for j < 5 and j >= n - 5) leave as one
// byte per thread; wave 0 then runs the greedy spacing rule (:110-123) over the tile's 64-bit
// words in scalar code, collecting up to 64 selections in one VGPR (lane k holds the k-th) and emitting
// them -- x, y, z from the LDS tile, intensity = indexInRow + row / 100.0 (:77) -- as float4
// stores into the row's own staging slots (ring position + rank).  k_compact then only copies
// contiguous per-row runs into the frame-major plane cloud.  Rows longer than a tile carry the
// greedy state (jstart) from tile to tile.
// kEdge (beyond the reference, off by default): wave 1 runs the edge rule -- greedy in index
// order, curvature > edge_min, spacing edge_span, centres in [5, n - 5) (oracle/edge_oracle.c) --
// on a second byte array, into its own staging slots.
constexpr int kCurvTile = 2048;                 // centres per tile (one tile per 64-beam 120k row)
constexpr int kCurvHalo = 8;                    // >= 5, and a multiple of 8 (aligned windows)
constexpr int kCurvSpan = kCurvTile + 2 * kCurvHalo;
constexpr int kCurvLoads = (kCurvSpan + 255) / 256;

// The greedy rule over one tile's candidate words (wave-uniform, run by ONE wave): selections at
// ring positions >= jstart, spaced by `span`; emitted 64 at a time from the LDS tile.
SSF_DEV void greedy_emit(const uint64_t* words, int t0, int tn, int span, int& jstart, int& cnt,
                         const float* sx, const float* sy, const float* sz, double rfrac,
                         float4* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    int nl = 0, selv = 0;
    auto flush = [&]() {
        if (lane < nl) {
            const int p = selv - (t0 - kCurvHalo);
            out[cnt + lane] = make_float4(sx[p], sy[p], sz[p], (float)((double)selv + rfrac));
        }
        cnt += nl;
        nl = 0;
    };
    const int nw = (tn + 63) >> 6;
    for (int wi = 0; wi < nw; ++wi) {
        const uint64_t wv = words[wi];                      // LDS broadcast
        uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wv >> 32)) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wv);
        const int j0 = t0 + 64 * wi;
        while (true) {
            const int lo = jstart - j0;
            if (lo >= 64) break;
            if (lo > 0) m &= ~((1ull << lo) - 1ull);
            if (!m) break;
            const int jj = j0 + (int)__builtin_ctzll(m);
            if (lane == nl) selv = jj;                 // lane nl keeps selection nl
            jstart = jj + span;
            if (++nl == 64) flush();
        }
    }
    flush();
}

template <bool kCurv, bool kEdge>
__global__ __launch_bounds__(256) void k_curv_select(const int64_t* __restrict__ frame_off,
                                                     int n_rows, int row_start, int row_end,
                                                     float plane_min, int plane_span,
                                                     const int32_t* __restrict__ ring_off,
                                                     const Xyz* __restrict__ rxyz,
                                                     float* __restrict__ curv,
                                                     float4* __restrict__ stage,
                                                     int32_t* __restrict__ sel_cnt,
                                                     float edge_min, int edge_span,
                                                     float4* __restrict__ estage,
                                                     int32_t* __restrict__ esel_cnt) {
    __shared__ __attribute__((aligned(16))) float sx[kCurvSpan], sy[kCurvSpan], sz[kCurvSpan];
    __shared__ __attribute__((aligned(16))) uint8_t pbits[kCurvTile / 8];
    __shared__ __attribute__((aligned(16))) uint8_t ebits[kEdge ? kCurvTile / 8 : 16];
    const int tid = threadIdx.x, w = tid >> 6;
    const int r = blockIdx.x, f = blockIdx.y;
    const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    const int rs = ro[r], n_r = ro[r + 1] - rs;
    const int64_t base = frame_off[f] + rs;
    const bool in_rows = (r >= row_start) && (r < n_rows - row_end);
    if (!in_rows || n_r == 0) {                                  // uniform
        if (kCurv)
            for (int j = tid; j < n_r; j += 256) curv[base + j] = 0.0f;
        if (tid == 0) sel_cnt[(int64_t)f * n_rows + r] = 0;
        if (kEdge && tid == 0) esel_cnt[(int64_t)f * n_rows + r] = 0;
        return;
    }
    const double rfrac = (double)r / 100.0;                    // :77
    const Xyz* src = rxyz + base;
    int cnt = 0, jstart = 0;                                   // wave 0's greedy state
    int ecnt = 0, ejstart = 0;                                 // wave 1's (kEdge)
    for (int t0 = 0; t0 < n_r; t0 += kCurvTile) {              // uniform
        const int tn = min(kCurvTile, n_r - t0);
        {   // positions [t0 - halo, t0 + tile + halo), clamped into the row: all loads first
            Xyz q[kCurvLoads];
#pragma unroll
            for (int k = 0; k < kCurvLoads; ++k) {
                const int pos = t0 - kCurvHalo + tid + 256 * k;
                q[k] = src[min(max(pos, 0), n_r - 1)];
            }
#pragma unroll
            for (int k = 0; k < kCurvLoads; ++k) {
                const int p = tid + 256 * k;
                if (p < kCurvSpan) { sx[p] = q[k].x; sy[p] = q[k].y; sz[p] = q[k].z; }
            }
        }
        __syncthreads();
        // centres j = t0 + 8 tid + i; their taps are tile entries 8 tid + 3 + i .. 8 tid + 13 + i
        float d0[8], d1[8];
        float v[8];
        auto coord = [&](const float* a, float (&d)[8]) {
            float h[24];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const float4 x4 = *reinterpret_cast<const float4*>(a + 8 * tid + 4 * k);
                h[4 * k] = x4.x; h[4 * k + 1] = x4.y; h[4 * k + 2] = x4.z; h[4 * k + 3] = x4.w;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float* u = h + 3 + i;                    // u[0 .. 10], centre u[5]
                float acc = u[0] + u[1];
#pragma unroll
                for (int k = 2; k < 11; ++k) acc = (k == 5) ? acc - 10.0f * u[5] : acc + u[k];
                d[i] = acc;
            }
        };
        if (8 * tid < tn) {
            coord(sx, d0);
            coord(sy, d1);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = d0[i] * d0[i] + d1[i] * d1[i];
            coord(sz, d0);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] + d0[i] * d0[i];
        }
        uint32_t pb = 0, eb = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int jl = 8 * tid + i, j = t0 + jl;
            if (jl < tn) {
                const bool inner = j >= 5 && j < n_r - 5;
                const float val = inner ? v[i] : 0.0f;
                if (kCurv) curv[base + j] = val;
                pb |= (uint32_t)(val < plane_min) << i;
                if (kEdge) eb |= (uint32_t)(inner && val > edge_min) << i;
            }
        }
        if (8 * tid < kCurvTile) pbits[tid] = (uint8_t)pb;
        if (kEdge && 8 * tid < kCurvTile) ebits[tid] = (uint8_t)eb;
        __syncthreads();
        if (w == 0)
            greedy_emit(reinterpret_cast<const uint64_t*>(pbits), t0, tn, plane_span, jstart, cnt,
                        sx, sy, sz, rfrac, stage + base);
        else if (kEdge && w == 1)
            greedy_emit(reinterpret_cast<const uint64_t*>(ebits), t0, tn, edge_span, ejstart, ecnt,
                        sx, sy, sz, rfrac, estage + base);
        __syncthreads();                                       // the tile is read; next tile
    }
    if (tid == 0) sel_cnt[(int64_t)f * n_rows + r] = cnt;
    if (kEdge && tid == 64) esel_cnt[(int64_t)f * n_rows + r] = ecnt;
}

// One work-group per frame: the row counts' prefix in LDS, then every output slot of the frame's
// plane cloud (row-major, framePlanePtr order) copies its float4 from its row's staging run.
__global__ __launch_bounds__(1024) void k_compact(const int64_t* __restrict__ frame_off, int n_rows,
                                                  const int32_t* __restrict__ ring_off,
                                                  const float4* __restrict__ stage,
                                                  const int32_t* __restrict__ sel_cnt,
                                                  float4* __restrict__ plane,
                                                  int32_t* __restrict__ plane_count) {
    __shared__ int pre[kMaxRows + 1];
    __shared__ int rbeg[kMaxRows];
    const int f = blockIdx.x, tid = threadIdx.x;
    if (tid < 64) {
        const int c = tid < n_rows ? sel_cnt[(int64_t)f * n_rows + tid] : 0;
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (tid >= o) incl += y;
        }
        if (tid < n_rows) {
            pre[tid] = incl - c;
            rbeg[tid] = ring_off[(int64_t)f * (n_rows + 1) + tid];
        }
        if (tid == 63) pre[n_rows] = incl;
    }
    __syncthreads();
    const int total = pre[n_rows];
    const int64_t fb = frame_off[f];
    if (tid == 0) plane_count[f] = total;
    for (int k = tid; k < total; k += blockDim.x) {
        int lo = 0, hi = n_rows - 1;                           // the row r with pre[r] <= k < pre[r + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pre[mid] <= k) lo = mid; else hi = mid - 1;
        }
        plane[fb + k] = stage[fb + rbeg[lo] + (k - pre[lo])];
    }
}

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, float* ring_xyz, float4* ring_xyzi, float* curv,
                                 float4* stage, int32_t* sel_cnt, float4* plane,
                                 int32_t* plane_count, const EdgeSel* edge) {
    const int R = cfg.n_rows;
    const int n_chunks = (int)((max_pts + kBinChunk - 1) / kBinChunk);
    if (n_frames <= 0) return hipSuccess;
    if (R > kMaxRows) return hipErrorInvalidValue;
    if (n_chunks > 0) {
        kmark(s, "k_bin_count");
        hipLaunchKernelGGL(k_bin_count, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, keep, rid, hist);
    }
    kmark(s, "k_bin_scan");
    hipLaunchKernelGGL(k_bin_scan, dim3(n_frames), dim3(64), 0, s, R, n_chunks, hist, ring_off);
    if (n_chunks > 0) {
        kmark(s, "k_bin_scatter");
        hipLaunchKernelGGL(k_bin_scatter, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, rid, hist, ring_off,
                           reinterpret_cast<Xyz*>(ring_xyz), ring_xyzi);
    }
    const dim3 cgrid(R, n_frames);
    kmark(s, "k_curv_select");
    const Xyz* rx = reinterpret_cast<const Xyz*>(ring_xyz);
    const float emin = edge ? edge->min_curv : 0.f;
    const int espan = edge ? edge->span : 1;
    float4* estage = edge ? edge->stage : nullptr;
    int32_t* ecnt = edge ? edge->sel_cnt : nullptr;
#define SSF_CURV_LAUNCH(C, E)                                                                      \
    hipLaunchKernelGGL((k_curv_select<C, E>), cgrid, dim3(256), 0, s, frame_off, R, cfg.row_start,  \
                       cfg.row_end, cfg.plane_min, cfg.plane_span, ring_off, rx, curv, stage, sel_cnt, \
                       emin, espan, estage, ecnt)
    if (edge) { if (curv) SSF_CURV_LAUNCH(true, true); else SSF_CURV_LAUNCH(false, true); }
    else { if (curv) SSF_CURV_LAUNCH(true, false); else SSF_CURV_LAUNCH(false, false); }
#undef SSF_CURV_LAUNCH
    kmark(s, "k_compact");
    hipLaunchKernelGGL(k_compact, dim3(n_frames), dim3(1024), 0, s, frame_off, R, ring_off, stage,
                       sel_cnt, plane, plane_count);
    if (edge) {
        kmark(s, "k_compact_edges");
        hipLaunchKernelGGL(k_compact, dim3(n_frames), dim3(1024), 0, s, frame_off, R, ring_off,
                           edge->stage, edge->sel_cnt, edge->out, edge->count);
    }
    return hipGetLastError();
}

}  // namespace ssf
