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
//   k_curv        the 11-tap stencil (:84-107) as a stream over 2048-point chunks of the ring
//                 cloud, evaluated left to right in float, 8 centres per thread; planar
//                 candidates out as a per-frame bit array
//   k_select      one work-group per frame: the greedy spacing rule (:110-123) with one row per
//                 lane, then the selected points (and their encoded intensity) written in
//                 framePlanePtr order (row major).
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

// k_curv: the 11-tap curvature (:84-107) as a pure stream over the frame's ring-ordered cloud,
// one work-group per 2048-point chunk of the rows in range (rows are contiguous there, row after
// row).  Each thread issues its 9 clamped 12-byte loads (the chunk and an 8-point halo on both
// sides) before the first use, the chunk lands in an LDS tile of x | y | z float arrays, and
// every thread owns 8 consecutive centres: it reads the 24 points around them as six aligned
// ds_read_b128 per coordinate and evaluates the sums left to right in float, exactly as the
// reference, one coordinate at a time.  A centre's row comes from the frame's row offsets (LDS);
// its value stays 0 for j < 5 and j >= n - 5 (never computed, :85).  The planar candidates
// (value < planeMin) leave as one byte per thread of a per-frame bit array (bit = ring position);
// the greedy spacing rule runs in k_select.  kEdge (beyond the reference, off by default): the
// edge candidates (curvature > edge_min, centres in [5, n - 5), oracle/edge_oracle.c) into a
// second bit array.  kCurv (debug / parity output): the curvature of every point, 0 outside the
// rows in range.
#ifndef SSF_CURV_PROBE
#define SSF_CURV_PROBE 0   // diagnostic variants only (tools/gpu): 2 = no stencil
#endif
constexpr int kCurvChunk = 2048;                // centres per work-group
constexpr int kCurvHalo = 8;                    // >= 5, and a multiple of 8 (aligned windows)
constexpr int kCurvLoads = (kCurvChunk + 2 * kCurvHalo + 255) / 256;   // 9

// 64-bit word where frame f's candidate bits start (frame-local bit i -> word + (i >> 6)):
// 8-byte aligned per frame, and frames never share a word
SSF_DEV int64_t cand_word0(const int64_t* frame_off, int f) { return (frame_off[f] >> 6) + f; }

template <bool kCurv, bool kEdge>
__global__ __launch_bounds__(256) void k_curv(const int64_t* __restrict__ frame_off, int n_rows,
                                              int row_start, int row_end, float plane_min,
                                              const int32_t* __restrict__ ring_off,
                                              const Xyz* __restrict__ rxyz,
                                              float* __restrict__ curv,
                                              uint8_t* __restrict__ pbits, float edge_min,
                                              uint8_t* __restrict__ ebits) {
    __shared__ __attribute__((aligned(16))) float sx[256 * kCurvLoads], sy[256 * kCurvLoads], sz[256 * kCurvLoads];
    __shared__ int ro[kMaxRows + 1];
    const int tid = threadIdx.x, c = blockIdx.x, f = blockIdx.y;
    // the chunk's bounds from uniform (scalar) loads, so the point loads issue after ONE memory
    // latency; the row table for the centres follows into LDS while they are in flight
    const int64_t fb = frame_off[f];
    const int32_t* rof = ring_off + (int64_t)f * (n_rows + 1);
    const int nr_tot = rof[n_rows];
    // the rows in range (every point for the debug curvature, which is 0 outside them); chunks
    // start at a multiple of 8 points, so every thread's 8 centres are one byte of the bit array
    const int lo = kCurv ? 0 : (rof[row_start] & ~7), hi = kCurv ? nr_tot : rof[n_rows - row_end];
    const int c0 = lo + c * kCurvChunk;                        // uniform
    if (c0 >= hi) return;
    const Xyz* src = rxyz + fb;
    {   // positions [c0 - halo, c0 + chunk + halo), clamped into the frame: all loads first
        Xyz q[kCurvLoads];
#pragma unroll
        for (int k = 0; k < kCurvLoads; ++k) {
            const int pos = c0 - kCurvHalo + tid + 256 * k;
            q[k] = src[min(max(pos, 0), nr_tot - 1)];
        }
        if (tid <= n_rows) ro[tid] = rof[tid];
        // every store unconditional (the tail lands in the pad): a store under a branch made the
        // compiler wait for the last load right after issuing it
#pragma unroll
        for (int k = 0; k < kCurvLoads; ++k) {
            const int p = tid + 256 * k;
            sx[p] = q[k].x; sy[p] = q[k].y; sz[p] = q[k].z;
        }
    }
    __syncthreads();
    const int i0 = c0 + 8 * tid;                               // this thread's 8 centres
    if (i0 >= hi) return;
    // its first centre's row: the last r with ro[r] <= i0
    int r = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
        if (r + st <= n_rows && ro[r + st] <= i0) r += st;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.0f;
    if (SSF_CURV_PROBE != 2) {
        // centres i0 + i; their taps are tile entries 8 tid + 3 + i .. 8 tid + 13 + i
        float d0[8], d1[8];
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
        const int ii = i0 + i;
        while (r < n_rows - 1 && ii >= ro[r + 1]) ++r;         // rows of >= 1 point ahead
        const int j = ii - ro[r], n_r = ro[r + 1] - ro[r];
        const bool row_in = r >= row_start && r < n_rows - row_end;
        const bool inner = j >= 5 && j < n_r - 5;
        const float val = inner ? v[i] : 0.0f;
        if (ii < hi) {
            if (kCurv) curv[fb + ii] = row_in ? val : 0.0f;
            pb |= (uint32_t)(row_in && val < plane_min) << i;
            if (kEdge) eb |= (uint32_t)(row_in && inner && val > edge_min) << i;
        }
    }
    const int64_t byte0 = cand_word0(frame_off, f) * 8 + (i0 >> 3);
    pbits[byte0] = (uint8_t)pb;
    if (kEdge) ebits[byte0] = (uint8_t)eb;
}

// k_select: one work-group per frame.  The greedy spacing rule (:110-123) for every row at once,
// ONE ROW PER LANE of wave 0 (wave 1: the edge rule, kEdge): each lane walks its row's candidate
// bits from the frame's bit array staged in LDS -- next candidate at or after jstart by a
// count-trailing-zeros of the word, jstart = selection + planeSpan -- so 64 rows advance in one
// VALU instruction stream (a scalar walk per row was ~180 cycles per step).  The selections
// (indexInRow) go to per-row slots in global scratch; after one barrier the row counts are
// prefixed and every thread of the work-group emits output slots in framePlanePtr order (row
// major): x, y, z gathered from the ring-ordered cloud, intensity = indexInRow + row / 100.0 (:77).
constexpr int kSelThreads = 1024;
constexpr int kSelWordsLds = 6144;              // candidate words staged per array (48 KiB: 393k points)

template <bool kEdge>
__global__ __launch_bounds__(kSelThreads) void k_select(const int64_t* __restrict__ frame_off, int n_rows,
                                                        int row_start, int row_end, int plane_span,
                                                        const int32_t* __restrict__ ring_off,
                                                        const Xyz* __restrict__ rxyz,
                                                        const uint64_t* __restrict__ pbits,
                                                        int32_t* __restrict__ sel,
                                                        float4* __restrict__ plane,
                                                        int32_t* __restrict__ plane_count,
                                                        int edge_span, const uint64_t* __restrict__ ebits,
                                                        int32_t* __restrict__ esel,
                                                        float4* __restrict__ edge,
                                                        int32_t* __restrict__ edge_count) {
    __shared__ uint64_t wl[kEdge ? 2 : 1][kSelWordsLds];
    __shared__ int ro[kMaxRows + 1];
    __shared__ int pre[2][kMaxRows + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int f = blockIdx.x;
    const int64_t fb = frame_off[f];
    const int nf = (int)(frame_off[f + 1] - fb);
    const int nw = (nf + 63) >> 6;
    const int64_t wb = cand_word0(frame_off, f);
    if (tid <= n_rows) ro[tid] = ring_off[(int64_t)f * (n_rows + 1) + tid];
    for (int k = tid; k < min(nw, kSelWordsLds); k += kSelThreads) {
        wl[0][k] = pbits[wb + k];
        if (kEdge) wl[kEdge ? 1 : 0][k] = ebits[wb + k];
    }
    __syncthreads();
    if (w < (kEdge ? 2 : 1)) {                                 // uniform: wave 0 planes, wave 1 edges
        const int r = lane;
        const bool e = kEdge && w == 1;
        const uint64_t* W = wl[e ? 1 : 0];
        const uint64_t* G = (e ? ebits : pbits) + wb;
        const int span = e ? edge_span : plane_span;
        int32_t* out = e ? esel : sel;
        int cnt = 0;
        if (r < n_rows && r >= row_start && r < n_rows - row_end) {
            const int rs = ro[r], n_r = ro[r + 1] - rs;
            if (n_r > 0) {
                auto word = [&](int k) { return k < kSelWordsLds ? W[k] : G[k]; };
                int js = 0;                                     // jstart, row-relative
                const int kend = (rs + n_r - 1) >> 6;
                uint64_t nxt = word(rs >> 6);
                for (int k = rs >> 6; k <= kend; ++k) {         // the row's words in order
                    uint64_t wv = nxt;
                    nxt = word(min(k + 1, kend));               // the next word in flight
                    const int gb = k * 64;
                    int low = rs + js - gb;                     // bits below jstart
                    if (low >= 64) continue;
                    if (low > 0) wv &= ~0ull << low;
                    const int top = rs + n_r - gb;              // bits past the row's end
                    if (top < 64) wv &= (1ull << top) - 1ull;
                    while (wv) {
                        const int j = gb + (int)__builtin_ctzll(wv) - rs;
                        out[fb + rs + cnt] = j;
                        ++cnt;
                        js = j + span;
                        low = rs + js - gb;
                        wv = low >= 64 ? 0ull : (wv & (~0ull << low));
                    }
                }
            }
        }
        int incl = cnt;                                         // prefix over the rows
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane < n_rows) pre[e ? 1 : 0][lane] = incl - cnt;
        if (lane == 63) pre[e ? 1 : 0][n_rows] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < (kEdge ? 2 : 1); ++e) {
        const int* P = pre[e];
        const int total = P[n_rows];
        if (tid == 0) (e ? edge_count : plane_count)[f] = total;
        const int32_t* S = e ? esel : sel;
        float4* O = e ? edge : plane;
        // four output slots per thread per trip, each stage's loads issued together (the
        // selection index, then the gathered point): three memory latencies per trip
        constexpr int U = 4;
        for (int k0 = 0; k0 < total; k0 += U * kSelThreads) {   // uniform
            int kk[U], rr[U], jj[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kk[u] = min(k0 + u * kSelThreads + tid, total - 1);
                int a = 0;                                      // the row r with P[r] <= k < P[r + 1]
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (a + st < n_rows && P[a + st] <= kk[u]) a += st;
                rr[u] = a;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) jj[u] = S[fb + ro[rr[u]] + (kk[u] - P[rr[u]])];
            Xyz q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = rxyz[fb + ro[rr[u]] + jj[u]];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k0 + u * kSelThreads + tid < total)
                    O[fb + kk[u]] = make_float4(q[u].x, q[u].y, q[u].z,
                                                (float)((double)jj[u] + (double)rr[u] / 100.0));
        }
    }
}

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, float* ring_xyz, float4* ring_xyzi, float* curv,
                                 uint64_t* bits, int32_t* sel, float4* plane,
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
    // k_curv: chunks of the rows in range (every point with the debug curvature)
    const int cchunks = (int)((max_pts + kCurvChunk - 1) / kCurvChunk);
    const dim3 cgrid(max(cchunks, 1), n_frames);
    kmark(s, "k_curv");
    const Xyz* rx = reinterpret_cast<const Xyz*>(ring_xyz);
    const float emin = edge ? edge->min_curv : 0.f;
    uint8_t* eb8 = edge ? reinterpret_cast<uint8_t*>(edge->bits) : nullptr;
#define SSF_CURV_LAUNCH(C, E)                                                                      \
    hipLaunchKernelGGL((k_curv<C, E>), cgrid, dim3(256), 0, s, frame_off, R, cfg.row_start,         \
                       cfg.row_end, cfg.plane_min, ring_off, rx, curv,                             \
                       reinterpret_cast<uint8_t*>(bits), emin, eb8)
    if (edge) { if (curv) SSF_CURV_LAUNCH(true, true); else SSF_CURV_LAUNCH(false, true); }
    else { if (curv) SSF_CURV_LAUNCH(true, false); else SSF_CURV_LAUNCH(false, false); }
#undef SSF_CURV_LAUNCH
    kmark(s, "k_select");
    if (edge)
        hipLaunchKernelGGL(k_select<true>, dim3(n_frames), dim3(kSelThreads), 0, s, frame_off, R,
                           cfg.row_start, cfg.row_end, cfg.plane_span, ring_off, rx, bits, sel, plane,
                           plane_count, edge->span, edge->bits, edge->sel, edge->out, edge->count);
    else
        hipLaunchKernelGGL(k_select<false>, dim3(n_frames), dim3(kSelThreads), 0, s, frame_off, R,
                           cfg.row_start, cfg.row_end, cfg.plane_span, ring_off, rx, bits, sel, plane,
                           plane_count, 1, nullptr, nullptr, nullptr, nullptr);
    return hipGetLastError();
}

}  // namespace ssf
