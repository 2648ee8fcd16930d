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
//   k_curv_select one wave per (frame,row): the row streams through a circular LDS window, the
//                 11-tap stencil (:84-107) is evaluated left to right in float, and the same
//                 wave runs the greedy spacing rule (:110-123) with a 64-bit ballot of
//                 candidates per 64 points (jstart is wave-uniform).
//   k_compact     row-major concatenation of the selected points (framePlanePtr order), with
//                 their encoded intensity.
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

// One WAVE per (frame, row), four rows per work-group, no block barrier.  The wave streams its
// row in 64-point groups (one coalesced 12-byte load per lane) into a 256-point circular LDS
// window (point p at p & 255, see stencil11w); group g-1's 11-tap stencil (:84-107, evaluated left to
// right in float exactly as the reference) is computed once group g has landed, and the greedy
// spacing rule (:110-123) runs on the same wave with a 64-bit ballot of candidates per group
// (jstart is wave-uniform).  Three register buffers with static roles (one loop trip = three
// groups; loads clamped and unconditional) keep three groups in flight: a rotation by register
// moves, or a load or store under a branch, makes the compiler wait for every load at each
// group.  The selected indices collect in LDS and leave once per trip.
#ifndef SSF_CURV_ROWS_PER_WG
#define SSF_CURV_ROWS_PER_WG 4
#endif
constexpr int kCurvRowsPerWG = SSF_CURV_ROWS_PER_WG;
#ifndef SSF_CURV_DEPTH
#define SSF_CURV_DEPTH 3
#endif
constexpr int kCurvDepth = SSF_CURV_DEPTH;   // 64-point groups in flight per wave (one trip)
#ifndef SSF_CURV_PROBE
#define SSF_CURV_PROBE 0                      // diagnostic variants only (tools/gpu scripts)
#endif

// The window holds 256 points (4 groups; point p at p & 255) plus a mirror of its first 16 at
// [256, 272), so the 11 taps of centre j are the contiguous a[b .. b + 10], b = (j - 5) & 255:
// one base address, immediate LDS offsets; (x, y, z) of a point in one float4.
constexpr int kWin = 256;
constexpr int kWinPad = kWin + 16;

// The 11 taps t[0 .. 10] (centre t[5]) from a float4 (x, y, z, -) window: 11 ds_read_b128 (16-B aligned,
// immediate offsets) serve all three coordinates; each coordinate's sum is evaluated left to
// right in float exactly as frameFeature.cpp:86-105.
SSF_DEV void stencil11t(const float4* t, float& dx, float& dy, float& dz) {
    float4 u[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) u[k] = t[k];
    // keep .w live: a whole-float4 read is ds_read_b128 (4 LDS cycles per wave), the x, y, z
    // read the compiler would otherwise emit is ds_read_b96 (8 cycles).  One statement after
    // all eleven reads: one per read made the compiler wait for each before issuing the next.
    asm volatile("" ::"v"(u[0].w), "v"(u[1].w), "v"(u[2].w), "v"(u[3].w), "v"(u[4].w), "v"(u[5].w),
                 "v"(u[6].w), "v"(u[7].w), "v"(u[8].w), "v"(u[9].w), "v"(u[10].w));
    float sx = u[0].x + u[1].x, sy = u[0].y + u[1].y, sz = u[0].z + u[1].z;
#pragma unroll
    for (int k = 2; k < 11; ++k) {
        if (k == 5) { sx = sx - 10.0f * u[5].x; sy = sy - 10.0f * u[5].y; sz = sz - 10.0f * u[5].z; }
        else { sx = sx + u[k].x; sy = sy + u[k].y; sz = sz + u[k].z; }
    }
    dx = sx; dy = sy; dz = sz;
}

// the taps of centre j in the circular window (t = a[(j - 5) & 255 ..], contiguous by the mirror)
SSF_DEV void stencil11w(const float4* a, int j, float& dx, float& dy, float& dz) {
    stencil11t(a + ((j - 5) & (kWin - 1)), dx, dy, dz);
}

// kHalves: 64-entry selection stores per trip (a trip selects <= 64 kCurvDepth / span + 1
// points: one store for span >= 4, two below)
// kEdge (beyond the reference, off by default): the same wave also runs the edge rule --
// greedy in index order, curvature > edge_min, spacing edge_span (the mirror image of :110-123;
// oracle/edge_oracle.c) -- into esel / esel_cnt.
template <bool kCurv, int kHalves, bool kEdge>
__global__ __launch_bounds__(64 * kCurvRowsPerWG) void k_curv_select(const int64_t* __restrict__ frame_off,
                                                     int n_rows, int row_start, int row_end,
                                                     float plane_min, int plane_span,
                                                     const int32_t* __restrict__ ring_off,
                                                     const Xyz* __restrict__ rxyz,
                                                     float* __restrict__ curv,
                                                     int32_t* __restrict__ sel,
                                                     int32_t* __restrict__ sel_cnt,
                                                     int32_t* __restrict__ sel_dump,
                                                     float edge_min, int edge_span,
                                                     int32_t* __restrict__ esel,
                                                     int32_t* __restrict__ esel_cnt) {
    __shared__ float4 win[kCurvRowsPerWG][kWinPad];
    __shared__ int32_t slist[kCurvRowsPerWG][64 * kHalves];
    __shared__ int32_t elist[kEdge ? kCurvRowsPerWG : 1][kEdge ? 64 * kHalves : 1];
    // the wave index through readfirstlane: the compiler then knows the row, its length and
    // every loop bound are wave-uniform (scalar loads, no exec-masked loops)
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r = blockIdx.x * kCurvRowsPerWG + w, f = blockIdx.y;
    if (r >= n_rows) return;                                   // wave-uniform
    const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
    const int rs = ro[r], n_r = ro[r + 1] - rs;
    const int64_t base = frame_off[f] + rs;
    const bool in_rows = (r >= row_start) && (r < n_rows - row_end);
    if (!in_rows || n_r == 0) {
        if (kCurv)
            for (int j = lane; j < n_r; j += 64) curv[base + j] = 0.0f;
        if (lane == 0) sel_cnt[(int64_t)f * n_rows + r] = 0;
        if (kEdge && lane == 0) esel_cnt[(int64_t)f * n_rows + r] = 0;
        return;
    }
    float4* wv = win[w];
    int32_t* sl = slist[w];
    const Xyz* src = rxyz + base;
    const int ng = (n_r + 63) >> 6;
#if SSF_CURV_PROBE == 3
    // diagnostic: the same bytes as lane-contiguous 16-B loads (48 lanes x 16 B = 64 points)
    const float4* src4 = reinterpret_cast<const float4*>(reinterpret_cast<uintptr_t>(src) & ~(uintptr_t)15);
    const int n4 = (3 * n_r + 3) / 4;
    auto load = [&](int g) {
        const float4 q = src4[min(48 * g + min(lane, 47), n4 - 1)];
        return Xyz{q.x + q.w, q.y, q.z};
    };
#else
    auto load = [&](int g) { return src[min(64 * g + lane, n_r - 1)]; };   // clamped
#endif
    int cnt = 0, nl = 0, jstart = 0;                           // wave-uniform
    int ecnt = 0, enl = 0, ejstart = 0;                        // wave-uniform (kEdge)
    int32_t* el = elist[kEdge ? w : 0];
    auto group = [&](Xyz& buf, int g) {
        {                                                      // group g into the window
            const int p = (64 * g + lane) & (kWin - 1);
            const float4 q = make_float4(buf.x, buf.y, buf.z, 0.0f);
            wv[p] = q;
            if (p < kWinPad - kWin) wv[p + kWin] = q;
            buf = load(g + kCurvDepth);
        }
        if (g == 0 || g > ng) return;                          // uniform
        const int j = 64 * (g - 1) + lane;                     // group g-1: its stencil is complete
        float v = 0.0f;
#if SSF_CURV_PROBE == 1 || SSF_CURV_PROBE == 3
        // diagnostic (tools/ variants only): the stream and the window, no stencil, no greedy
        v = wv[(j - 5) & (kWin - 1)].x;
#else
        if (j >= 5 && j < n_r - 5) {
            float dx, dy, dz;
            stencil11w(wv, j, dx, dy, dz);
            v = dx * dx + dy * dy;
            v = v + dz * dz;
        }
#endif
        if (kCurv) curv[base + min(j, n_r - 1)] = v;   // lanes past the row write its last value, 0
        uint64_t m = __ballot(j < n_r && v < plane_min);
#if SSF_CURV_PROBE
        // diagnostic: no greedy walk (one selection per group keeps the ballot live)
        if (m) { if (lane == 0) sl[nl] = 64 * (g - 1) + __ffsll((unsigned long long)m) - 1; nl++; }
        (void)jstart;
        if (true) return;
#endif
        const int j0 = 64 * (g - 1);
        while (true) {
            const int lo = jstart - j0;
            if (lo >= 64) break;
            if (lo > 0) m &= ~((1ull << lo) - 1ull);
            if (!m) break;
            const int l = __ffsll((unsigned long long)m) - 1;
            const int jj = __builtin_amdgcn_readfirstlane(j0 + l);
            if (lane == 0) sl[nl] = jj;
            nl++;
            jstart = jj + plane_span;
        }
        nl = __builtin_amdgcn_readfirstlane(nl);
        if (kEdge) {
            uint64_t me = __ballot(j >= 5 && j < n_r - 5 && v > edge_min);
            while (true) {
                const int lo = ejstart - j0;
                if (lo >= 64) break;
                if (lo > 0) me &= ~((1ull << lo) - 1ull);
                if (!me) break;
                const int l = __ffsll((unsigned long long)me) - 1;
                const int jj = __builtin_amdgcn_readfirstlane(j0 + l);
                if (lane == 0) el[enl] = jj;
                enl++;
                ejstart = jj + edge_span;
            }
            enl = __builtin_amdgcn_readfirstlane(enl);
        }
    };
    // a trip's selections (<= 64 kHalves) leave with unconditional stores; lanes without one write
    // the row's last slot, which no selection list reaches when the row has >= 2 points (at most
    // ceil(n_r / 2) entries for plane_span >= 2).  A ONE-point row selects its point 0, its last
    // slot: those lanes write a 64-slot dump after the last point of the batch instead.
    int32_t* const spare = n_r >= 2 ? sel + base + n_r - 1 : sel_dump + lane;
    // edges never select the row's last point (j < n_r - 5), so its slot is a safe spare too
    int32_t* const espare = kEdge ? (n_r >= 2 ? esel + base + n_r - 1 : sel_dump + lane) : nullptr;
    // prologue loads in buffer order (the loop's waits count on b[0] being the oldest)
    Xyz b[kCurvDepth];
#pragma unroll
    for (int k = 0; k < kCurvDepth; ++k) {
        b[k] = load(k);
        asm volatile("" ::: "memory");
    }
    for (int g = 0; g <= ng; g += kCurvDepth) {
#pragma unroll
        for (int k = 0; k < kCurvDepth; ++k) group(b[k], g + k);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int h = 0; h < kHalves; ++h)
            *(lane + 64 * h < nl ? sel + base + cnt + 64 * h + lane : spare) = sl[64 * h + lane];
        if (kEdge) {
#pragma unroll
            for (int h = 0; h < kHalves; ++h)
                *(lane + 64 * h < enl ? esel + base + ecnt + 64 * h + lane : espare) = el[64 * h + lane];
        }
        __builtin_amdgcn_wave_barrier();
        cnt += nl;
        nl = 0;
        ecnt += enl;
        enl = 0;
    }
    if (lane == 0) sel_cnt[(int64_t)f * n_rows + r] = cnt;
    if (kEdge && lane == 0) esel_cnt[(int64_t)f * n_rows + r] = ecnt;
}

__global__ __launch_bounds__(256) void k_compact(const int64_t* __restrict__ frame_off, int n_rows,
                                                 const int32_t* __restrict__ ring_off,
                                                 const Xyz* __restrict__ rxyz,
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
    const double rfrac = (double)r / 100.0;
    for (int k = tid; k < n; k += blockDim.x) {
        const int j = sel[base + k];                 // indexInRow
        const Xyz p = rxyz[base + j];
        plane[fb + pre + k] = make_float4(p.x, p.y, p.z, (float)((double)j + rfrac));   // :77
    }
}

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, float* ring_xyz, float4* ring_xyzi, float* curv,
                                 int32_t* sel,
                                 int32_t* sel_dump, int32_t* sel_cnt, float4* plane,
                                 int32_t* plane_count, const EdgeSel* edge) {
    const int R = cfg.n_rows;
    const int n_chunks = (int)((max_pts + kBinChunk - 1) / kBinChunk);
    if (n_frames <= 0) return hipSuccess;
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
    const dim3 cgrid((R + kCurvRowsPerWG - 1) / kCurvRowsPerWG, n_frames);
    kmark(s, "k_curv_select");
    const Xyz* rx = reinterpret_cast<const Xyz*>(ring_xyz);
    const bool two = cfg.plane_span < 4 || (edge && edge->span < 4);
    const float emin = edge ? edge->min_curv : 0.f;
    const int espan = edge ? edge->span : 1;
    int32_t* esel = edge ? edge->sel : nullptr;
    int32_t* ecnt = edge ? edge->sel_cnt : nullptr;
#define SSF_CURV_LAUNCH(C, H, E)                                                                  \
    hipLaunchKernelGGL((k_curv_select<C, H, E>), cgrid, dim3(64 * kCurvRowsPerWG), 0, s, frame_off, \
                       R, cfg.row_start, cfg.row_end, cfg.plane_min, cfg.plane_span, ring_off, rx,  \
                       curv, sel, sel_cnt, sel_dump, emin, espan, esel, ecnt)
    if (edge) {
        if (curv) { if (two) SSF_CURV_LAUNCH(true, 2, true); else SSF_CURV_LAUNCH(true, 1, true); }
        else { if (two) SSF_CURV_LAUNCH(false, 2, true); else SSF_CURV_LAUNCH(false, 1, true); }
    } else {
        if (curv) { if (two) SSF_CURV_LAUNCH(true, 2, false); else SSF_CURV_LAUNCH(true, 1, false); }
        else { if (two) SSF_CURV_LAUNCH(false, 2, false); else SSF_CURV_LAUNCH(false, 1, false); }
    }
#ifdef SSF_CURV_TWICE
    // diagnostic (tools/ variants only): the same launch again, on data the previous kernel
    // left settled (k_curv_select is idempotent)
    kmark(s, "k_curv_select_again");
    if (!edge) { if (curv) { if (two) SSF_CURV_LAUNCH(true, 2, false); else SSF_CURV_LAUNCH(true, 1, false); }
                 else { if (two) SSF_CURV_LAUNCH(false, 2, false); else SSF_CURV_LAUNCH(false, 1, false); } }
#endif
#undef SSF_CURV_LAUNCH
    kmark(s, "k_compact");
    hipLaunchKernelGGL(k_compact, dim3(R, n_frames), dim3(256), 0, s, frame_off, R, ring_off,
                       rx, sel, sel_cnt, plane, plane_count);
    if (edge) {
        kmark(s, "k_compact_edges");
        hipLaunchKernelGGL(k_compact, dim3(R, n_frames), dim3(256), 0, s, frame_off, R, ring_off,
                           rx, edge->sel, edge->sel_cnt, edge->out, edge->count);
    }
    return hipGetLastError();
}

}  // namespace ssf
