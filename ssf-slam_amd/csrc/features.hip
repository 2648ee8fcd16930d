// features.hip -- frameFeature::cloudHandler (src/frameFeature.cpp:35-139) on gfx950.
//
// Four kernels per batch of frames:
//   k_bin_count   ring id per point (frameFeature.cpp:57-72) + per-chunk ring histogram
//   k_bin_scan    per-frame exclusive scans -> per-(chunk,row) bases and row offsets
//   k_bin_curv    the stable per-row partition (:73-80) AND the 11-tap curvature (:84-107) of
//                 one 2048-point input chunk: the chunk plus a halo of input points on both
//                 sides is ranked per row (per-row lane words in LDS, waves in order -> the
//                 reference's push_back order), regrouped by row in LDS, and each
//                 chunk point's stencil is read from its row's run in that tile.  Out: per ring
//                 position the point's input index (4 B) and a candidate flag byte (planar, and
//                 edge when asked) -- the ring-ordered cloud itself is never written (debug only)
//   k_select      one work-group per frame: the flag bytes packed to bits in LDS, the stencils
//                 the halo did not cover (a row with < 5 points in the window, e.g. input not in
//                 azimuth order: the frame's fix-up list, normally empty) computed through the
//                 ring indices and OR-ed in, the greedy
//                 spacing rule (:110-123) with one row per lane, then the selected points (and
//                 their encoded intensity) gathered from the input in framePlanePtr order.
#include "ssf_device.hpp"
#include "ssf_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

namespace ssf {

// ---- the ring id by table ---------------------------------------------------------------------
// frameFeature.cpp:57-73: `float angle = atan(point.z / sqrt(x*x + y*y)) * 180 / M_PI`, then the
// bin arithmetic of :60 / :63-71 and int() truncation.  C++ overload resolution allows two
// evaluations (oracle/ssf_oracle.c orc_ring_angle), selected by ssf_config.ring_chain:
//   SSF_RING_CHAIN_FLOAT (default): the float overloads libstdc++'s <math.h> puts at global scope
//     -- ratio = z / sqrtf(r2) (float), atanf, `* 180` in float, `/ M_PI` in double, to float;
//   SSF_RING_CHAIN_DOUBLE: only ::sqrt / ::atan(double) -- ratio = (double)z / sqrt((double)r2).
// Either way the row id is a monotone step function of ONE ratio (float or double).  The host
// evaluates the exact chain with the host libm (glibc atanf / atan, as oracle/ssf_oracle.c) once per
// context and cuts the ratio axis into kRingCells uniform cells (cell = clamp((ratio - r0) * inv),
// float ops, the same on both sides; a double ratio takes the cell of its float rounding); a cell
// holds at most two ids (cells are narrower than the narrowest bin), so per cell {the threshold
// where the second id starts (float; and as the exact double for the double chain), id below,
// id from there}.  The device computes the ratio exactly as the reference and does ONE table
// lookup and one compare: no atan on the device at all.
#ifndef SSF_FEAT_EXACT_ID
#define SSF_FEAT_EXACT_ID 0                      // A/B: the exact ratio for every point
#endif
constexpr int kRingCells = 256;
constexpr int kRingChainFloat = SSF_RING_CHAIN_FLOAT, kRingChainDouble = SSF_RING_CHAIN_DOUBLE;
struct RingCell {
    float thr;          // ratios >= thr (float order) take id_b (double chain: thr rounded to float)
    int32_t ids;        // id_a (bits 0..7, signed), id_b (bits 8..15, signed)
};
struct RingTable {
    float r0, inv;
    RingCell cell[kRingCells];
    // per row, the float ratios of its interval [lo, hi) (the id is a monotone step function of
    // the ratio); an empty interval (lo >= hi) for a row that never occurs or is split.  Double
    // chain: the interval's ends rounded to float (the regular kernels' 1e-6 margins cover that)
    float rlo[kMaxRows], rhi[kMaxRows];
    int32_t chain, pad_;
    double dthr[kRingCells];   // per cell, the exact threshold of the double chain (float chain: thr)
};

SSF_DEV int ring_id_lookup(float ratio, float r0, float inv, const RingCell* T) {
    int ci = (int)((ratio - r0) * inv);          // v_cvt_i32_f32 saturates; NaN handled below
    ci = min(max(ci, 0), kRingCells - 1);
    const RingCell rc = T[ci];
    const int a = (int)(int8_t)(rc.ids & 0xff), b = (int)(int8_t)((rc.ids >> 8) & 0xff);
    const int id = ratio < rc.thr ? a : b;
    return ratio == ratio ? id : -1;             // 0 / 0 (a point at the origin): no row
}

// The reference's id from its exact ratio: the correctly rounded float z / sqrtf(r2) (float
// chain) or the correctly rounded double (double)z / sqrt((double)r2) against the cell's double
// threshold (double chain).  T: the cells (LDS or global), rt: the table (chain, dthr).
SSF_DEV int ring_id_exact(float x, float y, float z, float r0, float inv, const RingCell* T,
                          const RingTable* __restrict__ rt) {
    const float r2 = x * x + y * y;
    if (rt->chain != kRingChainDouble) return ring_id_lookup(z / sqrtf(r2), r0, inv, T);
    const double dr = (double)z / sqrt((double)r2);
    const float fr = (float)dr;
    int ci = (int)((fr - r0) * inv);
    ci = min(max(ci, 0), kRingCells - 1);
    const RingCell rc = T[ci];
    const int a = (int)(int8_t)(rc.ids & 0xff), b = (int)(int8_t)((rc.ids >> 8) & 0xff);
    const int id = dr < rt->dthr[ci] ? a : b;
    return dr == dr ? id : -1;
}

// The exact ratio needs a correctly rounded sqrt and divide (~30 instructions; f64 for the double
// chain).  The hardware reciprocal square root gives it to ~3e-7 relative (v_rsq_f32 1 ulp, one
// multiply, and the roundings of the exact form): that ratio takes the exact form's id unless a
// table threshold or a cell edge lies within 1e-6 of it (relative; a few in a million points), or
// r2 is tiny or not finite -- then the exact form decides (a rare, divergent branch).
SSF_DEV int ring_id_table(float x, float y, float z, float r0, float inv, const RingCell* T,
                          const RingTable* __restrict__ rt) {
    const float r2 = x * x + y * y;
    if (SSF_FEAT_EXACT_ID) return ring_id_exact(x, y, z, r0, inv, T, rt);   // A/B: no fast path
    const float ra = z * __builtin_amdgcn_rsqf(r2);
    int ci = (int)((ra - r0) * inv);
    ci = min(max(ci, 0), kRingCells - 1);
    const RingCell rc = T[ci];
    const float m = 1e-6f * fmaxf(1.0f, fabsf(ra));
    const float tc = (ra - r0) * inv, fr = tc - floorf(tc);
    // every test evaluated (no short-circuit: one exec mask, one branch)
    const int near = (int)!(fabsf(ra - rc.thr) > m) | (int)!(fr > m * inv) | (int)!(fr < 1.0f - m * inv) |
                     (int)!(r2 > 1e-30f) | (int)!(r2 < 1e30f);
    const int a = (int)(int8_t)(rc.ids & 0xff), b = (int)(int8_t)((rc.ids >> 8) & 0xff);
    int id = ra < rc.thr ? a : b;
    if (near) id = ring_id_exact(x, y, z, r0, inv, T, rt);
    return id;
}

// Each thread issues all of its kCountSteps point loads (clamped, unconditional) before the first ring
// id: one load latency per chunk instead of one per point.
constexpr int kCountSteps = kBinChunk / 256;

__global__ __launch_bounds__(256) void k_bin_count(const float* __restrict__ pts, int stride,
                                                   const int64_t* __restrict__ frame_off,
                                                   int n_rows, int n_chunks,
                                                   const uint8_t* __restrict__ keep,
                                                   const RingTable* __restrict__ rtab,
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
                const int id = (keep && !keep[i]) ? -1 : ring_id_table(px[k], py[k], pz[k], rtab->r0, rtab->inv,
                                                                        rtab->cell, rtab);
                rid[i] = (int8_t)id;
                if (id >= 0) atomicAdd(&h[id], 1);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < n_rows) hist[((int64_t)f * n_chunks + c) * n_rows + threadIdx.x] = h[threadIdx.x];
}

// One wave per frame: thread r scans its row's chunk counts in chunk order.  It also clears the
// frame's fix-up list count for the k_bin_curv launch that follows on this stream.
__global__ __launch_bounds__(64) void k_bin_scan(int n_rows, int n_chunks, int32_t* __restrict__ hist,
                                                 int32_t* __restrict__ ring_off,
                                                 uint32_t* __restrict__ fix_count) {
    const int f = blockIdx.x, r = threadIdx.x;
    if (r == 0) fix_count[f] = 0u;
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

// ---- k_bin_curv ------------------------------------------------------------------------------
// One work-group per (frame, 2048-point input chunk).  Its WINDOW is the chunk plus kCurvHalo
// input points on each side (clamped to the frame).  A row's points inside the window are
// consecutive ring positions of that row (the partition is stable and the window a contiguous
// input range), so once the window is regrouped by row, a chunk point's 11 taps are its
// neighbours in its row's run of the tile -- whenever the run holds 5 points on each side of it.
// With a 64-beam scan in azimuth order a row has a point every 64 inputs, so 384 halo points
// hold 6 per row; a stencil the halo does not cover goes to the frame's fix-up list (k_select).
//   rank   waves own contiguous parts of the window; a per-row lane word (LDS OR) ranks a
//          point among same-row lanes, a wave-private running count per row among the wave's
//          points, the per-wave counts are prefixed (waves in order, then rows): the tile
//          position.  Halo-before points per row are counted on the side (LDS adds).
//   place  every point decides at once, from its row's record (one ds_read_b128), its tile
//          slot, its ring position and its class: halo / chunk point whose stencil lies in the
//          window / chunk point with curvature 0 (row out of range, or within 5 of the row's
//          ends, :85) / chunk point whose taps the window lacks; one 32-bit word per tile entry
//          {ring position : 24, class : 2, flags : 2} and its window position (u16)
//   curv   ONE float array, filled with x, then y, then z (the points stay in registers):
//          every thread owns kCE consecutive tile entries and reads their taps as 7 aligned
//          ds_read_b128 per coordinate; sums left to right in float, exactly as the reference
//          (and the oracle), one coordinate at a time
//   out    per chunk point, at its ring position: the input index (frame-local, int32), and a
//          flag byte: bit 0 = planar candidate (row in range and curvature < planeMin, the
//          curvature being 0 outside [5, n - 5) as :85 leaves it), bit 1 = edge candidate
//          (kEdge, beyond the reference: row in range, centre in [5, n - 5), curvature >
//          edge_min, oracle/edge_oracle.c); tile order = contiguous per-row runs.  Debug only:
//          the ring-ordered cloud (x, y, z, intensity = indexInRow + row / 100.0, :77) and the
//          curvature of every point.
// Blocks are mapped XCD-aware: the dispatcher deals blocks round-robin over the 8 XCDs, so
// block b runs logical block (b % 8) * Q + b / 8 -- each XCD walks a contiguous range of
// chunks in order and a window's halo is the neighbouring chunk its own L2 just read.
#ifndef SSF_CURV_HALO
#define SSF_CURV_HALO 384
#endif
#ifndef SSF_CURV_SUB
#define SSF_CURV_SUB 1
#endif
constexpr int kCurvHalo = SSF_CURV_HALO;                 // multiple of 64, <= kBinChunk
constexpr int kCurvSub = SSF_CURV_SUB;                   // binning chunks per work-group
constexpr int kCurvNT = 256 * kCurvSub;                  // threads per work-group
constexpr int kCurvNW = kCurvNT / 64;
constexpr int kCurvOwn = kBinChunk * kCurvSub;           // chunk points per work-group
constexpr int kWin = kCurvOwn + 2 * kCurvHalo;           // window points at most
constexpr int kWinQ = ((kWin + kCurvNW - 1) / kCurvNW + 63) / 64;   // 64-point steps per wave part
constexpr int kCE = ((kWin + kCurvNT - 1) / kCurvNT + 3) & ~3;      // tile entries per thread (12)
constexpr int kTileE = kCE * kCurvNT;                    // tile entries (>= kWin)
constexpr int kTilePad = 8;
static_assert(kCurvHalo % 64 == 0 && kCurvHalo <= kBinChunk, "halo");
static_assert(kWin < 4096 || kCurvSub > 1, "");
static_assert(kWin < 8192, "window positions and run lengths use 13 bits");
// tile entry classes (meta bits 24..25)
constexpr uint32_t kClsHalo = 0, kClsStencil = 1, kClsZero = 2, kClsOpen = 3;

// byte where frame f's flag bytes start: 64-byte aligned per frame, frames disjoint
// (buffer: total + 64 F + 64 bytes)
SSF_DEV int64_t flag_base(const int64_t* frame_off, int f) { return (frame_off[f] & ~(int64_t)63) + 64 * (int64_t)f; }

// the 11-tap sum of one coordinate, left to right (u[5] is the centre): frameFeature.cpp:88-97
SSF_DEV float tap11(const float* u) {
    float acc = u[0] + u[1];
#pragma unroll
    for (int k = 2; k < 11; ++k) acc = (k == 5) ? acc - 10.0f * u[5] : acc + u[k];
    return acc;
}

SSF_DEV uint8_t cand_flags(bool row_in, bool inner, float v, float plane_min, bool edge, float edge_min) {
    const float val = inner ? v : 0.0f;
    return (uint8_t)((row_in && val < plane_min) ? 1 : 0) |
           (uint8_t)((edge && row_in && inner && v > edge_min) ? 2 : 0);
}

template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT) void k_bin_curv(const float* __restrict__ pts, int stride,
                                                  const int64_t* __restrict__ frame_off,
                                                  int n_frames, int n_rows, int n_chunks,
                                                  int row_start, int row_end, float plane_min,
                                                  float edge_min,
                                                  const int8_t* __restrict__ rid,
                                                  const int32_t* __restrict__ chunk_base,
                                                  const int32_t* __restrict__ ring_off,
                                                  int32_t* __restrict__ ring_idx,
                                                  uint8_t* __restrict__ flags,
                                                  int32_t* __restrict__ fix, uint32_t* __restrict__ fix_count,
                                                  float4* __restrict__ out4, float* __restrict__ curv) {
    __shared__ __attribute__((aligned(16))) float sc[kTileE + 2 * kTilePad];   // x, then y, then z
    __shared__ __attribute__((aligned(16))) uint32_t meta[kTileE];
    __shared__ uint16_t wpos[kTileE];
    __shared__ int wrun[kCurvNW][kMaxRows + 1];   // (+1: the slot of points in no row)
    __shared__ unsigned long long gmask[kCurvNW][kMaxRows + 1];   // a step's lanes per row (rank)
    __shared__ int nb[kMaxRows];                  // halo-before points per row
    // per (wave, row), in the rank space of the wave's points of that row: tile slot base, ring
    // position base, the ranks whose centre is in [5, n_r - 5) of a row in range (inner), and the
    // ranks whose 11 taps the window holds (covered)
    __shared__ int4 wrec[kCurvNW][kMaxRows];      // {k base, ring base, inner lo, inner hi}
    __shared__ int2 wcov[kCurvNW][kMaxRows];      // {covered lo, covered hi}
    __shared__ int4 rinfo[kMaxRows];              // debug: {run offset, cb - nb, ring offset, n_r}
    __shared__ int ntot;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // XCD-aware logical block (see above)
    const int nc2 = (n_chunks + kCurvSub - 1) / kCurvSub;      // work-group chunks per frame
    const int64_t nblk = (int64_t)nc2 * n_frames;
    const int64_t q8 = (nblk + 7) / 8;
    const int64_t lb = (int64_t)(blockIdx.x % 8) * q8 + blockIdx.x / 8;
    if (lb >= nblk) return;
    const int f = (int)(lb / nc2), c = (int)(lb - (int64_t)f * nc2) * kCurvSub;   // first binning chunk
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) return;                           // uniform
    const int64_t t = min(e, s + (int64_t)kCurvOwn);
    const int64_t ws = max(fb, s - (int64_t)kCurvHalo), we = min(e, t + (int64_t)kCurvHalo);
    const int L = (int)(we - ws), hb = (int)(s - ws), he = (int)(t - ws);   // own: [hb, he)
    const int qlen = ((L + kCurvNW - 1) / kCurvNW + 63) / 64 * 64;        // <= 64 kWinQ
    if (tid < kMaxRows) {
#pragma unroll
        for (int k = 0; k < kCurvNW; ++k) { wrun[k][tid] = 0; gmask[k][tid] = 0ull; }
        nb[tid] = 0;
    }
    if (tid < kCurvNW) { wrun[tid][kMaxRows] = 0; gmask[tid][kMaxRows] = 0ull; }
    // the rows' chunk bases and ring offsets, loaded now by wave 0 (used after the ranking):
    // their latency hides behind the point loads instead of stalling the work-group later
    int cbr = 0, ro0 = 0, ro1 = 0;
    if (tid < n_rows) {
        cbr = chunk_base[((int64_t)f * n_chunks + c) * n_rows + tid];
        const int32_t* ro = ring_off + (int64_t)f * (n_rows + 1);
        ro0 = ro[tid]; ro1 = ro[tid + 1];
    }
    __syncthreads();
    // all loads first (ids, then points at clamped indices, unconditionally)
    const int q0 = w * qlen, q1 = min(L, q0 + qlen);
    int idr[kWinQ];
    float px[kWinQ], py[kWinQ], pz[kWinQ];
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) idr[st] = (int)rid[ws + min(q0 + lane + 64 * st, L - 1)];   // clamped: no branch
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) if (q0 + lane + 64 * st >= q1) idr[st] = -1;
    const float* pw = pts + ws * stride;                     // the window's first point
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const float* pp = pw + (uint32_t)(min(q0 + lane + 64 * st, L - 1) * stride);   // < 2^32 floats
        px[st] = pp[0]; py[st] = pp[1]; pz[st] = pp[2];
    }
    // same-row lanes of a step: every lane ORs its bit into its row's 64-bit word of the wave
    // (ds_or_b64), reads the word back (the wave's LDS instructions complete in order, so every
    // OR of the step is in), ranks itself by the lanes below it, and the row's first lane clears
    // the word for the next step -- exact and order-free (OR commutes); the 6-bit ballot match it
    // replaces cost ~45 VALU instructions per step
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const int id = idr[st];
        const int rs = id >= 0 ? id : kMaxRows;              // points in no row: a spare slot
        unsigned long long* gm = &gmask[w][rs];
        __hip_atomic_fetch_or(gm, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t m = __hip_atomic_load(gm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int rin = __popcll(m & lanemask_lt());
        const int before = wrun[w][rs];                      // read by every lane first,
        if (rin == 0) {                                      // then the group leader adds, clears
            wrun[w][rs] = before + __popcll(m);
            __hip_atomic_store(gm, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (q0 + 64 * st < hb)                               // uniform: a step with halo-before points
            if (id >= 0 && q0 + lane + 64 * st < hb) atomicAdd(&nb[id], 1);
        idr[st] = (id & 0xff) | ((before + rin) << 8);       // rank among the wave's row points
    }
    __syncthreads();
    if (tid < 64) {                                          // rows on the lanes of wave 0
        const int r = tid;
        int tot = 0;
        if (r < n_rows) {
            int acc = 0;
            for (int k = 0; k < kCurvNW; ++k) { const int v = wrun[k][r]; wrun[k][r] = acc; acc += v; }
            tot = acc;
        }
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (r >= o) incl += y;
        }
        if (r < n_rows) {
            const int run0 = incl - tot, jb = cbr - nb[r], nr = ro1 - ro0;
            const bool row_in = r >= row_start && r < n_rows - row_end;
            if (kDebug) rinfo[r] = make_int4(run0, jb, ro0, nr);
#pragma unroll
            for (int k = 0; k < kCurvNW; ++k) {
                const int pw = wrun[k][r];                   // the wave's first position in the run
                // rank q of wave k: run position p = pw + q, row index j = jb + pw + q
                wrec[k][r] = make_int4(run0 + pw, ro0 + jb + pw,
                                       row_in ? 5 - jb - pw : 0, row_in ? nr - 5 - jb - pw : 0);
                wcov[k][r] = make_int2(5 - pw, tot - 5 - pw);
            }
        }
        if (r == 63) ntot = incl;
    }
    __syncthreads();
    const int nt = ntot;                                     // kept points in the window
    // ---- place: tile slot, ring position and class of every point; x into the tile
    int loc[kWinQ];
    // flags of a chunk point whose curvature is 0 (row in range, j outside [5, n_r - 5): :85)
    const uint32_t flz = (uint32_t)cand_flags(true, false, 0.0f, plane_min, kEdge, edge_min);
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const int id = (int)(int8_t)(idr[st] & 0xff);
        loc[st] = kTileE;                                    // no point: the pad slot
        if (id >= 0) {
            const int q = idr[st] >> 8;                      // rank among the wave's row points
            const int4 rw = wrec[w][id];
            const int2 cv = wcov[w][id];
            const int k = rw.x + q;
            const int wp = q0 + lane + 64 * st;
            const bool own = wp >= hb && wp < he;
            const bool inner = q >= rw.z && q < rw.w;        // row in range, centre in [5, n_r - 5)
            const bool covered = q >= cv.x && q < cv.y;
            const bool row_in = id >= row_start && id < n_rows - row_end;
            const uint32_t cls = !own ? kClsHalo : !inner ? kClsZero : covered ? kClsStencil : kClsOpen;
            const uint32_t fl = cls == kClsZero && row_in ? flz : 0u;
            meta[k] = (uint32_t)(rw.y + q) | (cls << 24) | (fl << 26);
            wpos[k] = (uint16_t)wp;
            sc[kTilePad + k] = px[st];
            loc[st] = k;
            if (kDebug && own) {
                const int j = rw.y + q - rinfo[id].z;
                const int64_t g = fb + rw.y + q;
                if (out4) out4[g] = make_float4(px[st], py[st], pz[st], (float)((double)j + (double)id / 100.0));
                if (curv && cls == kClsZero) curv[g] = 0.0f;
            }
        }
    }
    __syncthreads();
    // ---- curvature of this thread's kCE tile entries, one coordinate at a time
    const int k0 = kCE * tid;
    float v[kCE];
    auto coord = [&](float (&d)[kCE]) {
        float h[kCE + 16];                                   // tile entries k0 - 8 .. k0 + kCE + 8
#pragma unroll
        for (int k = 0; k < (kCE + 16) / 4; ++k) {
            const float4 x4 = *reinterpret_cast<const float4*>(sc + k0 + 4 * k);
            h[4 * k] = x4.x; h[4 * k + 1] = x4.y; h[4 * k + 2] = x4.z; h[4 * k + 3] = x4.w;
        }
#pragma unroll
        for (int i = 0; i < kCE; ++i) d[i] = tap11(h + 3 + i);   // centre h[8 + i]
    };
    {
        float d0[kCE], d1[kCE];
        coord(d0);
        __syncthreads();
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = py[st];
        __syncthreads();
        coord(d1);
#pragma unroll
        for (int i = 0; i < kCE; ++i) v[i] = d0[i] * d0[i] + d1[i] * d1[i];
        __syncthreads();
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = pz[st];
        __syncthreads();
        coord(d0);
#pragma unroll
        for (int i = 0; i < kCE; ++i) v[i] = v[i] + d0[i] * d0[i];
    }
    uint32_t mt[kCE];
#pragma unroll
    for (int i = 0; i < kCE; i += 4) {                       // k0 + kCE <= kTileE: 3 ds_read_b128
        const uint4 m4 = *reinterpret_cast<const uint4*>(meta + k0 + i);
        mt[i] = m4.x; mt[i + 1] = m4.y; mt[i + 2] = m4.z; mt[i + 3] = m4.w;
    }
    uint32_t fixm = 0;                                       // open stencils (bit i)
#pragma unroll
    for (int i = 0; i < kCE; ++i) {
        const uint32_t cls = (mt[i] >> 24) & 3u;
        if (k0 + i < nt && cls == kClsStencil) {
            const uint32_t fl = cand_flags(true, true, v[i], plane_min, kEdge, edge_min);
            meta[k0 + i] = mt[i] | (fl << 26);
            if (kDebug && curv) curv[fb + (mt[i] & 0xFFFFFFu)] = v[i];
        }
        fixm |= (k0 + i < nt && cls == kClsOpen) ? 1u << i : 0u;
    }
    // fix-up list (rare): wave-aggregated reservation, skipped by a wave with no open stencil
    if (__ballot(fixm != 0u)) {                              // wave-uniform
    const int nfx = __popc(fixm);
    int incl = nfx;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int wtot = __shfl(incl, 63, 64);
    {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&fix_count[f], (uint32_t)wtot);
        base = __shfl(base, 0, 64) + (uint32_t)(incl - nfx);
        while (fixm) {
            const int i = __builtin_ctz(fixm);
            fixm &= fixm - 1u;
            fix[fb + base++] = (int32_t)(mt[i] & 0xFFFFFFu);
        }
    }
    }
    __syncthreads();
    // ---- chunk points out, in tile order (contiguous per-row runs of ring positions)
    const int64_t fl0 = flag_base(frame_off, f);
    const int32_t ib = (int32_t)(ws - fb);
#pragma unroll 4
    for (int k = tid; k < nt; k += kCurvNT) {
        const uint32_t mk = meta[k];
        const int wp = wpos[k];
        if (((mk >> 24) & 3u) == kClsHalo) continue;
        const int g = (int)(mk & 0xFFFFFFu);
        ring_idx[fb + g] = ib + wp;
        flags[fl0 + g] = (uint8_t)(mk >> 26);
    }
}

// k_select: one work-group per frame.  The frame's flag bytes are packed into bit words in LDS
// (64 flags -> one word: byte LSBs gathered by a multiply); the stencils k_bin_curv left open (the
// frame's fix-up list) are evaluated through the ring index -- same taps, same sums, same order --
// and their flags OR-ed into the words; then the greedy spacing rule
// (:110-123) runs for every row at once, ONE ROW PER LANE of wave 0 (wave 1: the edge rule,
// kEdge): each lane walks its row's candidate bits -- next candidate at or after jstart by a
// count-trailing-zeros of the word, jstart = selection + planeSpan -- so 64 rows advance in one
// VALU instruction stream.  The selections (indexInRow) go to per-row slots in global scratch;
// after one barrier the row counts are prefixed and every thread of the work-group emits
// output slots in framePlanePtr order (row major): x, y, z gathered from the input through the
// ring index, intensity = indexInRow + row / 100.0 (:77).
#ifndef SSF_SEL_THREADS
#define SSF_SEL_THREADS 1024
#endif
constexpr int kSelThreads = SSF_SEL_THREADS;
constexpr int kSelWordsLds = 6144;              // candidate words staged per array (48 KiB: 393k points)

// bit b of the result = bit `bit` of byte b of x (bytes' bits gathered by one multiply: the
// products 2^(8k + 7m + 7) never collide, so no carries)
SSF_DEV uint32_t pack8(uint64_t x, int bit) {
    return (uint32_t)((((x >> bit) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
}

SSF_DEV uint64_t pack64(const uint64_t* b8, int bit) {
    uint64_t wv = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) wv |= (uint64_t)pack8(b8[k], bit) << (8 * k);
    return wv;
}

template <bool kEdge>
__global__ __launch_bounds__(kSelThreads) void k_select(const float* __restrict__ pts, int stride,
                                                        const int64_t* __restrict__ frame_off, int n_rows,
                                                        int row_start, int row_end, int plane_span,
                                                        float plane_min, float edge_min,
                                                        const int32_t* __restrict__ ring_off,
                                                        const int32_t* __restrict__ ring_idx,
                                                        uint8_t* __restrict__ flags,
                                                        const int32_t* __restrict__ fix,
                                                        const uint32_t* __restrict__ fix_count,
                                                        float* __restrict__ curv,
                                                        int32_t* __restrict__ sel,
                                                        float4* __restrict__ plane,
                                                        int32_t* __restrict__ plane_count,
                                                        int edge_span, int32_t* __restrict__ esel,
                                                        float4* __restrict__ edge,
                                                        int32_t* __restrict__ edge_count) {
    __shared__ uint64_t wl[kEdge ? 2 : 1][kSelWordsLds];
    __shared__ int ro[kMaxRows + 1];
    __shared__ int pre[2][kMaxRows + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int f = blockIdx.x;
    const int64_t fb = frame_off[f];
    if (tid <= n_rows) ro[tid] = ring_off[(int64_t)f * (n_rows + 1) + tid];
    __syncthreads();
    const int nr = ro[n_rows];                                 // kept points (ring positions)
    const int nw = (nr + 63) >> 6;
    uint8_t* F8 = flags + flag_base(frame_off, f);
    const uint64_t* F = reinterpret_cast<const uint64_t*>(F8);
    const uint32_t nfix = fix_count[f];
    for (int k = tid; k < min(nw, kSelWordsLds); k += kSelThreads) {
        uint64_t b8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) b8[u] = F[8 * k + u];
        wl[0][k] = pack64(b8, 0);
        if (kEdge) wl[kEdge ? 1 : 0][k] = pack64(b8, 1);
    }
    __syncthreads();
    if (nfix > 0) {                                            // uniform; normally not taken
        for (uint32_t q = tid; q < nfix; q += kSelThreads) {
            const int g = fix[fb + q];                         // in range and inner: 5 <= j < n_r - 5
            float ux[11], uy[11], uz[11];
#pragma unroll
            for (int m = 0; m < 11; ++m) {
                const float* p = pts + (fb + ring_idx[fb + g - 5 + m]) * stride;
                ux[m] = p[0]; uy[m] = p[1]; uz[m] = p[2];
            }
            const float d0 = tap11(ux), d1 = tap11(uy), d2 = tap11(uz);
            float v = d0 * d0 + d1 * d1;
            v = v + d2 * d2;
            const uint8_t fl = cand_flags(true, true, v, plane_min, kEdge, edge_min);
            if (curv) curv[fb + g] = v;
            if ((g >> 6) < kSelWordsLds) {
                if (fl & 1) atomicOr((unsigned long long*)&wl[0][g >> 6], 1ull << (g & 63));
                if (kEdge && (fl & 2)) atomicOr((unsigned long long*)&wl[kEdge ? 1 : 0][g >> 6], 1ull << (g & 63));
            } else {
                F8[g] = fl;                                    // read back by the walk below
            }
        }
        __syncthreads();
    }
    if (w < (kEdge ? 2 : 1)) {                                 // uniform: wave 0 planes, wave 1 edges
        const int r = lane;
        const bool e = kEdge && w == 1;
        const uint64_t* W = wl[e ? 1 : 0];
        const int span = e ? edge_span : plane_span;
        int32_t* out = e ? esel : sel;
        int cnt = 0;
        if (r < n_rows && r >= row_start && r < n_rows - row_end) {
            const int rs = ro[r], n_r = ro[r + 1] - rs;
            if (n_r > 0) {
                // beyond the LDS stage (frames > 393k points): the word straight from the flags
                auto word = [&](int k) {
                    if (k < kSelWordsLds) return W[k];
                    uint64_t b8[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) b8[u] = F[8 * k + u];
                    return pack64(b8, e ? 1 : 0);
                };
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
        // selection index, the ring index, then the gathered point)
        constexpr int U = 4;
        for (int k0 = 0; k0 < total; k0 += U * kSelThreads) {   // uniform
            int kk[U], rr[U], jj[U], ii[U];
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
#pragma unroll
            for (int u = 0; u < U; ++u) ii[u] = ring_idx[fb + ro[rr[u]] + jj[u]];
            float q[U][3];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float* p = pts + (fb + ii[u]) * stride;
                q[u][0] = p[0]; q[u][1] = p[1]; q[u][2] = p[2];
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k0 + u * kSelThreads + tid < total)
                    O[fb + kk[u]] = make_float4(q[u][0], q[u][1], q[u][2],
                                                (float)((double)jj[u] + (double)rr[u] / 100.0));
        }
    }
}

// ==== the single-read feature stage (round 4) ===================================================
// k_feat_chunk + k_feat_select (+ k_feat_debug for the parity outputs) replace k_bin_count,
// k_bin_scan, k_bin_curv and k_select for frames of up to kFeatMaxChunks chunks.  The points are
// read ONCE: k_feat_chunk computes the ring ids of its window itself, ranks and regroups it by row
// exactly like k_bin_curv, and evaluates every stencil the window covers -- but it needs no global
// ring position: its outputs are CHUNK-MAJOR, in the chunk's own-tile order (the chunk's own kept
// points, grouped by row, input order within a row):
//   cnt    [F][n_chunks + 1][64] own points per row (k_feat_select turns them into row bases)
//   gidx   u16 per own-tile slot: the point's position in the chunk (frame-local index = chunk *
//          2048 + gidx), at idx_base(f) + chunk * 2048 + slot
//   gbits  per chunk three 2048-bit planes: planar candidate, UNRESOLVED, edge candidate
// A chunk cannot know a point's indexInRow j, only its rank in the window; but a stencil the
// window covers (5 row points on each side in the window) has 5 <= j < n_r - 5 necessarily, so its
// curvature decides the flags (frameFeature.cpp:84-107).  Every other own point of a row in range
// is marked unresolved: k_feat_select, which has the whole frame's counts, gives it curvature 0
// when j < 5 or j >= n_r - 5 (:85; always a planar candidate) and evaluates the rest -- open
// stencils, rare for azimuth-ordered scans -- through the chunk-major index, the same taps in the
// same order.  Every write of k_feat_chunk is a whole, aligned, contiguous run (no per-row
// scatter); the greedy of k_feat_select walks each row as its sequence of (chunk, row) segments.
#ifndef SSF_FEAT_PACKED
#define SSF_FEAT_PACKED 0                        // packed-f32 stencil (A/B, see k_feat_chunk)
#endif
#ifndef SSF_FEAT_ZONES
#define SSF_FEAT_ZONES 0                         // A/B: one-zone steps count without masks (spills: slower)
#endif
#ifndef SSF_FEAT_REGULAR
#define SSF_FEAT_REGULAR 1                       // k_feat_chunk_reg for regular windows (A/B: 0)
#endif
#ifndef SSF_SEL_CUT
#define SSF_SEL_CUT 0                            // timing tools only: stop k_feat_select after phase 1..4
#endif
#ifndef SSF_FEAT_CUT
#define SSF_FEAT_CUT 0                           // timing tools only: stop k_feat_chunk after phase 1..4
#endif
#ifndef SSF_FEAT_WAVES
#define SSF_FEAT_WAVES 5                         // k_feat_chunk waves per SIMD (launch bound)
#endif
constexpr int kFeatMaxChunks = 128;              // 262144 points per frame (k_feat_select's LDS)
constexpr int kFeatPlanes = 3;                   // planar candidate, unresolved, edge candidate
constexpr int kFeatWords = kBinChunk / 64;       // 64-bit words per plane and chunk
constexpr uint8_t kFlP = 1, kFlU = 2, kFlE = 4;
// per (frame, chunk) block flag of the single-read stage: which kernel did the chunk and where
// k_feat_select finds a selected point's chunk position
//   kIrrRegular  k_feat_wave_reg / k_feat_chunk_reg: 64 x own column + the row's lane (lane map)
//   kIrrGeneral  not done yet -> k_feat_chunk_flagged, which writes the u16 position of every slot
//   kIrrRun      k_feat_wave_run: the row's run start (u16 at the chunk's first 64 index entries) + o
//   kIrrRunIdx   k_feat_wave_run with the debug outputs: the u16 position of every slot
constexpr uint8_t kIrrRegular = 0, kIrrGeneral = 1, kIrrRun = 2, kIrrRunIdx = 3;
static_assert(kCurvSub == 1 && kBinChunk == 2048, "own-tile slots and chunk positions use 11 bits");

// u16 index base of frame f: 64-entry aligned, frames disjoint with a gap of >= 33 entries (the
// chunk writes run up to 3 entries past the chunk's own points)
SSF_DEV int64_t idx_base(const int64_t* frame_off, int f) { return (frame_off[f] & ~(int64_t)31) + 64 * (int64_t)f; }

// LDS layouts of k_feat_chunk without write bank conflicts (ds_write_*: bank = (a / 4) mod 32,
// two 32-lane groups).  An azimuth-ordered scan puts one row per lane in every step, so a step's
// own-tile slots are p = seg(row) + q with seg spaced by the rows' own counts (32 for a full
// 2048-point chunk of a 64-beam scan): u16 slots 64 B apart (16-way), flag bytes 32 B apart
// (8-way).  XOR-swizzling bits 2..5 (idl) / 2..4 (flags) with the slot's row-size bits spreads
// them over every bank (2-way for the u16s: free for a store) and keeps 4-slot groups (8 B of
// idl) intact for the copy-out.  The f32 tile is padded by one float after every row run
// instead (runs of 44 floats: 12r mod 32 -> 45r mod 32), since its readers are 16-B loads.
static_assert(kTileE >= kWin + kMaxRows, "k_feat_chunk's tile holds the window plus one pad per row");
SSF_DEV int idl_sw(int p) { return p ^ (((p >> 6) & 15) << 2); }
SSF_DEV int fll_sw(int p) { return p ^ (((p >> 7) & 7) << 2); }

// The chunk's outputs from LDS (k_feat_chunk, k_feat_chunk_reg): the u16 chunk positions in
// own-tile order as whole 8-byte runs (idl, swizzled by idl_sw), and the candidate / unresolved
// (/ edge) bit planes packed from the flag bytes (fll, swizzled by fll_sw).
template <bool kEdge>
SSF_DEV void feat_chunk_out(int tid, int f, int c, int n_chunks, const int64_t* __restrict__ frame_off,
                            int clen, int no, const uint16_t* idl, const uint8_t* fll,
                            uint16_t* __restrict__ gidx, uint64_t* __restrict__ gbits, bool write_idx = true) {
    uint16_t* gi = gidx + idx_base(frame_off, f) + (int64_t)c * kBinChunk;   // 4 KiB aligned run
    if (write_idx)                                            // uniform
        for (int k = tid; 4 * k < clen; k += kCurvNT)         // 8-byte stores (4 slots)
            *reinterpret_cast<uint2*>(gi + 4 * k) = *reinterpret_cast<const uint2*>(idl + 4 * (k ^ ((k >> 4) & 15)));
    uint64_t* gb = gbits + ((int64_t)f * n_chunks + c) * (kFeatPlanes * kFeatWords);
    constexpr int kPl = kEdge ? 3 : 2;
    if (tid < kPl * kFeatWords) {
        const int pl = tid / kFeatWords, wi = tid - pl * kFeatWords;
        const int nbit = min(64, max(0, no - 64 * wi));
        uint64_t wv = 0;
        if (nbit > 0) {
            uint64_t b8[8];
            const int sw = (wi >> 1) & 7;                     // fll_sw of this word's 64 flags
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint64_t x = *reinterpret_cast<const uint64_t*>(fll + 8 * ((8 * wi + u) ^ (sw >> 1)));
                b8[u] = (sw & 1) ? ((x >> 32) | (x << 32)) : x;
            }
            wv = pack64(b8, pl);                              // bit pl of every flag byte
            if (nbit < 64) wv &= (1ull << nbit) - 1ull;
        }
        gb[pl * kFeatWords + wi] = wv;
    }
}

// One (frame, chunk) block of k_feat_chunk / k_feat_chunk_flagged (the work-group's LDS is
// declared here: one block at a time)
template <bool kDebug, bool kEdge>
SSF_DEV void feat_chunk_block(int64_t lb, const float* __restrict__ pts, int stride,
                                                    const int64_t* __restrict__ frame_off,
                                                    int n_frames, int n_rows, int n_chunks,
                                                    int row_start, int row_end, float plane_min,
                                                    float edge_min, const uint8_t* __restrict__ keep,
                                                    const RingTable* __restrict__ rtab,
                                                    int32_t* __restrict__ cnt,
                                                    uint16_t* __restrict__ gidx,
                                                    uint64_t* __restrict__ gbits,
                                                    float* __restrict__ curv_cm) {
    __shared__ __attribute__((aligned(16))) float sc[kTileE + 2 * kTilePad];   // x, then y, then z
    __shared__ __attribute__((aligned(16))) uint16_t meta[kTileE];   // own-tile slot | 0x8000: stencil
    // two LDS regions reused across phases (31 KiB in all: 5 work-groups per CU):
    //   A: the ring-id table (ids) -> u16 chunk position per own-tile slot (place, out)
    //   B: the per-row lane words (rank) -> the flag byte per own-tile slot (place, curvature, out)
    __shared__ __attribute__((aligned(16))) char regA[(kBinChunk + 4) * 2];
    __shared__ __attribute__((aligned(16))) char regB[kCurvNW * (kMaxRows + 1) * 8];
    static_assert(sizeof(regA) >= kRingCells * sizeof(RingCell) && sizeof(regB) >= kBinChunk, "LDS reuse");
    RingCell* rcell = reinterpret_cast<RingCell*>(regA);
    uint16_t* idl = reinterpret_cast<uint16_t*>(regA);
    auto gmask = reinterpret_cast<unsigned long long (*)[kMaxRows + 1]>(regB);
    uint8_t* fll = reinterpret_cast<uint8_t*>(regB);
    // per (wave, row): the wave's row points so far, packed {all : 16, halo-before : 16,
    // halo-before + own : 16} -- one word read and rewritten per step, no atomics
    __shared__ unsigned long long wrun[kCurvNW][kMaxRows + 1];
    // per (wave, row), in the rank space q of the wave's points of that row: tile slot base,
    // own-tile slot base, the ranks whose 11 taps the window holds
    __shared__ int4 wrec[kCurvNW][kMaxRows];
    __shared__ int ntot, nown;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: step masks in SGPRs
    const int f = (int)(lb / n_chunks), c = (int)(lb - (int64_t)f * n_chunks);
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) return;                                       // uniform
    const int64_t t = min(e, s + (int64_t)kBinChunk);
    const int64_t ws = max(fb, s - (int64_t)kCurvHalo), we = min(e, t + (int64_t)kCurvHalo);
    const int L = (int)(we - ws), hb = (int)(s - ws), he = (int)(t - ws);   // own: [hb, he)
    const int qlen = ((L + kCurvNW - 1) / kCurvNW + 63) / 64 * 64;
    const int q0 = w * qlen, q1 = min(L, q0 + qlen);
    int idr[kWinQ];
    float px[kWinQ], py[kWinQ], pz[kWinQ];
    const float* pw = pts + ws * stride;
    // every point load first (clamped, unconditional), in flight across the LDS set-up and its
    // barrier -- the ring table's load no longer goes ahead of them
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const float* pp = pw + (uint32_t)(min(q0 + lane + 64 * st, L - 1) * stride);
        px[st] = pp[0]; py[st] = pp[1]; pz[st] = pp[2];
    }
    uint8_t kp[kWinQ];
    if (keep) {
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) kp[st] = keep[ws + min(q0 + lane + 64 * st, L - 1)];
    }
    if (tid < kMaxRows) {
#pragma unroll
        for (int k = 0; k < kCurvNW; ++k) { wrun[k][tid] = 0ull; gmask[k][tid] = 0ull; }
    }
    if (tid < kCurvNW) { wrun[tid][kMaxRows] = 0ull; gmask[tid][kMaxRows] = 0ull; }
    for (int k = tid; k < kRingCells; k += kCurvNT) rcell[k] = rtab->cell[k];
    const float r0 = rtab->r0, rinv = rtab->inv;
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {                      // frameFeature.cpp:57-73
        const bool in = q0 + lane + 64 * st < q1 && (!keep || kp[st]);
        const int id = ring_id_table(px[st], py[st], pz[st], r0, rinv, rcell, rtab);   // every lane: no branch
        idr[st] = in ? id : -1;
    }
#if SSF_FEAT_CUT == 1                                         // timing only (tools): ring ids
    { int acc = 0; for (int st = 0; st < kWinQ; ++st) acc += idr[st]; if (acc == 0x7fffffff) cnt[0] = acc; return; }
#endif
    // rank among same-row points (the k_bin_curv ranking: per-row lane words, waves in order).
    // Every lane of a row computes the same new counter word and writes it (and clears the lane
    // word): the wave's LDS instructions complete in order, so all reads of the step precede
    // these writes -- no leader branch.  The halo-before / own lanes of a step are uniform masks.
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const int id = idr[st];
        const int rs = id >= 0 ? id : kMaxRows;
        unsigned long long* gm = &gmask[w][rs];
        __hip_atomic_fetch_or(gm, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t m = __hip_atomic_load(gm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t old = wrun[w][rs];
        const int s0 = q0 + 64 * st;                          // uniform
        const int hbl = __builtin_amdgcn_readfirstlane(min(64, max(0, hb - s0)));   // SGPRs
        const int hel = __builtin_amdgcn_readfirstlane(min(64, max(0, he - s0)));
        const int rin = __popcll(m & lanemask_lt());
        const uint64_t pm = (uint64_t)__popcll(m);
        uint64_t inc;
        if (SSF_FEAT_ZONES && (hbl == 0 || hbl == 64) && (hel == 0 || hel == 64)) {   // uniform: one zone
            inc = pm * (1ull + (hbl ? 1ull << 16 : 0ull) + (hel ? 1ull << 32 : 0ull));
        } else {                                              // the (at most two) boundary steps
            const uint64_t hm = hbl >= 64 ? ~0ull : ((1ull << hbl) - 1ull);   // lanes before the chunk
            const uint64_t om = hel >= 64 ? ~0ull : ((1ull << hel) - 1ull);   // lanes before its end
            inc = pm + ((uint64_t)__popcll(m & hm) << 16) + ((uint64_t)__popcll(m & om) << 32);
        }
        wrun[w][rs] = old + inc;
        __hip_atomic_store(gm, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        idr[st] = (id & 0xff) | (((int)(old & 0xffffu) + rin) << 8);
    }
    __syncthreads();
    if (tid < 64) {                                           // rows on the lanes of wave 0
        const int r = tid;
        int tot = 0, nbr = 0, obr = 0;
        int pwk[kCurvNW];
        if (r < n_rows) {
#pragma unroll
            for (int k = 0; k < kCurvNW; ++k) {
                const uint64_t v = wrun[k][r];
                pwk[k] = tot;                                 // the wave's first position in the run
                tot += (int)(v & 0xffffu);
                nbr += (int)((v >> 16) & 0xffffu);
                obr += (int)((v >> 32) & 0xffffu);
            }
        }
        const int own = r < n_rows ? obr - nbr : 0;
        int incl = tot, oincl = own;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64), yo = __shfl_up(oincl, o, 64);
            if (r >= o) { incl += y; oincl += yo; }
        }
        cnt[((int64_t)f * (n_chunks + 1) + c) * kMaxRows + r] = own;
        if (r < n_rows) {
            const int run0 = incl - tot, seg0 = oincl - own;
#pragma unroll
            for (int k = 0; k < kCurvNW; ++k)
                wrec[k][r] = make_int4(run0 + r + pwk[k], seg0 + pwk[k] - nbr, 5 - pwk[k], tot - 5 - pwk[k]);
            meta[run0 + r + tot] = 0;                         // the row run's pad entry: no stencil
        }
        if (r == 63) { ntot = incl + n_rows; nown = oincl; }  // tile entries incl. one pad per row
    }
    __syncthreads();
#if SSF_FEAT_CUT == 2                                         // timing only: + ranking, row scan
    { int acc = ntot; for (int st = 0; st < kWinQ; ++st) acc += idr[st]; if (acc == 0x7fffffff) cnt[0] = acc; return; }
#endif
    const int nt = ntot;
    const int64_t cm = fb + (int64_t)c * kBinChunk;           // chunk-major base (curvature)
    // ---- place: tile slot of every window point, own-tile slot + position of every own point
    int loc[kWinQ];
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const int id = (int)(int8_t)(idr[st] & 0xff);
        loc[st] = kTileE;                                     // no point: the pad slot
        if (id >= 0) {
            const int q = idr[st] >> 8;
            const int4 rw = wrec[w][id];
            const int k = rw.x + q;
            const int wp = q0 + lane + 64 * st;
            const bool own = wp >= hb && wp < he;
            const bool row_in = id >= row_start && id < n_rows - row_end;
            const bool covered = q >= rw.z && q < rw.w;
            uint16_t mk = 0;
            if (own) {
                const int p = rw.y + q;
                idl[idl_sw(p)] = (uint16_t)(wp - hb);
                if (row_in && covered) {
                    mk = (uint16_t)(p | 0x8000);
                } else {
                    fll[fll_sw(p)] = row_in ? kFlU : (uint8_t)0;
                    if (kDebug && curv_cm) curv_cm[cm + p] = 0.0f;
                }
            }
            meta[k] = mk;
            sc[kTilePad + k] = px[st];
            loc[st] = k;
        }
    }
    __syncthreads();
#if SSF_FEAT_CUT == 3                                         // timing only: + place
    { int acc = 0; for (int st = 0; st < kWinQ; ++st) acc += loc[st]; if (acc == 0x7fffffff) cnt[0] = acc; return; }
#endif
#if SSF_FEAT_PACKED
    // ---- curvature of this thread's kCE tile entries, one coordinate at a time, entries i and
    // i + kCE / 2 side by side in packed f32 (v_pk_add_f32 / v_pk_mul_f32: two IEEE operations,
    // the same rounding as two scalar ones): tap k of the pair is (t[k0 + i + k], t[k0 + i + 6 + k]),
    // one ds_read2_b32 -- the sums keep the reference's left-to-right order (frameFeature.cpp:88-97)
    static_assert(kCE == 12, "the packed stencil pairs entries i and i + 6");
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int k0 = kCE * tid;
    f2 v2[kCE / 2];
    auto coord = [&](bool first) {
        const float* t = sc + k0 + 3;                         // tap 0 of entry 0 (centre at + 5)
        f2 P[kCE / 2 + 10];                                   // P[j] = (t[j], t[j + 6])
#pragma unroll
        for (int j = 0; j < kCE / 2 + 10; ++j) P[j] = f2{t[j], t[j + kCE / 2]};
#pragma unroll
        for (int i = 0; i < kCE / 2; ++i) {
            f2 acc = P[i] + P[i + 1];
#pragma unroll
            for (int k = 2; k < 11; ++k) acc = (k == 5) ? acc - f2{10.0f, 10.0f} * P[i + 5] : acc + P[i + k];
            const f2 sq = acc * acc;
            v2[i] = first ? sq : v2[i] + sq;
        }
    };
    coord(true);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = py[st];
    __syncthreads();
    coord(false);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = pz[st];
    __syncthreads();
    coord(false);
    float v[kCE];
#pragma unroll
    for (int i = 0; i < kCE / 2; ++i) { v[i] = v2[i].x; v[i + kCE / 2] = v2[i].y; }
#else
    // ---- curvature of this thread's kCE tile entries, one coordinate at a time (k_bin_curv)
    const int k0 = kCE * tid;
    float v[kCE];
    auto coord = [&](float (&d)[kCE]) {
        float h[kCE + 16];
#pragma unroll
        for (int k = 0; k < (kCE + 16) / 4; ++k) {
            const float4 x4 = *reinterpret_cast<const float4*>(sc + k0 + 4 * k);
            h[4 * k] = x4.x; h[4 * k + 1] = x4.y; h[4 * k + 2] = x4.z; h[4 * k + 3] = x4.w;
        }
#pragma unroll
        for (int i = 0; i < kCE; ++i) d[i] = tap11(h + 3 + i);
    };
    {
        // ((dX dX + dY dY) + dZ dZ), each product rounded: the square of one coordinate's sum is
        // kept, not the sum itself (one kCE array live instead of two)
        float d0[kCE];
        coord(d0);
#pragma unroll
        for (int i = 0; i < kCE; ++i) v[i] = d0[i] * d0[i];
        __syncthreads();
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = py[st];
        __syncthreads();
        coord(d0);
#pragma unroll
        for (int i = 0; i < kCE; ++i) v[i] = v[i] + d0[i] * d0[i];
        __syncthreads();
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) sc[kTilePad + loc[st]] = pz[st];
        __syncthreads();
        coord(d0);
#pragma unroll
        for (int i = 0; i < kCE; ++i) v[i] = v[i] + d0[i] * d0[i];
    }
#endif
#if SSF_FEAT_CUT == 4                                         // timing only: + stencils
    { float acc = 0.f; for (int i = 0; i < kCE; ++i) acc += v[i]; if (acc == 1234.5f) cnt[0] = 1; return; }
#endif
    uint16_t mt[kCE];
#pragma unroll
    for (int i = 0; i < kCE; i += 4) {                        // k0 + kCE <= kTileE: 8-byte reads
        const uint2 m2 = *reinterpret_cast<const uint2*>(meta + k0 + i);
        mt[i] = (uint16_t)(m2.x & 0xffffu); mt[i + 1] = (uint16_t)(m2.x >> 16);
        mt[i + 2] = (uint16_t)(m2.y & 0xffffu); mt[i + 3] = (uint16_t)(m2.y >> 16);
    }
#pragma unroll
    for (int i = 0; i < kCE; ++i) {
        if (k0 + i < nt && (mt[i] & 0x8000)) {
            const int p = mt[i] & 0x7fff;
            const uint8_t fl = cand_flags(true, true, v[i], plane_min, kEdge, edge_min);
            fll[fll_sw(p)] = (uint8_t)((fl & 1) ? kFlP : 0) | (uint8_t)((fl & 2) ? kFlE : 0);
            if (kDebug && curv_cm) curv_cm[cm + p] = v[i];
        }
    }
    __syncthreads();
    // ---- out: the chunk's own-tile slots, whole aligned runs
    feat_chunk_out<kEdge>(tid, f, c, n_chunks, frame_off, (int)(t - s), nown, idl, fll, gidx, gbits);
}

#define SSF_FC_ARGS pts, stride, frame_off, n_frames, n_rows, n_chunks, row_start, row_end, plane_min, \
                    edge_min, keep, rtab, cnt, gidx, gbits, curv_cm
#define SSF_FC_PARAMS const float* __restrict__ pts, int stride, const int64_t* __restrict__ frame_off, \
    int n_frames, int n_rows, int n_chunks, int row_start, int row_end, float plane_min,              \
    float edge_min, const uint8_t* __restrict__ keep, const RingTable* __restrict__ rtab,             \
    int32_t* __restrict__ cnt, uint16_t* __restrict__ gidx, uint64_t* __restrict__ gbits,            \
    float* __restrict__ curv_cm
// every (frame, chunk) block, one per work-group (XCD-aware: each XCD walks a contiguous range, so
// a window's halo was just read into its own L2)
template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT, SSF_FEAT_WAVES) void k_feat_chunk(SSF_FC_PARAMS) {
    const int64_t nblk = (int64_t)n_chunks * n_frames;
    const int64_t q8 = (nblk + 7) / 8;
    const int64_t lb = (int64_t)(blockIdx.x % 8) * q8 + blockIdx.x / 8;
    if (lb >= nblk) return;
    feat_chunk_block<kDebug, kEdge>(lb, SSF_FC_ARGS);
}

// after k_feat_chunk_reg: only the blocks it flagged.  A work-group reads the flags of 16
// consecutive blocks in one 16-byte load and does the flagged ones in turn, so a launch of
// regular frames is nblk / 16 work-groups that return at once (one work-group per block cost
// ~9 us to drain for 15 k blocks)
constexpr int kFlagGroup = 16;
template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT, SSF_FEAT_WAVES) void k_feat_chunk_flagged(SSF_FC_PARAMS,
                                                                             const uint8_t* __restrict__ irregular) {
    const int64_t nblk = (int64_t)n_chunks * n_frames;
    const int64_t b0 = (int64_t)blockIdx.x * kFlagGroup;
    const uint4 fw = *reinterpret_cast<const uint4*>(irregular + b0);   // feat_irr_bytes: 16-B padded
    uint32_t m = 0;
    const uint32_t wd[4] = {fw.x, fw.y, fw.z, fw.w};
#pragma unroll
    for (int k = 0; k < kFlagGroup; ++k) m |= (uint32_t)(((wd[k >> 2] >> (8 * (k & 3))) & 0xffu) == kIrrGeneral) << k;
    while (m) {                                               // uniform
        const int k = __builtin_ctz(m);
        m &= m - 1u;
        if (b0 + k >= nblk) break;
        feat_chunk_block<kDebug, kEdge>(b0 + k, SSF_FC_ARGS);
        __syncthreads();                                      // the block's LDS readers are done
    }
}
#undef SSF_FC_ARGS
#undef SSF_FC_PARAMS

// k_feat_chunk_reg: the same outputs for REGULAR windows, the common layout of a 64-beam scan in
// azimuth order (the reference's driver order; the bench's synthetic scans): the window is whole
// columns of 64 points, each column holds every row once, and lane l of every column is the same
// row.  Then a row's points in the window are one lane's column sequence -- rank = column, the
// own-tile slot is row x own columns + (column - first own column), and the 11 taps of a stencil
// are that lane's columns c - 5 .. c + 5 -- so there is no ranking, no placement and no
// row-grouped tile: each coordinate goes through a column-major LDS image (conflict-free 4-byte
// stores and loads), the lane's 21 columns into registers, tap11 in the reference's order.
// Covered stencils, unresolved points, flags, positions and counts are exactly those of
// k_feat_chunk (same taps, same order, same rounding).  A window that is not regular (masked
// points, a ragged frame end, a point without a row, another order) is flagged, and k_feat_chunk,
// launched after it, does exactly the flagged blocks.
#ifndef SSF_FEAT_REG_LDS
#define SSF_FEAT_REG_LDS 0                       // k_feat_chunk_reg: halo columns from global (A/B 1: through LDS, 0.155 vs 0.147 ms)
#endif
#ifndef SSF_FEAT_REG_WAVES
#define SSF_FEAT_REG_WAVES 5                     // k_feat_chunk_reg waves per SIMD (launch bound)
#endif
template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT, SSF_FEAT_REG_WAVES) void k_feat_chunk_reg(
    const float* __restrict__ pts, int stride, const int64_t* __restrict__ frame_off, int n_frames,
    int n_rows, int n_chunks, int row_start, int row_end, float plane_min, float edge_min,
    const RingTable* __restrict__ rtab, int32_t* __restrict__ cnt, uint16_t* __restrict__ gidx,
    uint64_t* __restrict__ gbits, float* __restrict__ curv_cm, uint8_t* __restrict__ irregular,
    uint8_t* __restrict__ lanemap) {
    __shared__ __attribute__((aligned(16))) float sc[kWin];     // one coordinate, column-major
    __shared__ __attribute__((aligned(16))) uint16_t idl[kBinChunk + 4];
    __shared__ __attribute__((aligned(16))) uint8_t fll[kBinChunk];
    __shared__ int lid[kMaxRows];
    __shared__ unsigned long long lrows;
    static_assert(kWin % 64 == 0 && 64 * kCurvNW * kWinQ >= kWin, "columns");
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t nblk = (int64_t)n_chunks * n_frames;        // XCD-aware logical block
    const int64_t q8 = (nblk + 7) / 8;
    const int64_t lb = (int64_t)(blockIdx.x % 8) * q8 + blockIdx.x / 8;
    if (lb >= nblk) return;
    const int f = (int)(lb / n_chunks), c = (int)(lb - (int64_t)f * n_chunks);
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) {                                             // uniform: no chunk here at all
        if (tid == 0) irregular[lb] = 0;
        return;
    }
    const int64_t t = min(e, s + (int64_t)kBinChunk);
    const int64_t ws = max(fb, s - (int64_t)kCurvHalo), we = min(e, t + (int64_t)kCurvHalo);
    const int L = (int)(we - ws), hb = (int)(s - ws), he = (int)(t - ws);
    if (((L | hb | he) & 63) != 0) {                          // uniform: not whole columns
        if (tid == 0) irregular[lb] = 1;
        return;
    }
    const int ncols = L >> 6, c_hb = hb >> 6, own_cols = (he - hb) >> 6;
    const int cpw = (ncols + kCurvNW - 1) / kCurvNW;          // columns per wave (<= kWinQ)
    const int cw0 = w * cpw, nst = max(0, min(cpw, ncols - cw0));   // uniform
    float px[kWinQ], py[kWinQ], pz[kWinQ];
    // column col, lane l at pw + col x 64 stride (uniform: scalar) + l x stride (once per lane):
    // no per-load integer multiply
    const float* pw = pts + ws * stride + lane * stride;
    const int cstride = 64 * stride;
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {                      // every load first (clamped)
        const float* pp = pw + min(cw0 + st, ncols - 1) * cstride;
        px[st] = pp[0]; py[st] = pp[1]; pz[st] = pp[2];
    }
#if !SSF_FEAT_REG_LDS
    // the 5 columns on each side of the wave's 11 (stencil taps of its edge columns) straight
    // from global memory (L2: neighbouring waves load them as their own), in flight across the
    // ring ids and the regularity check
    float hx[10], hy[10], hz[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const int col = k < 5 ? max(cw0 - 5 + k, 0) : min(cw0 + kWinQ + k - 5, ncols - 1);
        const float* pp = pw + col * cstride;
        hx[k] = pp[0]; hy[k] = pp[1]; hz[k] = pp[2];
    }
#endif
    if (tid == 0) lrows = 0ull;
    // the row of the lane's first column (frameFeature.cpp:57-73 by the exact table, read from
    // L2), then every column's point checked INSIDE that row's ratio interval with the fast ratio
    // z * rsq(x^2 + y^2): 1e-6 (relative) clear of both ends, so the correctly rounded ratio, and
    // with it the reference's id, is that row too; a point near an end (a few in a million)
    // makes the window irregular
    const int mine = ring_id_table(px[0], py[0], pz[0], rtab->r0, rtab->inv, rtab->cell, rtab);
    const int mr = mine & (kMaxRows - 1);
    const float rlo = rtab->rlo[mr], rhi = rtab->rhi[mr];
    int ok = mine >= 0 && mine < kMaxRows;
    // the columns' ratios into one 0 / 1 word first (no ratio kept live across the loop)
    uint32_t inb = 0;
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const float r2 = px[st] * px[st] + py[st] * py[st];
        const float ra = pz[st] * __builtin_amdgcn_rsqf(r2);
        const float m = 1e-6f * fmaxf(1.0f, fabsf(ra));
        const bool in = ra >= rlo + m && ra < rhi - m && r2 > 1e-30f && r2 < 1e30f;
        inb |= (uint32_t)in << st;
    }
    const uint32_t need = nst >= 32 ? ~0u : ((1u << nst) - 1u);
    ok &= (int)((inb & need) == need);
    if (w == 0) lid[lane] = mine;
    __syncthreads();
    const int row = lid[lane];
    ok &= (int)(nst == 0) | (int)(mine == row);
    ok &= (int)(row >= 0);
    if (w == 0 && row >= 0)
        __hip_atomic_fetch_or(&lrows, 1ull << row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    ok &= (int)(lrows == ~0ull);                              // every row once per column
    if (!__syncthreads_and(ok)) {                             // uniform: the general kernel's block
        if (tid == 0) irregular[lb] = 1;
        return;
    }
    if (tid == 0) irregular[lb] = 0;
    // the chunk's row -> lane map (64 B): k_feat_select derives a selected point's chunk position
    // from it (64 x own column + lane) instead of gathering it from the u16 index, which this
    // kernel then writes only for the debug outputs
    if (w == 0) lanemap[lb * kMaxRows + row] = (uint8_t)lane;
    float v[kWinQ];
#if SSF_FEAT_REG_LDS
    auto coord = [&](const float (&P)[kWinQ], bool first) {
#pragma unroll
        for (int st = 0; st < kWinQ; ++st)
            if (st < nst) sc[(cw0 + st) * 64 + lane] = P[st];
        __syncthreads();
        float ext[kWinQ + 10];                                // columns cw0 - 5 .. cw0 + kWinQ + 4
#pragma unroll
        for (int k = 0; k < kWinQ + 10; ++k) ext[k] = sc[min(max(cw0 - 5 + k, 0), ncols - 1) * 64 + lane];
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) {
            const float d = tap11(ext + st);
            v[st] = first ? d * d : v[st] + d * d;            // ((dX dX + dY dY) + dZ dZ)
        }
        __syncthreads();                                      // before the next coordinate's stores
    };
    coord(px, true);
    coord(py, false);
    coord(pz, false);
#else
    auto coord = [&](const float (&P)[kWinQ], const float (&H)[10], bool first) {
        float ext[kWinQ + 10];                                // columns cw0 - 5 .. cw0 + kWinQ + 4
#pragma unroll
        for (int k = 0; k < 5; ++k) { ext[k] = H[k]; ext[kWinQ + 5 + k] = H[5 + k]; }
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) ext[5 + st] = P[st];   // px[st] is column cw0 + st (clamped)
#pragma unroll
        for (int st = 0; st < kWinQ; ++st) {
            const float d = tap11(ext + st);
            v[st] = first ? d * d : v[st] + d * d;            // ((dX dX + dY dY) + dZ dZ)
        }
    };
    coord(px, hx, true);
    coord(py, hy, false);
    coord(pz, hz, false);
#endif
    const bool row_in = row >= row_start && row < n_rows - row_end;
    const int64_t cm = fb + (int64_t)c * kBinChunk;           // chunk-major base (curvature)
#pragma unroll
    for (int st = 0; st < kWinQ; ++st) {
        const int col = cw0 + st;
        if (st < nst && col >= c_hb && col < c_hb + own_cols) {
            const int p = row * own_cols + (col - c_hb);
            const bool covered = col >= 5 && col < ncols - 5;
            uint8_t fl = row_in ? kFlU : (uint8_t)0;
            if (row_in && covered) {
                const uint8_t cf = cand_flags(true, true, v[st], plane_min, kEdge, edge_min);
                fl = (uint8_t)((cf & 1) ? kFlP : 0) | (uint8_t)((cf & 2) ? kFlE : 0);
            }
            idl[idl_sw(p)] = (uint16_t)(64 * (col - c_hb) + lane);
            fll[fll_sw(p)] = fl;
            if (kDebug && curv_cm) curv_cm[cm + p] = (row_in && covered) ? v[st] : 0.0f;
        }
    }
    if (tid < kMaxRows) cnt[((int64_t)f * (n_chunks + 1) + c) * kMaxRows + tid] = own_cols;
    __syncthreads();
    feat_chunk_out<kEdge>(tid, f, c, n_chunks, frame_off, (int)(t - s), kMaxRows * own_cols, idl, fll,
                          gidx, gbits, kDebug);
}

// k_feat_wave_reg: k_feat_chunk_reg's outputs with ONE WAVE per chunk (round 4).  In a regular
// window lane l of every column is the same row, so a chunk's whole stencil work is one lane's
// column sequence and needs no other wave: a work-group is kCurvNW independent chunks with no
// barrier at all.  Each wave loads the ring table into registers (lane l: cells 4l .. 4l + 3,
// rlo / rhi of row l; a lookup is a lane permute), then the chunk's 32 own columns and the 5 on
// each side (42 column loads of 768 B, streamed in blocks of kWB own columns, see stream below),
// checks regularity, evaluates every covered stencil from registers and builds the
// candidate / unresolved / edge bits of its own points as per-lane
// masks (bit i = own column i), OR-ed into the chunk's bit planes in the wave's LDS words
// (own-tile slot p = row x own columns + i) and stored as whole words.  The window's outermost
// columns (one each side of a full 6-column halo) are not loaded: no stencil of an own point
// reaches them, and they cannot change whether one is covered (a covered own point's 5 row
// neighbours on each side lie in the checked columns, which hold its row exactly once each), so
// the outputs are those of k_feat_chunk on every window this kernel calls regular.
#ifndef SSF_FEAT_WAVE_REG
#define SSF_FEAT_WAVE_REG 1                      // k_feat_wave_reg instead of k_feat_chunk_reg (A/B: 0)
#endif
#ifndef SSF_FEAT_WAVE_WAVES
#define SSF_FEAT_WAVE_WAVES 4                    // k_feat_wave_reg waves per SIMD (launch bound; 126 VGPRs)
#endif
constexpr int kWaveOwn = kBinChunk / 64;         // own columns of a full chunk (32)
constexpr int kWaveCols = kWaveOwn + 10;         // columns a wave loads
#ifndef SSF_FEAT_WAVE_BLOCK
#define SSF_FEAT_WAVE_BLOCK 8                    // own columns per streamed block
#endif
constexpr int kWB = SSF_FEAT_WAVE_BLOCK;
static_assert(kWaveOwn % kWB == 0, "whole blocks");
static_assert(kRingCells == 4 * 64 && kWaveOwn <= 32 && kCurvHalo >= 5 * 64,
              "ring table: 4 cells per lane; own-column masks are 32 bits; 5 halo columns");

// the table's cell ci from the lanes' registers (every lane must be active)
SSF_DEV RingCell cell_from_lanes(int ci, const float (&thr)[4], const int (&ids)[4]) {
    const int src = ci >> 2, q = ci & 3;
    float t4[4];
    int i4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { t4[k] = __shfl(thr[k], src, 64); i4[k] = __shfl(ids[k], src, 64); }
    RingCell rc;
    rc.thr = q == 0 ? t4[0] : q == 1 ? t4[1] : q == 2 ? t4[2] : t4[3];
    rc.ids = q == 0 ? i4[0] : q == 1 ? i4[1] : q == 2 ? i4[2] : i4[3];
    return rc;
}

template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT, (kDebug || kEdge) ? 3 : SSF_FEAT_WAVE_WAVES) void k_feat_wave_reg(
    const float* __restrict__ pts, int stride, const int64_t* __restrict__ frame_off, int n_frames,
    int n_rows, int n_chunks, int row_start, int row_end, float plane_min, float edge_min,
    const RingTable* __restrict__ rtab, int32_t* __restrict__ cnt, uint16_t* __restrict__ gidx,
    uint64_t* __restrict__ gbits, float* __restrict__ curv_cm, uint8_t* __restrict__ irregular,
    uint8_t* __restrict__ lanemap) {
    __shared__ unsigned long long wpl[kCurvNW][kFeatPlanes * kFeatWords];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t nblk = (int64_t)n_chunks * n_frames;
    const int64_t nwg = (nblk + kCurvNW - 1) / kCurvNW;       // XCD-aware logical work-group
    const int64_t q8 = (nwg + 7) / 8;
    const int64_t lw = (int64_t)(blockIdx.x % 8) * q8 + blockIdx.x / 8;
    const int64_t lb = lw * kCurvNW + w;                      // this wave's (frame, chunk)
    if (lw >= nwg || lb >= nblk) return;                      // uniform per wave (no barrier below)
    const int f = (int)(lb / n_chunks), c = (int)(lb - (int64_t)f * n_chunks);
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) {                                             // uniform: no chunk here at all
        if (lane == 0) irregular[lb] = 0;
        return;
    }
    const int64_t t = min(e, s + (int64_t)kBinChunk);
    const int64_t ws = max(fb, s - (int64_t)kCurvHalo), we = min(e, t + (int64_t)kCurvHalo);
    const int L = (int)(we - ws), hb = (int)(s - ws), he = (int)(t - ws);
    if (((L | hb | he) & 63) != 0) {                          // uniform: not whole columns
        if (lane == 0) irregular[lb] = 1;
        return;
    }
    // the table first: its loads are then the first to complete
    const float4 th4 = *reinterpret_cast<const float4*>(&rtab->cell[4 * lane]);          // cells 4l, 4l + 1
    const float4 th4b = *reinterpret_cast<const float4*>(&rtab->cell[4 * lane + 2]);     // 4l + 2, 4l + 3
    const float rlo_l = rtab->rlo[lane], rhi_l = rtab->rhi[lane];
    const float r0 = rtab->r0, rinv = rtab->inv;
    const bool dchain = rtab->chain == kRingChainDouble;      // uniform (a scalar load)
    const int ncols = L >> 6, c_hb = hb >> 6, oc = (he - hb) >> 6;
    const int j0 = c_hb - 5;                                  // window column of register k = 0
    const int klo = max(0, -j0), khi = min(kWaveCols, ncols - j0);   // registers holding real columns
    // x and y of a column side by side (the dwordx3 load's first two registers): the stencils of
    // x and y run as packed f32 pairs (v_pk_add_f32 / v_pk_mul_f32: two IEEE operations with
    // the rounding of two scalar ones, the reference's order kept), z alone
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 XY[kWaveCols];
    float Z[kWaveCols];
    // a column's base is uniform (SGPRs), the lane's byte offset one 32-bit VGPR for every column
    const uint32_t lob = (uint32_t)(lane * stride) * 4u;
    const char* wbase = reinterpret_cast<const char*>(pts + ws * stride);
    const uint32_t colb = 256u * (uint32_t)stride;            // bytes per column (< 2^31: checked at launch)
    auto load_col = [&](int k) {
        const uint32_t o = (uint32_t)min(max(j0 + k, 0), ncols - 1) * colb + lob;
        const float3 p3 = *reinterpret_cast<const float3*>(wbase + o);
        XY[k] = f2{p3.x, p3.y}; Z[k] = p3.z;
    };
    wpl[w][lane] = 0ull;                                      // the wave's plane words
    if (lane < kFeatPlanes * kFeatWords - 64) wpl[w][64 + lane] = 0ull;
    const float thr[4] = {th4.x, th4.z, th4b.x, th4b.z};
    const int ids[4] = {__float_as_int(th4.y), __float_as_int(th4.w), __float_as_int(th4b.y), __float_as_int(th4b.w)};
    int mine = -1, row = 0;
    float rlo = 0.f, rhi = 0.f;
    unsigned long long rows = 0ull;
    bool row_in = false;
    uint64_t inb = 0, need = 0;
    uint32_t mp = 0, mu = 0, me = 0;
    const int64_t cm = fb + (int64_t)c * kBinChunk;           // chunk-major base (curvature)
    uint16_t* gi = gidx + idx_base(frame_off, f) + (int64_t)c * kBinChunk;
    // every real column's point inside the row's ratio interval, clear of both ends by the row's
    // margin 1e-6 max(1, |rlo|, |rhi|) -- at least k_feat_chunk_reg's per-point 1e-6 max(1, |ra|)
    // for any ra inside, so it accepts a subset of what that check accepts -- folded into the
    // bounds once per lane (rlo / rhi below): per column one rsq, one multiply, four compares
    auto check_col = [&](int k) {
        const f2 q2 = XY[k] * XY[k];
        const float r2 = q2.x + q2.y;
        const float ra = Z[k] * __builtin_amdgcn_rsqf(r2);
        const bool in = ra >= rlo && ra < rhi && r2 > 1e-30f && r2 < 1e30f;
        inb |= (uint64_t)in << k;
        need |= (uint64_t)(k >= klo && k < khi) << k;         // uniform
    };
    // The columns stream in blocks of kWB own columns: the first block's window (kWB + 10
    // columns), then each block's loads issued before the previous block's stencils.  Even chunks
    // stream left to right, odd chunks right to left, so the 5 columns two neighbouring chunks
    // share are loaded by both at the same end of their streams, close in time (an L2 hit for the
    // later one: streaming both ways from the left, the right neighbour's copy had left the L2).
    constexpr int nb = kWaveOwn / kWB;
    auto stream = [&](auto rev) -> bool {
        constexpr bool R = decltype(rev)::value;
        constexpr int kf = R ? kWaveCols - 6 : 5;              // an own column of the first window
        constexpr int f0 = R ? kWB * (nb - 1) : 0;             // the first window [f0, f0 + kWB + 10)
        // that column first: a chunk whose first column is not one row per lane (any other layout,
        // e.g. channel-major CARLA sweeps) leaves before the other 41 columns are read
        load_col(kf);
        // the lane's row from that column (a clamped load is still a real column, and every real
        // column is checked below): ring_id_table's test with the cells from lane permutes (the
        // exact ratio's cell fetched for every lane, used where the fast one is near)
        {
            const float x = XY[kf].x, y = XY[kf].y, z = Z[kf];
            const float r2 = x * x + y * y;
            const float ra = z * __builtin_amdgcn_rsqf(r2);
            int ci = (int)((ra - r0) * rinv);
            ci = min(max(ci, 0), kRingCells - 1);
            const RingCell rc = cell_from_lanes(ci, thr, ids);
            const float m = 1e-6f * fmaxf(1.0f, fabsf(ra));
            const float tc = (ra - r0) * rinv, fr = tc - floorf(tc);
            const int near = (int)!(fabsf(ra - rc.thr) > m) | (int)!(fr > m * rinv) | (int)!(fr < 1.0f - m * rinv) |
                             (int)!(r2 > 1e-30f) | (int)!(r2 < 1e30f);
            // ring_id_exact's ratio: the float chain's z / sqrtf(r2), or the double chain's
            // double ratio (its cell from the float rounding, its threshold the cell's double)
            float rx;
            double dr = 0.0;
            if (dchain) { dr = (double)z / sqrt((double)r2); rx = (float)dr; }   // uniform
            else rx = z / sqrtf(r2);
            int cx = (int)((rx - r0) * rinv);
            cx = min(max(cx, 0), kRingCells - 1);
            const RingCell rcx = cell_from_lanes(cx, thr, ids);
            const int a = (int)(int8_t)(rc.ids & 0xff), b = (int)(int8_t)((rc.ids >> 8) & 0xff);
            const int ax = (int)(int8_t)(rcx.ids & 0xff), bx = (int)(int8_t)((rcx.ids >> 8) & 0xff);
            int idx = rx == rx ? (rx < rcx.thr ? ax : bx) : -1;
            if (dchain) idx = dr == dr ? (dr < rtab->dthr[cx] ? ax : bx) : -1;
            mine = near ? idx : (ra < rc.thr ? a : b);
        }
        row = mine & (kMaxRows - 1);
        {
            const float lo = __shfl(rlo_l, row, 64), hi = __shfl(rhi_l, row, 64);
            const float m = 1e-6f * fmaxf(1.0f, fmaxf(fabsf(lo), fabsf(hi)));
            rlo = lo + m;                                      // the check's bounds, margins in
            rhi = hi - m;
        }
        rows = 1ull << row;                                    // every row once per column
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) rows |= __shfl_xor(rows, o, 64);
        if (rows != ~0ull || !__all(mine >= 0 && mine < kMaxRows)) return false;   // uniform
        asm volatile("" ::: "memory");                         // no column load above the probe
#pragma unroll
        for (int k = f0; k < f0 + kWB + 10; ++k)
            if (k != kf) load_col(k);
        row_in = row >= row_start && row < n_rows - row_end;
#pragma unroll
        for (int k = f0; k < f0 + kWB + 10; ++k) check_col(k);
        // stencils of the own columns (window column c_hb + i, registers i .. i + 10), the flags
        // as bit i of per-lane masks: planar candidate, unresolved, edge candidate
#pragma unroll
        for (int bs = 0; bs < nb; ++bs) {
            const int bk = R ? nb - 1 - bs : bs;               // this block
            const int n0 = R ? kWB * (bk - 1) : kWB * (bk + 1) + 10;   // the next block's new columns
            if (bs + 1 < nb) {                                 // ... in flight
#pragma unroll
                for (int k = n0; k < n0 + kWB; ++k) load_col(k);
            }
#pragma unroll
            for (int i = kWB * bk; i < kWB * (bk + 1); ++i) { // no branch: columns past oc masked
                const int col = c_hb + i;
                const bool own = i < oc, covered = col >= 5 && col < ncols - 5;   // uniform
                f2 dxy = XY[i] + XY[i + 1];                   // tap11 of x and y (frameFeature.cpp:88-97)
#pragma unroll
                for (int k = 2; k < 11; ++k) dxy = (k == 5) ? dxy - f2{10.0f, 10.0f} * XY[i + 5] : dxy + XY[i + k];
                const float dz = tap11(Z + i);
                const f2 sq = dxy * dxy;
                float v = sq.x + sq.y;                        // ((dX dX + dY dY) + dZ dZ)
                v = v + dz * dz;
                const uint8_t cf = cand_flags(true, true, v, plane_min, kEdge, edge_min);
                const bool dec = own && row_in && covered;
                mp |= (uint32_t)(dec && (cf & 1)) << i;
                if (kEdge) me |= (uint32_t)(dec && (cf & 2)) << i;
                mu |= (uint32_t)(own && row_in && !covered) << i;
                if (kDebug && own) {                          // (an irregular chunk's are rewritten)
                    const int p = row * oc + i;
                    gi[p] = (uint16_t)(64 * i + lane);
                    if (curv_cm) curv_cm[cm + p] = dec ? v : 0.0f;
                }
            }
            // the block's stencils complete here, and no load moves across: 26 columns live, not 42
            asm volatile("" : "+v"(mp), "+v"(mu), "+v"(me), "+v"(inb) : : "memory");
            if (bs + 1 < nb) {
#pragma unroll
                for (int k = n0; k < n0 + kWB; ++k) check_col(k);
            }
        }
        return true;
    };
    const bool probed = (c & 1) ? stream(std::true_type{}) : stream(std::false_type{});   // uniform
    if (!probed) {                                            // not one row per lane: not regular
        if (lane == 0) irregular[lb] = kIrrGeneral;
        return;
    }
    const bool ok = mine >= 0 && mine < kMaxRows && (inb & need) == need && rows == ~0ull;
    if (!__all(ok)) {                                         // uniform: the general kernel's chunk
        if (lane == 0) irregular[lb] = 1;
        return;
    }
    // own-tile bits [row x oc, row x oc + oc) of each plane: at most two 64-bit words
    const int p0 = row * oc, wlo = p0 >> 6, sh = p0 & 63;
    const bool spill = sh + oc > 64;
    const uint32_t mk[kFeatPlanes] = {mp, mu, me};
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");    // the zeroed words before the ORs
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int pl = 0; pl < (kEdge ? 3 : 2); ++pl) {
        const uint64_t bm = mk[pl];
        if (bm) {
            __hip_atomic_fetch_or(&wpl[w][pl * kFeatWords + wlo], bm << sh, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            if (spill)
                __hip_atomic_fetch_or(&wpl[w][pl * kFeatWords + wlo + 1], bm >> (64 - sh), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    uint64_t* gb = gbits + ((int64_t)f * n_chunks + c) * (kFeatPlanes * kFeatWords);
    gb[lane] = __hip_atomic_load(&wpl[w][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   // planes 0, 1
    if (kEdge && lane < kFeatWords)
        gb[64 + lane] = __hip_atomic_load(&wpl[w][64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    cnt[((int64_t)f * (n_chunks + 1) + c) * kMaxRows + lane] = oc;
    lanemap[lb * kMaxRows + row] = (uint8_t)lane;
    if (lane == 0) irregular[lb] = 0;
}

// k_feat_wave_run: the single-read feature stage for chunks whose rows come as RUNS of consecutive
// inputs -- the layout of the reference's own data: a CARLA sweep is stored channel-major (every
// return of a channel in azimuth order, then the next channel), with the no-return rays and the
// road dropped (launch/run_noSeg.launch:4 reads a road-removed set; Scenario_Traj.py:307-315),
// so rows are ragged and no column holds one point per row.  A stencil (frameFeature.cpp:84-107)
// whose 11 taps are 11 CONSECUTIVE INPUTS of one row is exactly the reference's, whatever the rest
// of the frame holds: consecutive inputs of a row are consecutive in its ring order (:73-80).  So
// ONE WAVE per 2048-point chunk streams the chunk as 64-lane registers (lane l of register k =
// input s - 5 + 54k + l: 54 centres and 5 halo lanes each side; coalesced 768-B loads) and
// evaluates the stencil ALONG THE LANES: each of the reference's left-to-right additions is one
// v_add_f32 whose first operand is the partial sum one lane down (DPP wave_shr:1, free inside the
// instruction), so centre i's sum arrives in lane i + 5 after 11 dependent operations per
// coordinate, with tap11's roundings in tap11's order (lane_tap11x3).  Row ids: the fast ratio
// against the current row's interval (as k_feat_wave_reg's check); a register wholly inside it is
// one row, any other takes the table lookup where the check fails.  A centre is covered when its
// 10 neighbours share its row (a 10-bit window of one ballot); an own point of a row in range that
// is not covered is unresolved (row end or open stencil: k_feat_select decides it).  The chunk's
// runs (and gaps of points in no row) are logged in input order as they start.  Own-tile slots
// need each row to be at most one run in the chunk (slot = the row's base + the point's offset in
// its run): the bit planes are built in input order and moved run by run to slot order (nothing
// moves for runs in ascending row order without gaps), and k_feat_select finds a point at its
// row's run start (u16, the chunk's first 64 index entries) + its offset.  A chunk with a row in
// two runs, or more than kRunMax runs, is left to k_feat_chunk (kIrrGeneral).
#ifndef SSF_FEAT_WAVE_RUN
#define SSF_FEAT_WAVE_RUN 1                      // k_feat_wave_run for the non-regular chunks (A/B: 0)
#endif
#ifndef SSF_FEAT_RUN_WAVES
#define SSF_FEAT_RUN_WAVES 8                     // k_feat_wave_run waves per SIMD (launch bound)
#endif
constexpr int kRunStep = 54;                     // new centres per 64-lane register
constexpr int kRunMax = 64;                      // runs (and gaps) logged per chunk
#ifndef SSF_FEAT_RUN_PF
#define SSF_FEAT_RUN_PF 3                        // registers in flight per wave (r5ao: 3 0.0955 vs 4 0.0966 ms)
#endif
constexpr int kRunPF = SSF_FEAT_RUN_PF;
#ifndef SSF_FEAT_RUN_SOFF
#define SSF_FEAT_RUN_SOFF 0                      // A/B: the register step as the buffer load's SGPR offset
#endif
#ifndef SSF_FEAT_RUN_BALLOT1
#define SSF_FEAT_RUN_BALLOT1 0                   // A/B: the interior test as one ballot of a combined predicate
#endif

SSF_DEV float dpp_shr1(float v) {                // lane l <- lane l - 1 (lane 0 <- 0)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
SSF_DEV int dpp_shr1i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }

// tap11 along the lanes (see k_feat_wave_run), for x, y and z: lane L gets the sum of the centre in lane L - 5
// (valid for 10 <= L < 64).  P = x[l-1] + x[l]; three more `+ x` on the sum one lane down give
// x[l-4] + .. + x[l]; one lane down again `- 10 x[l]` is tap11's left half and centre; then five
// `+ x` on the sum one lane down add x[i+1] .. x[i+5] in order, the sum moving one lane each time.
// The three coordinates' chains step by step side by side: a DPP operand must not be read in the
// two cycles after the VALU op that wrote it, so one chain alone pays an s_nop per step.
SSF_DEV void lane_tap11x3(float x, float y, float z, float& dx, float& dy, float& dz) {
    float px = dpp_shr1(x) + x, py = dpp_shr1(y) + y, pz = dpp_shr1(z) + z;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        px = dpp_shr1(px) + x;
        py = dpp_shr1(py) + y;
        pz = dpp_shr1(pz) + z;
    }
    const float tx = 10.0f * x, ty = 10.0f * y, tz = 10.0f * z;
    px = dpp_shr1(px) - tx;
    py = dpp_shr1(py) - ty;
    pz = dpp_shr1(pz) - tz;
#pragma unroll
    for (int m = 0; m < 5; ++m) {
        px = dpp_shr1(px) + x;
        py = dpp_shr1(py) + y;
        pz = dpp_shr1(pz) + z;
    }
    dx = px; dy = py; dz = pz;
}

// bits [a, a + n) of a bit array of nw words as the low bits (0 < n <= 64)
SSF_DEV uint64_t bits_at(const unsigned long long* W, int a, int n, int nw) {
    const int wi = a >> 6, sh = a & 63;
    uint64_t v = W[wi] >> sh;
    if (sh && wi + 1 < nw) v |= (uint64_t)W[wi + 1] << (64 - sh);
    return n >= 64 ? v : (v & ((1ull << n) - 1ull));
}

template <bool kDebug, bool kEdge>
__global__ __launch_bounds__(kCurvNT, kDebug ? 2 : SSF_FEAT_RUN_WAVES) void k_feat_wave_run(
    const float* __restrict__ pts, int stride, const int64_t* __restrict__ frame_off, int n_frames,
    int n_rows, int n_chunks, int row_start, int row_end, float plane_min, float edge_min,
    const uint8_t* __restrict__ keep, const RingTable* __restrict__ rtab, int32_t* __restrict__ cnt,
    uint16_t* __restrict__ gidx, uint64_t* __restrict__ gbits, float* __restrict__ curv_cm,
    uint8_t* __restrict__ irregular, int all) {
    constexpr int kPl = kEdge ? 3 : 2;
    constexpr int kPW = kFeatPlanes * kFeatWords;
    __shared__ unsigned long long wpos[kCurvNW][kPW];    // the flags in input order
    __shared__ unsigned long long wslt[kCurvNW][kPW];    // ... in own-tile slot order
    __shared__ int2 wrun[kCurvNW][kRunMax];              // (row or -1 for a gap, first own position)
    __shared__ int wlen[kCurvNW][kMaxRows];              // own points per row
    __shared__ int wnum[kCurvNW][kMaxRows];              // runs per row
    __shared__ int wst[kCurvNW][kMaxRows];               // run start per row
    __shared__ float wcv[kDebug ? kCurvNW : 1][kDebug ? kBinChunk : 1];   // debug: curvature, input order
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t nblk = (int64_t)n_chunks * n_frames;
    const int64_t nwg = (nblk + kCurvNW - 1) / kCurvNW;       // XCD-aware logical work-group
    const int64_t q8 = (nwg + 7) / 8;
    const int64_t lw = (int64_t)(blockIdx.x % 8) * q8 + blockIdx.x / 8;
    const int64_t lb = lw * kCurvNW + w;                      // this wave's (frame, chunk)
    if (lw >= nwg || lb >= nblk) return;                      // uniform per wave (no barrier below)
    if (!all && irregular[lb] != kIrrGeneral) return;          // uniform: a regular chunk, done
    const int f = (int)(lb / n_chunks), c = (int)(lb - (int64_t)f * n_chunks);
    const int64_t fb = frame_off[f], e = frame_off[f + 1];
    const int64_t s = fb + (int64_t)c * kBinChunk;
    if (s >= e) {                                             // uniform: no chunk here at all
        if (lane == 0) irregular[lb] = kIrrRegular;
        return;
    }
    const int nf = (int)(e - fb);
    const int len = (int)(min(e, s + (int64_t)kBinChunk) - s);
    const int nreg = (len + kRunStep - 1) / kRunStep;         // registers with own centres
    const int q0 = (int)(s - fb) - 5;                         // frame index of register 0, lane 0
    for (int k = lane; k < kPW; k += 64) { wpos[w][k] = 0ull; wslt[w][k] = 0ull; }
    wlen[w][lane] = 0;
    wnum[w][lane] = 0;
    const float r0 = rtab->r0, rinv = rtab->inv;
    const int rlim = n_rows - row_end;
    // the wave's current row and its fast-ratio bounds, margins in (k_feat_wave_reg's check)
    int g = -1;
    float glo = INFINITY, ghi = -INFINITY;
    bool gin_row = false;                                     // g is a row in range
    // a register's points: frame index q = q0 + 54 k + lane through a buffer resource over the
    // frame's points: a lane outside the frame (q < 0 wraps) reads zeros from the range check and
    // is marked by INF (lanes [lo, hi) of the register are in the frame), so no clamp, no 64-bit
    // address per load: one add per register
    typedef int i3v __attribute__((ext_vector_type(3)));
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(pts + fb * stride), (short)0, nf * stride * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(keep ? keep + fb : keep), (short)0, keep ? nf : 0, 0x00020000);
    const uint32_t sb = (uint32_t)stride * 4u;
    const uint32_t voff0 = (uint32_t)(q0 + lane) * sb, vstep = (uint32_t)kRunStep * sb;
    auto load_reg = [&](int k, float& x, float& y, float& z, uint32_t& kp) {
#if SSF_FEAT_RUN_SOFF
        // the register's step as the scalar offset (SGPR): no vector add per load
        const i3v v = __builtin_amdgcn_raw_buffer_load_b96(prs, voff0, (int)((uint32_t)k * vstep), 0);
#else
        const i3v v = __builtin_amdgcn_raw_buffer_load_b96(prs, voff0 + (uint32_t)k * vstep, 0, 0);
#endif
        x = __int_as_float(v.x); y = __int_as_float(v.y); z = __int_as_float(v.z);
        kp = keep ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(krs, (uint32_t)(q0 + lane + kRunStep * k), 0, 0) : 1u;
    };
    auto lane_range = [](int lo, int hi) -> uint64_t {        // lanes [lo, hi) as a mask (0 <= lo, hi <= 64)
        if (hi <= lo) return 0ull;
        const uint64_t up = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
        return up & (~0ull << lo);
    };
    int nrun = 0;
    // the flag masks of register k (bits 0 .. 53: own positions 54 k .. 54 k + 53) go to lane k
    // of these VGPRs (v_writelane: no SALU, no LDS), and become the input-order words after the
    // loop.  The scalar unit is the one all 32 waves of a CU share: the steady state below keeps
    // it to a few instructions per register (SQ counters, r5e: 2.8 k SALU per chunk saturated it).
    uint32_t vPl = 0, vPh = 0, vUl = 0, vUh = 0, vEl = 0, vEh = 0;
    auto wl = [](uint32_t& dst, uint32_t val, int k) {        // lane k of dst <- val (uniform)
        asm("v_writelane_b32 %0, %1, %2" : "+v"(dst) : "s"(val), "{m0}"(k));   // lane select in m0
    };
    auto put = [&](int k, uint64_t mP, uint64_t mE) {
        wl(vPl, (uint32_t)mP, k);
        wl(vPh, (uint32_t)(mP >> 32), k);
        if (kEdge) {
            wl(vEl, (uint32_t)mE, k);
            wl(vEh, (uint32_t)(mE >> 32), k);
        }
    };
    // registers 1 .. kint: every lane in the frame, 54 own centres, no keep mask ("interior")
    const int kint = keep ? 0 : min((nf - 64 - q0) / kRunStep, len / kRunStep - 1);
    // one register's work (k: register, c*: its points); false when the chunk has too many runs
    auto reg = [&](int k, float cx, float cy, float cz, uint32_t ck) -> bool {
        const float r2 = cx * cx + cy * cy;
        const float ra = cz * __builtin_amdgcn_rsqf(r2);
        // (no upper bound on r2 needed: r2 = +inf gives ra = 0 = the exact z / sqrtf(inf); the
        // lower one keeps zero and denormal r2 off the fast path)
#if SSF_FEAT_RUN_BALLOT1
        const uint64_t INR = __builtin_amdgcn_ballot_w64((ra >= glo) & (ra < ghi) & (r2 > 1e-30f));
#else
        const uint64_t INR = __builtin_amdgcn_ballot_w64(ra >= glo) & __builtin_amdgcn_ballot_w64(ra < ghi) &
                             __builtin_amdgcn_ballot_w64(r2 > 1e-30f);
#endif
        if (k >= 1 && k <= kint && INR == ~0ull) {           // uniform: an interior register, all row g
            float dx, dy, dz;
            lane_tap11x3(cx, cy, cz, dx, dy, dz);
            float v = dx * dx + dy * dy;                      // ((dX dX + dY dY) + dZ dZ)
            v = v + dz * dz;
            const uint64_t R = gin_row ? ~0x3FFull : 0ull;    // own, row in range, covered
            const uint64_t mP = (R & __builtin_amdgcn_ballot_w64(v < plane_min)) >> 10;
            const uint64_t mE = kEdge ? ((R & __builtin_amdgcn_ballot_w64(v > edge_min)) >> 10) : 0ull;
            put(k, mP, mE);                                   // nothing unresolved (lanes k of vU stay 0)
            if (kDebug && lane >= 10) wcv[kDebug ? w : 0][kRunStep * k + lane - 10] = gin_row ? v : 0.0f;
            return true;
        }
        const int q = q0 + kRunStep * k;                      // frame index of lane 0 (uniform)
        const uint64_t INF = lane_range(max(0, -q), min(64, nf - q));
        const uint64_t OK = keep ? (INF & __builtin_amdgcn_ballot_w64(ck != 0u)) : INF;
        const uint64_t IN = OK & INR;
        const bool uni = IN == ~0ull;                         // the whole register is row g
        int id = g;
        if (!uni) {
            const bool in = (IN >> lane) & 1ull, ok = (OK >> lane) & 1ull;
            if (!in) id = ok ? ring_id_table(cx, cy, cz, r0, rinv, rtab->cell, rtab) : -1;
            const int last = __builtin_amdgcn_readlane(id, 63);
            if (last >= 0 && last != g) {                     // uniform: follow the last lane's row
                g = last;
                const float lo = rtab->rlo[g], hi = rtab->rhi[g];
                const float m = 1e-6f * fmaxf(1.0f, fmaxf(fabsf(lo), fabsf(hi)));
                glo = lo + m;
                ghi = hi - m;
                gin_row = g >= row_start && g < rlim;
            }
        }
        float dx, dy, dz;
        lane_tap11x3(cx, cy, cz, dx, dy, dz);
        float v = dx * dx + dy * dy;                          // ((dX dX + dY dY) + dZ dZ)
        v = v + dz * dz;
        // lane L >= 10: the centre in lane L - 5, own position a0 + L - 10
        const int a0 = kRunStep * k;
        const int nown = min(kRunStep, len - a0);             // >= 1
        const uint64_t OWN = lane_range(10, 10 + nown);
        uint64_t COV, ROWIN;
        if (uni) {                                            // from the wave's row g (SGPRs)
            COV = ~0ull;
            ROWIN = gin_row ? ~0ull : 0ull;
        } else {
            const int idp = dpp_shr1i(id);
            const uint64_t E = __builtin_amdgcn_ballot_w64(id >= 0) & __builtin_amdgcn_ballot_w64(id == idp);
            const uint64_t sh = E >> max(lane - 9, 0);       // inputs l - 1, l one row: bit l
            COV = __builtin_amdgcn_ballot_w64(lane >= 10 && (sh & 0x3FFull) == 0x3FFull);
            const int idc = __shfl(id, max(lane - 5, 0), 64);
            ROWIN = __builtin_amdgcn_ballot_w64(idc >= row_start) & __builtin_amdgcn_ballot_w64(idc < rlim);
        }
        const uint64_t DEC = OWN & ROWIN & COV;
        const uint64_t mP = (DEC & __builtin_amdgcn_ballot_w64(v < plane_min)) >> 10;   // cand_flags
        const uint64_t mU = (OWN & ROWIN & ~COV) >> 10;
        const uint64_t mE = kEdge ? ((DEC & __builtin_amdgcn_ballot_w64(v > edge_min)) >> 10) : 0ull;
        put(k, mP, mE);
        wl(vUl, (uint32_t)mU, k);
        wl(vUh, (uint32_t)(mU >> 32), k);
        if (kDebug && lane >= 10 && lane < 10 + nown) wcv[kDebug ? w : 0][a0 + lane - 10] = ((DEC >> lane) & 1ull) ? v : 0.0f;
        // the runs starting here: an own centre whose input before it is another row (or none)
        uint64_t RS;
        if (uni) RS = k == 0 ? (1ull << 5) : 0ull;
        else {
            const int idm = dpp_shr1i(id);
            RS = lane_range(5, 5 + nown) & (__builtin_amdgcn_ballot_w64(id != idm) | (k == 0 ? (1ull << 5) : 0ull));
        }
        while (RS) {                                          // uniform (SGPRs), in input order
            const int i = (int)__builtin_ctzll(RS);
            RS &= RS - 1ull;
            const int r = __builtin_amdgcn_readlane(id, i);
            if (nrun < kRunMax && lane == 0) wrun[w][nrun] = make_int2(r, a0 + i - 5);
            ++nrun;
        }
        return nrun <= kRunMax;
    };
    // SSF_FEAT_RUN_PF registers in flight per wave: a register is reloaded with the one
    // SSF_FEAT_RUN_PF ahead as soon as its points are taken (reloading after its use, in place,
    // measured slower: 0.101 against 0.099 ms, r5j)
    float X[kRunPF], Y[kRunPF], Z[kRunPF];
    uint32_t KP[kRunPF];
#pragma unroll
    for (int j = 0; j < kRunPF; ++j) load_reg(j, X[j], Y[j], Z[j], KP[j]);
    bool go = true;
    for (int k0 = 0; k0 < nreg && go; k0 += kRunPF) {        // uniform
#pragma unroll
        for (int j = 0; j < kRunPF; ++j) {
            if (go && k0 + j < nreg) {                        // uniform
                const float cx = X[j], cy = Y[j], cz = Z[j];
                const uint32_t ck = KP[j];
                load_reg(k0 + j + kRunPF, X[j], Y[j], Z[j], KP[j]);
                go = reg(k0 + j, cx, cy, cz, ck);
            }
        }
    }
    // the input-order words: lane t < 32 word t of the candidate plane, lane 32 + t of the
    // unresolved one (the edge plane next), each from the 1 .. 3 registers overlapping its bits
    {
        auto word = [&](uint32_t lo, uint32_t hi, int t) -> uint64_t {
            uint64_t wv = 0;
            const int k0 = (64 * t) / kRunStep;
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const int k = min(k0 + d, 63);
                const uint64_t m = ((uint64_t)(uint32_t)__shfl((int)hi, k, 64) << 32) |
                                   (uint32_t)__shfl((int)lo, k, 64);             // own bits 0 .. 53
                const int o = kRunStep * k - 64 * t;           // bit offset of the register in the word
                if (k0 + d < nreg && o < 64 && o > -kRunStep) wv |= o >= 0 ? (m << o) : (m >> -o);
            }
            return wv;
        };
        const int t = lane & 31;
        // (every lane shuffles the same plane's VGPRs: a shuffle reads the SOURCE lane's value)
        const uint64_t a0 = word(vPl, vPh, t), a1 = word(vUl, vUh, t);
        if (64 * t < len) wpos[w][lane < 32 ? t : kFeatWords + t] = lane < 32 ? a0 : a1;
        if (kEdge) {
            const uint64_t e2 = word(vEl, vEh, t);
            if (lane < 32 && 64 * t < len) wpos[w][2 * kFeatWords + t] = e2;
        }
    }
    bool fail = nrun > kRunMax;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");    // the loop's LDS writes before the reads
    __builtin_amdgcn_wave_barrier();
    int2 rj = make_int2(-1, len);
    int nj = 0;
    if (!fail && lane < nrun) {
        rj = wrun[w][lane];
        nj = (lane + 1 < nrun ? wrun[w][lane + 1].y : len) - rj.y;
        if (rj.x >= 0) {
            atomicAdd(&wnum[w][rj.x], 1);
            atomicAdd(&wlen[w][rj.x], nj);
            wst[w][rj.x] = rj.y;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const int cr = wlen[w][lane];                             // lane r: row r's own points
    fail = fail || __any(wnum[w][lane] > 1);
    if (fail) {                                               // uniform: a row in two runs, or too many runs
        if (lane == 0) irregular[lb] = kIrrGeneral;
        return;
    }
    int incl = cr;                                            // own-tile slot base of every row
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int base = incl - cr;
    const int bj = __shfl(base, rj.x & 63, 64);               // run lane j: its slot start
    const bool ident = __all(lane >= nrun || rj.x < 0 || bj == rj.y);   // slots = positions
    if (!ident) {                                             // uniform: move the runs' bits
        for (int j = 0; j < nrun; ++j) {
            const int r = __shfl(rj.x, j, 64), a = __shfl(rj.y, j, 64), n = __shfl(nj, j, 64);
            const int b = __shfl(bj, j, 64);
            if (r < 0 || n <= 0) continue;
            const int d0 = b >> 6, nd = ((b + n - 1) >> 6) - d0 + 1;
            for (int t = lane; t < kPl * nd; t += 64) {
                const int pl = t / nd, d = d0 + (t - pl * nd);
                const int lo = max(b, 64 * d), hi = min(b + n, 64 * d + 64);
                const uint64_t bits = bits_at(&wpos[w][pl * kFeatWords], lo - b + a, hi - lo, kFeatWords);
                if (bits)
                    __hip_atomic_fetch_or(&wslt[w][pl * kFeatWords + d], bits << (lo - 64 * d), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    const unsigned long long* PL = ident ? &wpos[w][0] : &wslt[w][0];
    uint64_t* gb = gbits + ((int64_t)f * n_chunks + c) * kPW;
    for (int t = lane; t < kPl * kFeatWords; t += 64) gb[t] = PL[t];
    cnt[((int64_t)f * (n_chunks + 1) + c) * kMaxRows + lane] = cr;
    uint16_t* gi = gidx + idx_base(frame_off, f) + (int64_t)c * kBinChunk;
    if (!kDebug) {
        gi[lane] = (uint16_t)(cr > 0 ? wst[w][lane] : 0);     // the row's run start
    } else {                                                  // every slot's position (kIrrRunIdx)
        for (int j = 0; j < nrun; ++j) {
            const int r = __shfl(rj.x, j, 64), a = __shfl(rj.y, j, 64), n = __shfl(nj, j, 64);
            const int b = __shfl(bj, j, 64);
            if (r < 0) continue;
            for (int o = lane; o < n; o += 64) {
                gi[b + o] = (uint16_t)(a + o);
                if (curv_cm) curv_cm[s + b + o] = wcv[kDebug ? w : 0][a + o];
            }
        }
    }
    if (lane == 0) irregular[lb] = kDebug ? kIrrRunIdx : kIrrRun;
}

// k_feat_select: one 1024-thread work-group per frame.  The chunks' row counts become, in LDS,
// each row's base per chunk (exclusive prefix over chunks: indexInRow of the segment's first
// point; the row lengths n_r and the ring offsets follow) and each segment's start in its chunk's
// own-tile order (exclusive prefix over rows).  Every (chunk, row) segment of the candidate planes
// is then copied, 64 bits at a time, to its row's place in ring order (bit ro[r] + indexInRow):
// the frame's candidates as row-major bit words in LDS, as k_select had them.  The unresolved
// points are decided (row ends -> curvature 0, :85; open stencils evaluated through the
// chunk-major index, the same taps in the same order) and OR-ed in; then the greedy spacing rule
// (:110-123) with one row per lane of wave 0 (wave 1: the edge rule), count-trailing-zeros walks
// over the row's words; each selection is stored as its chunk-major slot (the walk tracks the
// chunk its indexInRow falls in).  After a row prefix every thread emits framePlanePtr-ordered
// output: the point gathered through the slot's index, intensity = indexInRow + row / 100.0 (:77).
constexpr int kFeatRowWords = kFeatMaxChunks * kFeatWords + 1;   // ring-order words of a frame (+1)
#ifndef SSF_SEL_OUT_U
#define SSF_SEL_OUT_U 1                          // r5az: 1 0.0477, 2 0.0495, 4 0.0515, 8 0.0556 ms
#endif

template <bool kEdge>
__global__ __launch_bounds__(kSelThreads) void k_feat_select(const float* __restrict__ pts, int stride,
                                                             const int64_t* __restrict__ frame_off,
                                                             int n_rows, int n_chunks, int row_start,
                                                             int row_end, int plane_span,
                                                             float plane_min, float edge_min,
                                                             int32_t* __restrict__ cnt,
                                                             const uint16_t* __restrict__ gidx,
                                                             const uint64_t* __restrict__ gbits,
                                                             int32_t* __restrict__ ring_off,
                                                             float* __restrict__ curv_cm,
                                                             int32_t* __restrict__ sel,
                                                             float4* __restrict__ plane,
                                                             int32_t* __restrict__ plane_count,
                                                             int edge_span, int32_t* __restrict__ esel,
                                                             float4* __restrict__ edge,
                                                             int32_t* __restrict__ edge_count,
                                                             const uint8_t* __restrict__ irregular,
                                                             const uint8_t* __restrict__ lanemap) {
    constexpr int kRB = kFeatMaxChunks + 1;                   // odd stride: conflict-free columns
    __shared__ int rb[kMaxRows][kRB];                         // row base per chunk; [.][ncf] = n_r
    __shared__ uint16_t ss[kFeatMaxChunks][kMaxRows];         // segment start in the chunk's slots
    __shared__ uint64_t wl[kEdge ? 2 : 1][kFeatRowWords];     // candidates in ring order
    // one chunk-major candidate plane staged from global (coalesced) for the transposition, then
    // reused for the planar selections (indexInRow per output slot) when they fit
    __shared__ uint64_t stg[kFeatMaxChunks * kFeatWords];
    __shared__ int ro[kMaxRows + 1];
    __shared__ int lb[kMaxRows + 1];                          // per-row slot bases of the LDS selections
    __shared__ int pre[2][kMaxRows + 1];
    // per chunk: 1 = general-kernel block (positions from the u16 index), else its row -> lane map
    // (k_feat_chunk_reg: a selected point's chunk position is 64 x its own column + that lane)
    __shared__ uint8_t irc[kFeatMaxChunks];
    __shared__ uint8_t lmc[kFeatMaxChunks][kMaxRows];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int nwv = kSelThreads / 64;
    const int f = blockIdx.x;
    const int64_t fb = frame_off[f];
    const int nf = (int)(frame_off[f + 1] - fb);
    const int ncf = (nf + kBinChunk - 1) / kBinChunk;
    int32_t* C = cnt + (int64_t)f * (n_chunks + 1) * kMaxRows;
    const uint64_t* Bf = gbits + (int64_t)f * n_chunks * (kFeatPlanes * kFeatWords);
    const uint16_t* GI = gidx + idx_base(frame_off, f);
    // every global load of the set-up issued first, into registers (one latency, not one per
    // loop trip): the chunks' row counts (a wave's chunks), their candidate and unresolved words,
    // the block flags and the lane maps (4-byte words)
    constexpr int kCPW = kFeatMaxChunks / nwv;                // chunks per wave at most
    constexpr int kWPT = kFeatMaxChunks * kFeatWords / kSelThreads;   // plane words per thread
    constexpr int kLPT = kFeatMaxChunks * kMaxRows / 4 / kSelThreads; // lane-map words per thread
    int cv[kCPW];
#pragma unroll
    for (int i = 0; i < kCPW; ++i) {
        const int c = w + i * nwv;
        cv[i] = c < ncf ? C[c * kMaxRows + lane] : 0;
    }
    uint64_t pwd[kWPT], uwd[kWPT];
#pragma unroll
    for (int i = 0; i < kWPT; ++i) {
        const int k = tid + i * kSelThreads, cc = k / kFeatWords, wi = k - cc * kFeatWords;
        const bool in = k < ncf * kFeatWords;
        pwd[i] = in ? Bf[cc * (kFeatPlanes * kFeatWords) + wi] : 0ull;
        uwd[i] = in ? Bf[cc * (kFeatPlanes * kFeatWords) + kFeatWords + wi] : 0ull;
    }
    uint32_t lmw[kLPT];
    const uint32_t* LM = reinterpret_cast<const uint32_t*>(lanemap + (lanemap ? (int64_t)f * n_chunks * kMaxRows : 0));
#pragma unroll
    for (int i = 0; i < kLPT; ++i) {
        const int k = tid + i * kSelThreads;
        lmw[i] = (lanemap && k < ncf * (kMaxRows / 4)) ? LM[k] : 0u;
    }
    const uint8_t irv = (tid < ncf && irregular) ? irregular[(int64_t)f * n_chunks + tid] : (uint8_t)1;
    if (tid < ncf) irc[tid] = irv;
#pragma unroll
    for (int i = 0; i < kLPT; ++i) {
        const int k = tid + i * kSelThreads;
        if (k < ncf * (kMaxRows / 4)) reinterpret_cast<uint32_t*>(&lmc[0][0])[k] = lmw[i];
    }
    // the frame-local input index of row r's point j (indexInRow) in chunk cc (rb: row bases)
    auto point_of = [&](int cc, int r, int j) -> int {
        const int o = j - rb[r][cc];                          // its place in the (chunk, row) segment
        const uint8_t m = irc[cc];
        return cc * kBinChunk + (m == kIrrRun ? (int)GI[(int64_t)cc * kBinChunk + r] + o
                                 : m ? (int)GI[(int64_t)cc * kBinChunk + ss[cc][r] + o] : 64 * o + lmc[cc][r]);
    };
    // counts -> segment starts (prefix over rows, per chunk); counts into rb
#pragma unroll
    for (int i = 0; i < kCPW; ++i) {
        const int c = w + i * nwv;
        if (c >= ncf) break;                                  // uniform
        const int v = cv[i];
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        ss[c][lane] = (uint16_t)(incl - v);
        rb[lane][c] = v;
    }
    const int nwf = (nf + 63) / 64 + 1;                       // ring-order words of this frame
    for (int k = tid; k < nwf; k += kSelThreads) {
        wl[0][k] = 0ull;
        if (kEdge) wl[kEdge ? 1 : 0][k] = 0ull;
    }
    __syncthreads();
    for (int r = w; r < kMaxRows; r += nwv) {                 // per row: prefix over the chunks
        int carry = 0;
        for (int c0 = 0; c0 < ncf; c0 += 64) {                // uniform
            const int c = c0 + lane;
            const int v = c < ncf ? rb[r][c] : 0;
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            if (c < ncf) rb[r][c] = carry + incl - v;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) rb[r][ncf] = carry;
    }
    __syncthreads();
    if (tid < 64) {                                           // ring offsets: prefix over rows
        const int nr = tid < n_rows ? rb[tid][ncf] : 0;
        int incl = nr;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (tid >= o) incl += y;
        }
        if (tid < n_rows) ro[tid] = incl - nr;
        if (tid == 63) ro[n_rows] = incl;
        // a row of n_r points makes at most ceil(n_r / planeSpan) selections: slot bases for
        // the LDS copy of the planar selections
        const int cap = tid < n_rows ? (nr + plane_span - 1) / max(1, plane_span) : 0;
        int ci = cap;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(ci, o, 64);
            if (tid >= o) ci += y;
        }
        if (tid < n_rows) lb[tid] = ci - cap;
        if (tid == 63) lb[n_rows] = ci;
    }
    __syncthreads();
    if (tid <= n_rows) ring_off[(int64_t)f * (n_rows + 1) + tid] = ro[tid];
    if (curv_cm)                                              // debug: the row bases for k_feat_debug
        for (int k = tid; k < (ncf + 1) * kMaxRows; k += kSelThreads)
            C[k] = rb[k % kMaxRows][k / kMaxRows];
#if SSF_SEL_CUT == 1                                          // timing only (tools)
    __syncthreads();
    if (tid == 0) plane_count[f] = 0;
    return;
#endif
    // candidate planes: every (chunk, row) segment of a row in range to its ring-order bits,
    // one plane at a time through the staging copy
#pragma unroll
    for (int pl = 0; pl < (kEdge ? 2 : 1); ++pl) {
        if (pl) __syncthreads();                              // the previous plane's reads are done
        if (pl == 0) {
#pragma unroll
            for (int i = 0; i < kWPT; ++i) {
                const int k = tid + i * kSelThreads;
                if (k < ncf * kFeatWords) stg[k] = pwd[i];
            }
        } else {
            for (int k = tid; k < ncf * kFeatWords; k += kSelThreads) {
                const int c = k / kFeatWords, wi = k - c * kFeatWords;
                stg[k] = Bf[c * (kFeatPlanes * kFeatWords) + 2 * kFeatWords + wi];
            }
        }
        __syncthreads();
        for (int k = tid; k < ncf * kMaxRows; k += kSelThreads) {
            const int c = k / kMaxRows, r = k - c * kMaxRows;
            if (r < row_start || r >= n_rows - row_end) continue;
            const int L = rb[r][c + 1] - rb[r][c];
            const int src0 = c * kBinChunk + ss[c][r], dst0 = ro[r] + rb[r][c];
            for (int b = 0; b < L; b += 64) {
                const int sb = src0 + b, wi = sb >> 6, sh = sb & 63;
                uint64_t v = stg[wi] >> sh;
                if (sh && wi + 1 < ncf * kFeatWords) v |= stg[wi + 1] << (64 - sh);
                const int nb = L - b;
                if (nb < 64) v &= (1ull << nb) - 1ull;
                if (!v) continue;
                const int db = dst0 + b, di = db >> 6, dh = db & 63;
                atomicOr((unsigned long long*)&wl[pl][di], v << dh);
                if (dh) atomicOr((unsigned long long*)&wl[pl][di + 1], v >> (64 - dh));
            }
        }
    }
#if SSF_SEL_CUT == 2                                          // timing only (tools)
    __syncthreads();
    if (tid == 0) plane_count[f] = 0;
    return;
#endif
    // the unresolved own points of rows in range
#pragma unroll
    for (int i = 0; i < kWPT; ++i) {
        const int k = tid + i * kSelThreads;
        const int c = k / kFeatWords, wi = k - c * kFeatWords;
        uint64_t u = uwd[i];                                  // 0 beyond the frame's words
        while (u) {
            const int p = 64 * wi + (int)__builtin_ctzll(u);
            u &= u - 1ull;
            int r = 0;                                        // the last row whose segment starts <= p
#pragma unroll
            for (int st = 32; st > 0; st >>= 1)
                if (r + st < kMaxRows && ss[c][r + st] <= p) r += st;
            const int j = rb[r][c] + (p - ss[c][r]), nr = rb[r][ncf];
            const int g = ro[r] + j;                          // ring position
            if (j < 5 || j >= nr - 5) {                       // curvature 0: a planar candidate
                atomicOr((unsigned long long*)&wl[0][g >> 6], 1ull << (g & 63));
                continue;
            }
            float ux[11], uy[11], uz[11];                     // an open stencil, through the index
#pragma unroll
            for (int m = 0; m < 11; ++m) {
                const int jj = j - 5 + m;
                int cc = 0;                                   // the last chunk whose base <= jj
                for (int st = 64; st > 0; st >>= 1)
                    if (cc + st < ncf && rb[r][cc + st] <= jj) cc += st;
                const int ii = point_of(cc, r, jj);
                const float* q = pts + (fb + ii) * stride;
                ux[m] = q[0]; uy[m] = q[1]; uz[m] = q[2];
            }
            const float d0 = tap11(ux), d1 = tap11(uy), d2 = tap11(uz);
            float val = d0 * d0 + d1 * d1;
            val = val + d2 * d2;
            const uint8_t fl = cand_flags(true, true, val, plane_min, kEdge, edge_min);
            if (fl & 1) atomicOr((unsigned long long*)&wl[0][g >> 6], 1ull << (g & 63));
            if (kEdge && (fl & 2)) atomicOr((unsigned long long*)&wl[kEdge ? 1 : 0][g >> 6], 1ull << (g & 63));
            if (curv_cm) curv_cm[fb + (int64_t)c * kBinChunk + p] = val;
        }
    }
    __syncthreads();
#if SSF_SEL_CUT == 3                                          // timing only (tools)
    __syncthreads();
    if (tid == 0) plane_count[f] = 0;
    return;
#endif
    // the planar selections (indexInRow per slot) stay in LDS when a frame cannot make more than
    // the staging region holds (sum over rows of ceil(n_r / span) <= nf / span + rows)
    const bool sel_lds = lb[n_rows] <= kFeatMaxChunks * kFeatWords * 2;
    int32_t* sel_l = reinterpret_cast<int32_t*>(stg);
    if (w < (kEdge ? 2 : 1)) {                                // wave 0 planes, wave 1 edges
        const int r = lane;
        const bool e = kEdge && w == 1;
        const uint64_t* W = wl[e ? 1 : 0];
        const int span = e ? edge_span : plane_span;
        const bool lds_out = !e && sel_lds;
        int32_t* out = e ? esel + fb : (lds_out ? sel_l : sel + fb);
        int cnt_r = 0;
        if (r < n_rows && r >= row_start && r < n_rows - row_end) {
            const int rs = ro[r], n_r = ro[r + 1] - rs;
            if (n_r > 0) {
                int js = 0;                                   // jstart, row-relative
                const int kend = (rs + n_r - 1) >> 6;
                int32_t* orow = out + (lds_out ? lb[r] : rs);  // this row's selection slots
                uint64_t nxt = W[rs >> 6];
                for (int k = rs >> 6; k <= kend; ++k) {       // the row's words in order
                    uint64_t wv = nxt;
                    nxt = W[min(k + 1, kend)];                // the next word in flight
                    const int gb = k * 64;
                    int low = rs + js - gb;
                    if (low >= 64) continue;
                    if (low > 0) wv &= ~0ull << low;
                    const int top = rs + n_r - gb;
                    if (top < 64) wv &= (1ull << top) - 1ull;
                    while (wv) {
                        const int j = gb + (int)__builtin_ctzll(wv) - rs;
                        orow[cnt_r] = j;                      // indexInRow
                        ++cnt_r;
                        js = j + span;
                        low = rs + js - gb;
                        wv = low >= 64 ? 0ull : (wv & (~0ull << low));
                    }
                }
            }
        }
        int incl = cnt_r;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane < n_rows) pre[e ? 1 : 0][lane] = incl - cnt_r;
        if (lane == 63) pre[e ? 1 : 0][n_rows] = incl;
    }
    __syncthreads();
#if SSF_SEL_CUT == 4                                          // timing only (tools)
    if (tid == 0) plane_count[f] = 0;
    return;
#endif
#pragma unroll
    for (int e = 0; e < (kEdge ? 2 : 1); ++e) {
        const int* P = pre[e];
        const int total = P[n_rows];
        if (tid == 0) (e ? edge_count : plane_count)[f] = total;
        const bool lds_in = !e && sel_lds;
        const int32_t* S = e ? esel + fb : (lds_in ? sel_l : sel + fb);
        const int* SB = lds_in ? lb : ro;                     // per-row slot bases
        float4* O = e ? edge : plane;
        constexpr int U = SSF_SEL_OUT_U;          // outputs per thread per trip (loads in flight)
        for (int k0 = 0; k0 < total; k0 += U * kSelThreads) {   // uniform
            int kk[U], rr[U], jj[U], ii[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kk[u] = min(k0 + u * kSelThreads + tid, total - 1);
                int a = 0;
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (a + st < n_rows && P[a + st] <= kk[u]) a += st;
                rr[u] = a;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) jj[u] = S[SB[rr[u]] + (kk[u] - P[rr[u]])];
#pragma unroll
            for (int u = 0; u < U; ++u) {                     // indexInRow -> chunk, slot, position
                const int r = rr[u], j = jj[u];
                int cc = 0;                                   // the last chunk whose base <= j
#pragma unroll
                for (int st = 64; st > 0; st >>= 1)
                    if (cc + st < ncf && rb[r][cc + st] <= j) cc += st;
                ii[u] = point_of(cc, r, j);
            }
            float q[U][3];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float* p = pts + (fb + ii[u]) * stride;
                q[u][0] = p[0]; q[u][1] = p[1]; q[u][2] = p[2];
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k0 + u * kSelThreads + tid < total)
                    O[fb + kk[u]] = make_float4(q[u][0], q[u][1], q[u][2],
                                                (float)((double)jj[u] + (double)rr[u] / 100.0));
        }
    }
}

// Parity outputs of the single-read stage (debug only): per own-tile slot of a chunk, its row and
// indexInRow from the row bases k_feat_select left in cnt, and at its ring position the point
// (x, y, z, intensity = indexInRow + row / 100.0) and its curvature (chunk-major -> ring order).
__global__ __launch_bounds__(256) void k_feat_debug(const float* __restrict__ pts, int stride,
                                                    const int64_t* __restrict__ frame_off,
                                                    int n_rows, int n_chunks,
                                                    const int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ ring_off,
                                                    const uint16_t* __restrict__ gidx,
                                                    const float* __restrict__ curv_cm,
                                                    float4* __restrict__ out4, float* __restrict__ curv) {
    __shared__ int base[kMaxRows], segs[kMaxRows + 1], ro[kMaxRows];
    const int c = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const int64_t fb = frame_off[f];
    const int nf = (int)(frame_off[f + 1] - fb);
    if ((int64_t)c * kBinChunk >= nf) return;
    const int32_t* Cb = cnt + (int64_t)f * (n_chunks + 1) * kMaxRows;
    if (tid < 64) {
        const int b0 = Cb[c * kMaxRows + tid], b1 = Cb[(c + 1) * kMaxRows + tid];
        const int v = b1 - b0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (tid >= o) incl += y;
        }
        base[tid] = b0;
        segs[tid] = incl - v;
        if (tid == 63) segs[64] = incl;
        ro[tid] = tid < n_rows ? ring_off[(int64_t)f * (n_rows + 1) + tid] : 0;
    }
    __syncthreads();
    const int no = segs[64];
    const uint16_t* GI = gidx + idx_base(frame_off, f) + (int64_t)c * kBinChunk;
    for (int p = tid; p < no; p += 256) {
        int r = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
            if (r + st < kMaxRows && segs[r + st] <= p) r += st;
        const int j = base[r] + (p - segs[r]);
        const int64_t g = fb + ro[r] + j;
        const int ii = c * kBinChunk + (int)GI[p];
        const float* q = pts + (fb + ii) * stride;
        if (out4) out4[g] = make_float4(q[0], q[1], q[2], (float)((double)j + (double)r / 100.0));
        if (curv) curv[g] = curv_cm[fb + (int64_t)c * kBinChunk + p];
    }
}

// ---- host: the ring-id table ------------------------------------------------------------------
namespace {
constexpr double kPi = 3.14159265358979323846;       // M_PI
// the bin arithmetic of a float angle (frameFeature.cpp:58-73; oracle/ssf_oracle.c orc_ring_id_of_angle)
int angle_id(float angle, int n_rows) {
    if (angle != angle) return -1;
    int id = -1;
    if (n_rows == 16) {
        const double v = (double)((angle + 15.0f) / 2.0f) + 0.5;
        id = v > -2147483648.0 && v < 2147483647.0 ? (int)v : -1;
    } else if (n_rows == 64) {
        const double v = (double)angle >= -8.83 ? (double)(2.0f - angle) * 3.0 + 0.5 : (-8.83 - (double)angle) * 2.0 + 0.5;
        const int t = v > -2147483648.0 && v < 2147483647.0 ? (int)v : -1000;
        id = (double)angle >= -8.83 ? t : (t == -1000 ? -1 : n_rows / 2 + t);
    }
    return (id > -1 && id < n_rows) ? id : -1;
}
// the float chain's id of its float ratio: atanf, `* 180` in float, `/ M_PI` in double, to float
int id_float_chain(float ratio, int n_rows) {
    if (ratio != ratio) return -1;
    const float deg = ::atanf(ratio) * 180.0f;
    return angle_id((float)((double)deg / kPi), n_rows);
}
// the double chain's id of its double ratio
int id_double_chain(double ratio, int n_rows) {
    if (ratio != ratio) return -1;
    return angle_id((float)(::atan(ratio) * 180.0 / kPi), n_rows);
}
uint32_t fkey(float f) { uint32_t b; std::memcpy(&b, &f, 4); return (b & 0x80000000u) ? ~b : (b | 0x80000000u); }
float kfloat(uint32_t k) { const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k; float f; std::memcpy(&f, &b, 4); return f; }
uint64_t dkey(double d) { uint64_t b; std::memcpy(&b, &d, 8); return (b >> 63) ? ~b : (b | (1ull << 63)); }
double kdouble(uint64_t k) { const uint64_t b = (k >> 63) ? (k & ~(1ull << 63)) : ~k; double d; std::memcpy(&d, &b, 8); return d; }
int host_cell(float ratio, float r0, float inv) {   // the device's cell, the same float ops
    const float tc = (ratio - r0) * inv;
    return tc < 0.0f ? 0 : (tc >= (float)kRingCells ? kRingCells - 1 : std::min((int)tc, kRingCells - 1));
}
// smallest key in [lo, hi] with pred true (pred monotone false -> true on the range; hi must satisfy it)
template <class K, class P> K first_key(K lo, K hi, P pred) {
    while (lo < hi) {
        const K m = lo + (hi - lo) / 2;
        if (pred(m)) hi = m; else lo = m + 1;
    }
    return lo;
}
}  // namespace

int build_ring_table(int n_rows, int chain, void* out_host) {
    if (chain != kRingChainFloat && chain != kRingChainDouble) return -5;
    const bool dbl = chain == kRingChainDouble;
    RingTable& T = *reinterpret_cast<RingTable*>(out_host);
    std::memset(&T, 0, sizeof(T));
    T.chain = chain;
    if (n_rows == 64) { T.r0 = -0.5f; T.inv = (float)kRingCells / 0.6f; }
    else { T.r0 = -0.4f; T.inv = (float)kRingCells / 0.8f; }
    // the id of a ratio given as a double (the float chain's ratios are floats: exact in double)
    auto id_of = [&](double r) { return dbl ? id_double_chain(r, n_rows) : id_float_chain((float)r, n_rows); };
    if (id_of(-INFINITY) != id_of(-2.0) || id_of(INFINITY) != id_of(2.0)) return -1;
    // the id's change points: brackets from a dense sweep of [-2, 2] (the ids are -1 beyond),
    // each refined to the exact first ratio of the new id (first float / first double)
    std::vector<double> chg;
    double prev_r = -2.0;
    int prev_id = id_of(prev_r);
    for (int k = 1; k <= 40000; ++k) {
        const double r = (double)(-2.0f + 4.0f * (float)k / 40000.0f);
        const int id = id_of(r);
        if (id != prev_id) {
            const int a = prev_id;
            if (dbl) chg.push_back(kdouble(first_key<uint64_t>(dkey(prev_r) + 1, dkey(r), [&](uint64_t q) { return id_of(kdouble(q)) != a; })));
            else chg.push_back(kfloat(first_key<uint32_t>(fkey((float)prev_r) + 1, fkey((float)r), [&](uint32_t q) { return id_of(kfloat(q)) != a; })));
            if (id_of(chg.back()) != id) return -2;                           // two changes in one bracket
        }
        prev_r = r; prev_id = id;
    }
    int seen[kMaxRows] = {};
    for (int r = 0; r < kMaxRows; ++r) { T.rlo[r] = INFINITY; T.rhi[r] = -INFINITY; }
    for (size_t i = 0; i + 1 < chg.size(); ++i) {             // the constant-id intervals between changes
        const int id = id_of(chg[i]);
        if (id < 0 || id >= kMaxRows) continue;
        if (++seen[id] == 1) { T.rlo[id] = (float)chg[i]; T.rhi[id] = (float)chg[i + 1]; }
        else { T.rlo[id] = INFINITY; T.rhi[id] = -INFINITY; }   // a split row: never regular
    }
    const uint32_t kmin = fkey(-INFINITY), kmax = fkey(INFINITY);
    for (int c = 0; c < kRingCells; ++c) {
        // the cell's floats [ks, ke]; a change point T belongs to the cell of its float rounding
        // (the device looks a double ratio up in the cell of its float rounding; a float chain
        // ratio is its own rounding)
        const uint32_t ks = c == 0 ? kmin : first_key<uint32_t>(kmin, kmax, [&](uint32_t q) { return host_cell(kfloat(q), T.r0, T.inv) >= c; });
        if (c > 0 && host_cell(kfloat(ks), T.r0, T.inv) != c) return -3;   // an empty cell
        int nchg = 0;
        double at = 0.0;
        for (double q : chg) if (host_cell((float)q, T.r0, T.inv) == c) { ++nchg; at = q; }
        if (nchg > 1) return -4;                                             // cells too wide
        // below the change (or the whole cell): the id of the cell's first float
        const int a = nchg ? id_of(dbl ? kdouble(dkey(at) - 1) : (double)kfloat(fkey((float)at) - 1))
                           : id_of((double)kfloat(ks));
        const int b = nchg ? id_of(at) : a;
        T.cell[c].thr = nchg ? (float)at : INFINITY;
        T.dthr[c] = nchg ? at : INFINITY;
        T.cell[c].ids = (int32_t)(((uint32_t)(uint8_t)(int8_t)a) | ((uint32_t)(uint8_t)(int8_t)b << 8));
    }
    return 0;
}
size_t ring_table_bytes() { return sizeof(RingTable); }

size_t feat_idx_bytes(int64_t total, int n_frames) { return sizeof(uint16_t) * (size_t)(total + 64 * (int64_t)n_frames + 64); }
size_t feat_bits_bytes(int n_frames, int64_t max_pts) {
    const int64_t nc = (max_pts + kBinChunk - 1) / kBinChunk;
    return sizeof(uint64_t) * (size_t)std::max<int64_t>(1, (int64_t)n_frames * nc) * kFeatPlanes * kFeatWords;
}
size_t feat_cnt_bytes(int n_frames, int64_t max_pts) {
    const int64_t nc = (max_pts + kBinChunk - 1) / kBinChunk;
    return sizeof(int32_t) * (size_t)std::max(1, n_frames) * (nc + 1) * kMaxRows;
}
size_t feat_lmap_bytes(int n_frames, int64_t max_pts) {
    const int64_t nc = (max_pts + kBinChunk - 1) / kBinChunk;
    return (size_t)std::max<int64_t>(1, (int64_t)n_frames * nc) * kMaxRows;
}
size_t feat_irr_bytes(int n_frames, int64_t max_pts) {
    const int64_t nc = (max_pts + kBinChunk - 1) / kBinChunk;
    return (size_t)std::max<int64_t>(16, ((int64_t)n_frames * nc + 15) & ~(int64_t)15);
}
bool feat_single_read(int64_t max_pts) {
#ifdef SSF_FEAT_LEGACY
    (void)max_pts;
    return false;
#else
    return (max_pts + kBinChunk - 1) / kBinChunk <= kFeatMaxChunks;
#endif
}

size_t flag_bytes(int64_t total, int n_frames) { return (size_t)(total + 64 * (int64_t)n_frames + 64); }
// per-frame fix-up counts (64-byte aligned block), then the entries at the frame offsets
static size_t fix_head(int n_frames) { return ((size_t)n_frames * sizeof(uint32_t) + 63) & ~(size_t)63; }
size_t fix_bytes(int64_t total, int n_frames) { return fix_head(n_frames) + sizeof(int32_t) * (size_t)(total + 1); }

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, int32_t* ring_idx, float4* ring_xyzi, float* curv,
                                 uint8_t* flags, void* fix, int32_t* sel, float4* plane,
                                 int32_t* plane_count, const EdgeSel* edge, const FeatScratch* fs) {
    const int R = cfg.n_rows;
    const int n_chunks = (int)((max_pts + kBinChunk - 1) / kBinChunk);
    if (n_frames <= 0) return hipSuccess;
    if (R > kMaxRows) return hipErrorInvalidValue;
    if (max_pts >= (int64_t)1 << 24) return hipErrorInvalidValue;   // ring positions: 24 bits
    const bool dbg = curv != nullptr || ring_xyzi != nullptr;
    const float emin = edge ? edge->min_curv : 0.f;
    if (fs && feat_single_read(max_pts) && n_chunks > 0) {
        // the single-read stage: k_feat_chunk -> k_feat_select (-> k_feat_debug)
        float* ccm = dbg ? fs->curv_cm : nullptr;
        const int64_t nblk = (int64_t)n_chunks * n_frames;
        const dim3 grid((unsigned)((nblk + 7) / 8 * 8));
        // unmasked 64-beam frames: the regular-window kernel first, then the general one for the
        // blocks it flagged (every other block returns at once)
        const bool regular = SSF_FEAT_REGULAR && !keep && R == kMaxRows && fs->irr && fs->lmap &&
                             stride <= 4096;              // k_feat_wave_reg: 32-bit window offsets
        // the run kernel next, for the chunks k_feat_wave_reg left (every chunk when it did not
        // run: masked frames, 16 beams); then k_feat_chunk for the rest
        const bool run = SSF_FEAT_WAVE_RUN && fs->irr && stride <= 4096;
        uint8_t* irr = (regular || run) ? fs->irr : nullptr;
        const RingTable* rt = reinterpret_cast<const RingTable*>(fs->rtab);
        if (regular && SSF_FEAT_WAVE_REG) {                   // one wave per chunk
            kmark(s, "k_feat_wave_reg");
            const int64_t nwg = (nblk + kCurvNW - 1) / kCurvNW;
            const dim3 wgrid((unsigned)((nwg + 7) / 8 * 8));
#define SSF_FR_LAUNCH(D, E)                                                                         \
            hipLaunchKernelGGL((k_feat_wave_reg<D, E>), wgrid, dim3(kCurvNT), 0, s, pts, stride,     \
                               frame_off, n_frames, R, n_chunks, cfg.row_start, cfg.row_end,         \
                               cfg.plane_min, emin, rt, fs->cnt, fs->gidx, fs->gbits, ccm, irr,    \
                               fs->lmap)
            if (edge) { if (dbg) SSF_FR_LAUNCH(true, true); else SSF_FR_LAUNCH(false, true); }
            else { if (dbg) SSF_FR_LAUNCH(true, false); else SSF_FR_LAUNCH(false, false); }
#undef SSF_FR_LAUNCH
        } else if (regular) {
            kmark(s, "k_feat_chunk_reg");
#define SSF_FR_LAUNCH(D, E)                                                                         \
            hipLaunchKernelGGL((k_feat_chunk_reg<D, E>), grid, dim3(kCurvNT), 0, s, pts, stride,     \
                               frame_off, n_frames, R, n_chunks, cfg.row_start, cfg.row_end,         \
                               cfg.plane_min, emin, rt, fs->cnt, fs->gidx, fs->gbits, ccm, irr,    \
                               fs->lmap)
            if (edge) { if (dbg) SSF_FR_LAUNCH(true, true); else SSF_FR_LAUNCH(false, true); }
            else { if (dbg) SSF_FR_LAUNCH(true, false); else SSF_FR_LAUNCH(false, false); }
#undef SSF_FR_LAUNCH
        }
        if (run) {
            kmark(s, "k_feat_wave_run");
            const int64_t nwg = (nblk + kCurvNW - 1) / kCurvNW;
            const dim3 wgrid((unsigned)((nwg + 7) / 8 * 8));
#define SSF_RUN_LAUNCH(D, E)                                                                        \
            hipLaunchKernelGGL((k_feat_wave_run<D, E>), wgrid, dim3(kCurvNT), 0, s, pts, stride,     \
                               frame_off, n_frames, R, n_chunks, cfg.row_start, cfg.row_end,         \
                               cfg.plane_min, emin, keep, rt, fs->cnt, fs->gidx, fs->gbits, ccm, irr, \
                               regular ? 0 : 1)
            if (edge) { if (dbg) SSF_RUN_LAUNCH(true, true); else SSF_RUN_LAUNCH(false, true); }
            else { if (dbg) SSF_RUN_LAUNCH(true, false); else SSF_RUN_LAUNCH(false, false); }
#undef SSF_RUN_LAUNCH
        }
#define SSF_FC_COMMON pts, stride, frame_off, n_frames, R, n_chunks, cfg.row_start, cfg.row_end,         \
                      cfg.plane_min, emin, keep, rt, fs->cnt, fs->gidx, fs->gbits, ccm
        if (irr) {
            kmark(s, "k_feat_chunk_flagged");
            const dim3 fgrid((unsigned)((nblk + kFlagGroup - 1) / kFlagGroup));
#define SSF_FC_LAUNCH(D, E) hipLaunchKernelGGL((k_feat_chunk_flagged<D, E>), fgrid, dim3(kCurvNT), 0, s, SSF_FC_COMMON, irr)
            if (edge) { if (dbg) SSF_FC_LAUNCH(true, true); else SSF_FC_LAUNCH(false, true); }
            else { if (dbg) SSF_FC_LAUNCH(true, false); else SSF_FC_LAUNCH(false, false); }
#undef SSF_FC_LAUNCH
        } else {
            kmark(s, "k_feat_chunk");
#define SSF_FC_LAUNCH(D, E) hipLaunchKernelGGL((k_feat_chunk<D, E>), grid, dim3(kCurvNT), 0, s, SSF_FC_COMMON)
            if (edge) { if (dbg) SSF_FC_LAUNCH(true, true); else SSF_FC_LAUNCH(false, true); }
            else { if (dbg) SSF_FC_LAUNCH(true, false); else SSF_FC_LAUNCH(false, false); }
#undef SSF_FC_LAUNCH
        }
#undef SSF_FC_COMMON
#if SSF_FEAT_CUT
        // timing variants (tools only): the chunk kernel stopped early and wrote nothing, so the
        // select must not read its outputs; empty plane lists instead
        (void)ring_off; (void)sel;
        return hipMemsetAsync(plane_count, 0, sizeof(int32_t) * (size_t)n_frames, s);
#endif
        kmark(s, "k_feat_select");
        if (edge)
            hipLaunchKernelGGL(k_feat_select<true>, dim3(n_frames), dim3(kSelThreads), 0, s, pts, stride,
                               frame_off, R, n_chunks, cfg.row_start, cfg.row_end, cfg.plane_span,
                               cfg.plane_min, emin, fs->cnt, fs->gidx, fs->gbits, ring_off, ccm, sel,
                               plane, plane_count, edge->span, edge->sel, edge->out, edge->count, irr,
                               regular ? fs->lmap : nullptr);
        else
            hipLaunchKernelGGL(k_feat_select<false>, dim3(n_frames), dim3(kSelThreads), 0, s, pts, stride,
                               frame_off, R, n_chunks, cfg.row_start, cfg.row_end, cfg.plane_span,
                               cfg.plane_min, emin, fs->cnt, fs->gidx, fs->gbits, ring_off, ccm, sel,
                               plane, plane_count, 1, nullptr, nullptr, nullptr, irr,
                               regular ? fs->lmap : nullptr);
        if (dbg) {
            kmark(s, "k_feat_debug");
            hipLaunchKernelGGL(k_feat_debug, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                               frame_off, R, n_chunks, fs->cnt, ring_off, fs->gidx, fs->curv_cm,
                               ring_xyzi, curv);
        }
        return hipGetLastError();
    }
    // fix-up lists: per-frame counts, then the entries at the frame offsets
    uint32_t* fix_count = reinterpret_cast<uint32_t*>(fix);
    int32_t* fixl = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(fix) + fix_head(n_frames));
    if (n_chunks > 0) {
        kmark(s, "k_bin_count");
        if (!fs || !fs->rtab) return hipErrorInvalidValue;          // the ring-id table is required
        hipLaunchKernelGGL(k_bin_count, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, keep, reinterpret_cast<const RingTable*>(fs->rtab),
                           rid, hist);
    }
    kmark(s, "k_bin_scan");
    hipLaunchKernelGGL(k_bin_scan, dim3(n_frames), dim3(64), 0, s, R, n_chunks, hist, ring_off, fix_count);
    if (n_chunks > 0) {
        const int64_t nblk = (int64_t)((n_chunks + kCurvSub - 1) / kCurvSub) * n_frames;
        const dim3 grid((unsigned)((nblk + 7) / 8 * 8));
        kmark(s, "k_bin_curv");
#define SSF_BC_LAUNCH(D, E)                                                                        \
        hipLaunchKernelGGL((k_bin_curv<D, E>), grid, dim3(kCurvNT), 0, s, pts, stride, frame_off,       \
                           n_frames, R, n_chunks, cfg.row_start, cfg.row_end, cfg.plane_min, emin,  \
                           rid, hist, ring_off, ring_idx, flags, fixl, fix_count, ring_xyzi, curv)
        if (edge) { if (dbg) SSF_BC_LAUNCH(true, true); else SSF_BC_LAUNCH(false, true); }
        else { if (dbg) SSF_BC_LAUNCH(true, false); else SSF_BC_LAUNCH(false, false); }
#undef SSF_BC_LAUNCH
    }
    kmark(s, "k_select");
    if (edge)
        hipLaunchKernelGGL(k_select<true>, dim3(n_frames), dim3(kSelThreads), 0, s, pts, stride, frame_off,
                           R, cfg.row_start, cfg.row_end, cfg.plane_span, cfg.plane_min, emin, ring_off,
                           ring_idx, flags, fixl, fix_count, curv, sel, plane, plane_count, edge->span,
                           edge->sel, edge->out, edge->count);
    else
        hipLaunchKernelGGL(k_select<false>, dim3(n_frames), dim3(kSelThreads), 0, s, pts, stride, frame_off,
                           R, cfg.row_start, cfg.row_end, cfg.plane_span, cfg.plane_min, emin, ring_off,
                           ring_idx, flags, fixl, fix_count, curv, sel, plane, plane_count, 1, nullptr,
                           nullptr, nullptr);
    return hipGetLastError();
}

}  // namespace ssf
