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
constexpr int kSelThreads = 1024;
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

size_t flag_bytes(int64_t total, int n_frames) { return (size_t)(total + 64 * (int64_t)n_frames + 64); }
// per-frame fix-up counts (64-byte aligned block), then the entries at the frame offsets
static size_t fix_head(int n_frames) { return ((size_t)n_frames * sizeof(uint32_t) + 63) & ~(size_t)63; }
size_t fix_bytes(int64_t total, int n_frames) { return fix_head(n_frames) + sizeof(int32_t) * (size_t)(total + 1); }

hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, int32_t* ring_idx, float4* ring_xyzi, float* curv,
                                 uint8_t* flags, void* fix, int32_t* sel, float4* plane,
                                 int32_t* plane_count, const EdgeSel* edge) {
    const int R = cfg.n_rows;
    const int n_chunks = (int)((max_pts + kBinChunk - 1) / kBinChunk);
    if (n_frames <= 0) return hipSuccess;
    if (R > kMaxRows) return hipErrorInvalidValue;
    if (max_pts >= (int64_t)1 << 24) return hipErrorInvalidValue;   // ring positions: 24 bits
    // fix-up lists: per-frame counts, then the entries at the frame offsets
    uint32_t* fix_count = reinterpret_cast<uint32_t*>(fix);
    int32_t* fixl = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(fix) + fix_head(n_frames));
    if (n_chunks > 0) {
        kmark(s, "k_bin_count");
        hipLaunchKernelGGL(k_bin_count, dim3(n_chunks, n_frames), dim3(256), 0, s, pts, stride,
                           frame_off, R, n_chunks, keep, rid, hist);
    }
    kmark(s, "k_bin_scan");
    hipLaunchKernelGGL(k_bin_scan, dim3(n_frames), dim3(64), 0, s, R, n_chunks, hist, ring_off, fix_count);
    const bool dbg = curv != nullptr || ring_xyzi != nullptr;
    const float emin = edge ? edge->min_curv : 0.f;
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
