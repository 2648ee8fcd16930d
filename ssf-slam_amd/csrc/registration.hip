// registration.hip -- lidarOdometry_onlyPC::frameRegistration (src/lidarOdometry_onlyPC.cpp:147-252)
// on gfx950, batched over independent frame pairs.
//
//   k_plane_table  per LAST-frame plane point a: exact 30-NN (FLANN L2_Simple float distances,
//                  ties to the lower index) over the frame's plane cloud streamed through LDS
//                  tiles, ring-diverse 5-point pick (:180-205), gate d2[n] < 1 (:207), 5x3
//                  column-pivoted Householder least squares (:208-220), coplanarity gate (:222-232).
//                  Everything there depends only on (last frame, a), so it is computed once per
//                  frame here instead of twice per correspondence.
//   k_associate    per CURRENT plane point: transformToLast in double (:74-82) -> exact 1-NN in the
//                  last plane cloud (:168, unbounded) -> correspondence record {po, pa, n, valid}.
//   k_solve        one work-group per pair runs the whole Ceres-LM (or GN) loop on device:
//                  residual/Jacobian/Huber evaluation in f64 over the records, deterministic
//                  block reduction of the 28 normal-equation terms, and the 6x6 trust-region
//                  step on one lane -- no host round trip between iterations.
#include "ssf_device.hpp"
#include "ssf_internal.hpp"

#include <float.h>

#include <rocprim/block/block_radix_sort.hpp>

namespace ssf {

// ------------------------------------------------------------------------------------------
// Eigen ColPivHouseholderQR<Matrix<float,5,3>>::solve(-1) -- same sequence as the oracle's
// qr_solve_5x3 (oracle/ssf_oracle.c), float, no FMA contraction.
SSF_DEV float sqnorm_f(const float* v, int n) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < n; ++i) s = s + v[i] * v[i];
    return s;
}

// Every loop is unrolled and every runtime index (the pivot column, the permutation, the rank)
// is applied as a predicate on compile-time indices: the 5x3 system stays in registers (with
// runtime indices it lived in scratch, ~90 B of private-memory traffic per plane point).  The
// floating-point operations and their order are those of the oracle's loops.
SSF_DEV void qr_solve_5x3(float m[3][5], float x[3]) {
    float hc[3] = {0.f, 0.f, 0.f};
    int tr[3] = {0, 1, 2};
    float nu[3], nd[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { nd[k] = sqrtf(sqnorm_f(m[k], 5)); nu[k] = nd[k]; }
    float mx = nu[0];
#pragma unroll
    for (int k = 1; k < 3; ++k) if (nu[k] > mx) mx = nu[k];
    float th = mx * FLT_EPSILON;
    th = (th * th) / 5.0f;
    const float ndt = sqrtf(FLT_EPSILON);
    int nz = 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int bi = k;
        float bv = nu[k];
#pragma unroll
        for (int j = k + 1; j < 3; ++j) if (nu[j] > bv) { bv = nu[j]; bi = j; }
        const float bsq = bv * bv;
        if (nz == 3 && bsq < th * (float)(5 - k)) nz = k;
        tr[k] = bi;
#pragma unroll
        for (int j = k + 1; j < 3; ++j) {
            if (j == bi) {
#pragma unroll
                for (int r = 0; r < 5; ++r) { float t = m[k][r]; m[k][r] = m[j][r]; m[j][r] = t; }
                float t = nu[k]; nu[k] = nu[j]; nu[j] = t;
                t = nd[k]; nd[k] = nd[j]; nd[j] = t;
            }
        }
        constexpr int L0 = 5;
        const int L = L0 - k;
        float* v = &m[k][k];
        const float tail = sqnorm_f(v + 1, L - 1);
        const float c0 = v[0];
        float beta, tau;
        if (tail <= FLT_MIN) {
            tau = 0.0f; beta = c0;
#pragma unroll
            for (int i = 1; i < L; ++i) v[i] = 0.0f;
        } else {
            beta = sqrtf(c0 * c0 + tail);
            if (c0 >= 0.0f) beta = -beta;
            const float den = c0 - beta;
#pragma unroll
            for (int i = 1; i < L; ++i) v[i] = v[i] / den;
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        v[0] = beta;
        if (tau != 0.0f) {
#pragma unroll
            for (int c = k + 1; c < 3; ++c) {
                float tmp = 0.0f;
#pragma unroll
                for (int i = 1; i < L; ++i) tmp = tmp + v[i] * m[c][k + i];
                tmp = tmp + m[c][k];
                m[c][k] = m[c][k] - tau * tmp;
#pragma unroll
                for (int i = 1; i < L; ++i) m[c][k + i] = m[c][k + i] - (tau * v[i]) * tmp;
            }
        }
#pragma unroll
        for (int j = k + 1; j < 3; ++j) {
            if (nu[j] != 0.0f) {
                float t = fabsf(m[j][k]) / nu[j];
                t = (1.0f + t) * (1.0f - t);
                if (t < 0.0f) t = 0.0f;
                const float rr = nu[j] / nd[j];
                const float t2 = t * (rr * rr);
                if (t2 <= ndt) {
                    nd[j] = sqrtf(sqnorm_f(&m[j][k + 1], 5 - k - 1));
                    nu[j] = nd[j];
                } else {
                    nu[j] = nu[j] * sqrtf(t);
                }
            }
        }
    }
    int perm[3] = {0, 1, 2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {                       // swap perm[k] and perm[tr[k]] (tr[k] >= k)
        const int pk0 = perm[k];
        int pt = pk0;
#pragma unroll
        for (int j = k; j < 3; ++j) if (j == tr[k]) pt = perm[j];
#pragma unroll
        for (int j = k; j < 3; ++j) if (j == tr[k]) perm[j] = pk0;
        perm[k] = pt;
    }
    x[0] = x[1] = x[2] = 0.0f;
    if (nz == 0) return;
    float c[5] = {-1.0f, -1.0f, -1.0f, -1.0f, -1.0f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k >= nz) break;
        const float tau = hc[k];
        const int L = 5 - k;
        if (tau != 0.0f) {
            const float* v = &m[k][k];
            float tmp = 0.0f;
#pragma unroll
            for (int i = 1; i < L; ++i) tmp = tmp + v[i] * c[k + i];
            tmp = tmp + c[k];
            c[k] = c[k] - tau * tmp;
#pragma unroll
            for (int i = 1; i < L; ++i) c[k + i] = c[k + i] - (tau * v[i]) * tmp;
        }
    }
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        if (i < nz && c[i] != 0.0f) {
            c[i] = c[i] / m[i][i];
#pragma unroll
            for (int s2 = 0; s2 < i; ++s2) c[s2] = c[s2] - c[i] * m[i][s2];
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int p2 = 0; p2 < 3; ++p2)
            if (i < nz && perm[i] == p2) x[p2] = c[i];
}

constexpr int kKnnTile = 2048;
constexpr int kK = 30;

SSF_DEV bool lex_less(float ka, int ia, float kb, int ib) { return ka < kb || (ka == kb && ia < ib); }

SSF_DEV float l2_simple(const float4& q, const float4& p) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    float d = dx * dx + dy * dy;
    return d + dz * dz;
}

// A (distance, index) pair packed into one f64: high word = the non-negative f32 distance
// bits, low word = the index.  For non-negative, non-NaN values the f64 order is the u64 order
// of the bits, i.e. exactly the lexicographic (distance, index) order, so a sorted insertion is
// one v_min_f64 + one v_max_f64 per slot.  (Keys with distance 0 are f64 denormals; the kernel
// keeps f64 denormals, the default, so they compare correctly.)
SSF_DEV double knn_key(float d, int id) { return __hiloint2double(__float_as_int(d), id); }
SSF_DEV float key_dist(double k) { return __int_as_float(__double2hiint(k)); }
SSF_DEV int key_index(double k) { return __double2loint(k); }

// Branch-free.  Measured and reverted (round 2d): skipping the slots when no active lane's key
// beats its list's last (exact: keys are unique) made k_plane_table_sorted 0.40 -> 0.67 ms.
template <int K>
SSF_DEV void key_insert(double (&kk)[K], double key) {
#pragma unroll
    for (int s = 0; s < K; ++s) {
        // plain v_max/v_min (keys are never NaN: no canonicalisation), the slot updated in place
        double hi;
        asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(kk[s]), "v"(key));
        asm("v_min_f64 %0, %0, %1" : "+v"(kk[s]) : "v"(key));
        key = hi;
    }
}
// key_insert that returns the key leaving the list (the new key itself when it does not enter)
template <int K>
SSF_DEV double key_insert_out(double (&kk)[K], double key) {
#pragma unroll
    for (int s = 0; s < K; ++s) {
        double hi;
        asm("v_max_f64 %0, %1, %2" : "=v"(hi) : "v"(kk[s]), "v"(key));
        asm("v_min_f64 %0, %0, %1" : "+v"(kk[s]) : "v"(key));
        key = hi;
    }
    return key;
}

// Ring-diverse 5-point pick (:180-205), gate d2[n] < 1 (:207), 5x3 least-squares plane
// (:208-220) and coplanarity gate (:222-232) from the sorted 30-NN key list kk of a point.
SSF_DEV void plane_from_knn(const float4* __restrict__ P, const double (&kk)[30],
                            int m, float plane_max, float nrm[3], uint8_t& ok) {
    const int K = m < 30 ? m : 30;
    nrm[0] = nrm[1] = nrm[2] = 0.f;
    ok = 0;
    if (K < 5) return;                                                 // :177
    int v5[5];
    int prow = -1, vr0 = -1, vr1 = -1, nvr = 0, n = 5;
#pragma unroll
    for (int ik = 0; ik < 30; ++ik) {                                  // :180-198
        if (ik < K && nvr < 2) {
            const int id = key_index(kk[ik]);
            if ((unsigned)id >= (unsigned)m) { ok = 0; return; }       // never reached: lists are complete
            const float fi = P[id].w;
            const int ii = (int)fi;
            const int row = (int)(100.0 * ((double)(fi - (float)ii) + 0.002));
            if (ik == 0) prow = row;
            if (ik < 5) {
                v5[ik] = id;
            } else if (row != prow && row >= 0 && row <= 63) {
                if (nvr == 0) vr0 = id; else vr1 = id;
                nvr++;
                n = ik;
            }
        }
    }
    if (nvr == 1) v5[4] = vr0;                                         // :199-205
    if (nvr == 2) { v5[3] = vr0; v5[4] = vr1; }
    float dn = key_dist(kk[0]);
#pragma unroll
    for (int ik = 0; ik < 30; ++ik) if (ik == n) dn = key_dist(kk[ik]);
    if (!(dn < 1.0f)) return;                                          // :207
    float Am[3][5];
    float pts[5][3];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float4 p = P[v5[j]];
        pts[j][0] = p.x; pts[j][1] = p.y; pts[j][2] = p.z;
        Am[0][j] = p.x; Am[1][j] = p.y; Am[2][j] = p.z;
    }
    qr_solve_5x3(Am, nrm);                                             // :219
    float z = nrm[0] * nrm[0] + nrm[1] * nrm[1];
    z = z + nrm[2] * nrm[2];
    if (z > 0.0f) {                                                    // :220
        const float sq = sqrtf(z);
        nrm[0] = nrm[0] / sq; nrm[1] = nrm[1] / sq; nrm[2] = nrm[2] / sq;
    }
    ok = 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {                                      // :222-232
        const double vx = (double)(pts[k][0] - pts[k + 1][0]);
        const double vy = (double)(pts[k][1] - pts[k + 1][1]);
        const double vz = (double)(pts[k][2] - pts[k + 1][2]);
        double dd = (double)nrm[0] * vx + (double)nrm[1] * vy;
        dd = dd + (double)nrm[2] * vz;
        if (fabs(dd) > (double)plane_max) { ok = 0; break; }
    }
}

__global__ __launch_bounds__(256) void k_plane_table(const float4* __restrict__ plane,
                                                     const int64_t* __restrict__ frame_off,
                                                     const int32_t* __restrict__ count,
                                                     float plane_max, float* __restrict__ normal,
                                                     uint8_t* __restrict__ valid) {
    __shared__ float4 tile[kKnnTile];
    const int f = blockIdx.y;
    const int m = count[f];
    if ((int)(blockIdx.x * blockDim.x) >= m) return;  // uniform
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = a < m;
    const float4* P = plane + frame_off[f];
    const float4 q = active ? P[a] : make_float4(0.f, 0.f, 0.f, 0.f);
    double kk[kK];
#pragma unroll
    for (int k = 0; k < kK; ++k) kk[k] = knn_key(__builtin_inff(), 0x7fffffff);
    for (int t0 = 0; t0 < m; t0 += kKnnTile) {
        const int nt = min(kKnnTile, m - t0);
        for (int k = threadIdx.x; k < nt; k += blockDim.x) tile[k] = P[t0 + k];
        __syncthreads();
        if (active) {
            for (int k = 0; k < nt; ++k) {
                const double key = knn_key(l2_simple(q, tile[k]), t0 + k);
                if (key < kk[kK - 1]) key_insert<kK>(kk, key);
            }
        }
        __syncthreads();
    }
    if (!active) return;
    float nrm[3];
    uint8_t ok;
    plane_from_knn(P, kk, m, plane_max, nrm, ok);
    const int64_t o = frame_off[f] + a;
    normal[3 * o] = nrm[0]; normal[3 * o + 1] = nrm[1]; normal[3 * o + 2] = nrm[2];
    valid[o] = ok;
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_associate(const float4* __restrict__ last,
                                                   const int64_t* __restrict__ last_off,
                                                   const int32_t* __restrict__ last_count,
                                                   const float* __restrict__ last_normal,
                                                   const uint8_t* __restrict__ last_valid,
                                                   const float4* __restrict__ curr,
                                                   const int64_t* __restrict__ curr_off,
                                                   const int32_t* __restrict__ curr_count,
                                                   const double* __restrict__ pose_rel,
                                                   CorrRec* __restrict__ corr,
                                                   int32_t* __restrict__ nn_out) {
    __shared__ float4 tile[kKnnTile];
    const int p = blockIdx.y;
    const int mc = curr_count[p], ml = last_count[p];
    if ((int)(blockIdx.x * blockDim.x) >= mc || ml <= 10) return;  // uniform (:158)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < mc;
    const float4* L = last + last_off[p];
    const int64_t co = curr_off[p];
    const double q[4] = {pose_rel[7 * p], pose_rel[7 * p + 1], pose_rel[7 * p + 2], pose_rel[7 * p + 3]};
    const double t[3] = {pose_rel[7 * p + 4], pose_rel[7 * p + 5], pose_rel[7 * p + 6]};
    float4 pc = make_float4(0.f, 0.f, 0.f, 0.f), qs = pc;
    if (active) {
        pc = curr[co + i];
        const double v[3] = {(double)pc.x, (double)pc.y, (double)pc.z};
        double r[3];
        quat_rotate(q, v, r);                                           // :74-82
        qs.x = (float)(r[0] + t[0]); qs.y = (float)(r[1] + t[1]); qs.z = (float)(r[2] + t[2]);
    }
    float best = __builtin_inff();
    int bi = -1;
    for (int t0 = 0; t0 < ml; t0 += kKnnTile) {
        const int nt = min(kKnnTile, ml - t0);
        for (int k = threadIdx.x; k < nt; k += blockDim.x) tile[k] = L[t0 + k];
        __syncthreads();
        if (active) {
            for (int k = 0; k < nt; ++k) {
                const float d = l2_simple(qs, tile[k]);
                if (d < best) { best = d; bi = t0 + k; }
            }
        }
        __syncthreads();
    }
    if (!active) return;
    const int64_t lo = last_off[p];
    CorrRec rec;
    const bool ok = bi >= 0 && last_valid[lo + bi];
    const float4 pa = L[bi >= 0 ? bi : 0];
    rec.po[0] = pc.x; rec.po[1] = pc.y; rec.po[2] = pc.z; rec.valid = ok ? 1.0f : 0.0f;
    rec.pa[0] = pa.x; rec.pa[1] = pa.y; rec.pa[2] = pa.z; rec.pad0 = 0.f;
    const float* nr = last_normal + 3 * (lo + (bi >= 0 ? bi : 0));
    rec.n[0] = nr[0]; rec.n[1] = nr[1]; rec.n[2] = nr[2]; rec.pad1 = 0.f;
    corr[co + i] = rec;
    if (nn_out) nn_out[co + i] = bi;
}

// ------------------------------------------------------------------------------------------
// x-sorted exact k-NN.  One work-group per frame bitonic-sorts the frame's plane points by
// (x, index) in LDS; every query then walks outward from its own position in x order and stops a
// direction once fl(dx*dx) exceeds its current K-th distance: since the float distance
// ((dx*dx + dy*dy) + dz*dz) >= fl(dx*dx) and fl(dx*dx) grows monotonically along the sorted
// order, no point beyond the stop can enter the list.  Lists are ordered by (distance, original
// index), so the result is exactly the brute-force (index-order) result.  Typical frames touch a
// few hundred candidates per query instead of all M.  The sorted points / permutation are
// written out and reused as the LAST frame of the next pair's association.
constexpr int kSortMax = 16384;           // plane points per frame sorted in LDS (128 KiB)
constexpr int kTableThreads = 1024;
#ifndef SSF_TABLE_MAX_SPLIT
#define SSF_TABLE_MAX_SPLIT 8                     // work-groups per frame at most (small batches)
#endif

constexpr int kTableStripF4Max = 9216;    // after the sort, frames up to this size search strips of
// 16-B points in LDS (16 m + the 12 KiB strip table + >= 2 KiB of deferred queue) ...
constexpr int kTableStripSoaMax = 10624;  // ... and up to this size strips of 14-B SoA points

// Diagnostic build only (-DSSF_TABLE_STAMPS): lane 0 writes s_memtime deltas after the sort,
// the bounded walks and the deferred walks into sorted_idx[m .. m+3] (frame padding, read by
// tools/diag_table_phases.py); the product library never executes it.
#ifdef SSF_TABLE_STAMPS
#define SSF_TSTAMP(k) do { __syncthreads(); if (threadIdx.x == 0) SI[m + (k)] = (int32_t)((__builtin_amdgcn_s_memtime() - tstamp0) >> 4); } while (0)
#else
#define SSF_TSTAMP(k) do { } while (0)
#endif

// Outward x-walk from sorted rank r.  bounded: the list is seeded with the sentinel distance 1,
// so only points with d2 < 1 enter it, and the walk stops once dx^2 >= 1 (only those points are
// needed to decide most queries, see bounded_decides).
// Sorted-point views the walks read through (all inlined; the address space of each pointer --
// LDS or global -- is inferred at the call site):
//   PtsF4  16-B points (x, y, z, -) + a separate int permutation (sorted rank -> original index)
//   PtsSoA x / y / z float arrays + a u16 permutation: 14 B per point, so ~9k-point frames fit in
//          LDS next to the deferred-query grid
struct PtsF4 {
    const float4* S;
    const int* I;
    SSF_DEV float4 pt(int c) const { return S[c]; }
    SSF_DEV int id(int c) const { return I[c]; }
};
struct PtsSoA {
    const float* X;
    const float* Y;
    const float* Z;
    const uint16_t* I;
    SSF_DEV float4 pt(int c) const { return make_float4(X[c], Y[c], Z[c], 0.f); }
    SSF_DEV int id(int c) const { return (int)I[c]; }
};

struct PtsF4W {                     // 16-B points with the original index in .w
    const float4* S;
    SSF_DEV float4 pt(int c) const { return S[c]; }
    SSF_DEV int id(int c) const { return __float_as_int(S[c].w); }
};

template <class V>
SSF_DEV void knn_walk(const V& v, int m, int r, const float4& q, bool bounded, double (&kk)[kK]) {
    const float lim = bounded ? 1.0f : __builtin_inff();
#pragma unroll
    for (int k = 0; k < kK; ++k) kk[k] = knn_key(lim, 0x7fffffff);
    for (int c = r; c < m; ++c) {                         // rightwards (x non-decreasing)
        const float4 p = v.pt(c);
        const float dx = q.x - p.x;
        const float dx2 = dx * dx;
        if (dx2 > key_dist(kk[kK - 1]) || dx2 >= lim) break;
        const double key = knn_key(l2_simple(q, p), v.id(c));
        key_insert<kK>(kk, key);              // branch-free: a key >= kk[K-1] passes through
    }
    for (int c = r - 1; c >= 0; --c) {                    // leftwards
        const float4 p = v.pt(c);
        const float dx = q.x - p.x;
        const float dx2 = dx * dx;
        if (dx2 > key_dist(kk[kK - 1]) || dx2 >= lim) break;
        const double key = knn_key(l2_simple(q, p), v.id(c));
        key_insert<kK>(kk, key);              // branch-free: a key >= kk[K-1] passes through
    }
}

SSF_DEV int row_of(float fi) {                           // lidarOdometry_onlyPC.cpp:181-183
    const int ii = (int)fi;
    return (int)(100.0 * ((double)(fi - (float)ii) + 0.002));
}

// Is the 1-m-bounded list (kd, ki) enough to reproduce :177-232 exactly?  Let K1 = #points with
// d2 < 1 (all of them are in the list: they have |dx| < 1).  The gate d2[n] < 1 (:207) holds iff
// n < K1.  K1 <= 5 -> n >= 5 fails;  K1 >= 30 -> the list is the exact 30-NN;  two qualifying
// different-row points among ranks 5..K1-1 -> n < K1 and only ranks < K1 are used.  Otherwise
// the answer depends on ranks beyond 1 m and the query takes the full walk.
// returns 0 undecided, 1 decided (the list is exact for every rank the pick uses), 2 decided
// invalid (K1 <= 5: the list may be short, the plane is rejected without reading it).
SSF_DEV int bounded_decides(const float4* __restrict__ P, int m, const double (&kk)[kK]) {
    if (m <= kK) return 0;
    int K1 = 0;
#pragma unroll
    for (int k = 0; k < kK; ++k) K1 += key_dist(kk[k]) < 1.0f;
    if (K1 <= 5) return 2;
    if (K1 >= kK) return 1;
    const int prow = row_of(P[key_index(kk[0])].w);
    int nq = 0;
#pragma unroll
    for (int k = 5; k < kK; ++k)
        if (k < K1) {
            const int row = row_of(P[key_index(kk[k])].w);
            nq += (row != prow && row >= 0 && row <= 63);
        }
    return nq >= 2 ? 1 : 0;
}

// A deferred query (6 <= K1 < 30 keys inside 1 m, fewer than two other-ring points among ranks
// 5..K1-1) has a valid plane only if NO point of ranks K1..29 lies on another ring (0..63):
// the pick (lidarOdometry_onlyPC.cpp:180-198) takes the first such point, n becomes its rank and
// dis2[n] >= 1 fails :207.  If none is there, n is a rank inside 1 m and the plane uses only
// points inside 1 m.  kk is exact for every key closer than lim.  Returns 1 when the list
// is complete (table_finish decides), 2 when an other-ring point among the exact ranks >= K1
// decides it invalid, 0 when the ranks beyond lim are still needed.
SSF_DEV int deferred_decides(const float4* __restrict__ P, const double (&kk)[kK], float lim) {
    if (key_dist(kk[kK - 1]) < lim) return 1;
    const int prow = row_of(P[key_index(kk[0])].w);
    int dec = 0;
#pragma unroll
    for (int k = 5; k < kK; ++k) {
        const float d = key_dist(kk[k]);
        if (d >= 1.0f && d < lim) {
            const int row = row_of(P[key_index(kk[k])].w);
            if (row != prow && row >= 0 && row <= 63) dec = 2;
        }
    }
    return dec;
}

SSF_DEV void table_finish(const float4* __restrict__ P, int m, float plane_max, int64_t o,
                          const double (&kk)[kK], float* __restrict__ normal,
                          uint8_t* __restrict__ valid) {
    float nrm[3];
    uint8_t ok;
    plane_from_knn(P, kk, m, plane_max, nrm, ok);
    normal[3 * o] = nrm[0]; normal[3 * o + 1] = nrm[1]; normal[3 * o + 2] = nrm[2];
    valid[o] = ok;
}

// Queries in sorted order (adjacent lanes ~ adjacent x): 1-m-bounded walk for everyone; the
// undecided few go to an LDS queue and are re-walked in full afterwards, one per lane, so a
// handful of long walks no longer stalls whole waves.  queue == nullptr: walk in full at once.
template <class V>
SSF_DEV void table_walks(const float4* __restrict__ P, const V& v, int m, float plane_max,
                         int64_t base, float* __restrict__ normal, uint8_t* __restrict__ valid,
                         int* queue, int qcap, int* qlen, int32_t* stamp_out = nullptr,
                         unsigned long long stamp0 = 0) {
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
        const float4 q = v.pt(r);
        double kk[kK];
        bool bounded = true;
        int dec;
        for (;;) {                                        // one walk call site: one live list
            knn_walk(v, m, r, q, bounded, kk);
            if (!bounded) { dec = 1; break; }
            dec = bounded_decides(P, m, kk);
            if (dec != 0) break;
            const int slot = queue ? atomicAdd(qlen, 1) : qcap;
            if (slot < qcap) { queue[slot] = r; break; }
            bounded = false;
        }
        if (dec == 2) {                                   // gate d2[n] < 1 fails for any n >= 5
            const int64_t o = base + v.id(r);
            normal[3 * o] = 0.f; normal[3 * o + 1] = 0.f; normal[3 * o + 2] = 0.f;
            valid[o] = 0;
        } else if (dec == 1) {
            table_finish(P, m, plane_max, base + v.id(r), kk, normal, valid);
        }
    }
    if (!queue) return;
    __syncthreads();
#ifdef SSF_TABLE_STAMPS
    if (threadIdx.x == 0 && stamp_out) *stamp_out = (int32_t)((__builtin_amdgcn_s_memtime() - stamp0) >> 4);
    if (threadIdx.x == 0 && stamp_out) stamp_out[1] = *qlen;
#endif
    const int nq = min(*qlen, qcap);
    for (int k = threadIdx.x; k < nq; k += blockDim.x) {
        const int r = queue[k];
        const float4 q = v.pt(r);
        double kk[kK];
        knn_walk(v, m, r, q, false, kk);
        table_finish(P, m, plane_max, base + v.id(r), kk, normal, valid);
    }
}

// ------------------------------------------------------------------------------------------
// y-strips (shared by the plane table and the association; see k_associate_strips for the
// search and its exactness argument)
constexpr int kStripThreads = 1024;
constexpr int kStripMax = 256;             // strips per frame (W widened beyond 255 m of y)
constexpr int kStripWaves = kStripThreads / 64;
constexpr int kAssocStripF4Max = 6144;     // 16-B points (x, y, z, index) staged: 96 KiB
constexpr int kAssocStripSoaMax = 10752;   // x | y | z + u16 index (14 B): 147 KiB

struct StripLds {
    int start[kStripMax + 1];
    int cursor[kStripMax];
    float ylo[kStripMax], yhi[kStripMax];
    uint16_t wc[kStripWaves][kStripMax];
    float red[2 * kStripWaves];
};

struct StripGeo {
    float y0, W, invW;
    int ns;
    SSF_DEV int strip_of(float y) const { return min(ns - 1, max(0, (int)((y - y0) * invW))); }
};

// The plane table's strip image, kept for the association of the pairs whose LAST frame it is
// (strips_build is deterministic and both kernels run it on the same x-sorted points with the
// same work-group size, so the image is the one the association would build).  Per frame of
// m points, at the frame's offset: m float4 strip-major points (original index in the low 16
// bits of .w), and kStripHeadWords int32 words {start[kStripMax + 1], ylo[kStripMax],
// yhi[kStripMax], y0, W, invW, ns}.  Frames with kStripHeadWords <= m <= kAssocStripF4Max only
// (the header lives in the frame's own m words; the association stages float4 up to there).
constexpr int kStripHeadWords = (kStripMax + 1) + 2 * kStripMax + 4;
SSF_DEV bool strip_image_frame(int m) { return m >= kStripHeadWords && m <= kAssocStripF4Max; }
// every frame the association may stage from an image is one the table imaged: the table sorts
// it (<= kSortMax) and keeps its float4 strips (<= kTableStripF4Max)
static_assert(kTableStripF4Max >= kAssocStripF4Max && kSortMax >= kAssocStripF4Max,
              "strip image: the table must image every frame the association stages as float4");
// The header's last word is ns | kStripImageMagic << 16; a frame whose table launch did not image
// it carries 0 there (k_plane_table_sorted's other branches, k_strip_invalidate), and the
// association builds its strips itself unless the word checks out.
constexpr int32_t kStripImageMagic = 0x57A1;
SSF_DEV bool strip_image_valid(const int32_t* __restrict__ head) {
    const int32_t v = head[3 * kStripMax + 1 + 3];
    const int ns = v & 0xffff;
    return (v >> 16) == kStripImageMagic && ns >= 1 && ns <= kStripMax;
}

SSF_DEV void strip_image_store(const float4* F, const StripLds& T, const StripGeo& g, int m,
                               float4* __restrict__ img, int32_t* __restrict__ head) {
    for (int r = threadIdx.x; r < m; r += blockDim.x) img[r] = F[r];
    for (int j = threadIdx.x; j <= kStripMax; j += blockDim.x) head[j] = T.start[j];
    for (int j = threadIdx.x; j < g.ns; j += blockDim.x) {
        head[kStripMax + 1 + j] = __float_as_int(T.ylo[j]);
        head[2 * kStripMax + 1 + j] = __float_as_int(T.yhi[j]);
    }
    if (threadIdx.x == 0) {
        int32_t* gh = head + 3 * kStripMax + 1;
        gh[0] = __float_as_int(g.y0); gh[1] = __float_as_int(g.W); gh[2] = __float_as_int(g.invW);
        gh[3] = g.ns | (kStripImageMagic << 16);
    }
}

// The association's side: the image into its LDS (F, T), the geometry returned.
SSF_DEV StripGeo strip_image_load(const float4* __restrict__ img, const int32_t* __restrict__ head, int m,
                                  float4* F, StripLds& T) {
    const int32_t* gh = head + 3 * kStripMax + 1;
    StripGeo g;
    g.y0 = __int_as_float(gh[0]); g.W = __int_as_float(gh[1]); g.invW = __int_as_float(gh[2]); g.ns = gh[3] & 0xffff;
    for (int r = threadIdx.x; r < m; r += blockDim.x) F[r] = img[r];
    for (int j = threadIdx.x; j <= kStripMax; j += blockDim.x) T.start[j] = head[j];
    for (int j = threadIdx.x; j < g.ns; j += blockDim.x) {
        T.ylo[j] = __int_as_float(head[kStripMax + 1 + j]);
        T.yhi[j] = __int_as_float(head[2 * kStripMax + 1 + j]);
    }
    __syncthreads();
    return g;
}

// The strip-major points, either layout: float4 (x, y, z, original index in .w) or x | y | z
// float arrays + a u16 original index.
template <bool kSoa>
struct StripView {
    const float4* F;
    const float* X;
    const uint16_t* I;
    int m;
    SSF_DEV float4 pt(int c) const { return kSoa ? make_float4(X[c], X[m + c], X[2 * m + c], 0.f) : F[c]; }
    SSF_DEV float x(int c) const { return kSoa ? X[c] : F[c].x; }
    SSF_DEV float y(int c) const { return kSoa ? X[m + c] : F[c].y; }
    // 16-B layout: original index in the low 16 bits of .w; the plane table packs the point's
    // ring code (row_code) in bits 16..23
    SSF_DEV int id(int c) const { return kSoa ? (int)I[c] : (__float_as_int(F[c].w) & 0xFFFF); }
};

constexpr int kStripPerMax = kSortMax / kStripThreads;   // x-order points per thread (16)

// Whole work-group (kStripThreads): partition m x-sorted points into y-strips, x order kept in
// each strip (stable: per-wave match masks on the strip id, per-wave strip counts, one chunk of
// kStripThreads points in x order at a time).  get(k, r) returns the point of x-sorted rank
// r = k kStripThreads + tid with its original index in .w.  Writes the strip-major points (F,
// or X | Y | Z + I16), T.start / T.ylo / T.yhi; returns the strip geometry.
template <bool kSoa, int kPer, class Get>
SSF_DEV StripGeo strips_build(Get get, int m, StripLds& T, float4* F, float* X, uint16_t* I16,
                              float wmin = 1.001f) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float y0 = __builtin_inff(), y1 = -__builtin_inff();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int r = k * kStripThreads + tid;
        if (r < m) { const float y = get(k, r).y; y0 = fminf(y0, y); y1 = fmaxf(y1, y); }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { y0 = fminf(y0, __shfl_xor(y0, o, 64)); y1 = fmaxf(y1, __shfl_xor(y1, o, 64)); }
    if (lane == 0) { T.red[2 * w] = y0; T.red[2 * w + 1] = y1; }
    for (int k = tid; k < kStripWaves * kStripMax; k += kStripThreads) (&T.wc[0][0])[k] = 0;
    for (int k = tid; k < kStripMax; k += kStripThreads) T.cursor[k] = 0;
    __syncthreads();
    StripGeo g;
    y0 = __builtin_inff(); y1 = -__builtin_inff();
    for (int k = 0; k < kStripWaves; ++k) { y0 = fminf(y0, T.red[2 * k]); y1 = fmaxf(y1, T.red[2 * k + 1]); }
    g.y0 = y0;
    // W > 1 m (wmin) by a margin far above the float error of the strip assignment: a point two
    // strips away from the query's is then always more than 1 m away (the bounded 30-NN searches
    // the query's strip and its two neighbours only).  The plane table's pick walks take
    // wmin = 0.5005 (visit_1m then covers two strips on each side).
    g.W = fmaxf(wmin, (y1 - y0) / (float)(kStripMax - 1));
    g.invW = 1.0f / g.W;
    g.ns = min(kStripMax, (int)((y1 - y0) * g.invW) + 1);
    // histogram (cursor holds the counts), exclusive scan into start
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int r = k * kStripThreads + tid;
        if (r < m) atomicAdd(&T.cursor[g.strip_of(get(k, r).y)], 1);
    }
    __syncthreads();
    if (w == 0) {
        constexpr int per = (kStripMax + 63) / 64;                      // 4 strips per lane
        int run = 0;
        for (int k = 0; k < per; ++k) run += T.cursor[lane * per + k];
        int incl = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int y = __shfl_up(incl, o, 64); if (lane >= o) incl += y; }
        int pre = incl - run;
        for (int k = 0; k < per; ++k) {
            const int sidx = lane * per + k;
            T.start[sidx] = pre;
            pre += T.cursor[sidx];
            T.cursor[sidx] = T.start[sidx];
        }
        if (lane == 63) T.start[kStripMax] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {                                    // stable scatter by chunk
        if (k * kStripThreads >= m) break;                              // uniform
        const int r = k * kStripThreads + tid;
        const bool v = r < m;
        float4 pt = make_float4(0.f, 0.f, 0.f, 0.f);
        int sidx = 0;
        if (v) { pt = get(k, r); sidx = g.strip_of(pt.y); }
        uint64_t eq = __ballot(v);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((sidx >> b) & 1);
            eq &= ((sidx >> b) & 1) ? bb : ~bb;
        }
        const int rank = __popcll(eq & lanemask_lt());
        if (v && rank == 0) T.wc[w][sidx] = (uint16_t)__popcll(eq);
        __syncthreads();
        if (v) {
            int before = T.cursor[sidx];
            for (int j = 0; j < w; ++j) before += T.wc[j][sidx];
            const int dst = before + rank;
            if (kSoa) {
                X[dst] = pt.x; X[m + dst] = pt.y; X[2 * m + dst] = pt.z;
                I16[dst] = (uint16_t)__float_as_int(pt.w);
            } else {
                F[dst] = pt;
            }
        }
        __syncthreads();
        for (int j = tid; j < kStripMax; j += kStripThreads) {
            int add = 0;
            for (int u = 0; u < kStripWaves; ++u) { add += T.wc[u][j]; T.wc[u][j] = 0; }
            T.cursor[j] += add;
        }
        __syncthreads();
    }
    // actual y extent of every strip (the in-strip lower bound of |dy|)
    const StripView<kSoa> v{F, X, I16, m};
    for (int j = tid; j < g.ns; j += kStripThreads) {
        float a = __builtin_inff(), b = -__builtin_inff();
        for (int c = T.start[j]; c < T.start[j + 1]; ++c) { const float y = v.y(c); a = fminf(a, y); b = fmaxf(b, y); }
        T.ylo[j] = a; T.yhi[j] = b;
    }
    __syncthreads();
    return g;
}

// One strip of the k-NN search: binary search of q.x (or the query's own position `start`),
// outward walks while fl(dx^2) + fl(dymin^2) can still beat the 30th key and stays below lim.
template <bool kSoa>
SSF_DEV void strip_search(const StripView<kSoa>& v, const StripLds& T, int sidx, int start,
                          const float4& q, float lim, double (&kk)[kK]) {
    const int a = T.start[sidx], b = T.start[sidx + 1];
    if (a >= b) return;
    const float yl = T.ylo[sidx], yh = T.yhi[sidx];
    const float dyl = q.y < yl ? yl - q.y : (q.y > yh ? q.y - yh : 0.0f);
    const float dy2 = dyl * dyl;
    if (dy2 > key_dist(kk[kK - 1]) || dy2 >= lim) return;
    int l = start;
    if (l < 0) {
        l = a;
        int h = b;                                                       // first x >= q.x
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (v.x(mid) < q.x) l = mid + 1; else h = mid;
        }
    }
    for (int c = l; c < b; ++c) {                                        // rightwards
        const float4 p = v.pt(c);
        const float dx = q.x - p.x;
        const float t = dx * dx + dy2;
        if (t > key_dist(kk[kK - 1]) || t >= lim) break;
        key_insert<kK>(kk, knn_key(l2_simple(q, p), v.id(c)));
    }
    for (int c = l - 1; c >= a; --c) {                                   // leftwards
        const float4 p = v.pt(c);
        const float dx = q.x - p.x;
        const float t = dx * dx + dy2;
        if (t > key_dist(kk[kK - 1]) || t >= lim) break;
        key_insert<kK>(kk, knn_key(l2_simple(q, p), v.id(c)));
    }
}

// k-NN within radius R = kRings m (keys seeded (R^2, INT_MAX), walks stop at R^2): with
// W > 1 m only the query's strip (searched from its own position) and kRings strips on either
// side can hold points within R.  Keys are (distance, original index), so the list equals the
// x-walk's for every point closer than R; kRings = 1 is knn_walk's 1-m bounded mode.  The
// strips are unrolled (no loop nest around the walks: that spilled the 30 keys).
template <int kRings, bool kSoa>
SSF_DEV void strip_knn_radius(const StripView<kSoa>& v, const StripLds& T, const StripGeo& g,
                              int self, const float4& q, double (&kk)[kK]) {
    constexpr float R2 = (float)(kRings * kRings);
#pragma unroll
    for (int k = 0; k < kK; ++k) kk[k] = knn_key(R2, 0x7fffffff);
    const int s0 = g.strip_of(q.y);
    strip_search(v, T, s0, self, q, R2, kk);
#pragma unroll
    for (int rr = 1; rr <= kRings; ++rr) {
        if (s0 + rr < g.ns) strip_search(v, T, s0 + rr, -1, q, R2, kk);
        if (s0 - rr >= 0) strip_search(v, T, s0 - rr, -1, q, R2, kk);
    }
}

// The table's walks over the strips, queries in strip-major order (adjacent lanes: the same
// strip, adjacent x).  1-m bounded search for everyone; the undecided few are queued and
// searched in full afterwards (as table_walks).
#ifndef SSF_DEFER_RINGS
#define SSF_DEFER_RINGS 6
#endif
constexpr int kDeferRings = SSF_DEFER_RINGS;     // deferred queries: strips within this many metres
#ifndef SSF_DEFER_FIRST
#define SSF_DEFER_FIRST 2
#endif
#ifndef SSF_DEFER_MID
#define SSF_DEFER_MID 0
#endif
constexpr int kDeferFirst = SSF_DEFER_FIRST;     // ... searched first within this many metres

SSF_DEV void table_deferred_walk(const float4* __restrict__ P, const float4* __restrict__ SP,
                                 const int32_t* __restrict__ SI, int m, int qi, const float4& q,
                                 double (&kk)[kK]) {
    int l = 0, h = m;                                  // x rank of (q.x, qi) in the sorted copy
    while (l < h) {
        const int mid = (l + h) >> 1;
        if (lex_less(SP[mid].x, SI[mid], q.x, qi)) l = mid + 1; else h = mid;
    }
    knn_walk(PtsF4{SP, SI}, m, l, q, false, kk);
}

// ---- the plane table's pick without the 30-key list (16-B strip layout) ---------------------
// The pick (lidarOdometry_onlyPC.cpp:180-207) reads, from the sorted 30-NN list: the ranks 0..4,
// prow = the row of rank 0, and in rank order from rank 5 the first two points on another ring
// (0..63); n = the rank of the last one found (5 if none) must satisfy d2[n] < 1.  With K1 = the
// number of points within 1 m (the query itself included):
//   K1 <= 5                      -> invalid (n >= 5 >= K1);
//   D1 < D2: the two smallest keys of other-ring points of rank >= 5 within 1 m;
//   K1 >= 30                     -> n = rank of the last of D1, D2 whose rank (= number of keys
//                                   below it) is < 30, else 5; always valid-gated (d2 < 1);
//   K1 < 30, D2 found            -> n = rank(D2) < K1, D1 and D2 replace ranks 3 and 4;
//   K1 < 30, D2 not found        -> the ranks K1..29 lie beyond 1 m: the plane is invalid iff
//                                   an other-ring point has rank < 30, i.e. iff E, the smallest
//                                   key of an other-ring point beyond 1 m, has fewer than
//                                   30 - K1 keys beyond 1 m below it; else valid with D1 (if any).
// The planes are computed from the same five points as plane_from_knn; each stage walks the
// strips with a few registers instead of inserting every candidate into a 30-key list.
constexpr uint32_t kRowCodeBad = 255u;
SSF_DEV uint32_t row_code(float fi) {
    const int r = row_of(fi);
    return (r >= 0 && r < (int)kRowCodeBad) ? (uint32_t)r : kRowCodeBad;
}
SSF_DEV int pt_row(const float4& p) { return (__float_as_int(p.w) >> 16) & 0xFF; }
SSF_DEV int pt_id(const float4& p) { return __float_as_int(p.w) & 0xFFFF; }
// The pick walks' keys carry the point's ring code too (round 6): low word = index << 8 | ring
// code.  Indices are unique, so the key order is still exactly (distance, index); a key that
// leaves the top-five list tells its ring by itself (pick_1m keeps two other-ring keys instead of
// six).  The sentinel knn_key(d, 0x7fffffff) decodes as ring 255 (never another ring in 0..63).
SSF_DEV double pick_key(float d, const float4& p) {
    const int w = __float_as_int(p.w);
    return __hiloint2double(__float_as_int(d), ((w & 0xFFFF) << 8) | ((w >> 16) & 0xFF));
}
SSF_DEV int pick_index(double k) { return (int)((uint32_t)__double2loint(k) >> 8); }
SSF_DEV int pick_row(double k) { return __double2loint(k) & 0xFF; }

// Visit the points of one strip with dx^2 + dy_lb^2 <= bound() (bound re-read at every step)
// and < lim, from q's x position (start: the query's own strip position, or -1 = binary search).
// start: in, the query's own strip position or a position found before; -1: binary search
// (the result is stored back, so later walks of the same strip skip the search).
template <class Bound, class Body>
SSF_DEV void strip_visit(const StripView<false>& v, const StripLds& T, int sidx, int& start, const float4& q,
                         float lim, Bound&& bound, Body&& body) {
    const int a = T.start[sidx], b = T.start[sidx + 1];
    if (a >= b) return;
    const float yl = T.ylo[sidx], yh = T.yhi[sidx];
    const float dyl = q.y < yl ? yl - q.y : (q.y > yh ? q.y - yh : 0.0f);
    const float dy2 = dyl * dyl;
    if (dy2 > bound() || dy2 >= lim) return;
    int l = start;
    if (l < 0) {
        l = a;
        int h = b;
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (v.F[mid].x < q.x) l = mid + 1; else h = mid;
        }
        start = l;
    }
    // the next record is read while the current one is processed (clamped: always in the strip)
    if (l < b) {
        float4 pn = v.F[l];
        for (int c = l; c < b; ++c) {
            const float4 p = pn;
            pn = v.F[min(c + 1, b - 1)];
            const float dx = q.x - p.x;
            const float t = dx * dx + dy2;
            if (t > bound() || t >= lim) break;
            body(p);
        }
    }
    if (l > a) {
        float4 pn = v.F[l - 1];
        for (int c = l - 1; c >= a; --c) {
            const float4 p = pn;
            pn = v.F[max(c - 1, a)];
            const float dx = q.x - p.x;
            const float t = dx * dx + dy2;
            if (t > bound() || t >= lim) break;
            body(p);
        }
    }
}

// The 1-m region: the query's strip and its neighbours -- one on each side for strips wider
// than 1 m, two for strips of 0.5 .. 1 m (SSF_TABLE_PICK_W).  pos: the start positions in the
// query's strip (its own) and the neighbours (-1 until found).
#ifndef SSF_TABLE_PICK_W
#define SSF_TABLE_PICK_W 1.001f                  // pick-walk strip width floor (0.5005f: five strips, r5aq: 0.342 vs 0.276 ms, slower)
#endif
constexpr float kPickStripW = SSF_TABLE_PICK_W;
constexpr int kPos1m = kPickStripW < 1.0f ? 5 : 3;
template <class Bound, class Body>
SSF_DEV void visit_1m(const StripView<false>& v, const StripLds& T, const StripGeo& g, int (&pos)[kPos1m],
                      const float4& q, Bound&& bound, Body&& body) {
    const int s0 = g.strip_of(q.y);
    strip_visit(v, T, s0, pos[0], q, 1.0f, bound, body);
    if (s0 + 1 < g.ns) strip_visit(v, T, s0 + 1, pos[1], q, 1.0f, bound, body);
    if (s0 - 1 >= 0) strip_visit(v, T, s0 - 1, pos[2], q, 1.0f, bound, body);
    if (kPos1m == 5 && g.W < 1.0f) {                                   // uniform per frame
        if (s0 + 2 < g.ns) strip_visit(v, T, s0 + 2, pos[kPos1m == 5 ? 3 : 0], q, 1.0f, bound, body);
        if (s0 - 2 >= 0) strip_visit(v, T, s0 - 2, pos[kPos1m == 5 ? 4 : 0], q, 1.0f, bound, body);
    }
}

// Every strip outward from q's, in rings of strips, while a strip can still hold a point with
// d2 <= bound(): strip s0 +- r has |dy| >= (r - 1) W (less 1 mm of rounding slack).
template <class Bound, class Body>
SSF_DEV void visit_all(const StripView<false>& v, const StripLds& T, const StripGeo& g, int self, const float4& q,
                       Bound&& bound, Body&& body) {
    const float inf = __builtin_inff();
    const int s0 = g.strip_of(q.y);
    int p0 = self;
    strip_visit(v, T, s0, p0, q, inf, bound, body);
    for (int r = 1; r < g.ns; ++r) {
        const float lb = (float)(r - 1) * g.W - 0.001f;
        if (lb > 0.0f && lb * lb > bound()) break;
        int pu = -1, pd = -1;
        if (s0 + r < g.ns) strip_visit(v, T, s0 + r, pu, q, inf, bound, body);
        if (s0 - r >= 0) strip_visit(v, T, s0 - r, pd, q, inf, bound, body);
    }
}

// The plane of the five picked points: plane_from_knn from the least-squares solve on
// (identical arithmetic).
SSF_DEV void plane_from_pick(const float4* __restrict__ P, const int (&v5)[5], float plane_max, float nrm[3],
                             uint8_t& ok) {
    float Am[3][5];
    float pts[5][3];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float4 p = P[v5[j]];
        pts[j][0] = p.x; pts[j][1] = p.y; pts[j][2] = p.z;
        Am[0][j] = p.x; Am[1][j] = p.y; Am[2][j] = p.z;
    }
    qr_solve_5x3(Am, nrm);                                             // :219
    float z = nrm[0] * nrm[0] + nrm[1] * nrm[1];
    z = z + nrm[2] * nrm[2];
    if (z > 0.0f) {                                                    // :220
        const float sq = sqrtf(z);
        nrm[0] = nrm[0] / sq; nrm[1] = nrm[1] / sq; nrm[2] = nrm[2] / sq;
    }
    ok = 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {                                      // :222-232
        const double vx = (double)(pts[k][0] - pts[k + 1][0]);
        const double vy = (double)(pts[k][1] - pts[k + 1][1]);
        const double vz = (double)(pts[k][2] - pts[k + 1][2]);
        double dd = (double)nrm[0] * vx + (double)nrm[1] * vy;
        dd = dd + (double)nrm[2] * vz;
        if (fabs(dd) > (double)plane_max) { ok = 0; break; }
    }
}

struct PickState {
    int pos[kPos1m];    // strip start positions of the 1-m region (visit_1m)
    double t5[5];       // ranks 0..4
    double d1, d2;      // the first two other-ring keys of rank >= 5 within 1 m (sentinel: 1 m)
    int K1, prow;
    int sl;             // keys that left the top five and are not other-ring (an upper bound
                        // when d1 / d2 come from the second walk: then 1 << 30)
};

// Inside 1 m for query j, one walk: K1, the top five, and the six smallest keys of points on
// another ring than the query's own (at most four of them can be in the top five, so D1 / D2 are
// the first two of them above rank 4).  prow is the ring of rank 0: the query itself unless an
// exact duplicate with a lower index precedes it -- then a second walk with that ring.
SSF_DEV void pick_1m(const float4* __restrict__ P, const StripView<false>& v, const StripLds& T, const StripGeo& g,
                     int j, const float4& q, PickState& s) {
    const double sent = knn_key(1.0f, 0x7fffffff);
#pragma unroll
    for (int k = 0; k < 5; ++k) s.t5[k] = sent;
    // o2: the two smallest other-ring keys that LEFT the top five.  Every key within 1 m either
    // ends in the final top five or leaves it exactly once (the list only improves), so the keys
    // that left are exactly those above the final rank-4 key: o2 = D1, D2 (when rank 0's ring is
    // the query's own; otherwise the second walk below)
    double o2[2] = {sent, sent};
    const int qrow = pt_row(q);
    int K1 = 0, sl = 0;
    s.pos[0] = j;
#pragma unroll
    for (int k = 1; k < kPos1m; ++k) s.pos[k] = -1;
    visit_1m(v, T, g, s.pos, q, [] { return 1.0f; }, [&](const float4& p) {
        const float d = l2_simple(q, p);
        if (d < 1.0f) {
            ++K1;
            const double out = key_insert_out<5>(s.t5, pick_key(d, p));
            const int row = pick_row(out);
            if (row != qrow && row <= 63) key_insert<2>(o2, out);
            else ++sl;
        }
    });
    s.K1 = K1;
    s.sl = 1 << 30;
    s.d1 = sent; s.d2 = sent;
    s.prow = -1;
    if (K1 <= 5) return;
    s.prow = pick_row(s.t5[0]);                                        // row_of(P[rank 0].w)
    const double k5 = s.t5[4];
    if (pick_index(s.t5[0]) == pt_id(q) || s.prow == qrow) {
        s.d1 = o2[0]; s.d2 = o2[1];
        s.sl = sl;
        return;
    }
    const int prow = s.prow;
    double dd[2] = {sent, sent};
    visit_1m(v, T, g, s.pos, q, [&] { return key_dist(dd[1]); }, [&](const float4& p) {
        const float d = l2_simple(q, p);
        const int row = pt_row(p);
        const double key = pick_key(d, p);
        if (d < 1.0f && key > k5 && row != prow && row <= 63) key_insert<2>(dd, key);
    });
    s.d1 = dd[0]; s.d2 = dd[1];
}

SSF_DEV void pick_finish(const float4* __restrict__ P, const PickState& s, int nvr, float plane_max, int64_t o,
                         float* __restrict__ normal, uint8_t* __restrict__ valid) {
    int v5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) v5[k] = pick_index(s.t5[k]);
    if (nvr == 1) v5[4] = pick_index(s.d1);                            // :199-205
    if (nvr == 2) { v5[3] = pick_index(s.d1); v5[4] = pick_index(s.d2); }
    float nrm[3];
    uint8_t ok;
    plane_from_pick(P, v5, plane_max, nrm, ok);
    normal[3 * o] = nrm[0]; normal[3 * o + 1] = nrm[1]; normal[3 * o + 2] = nrm[2];
    valid[o] = ok;
}

SSF_DEV void pick_invalid(int64_t o, float* __restrict__ normal, uint8_t* __restrict__ valid) {
    normal[3 * o] = 0.f; normal[3 * o + 1] = 0.f; normal[3 * o + 2] = 0.f;
    valid[o] = 0;
}

// Beyond 1 m (K1 < 30, fewer than two other-ring points inside): invalid iff E, the smallest
// key of an other-ring point beyond 1 m, has fewer than 30 - K1 keys beyond 1 m below it.
SSF_DEV bool pick_beyond_invalid(const StripView<false>& v, const StripLds& T, const StripGeo& g, int j,
                                 const float4& q, const PickState& s) {
    double E = knn_key(__builtin_inff(), 0x7fffffff);
    const int prow = s.prow;
    visit_all(v, T, g, j, q, [&] { return key_dist(E); }, [&](const float4& p) {
        const float d = l2_simple(q, p);
        const int row = pt_row(p);
        const double key = pick_key(d, p);
        if (d >= 1.0f && row != prow && row <= 63 && key < E) E = key;
    });
    if (!(key_dist(E) < __builtin_inff())) return false;          // no other-ring point at all
    int C = 0;
    const int need = 30 - s.K1;
    const float lim = key_dist(E);
    visit_all(v, T, g, j, q, [&] { return C >= need ? -1.0f : lim; }, [&](const float4& p) {
        const float d = l2_simple(q, p);
        C += (d >= 1.0f && pick_key(d, p) < E);
    });
    return C < need;
}

#ifndef SSF_TABLE_COOP_G
#define SSF_TABLE_COOP_G 4                       // lanes per deferred pick query (0: one lane each)
#endif
constexpr int kTableCoopG = SSF_TABLE_COOP_G;
// Whole work-group: every query of the frame (m > 30, every ring code < 255).  Queries that need
// points beyond 1 m (K1 < 30, fewer than two other-ring points inside) are queued and finished
// afterwards, spread over the waves.
SSF_DEV void table_pick_walks(const float4* __restrict__ P, const StripView<false>& v, const StripLds& T,
                              const StripGeo& g, int m, float plane_max, int64_t base, float* __restrict__ normal,
                              uint8_t* __restrict__ valid, int* queue, int qcap, int* qlen,
                              int32_t* stamp_out = nullptr, unsigned long long stamp0 = 0,
                              int share = 0, int nshare = 1) {
    // queries of this work-group's share: every nshare-th one (k_plane_table_sorted splits a
    // frame's queries over nshare work-groups for small batches)
    for (int j = share + nshare * (int)threadIdx.x; j < m; j += nshare * (int)blockDim.x) {
        const float4 q = v.pt(j);
        const int64_t o = base + v.id(j);
        PickState s;
        pick_1m(P, v, T, g, j, q, s);
        if (s.K1 <= 5) { pick_invalid(o, normal, valid); continue; }
        const bool f1 = key_dist(s.d1) < 1.0f, f2 = key_dist(s.d2) < 1.0f;
        if (s.K1 >= 30) {
            int r1 = 0, r2 = 0;                                            // ranks of D1, D2
            // the keys below D2 are the top five, D1 and left keys that are not other-ring (D1 /
            // D2 are the two smallest other-ring keys that left): with L such keys r1 <= 5 + L,
            // r2 <= 6 + L, so L <= 23 puts both inside the 30 without the rank walk.  sl = L + 5
            // (the five sentinels left the list too: K1 >= 30)
            if (f1 && s.sl > 28) {
                const double b1 = s.d1, b2 = s.d2;
                const float lim = f2 ? key_dist(b2) : key_dist(b1);
                visit_1m(v, T, g, s.pos, q, [&] { return lim; }, [&](const float4& p) {
                    const double key = pick_key(l2_simple(q, p), p);
                    r1 += key < b1;
                    r2 += key < b2;
                });
            }
            const int nvr = (f1 && r1 < 30) + (f2 && r2 < 30);
            pick_finish(P, s, nvr, plane_max, o, normal, valid);
        } else if (f2) {
            pick_finish(P, s, 2, plane_max, o, normal, valid);
        } else {
            const int slot = atomicAdd(qlen, 1);
            if (slot < qcap) { queue[slot] = j; continue; }
            if (pick_beyond_invalid(v, T, g, j, q, s)) pick_invalid(o, normal, valid);   // queue full
            else pick_finish(P, s, f1 ? 1 : 0, plane_max, o, normal, valid);
        }
    }
    __syncthreads();
#ifdef SSF_TABLE_STAMPS
    if (threadIdx.x == 0 && stamp_out) { stamp_out[0] = (int32_t)((__builtin_amdgcn_s_memtime() - stamp0) >> 4); stamp_out[1] = *qlen; }
#endif
    const int nq = min(*qlen, qcap);
#if SSF_TABLE_COOP_G
    // one deferred query per group of kTableCoopG lanes: the group's lanes run the 1-m pick
    // redundantly (same bits), then both beyond-1-m searches of pick_beyond_invalid with the
    // strips of each ring round one per lane (strip i of the round order s0, s0+1, s0-1, s0+2,
    // ...), the group's minimum E / sum C after each round -- a lane alone walked every ring
    // (the slowest deferred query set the frame's time: ~0.127 M of ~0.60 M cycles, r03 stamps)
    {
        constexpr int G = kTableCoopG;
        const int gl = threadIdx.x % G, ng = blockDim.x / G;
        for (int k = threadIdx.x / G; k < nq; k += ng) {
            const int j = queue[k];                                       // uniform per group
            const float4 q = v.pt(j);
            const int64_t o = base + v.id(j);
            PickState s;
            pick_1m(P, v, T, g, j, q, s);
            const bool f1 = key_dist(s.d1) < 1.0f;
            const int prow = s.prow, s0 = g.strip_of(q.y), nstrip = 2 * g.ns;   // round order
            auto strip_at = [&](int i) { return i == 0 ? s0 : ((i & 1) ? s0 + (i + 1) / 2 : s0 - i / 2); };
            auto ring_at = [&](int i) { return (i + 1) / 2; };
            // E: the smallest key of an other-ring point beyond 1 m
            double E = knn_key(__builtin_inff(), 0x7fffffff);
            for (int i0 = 0; i0 < nstrip; i0 += G) {
                // a round's strips all have rings >= ring_at(i0): their |dy| >= (r - 1) W
                const float lb = (float)(ring_at(i0) - 1) * g.W - 0.001f;
                if (i0 > 0 && lb > 0.0f && lb * lb > key_dist(E)) break;   // uniform per group
                const int i = i0 + gl, sidx = strip_at(i);
                if (i < nstrip && sidx >= 0 && sidx < g.ns) {
                    int st = sidx == s0 ? j : -1;
                    strip_visit(v, T, sidx, st, q, __builtin_inff(), [&] { return key_dist(E); },
                                [&](const float4& p) {
                                    const float d = l2_simple(q, p);
                                    const int row = pt_row(p);
                                    const double key = pick_key(d, p);
                                    if (d >= 1.0f && row != prow && row <= 63 && key < E) E = key;
                                });
                }
#pragma unroll
                for (int x = G / 2; x >= 1; x >>= 1) {
                    const double y = __shfl_xor(E, x, kWave);
                    E = y < E ? y : E;
                }
            }
            bool inval = false;
            if (key_dist(E) < __builtin_inff()) {
                // C: keys beyond 1 m below E; invalid iff C < 30 - K1
                const int need = 30 - s.K1;
                const float lim = key_dist(E);
                int C = 0;
                for (int i0 = 0; i0 < nstrip; i0 += G) {
                    const float lb = (float)(ring_at(i0) - 1) * g.W - 0.001f;
                    if (C >= need || (i0 > 0 && lb > 0.0f && lb * lb > lim)) break;   // uniform per group
                    const int i = i0 + gl, sidx = strip_at(i);
                    int c = 0;
                    if (i < nstrip && sidx >= 0 && sidx < g.ns) {
                        int st = sidx == s0 ? j : -1;
                        strip_visit(v, T, sidx, st, q, __builtin_inff(), [&] { return lim; },
                                    [&](const float4& p) {
                                        const float d = l2_simple(q, p);
                                        c += (d >= 1.0f && pick_key(d, p) < E);
                                    });
                    }
#pragma unroll
                    for (int x = G / 2; x >= 1; x >>= 1) c += __shfl_xor(c, x, kWave);
                    C += c;
                }
                inval = C < need;
            }
            if (gl == 0) {
                if (inval) pick_invalid(o, normal, valid);
                else pick_finish(P, s, f1 ? 1 : 0, plane_max, o, normal, valid);
            }
        }
    }
#else
    const int nw = blockDim.x >> 6, t2 = (threadIdx.x & 63) * nw + (threadIdx.x >> 6);
    for (int k = t2; k < nq; k += blockDim.x) {
        const int j = queue[k];
        const float4 q = v.pt(j);
        const int64_t o = base + v.id(j);
        PickState s;
        pick_1m(P, v, T, g, j, q, s);
        const bool f1 = key_dist(s.d1) < 1.0f;
        const bool inval = pick_beyond_invalid(v, T, g, j, q, s);
        if (inval) pick_invalid(o, normal, valid);
        else pick_finish(P, s, f1 ? 1 : 0, plane_max, o, normal, valid);
    }
#endif
#ifdef SSF_TABLE_STAMPS
    __syncthreads();
    if (threadIdx.x == 0 && stamp_out) stamp_out[4] = (int32_t)((__builtin_amdgcn_s_memtime() - stamp0) >> 4);
#endif
}

// The deferred few (no decision inside 1 m: sparse, far regions) walk the x-sorted copy the
// sort left in global memory (SP / SI, L2-resident), unbounded, from their x rank (binary
// search on (x, index)): a strip ring search there would need a loop nest whose register
// pressure spills the bounded walks that share the kernel.
template <bool kSoa>
SSF_DEV void table_strip_walks(const float4* __restrict__ P, const StripView<kSoa>& v,
                               const StripLds& T, const StripGeo& g, int m, float plane_max,
                               int64_t base, float* __restrict__ normal, uint8_t* __restrict__ valid,
                               int* queue, int qcap, int* qlen, const float4* __restrict__ SP,
                               const int32_t* __restrict__ SI, int32_t* stamp_out,
                               unsigned long long stamp0, int share = 0, int nshare = 1) {
    for (int j = share + nshare * (int)threadIdx.x; j < m; j += nshare * (int)blockDim.x) {
        const float4 q = v.pt(j);
        double kk[kK];
        int dec;
        strip_knn_radius<1>(v, T, g, j, q, kk);
        dec = bounded_decides(P, m, kk);
        if (dec == 0) {
            const int slot = atomicAdd(qlen, 1);
            if (slot < qcap) queue[slot] = j;
            else { table_deferred_walk(P, SP, SI, m, v.id(j), q, kk); dec = 1; }   // queue full
        }
        if (dec == 2) {
            const int64_t o = base + v.id(j);
            normal[3 * o] = 0.f; normal[3 * o + 1] = 0.f; normal[3 * o + 2] = 0.f;
            valid[o] = 0;
        } else if (dec == 1) {
            table_finish(P, m, plane_max, base + v.id(j), kk, normal, valid);
        }
    }
    __syncthreads();
#ifdef SSF_TABLE_STAMPS
    if (threadIdx.x == 0 && stamp_out) { stamp_out[0] = (int32_t)((__builtin_amdgcn_s_memtime() - stamp0) >> 4); stamp_out[1] = *qlen; }
#endif
    const int nq = min(*qlen, qcap);
    // spread the deferred queries over the waves (entry k -> wave k % nw)
    const int nw = blockDim.x >> 6, t2 = (threadIdx.x & 63) * nw + (threadIdx.x >> 6);
    for (int k = t2; k < nq; k += blockDim.x) {
        const int j = queue[k];
        const float4 q = v.pt(j);
        double kk[kK];
        // within 2 m, then within kDeferRings m, from the strips: decided as soon as the exact
        // part of the list settles it (deferred_decides); else the x-sorted global copy, unbounded
        strip_knn_radius<kDeferFirst>(v, T, g, j, q, kk);
        int dec = deferred_decides(P, kk, (float)(kDeferFirst * kDeferFirst));
#if SSF_DEFER_MID
        if (dec == 0) {
            strip_knn_radius<SSF_DEFER_MID>(v, T, g, j, q, kk);
            dec = deferred_decides(P, kk, (float)(SSF_DEFER_MID * SSF_DEFER_MID));
        }
#endif
        if (dec == 0) {
            strip_knn_radius<kDeferRings>(v, T, g, j, q, kk);
            dec = deferred_decides(P, kk, (float)(kDeferRings * kDeferRings));
        }
        if (dec == 0) table_deferred_walk(P, SP, SI, m, v.id(j), q, kk);
        const int64_t o = base + v.id(j);
        if (dec == 2) {
            normal[3 * o] = 0.f; normal[3 * o + 1] = 0.f; normal[3 * o + 2] = 0.f;
            valid[o] = 0;
        } else {
            table_finish(P, m, plane_max, o, kk, normal, valid);
        }
    }
}

// The (x, index) bitonic sort of k_plane_table_sorted with each thread's E elements in registers
// (element t = e kTableThreads + tid): partners 64 <= j < kTableThreads apart go through LDS (one
// barrier per half-stage), j < 64 through wave shuffles, j >= kTableThreads within the thread.
// The same comparator network as the LDS loop (same pairs, directions and comparisons), so the
// same permutation for any input.  Leaves the sorted indices in idx[].
template <int E>
SSF_DEV void table_sort_regs(const float4* __restrict__ P, int m, float* key, int* idx) {
    constexpr int NT = kTableThreads, NP = E * NT;
    const int tid = threadIdx.x;
    float k[E];
    int ix[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int t = e * NT + tid;
        k[e] = t < m ? P[t].x : __builtin_inff();
        ix[e] = t;
    }
    for (int kk = 2; kk <= NP; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j >= NT) {                                          // partner in this thread
                const int je = j / NT;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int e2 = e ^ je;
                    if (e2 > e) {
                        const int t = e * NT + tid;
                        const bool asc = (t & kk) == 0;
                        const bool sw = asc ? lex_less(k[e2], ix[e2], k[e], ix[e]) : lex_less(k[e], ix[e], k[e2], ix[e2]);
                        if (sw) {
                            const float tk = k[e]; k[e] = k[e2]; k[e2] = tk;
                            const int ti = ix[e]; ix[e] = ix[e2]; ix[e2] = ti;
                        }
                    }
                }
            } else if (j >= 64) {                                   // partner in another wave
#pragma unroll
                for (int e = 0; e < E; ++e) { key[e * NT + tid] = k[e]; idx[e * NT + tid] = ix[e]; }
                __syncthreads();
                const bool lower = (tid & j) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int t = e * NT + tid;
                    const float pk = key[t ^ j];
                    const int pi = idx[t ^ j];
                    const bool asc = (t & kk) == 0;
                    const bool take = (lower == asc) ? lex_less(pk, pi, k[e], ix[e]) : lex_less(k[e], ix[e], pk, pi);
                    if (take) { k[e] = pk; ix[e] = pi; }
                }
                __syncthreads();
            } else {                                                // partner in this wave
                const bool lower = (tid & j) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int t = e * NT + tid;
                    const float pk = __shfl_xor(k[e], j, 64);
                    const int pi = __shfl_xor(ix[e], j, 64);
                    const bool asc = (t & kk) == 0;
                    const bool take = (lower == asc) ? lex_less(pk, pi, k[e], ix[e]) : lex_less(k[e], ix[e], pk, pi);
                    if (take) { k[e] = pk; ix[e] = pi; }
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) { key[e * NT + tid] = k[e]; idx[e * NT + tid] = ix[e]; }
    __syncthreads();
}

// The same (x, index) order by a stable LSD radix sort of the x bits (rocPRIM
// block_radix_sort, keys and the index in registers, E per thread in blocked order, so equal
// keys keep index order): x + 0 turns -0 into +0 (lex_less compares them equal), the sign-flip
// encoding orders the floats as unsigned words, and slots past m take the largest key.
// -DSSF_TABLE_BITONIC restores the bitonic network (A/B).
template <int E>
SSF_DEV void table_sort_radix(const float4* __restrict__ P, int m, void* storage, int* idx) {
    using Sort = rocprim::block_radix_sort<unsigned int, kTableThreads, E, int>;
    // the exchange storage lives in the key region; the index stores below follow the sort with
    // no barrier, so the storage must not reach the index region
    static_assert(sizeof(typename Sort::storage_type) <= kSortMax * 4, "radix sort storage exceeds the key region");
    auto& st = *reinterpret_cast<typename Sort::storage_type*>(storage);
    const int tid = threadIdx.x;
    unsigned int k[E];
    int ix[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int t = tid * E + e;
        const unsigned int b = __float_as_uint(t < m ? P[t].x + 0.0f : 0.0f);
        k[e] = t < m ? (b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u)) : 0xFFFFFFFFu;
        ix[e] = t;
    }
    Sort().sort(k, ix, st);
#pragma unroll
    for (int e = 0; e < E; ++e) idx[tid * E + e] = ix[e];
    __syncthreads();
}

__global__ __launch_bounds__(kTableThreads) void k_plane_table_sorted(
    const float4* __restrict__ plane, const int64_t* __restrict__ frame_off,
    const int32_t* __restrict__ count, float plane_max, float* __restrict__ normal,
    uint8_t* __restrict__ valid, float4* __restrict__ sorted_xyzi, int32_t* __restrict__ sorted_idx,
    float4* __restrict__ strip_xyzi, int32_t* __restrict__ strip_head) {
    // 160 KiB of LDS: [0, 64K) keys, [64K, 128K) permutation, [128K, 160K) spare.  After the
    // sort, frames <= kTableStripSoaMax rebuild the whole image as y-strips of the sorted points
    // + the strip table + the deferred queue; larger frames walk the sorted copy in global memory.
    __shared__ __attribute__((aligned(16))) char lds[kSortMax * 8 + 32768];
    float* key = reinterpret_cast<float*>(lds);
    int* idx = reinterpret_cast<int*>(lds + kSortMax * 4);
    const int f = blockIdx.x, tid = threadIdx.x;
    // small batches: gridDim.y work-groups per frame, each sorting and building the strips
    // (identical results) and walking every gridDim.y-th query; share 0 alone
    // writes the strip image and the stamps (every share writes the sorted copy, see below)
    const int share = (int)blockIdx.y, nshare = (int)gridDim.y;
    const int m = count[f];
    const int64_t base = frame_off[f];
    const float4* P = plane + base;
    if (m <= 0) return;
    if (share > 0 && (m > kTableStripSoaMax || m <= share)) return;   // uniform: no queries here
#ifdef SSF_TABLE_STAMPS
    const unsigned long long tstamp0 = __builtin_amdgcn_s_memtime();
#endif
    int np = 1;
    while (np < m) np <<= 1;
#ifndef SSF_TABLE_BITONIC
    // the key region [0, 64 KiB) holds the radix sort's storage (the keys stay in registers)
    if (np <= kTableThreads) table_sort_radix<1>(P, m, lds, idx);
    else if (np == 2 * kTableThreads) table_sort_radix<2>(P, m, lds, idx);
    else if (np == 4 * kTableThreads) table_sort_radix<4>(P, m, lds, idx);
    else if (np == 8 * kTableThreads) table_sort_radix<8>(P, m, lds, idx);
    else
#endif
    if (np == 4 * kTableThreads) table_sort_regs<4>(P, m, key, idx);
    else if (np == 2 * kTableThreads) table_sort_regs<2>(P, m, key, idx);
    else if (np == kTableThreads) table_sort_regs<1>(P, m, key, idx);
    else if (np == 8 * kTableThreads) table_sort_regs<8>(P, m, key, idx);
    else if (np == 16 * kTableThreads) table_sort_regs<16>(P, m, key, idx);
    else {
    for (int r = tid; r < np; r += blockDim.x) {
        key[r] = r < m ? P[r].x : __builtin_inff();
        idx[r] = r;
    }
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < np; t += blockDim.x) {
                const int u = t ^ j;
                if (u > t) {
                    const float ka = key[t], kb = key[u];
                    const int ia = idx[t], ib = idx[u];
                    const bool asc = (t & k) == 0;
                    if (asc ? lex_less(kb, ib, ka, ia) : lex_less(ka, ia, kb, ib)) {
                        key[t] = kb; key[u] = ka; idx[t] = ib; idx[u] = ia;
                    }
                }
            }
            __syncthreads();
        }
    }
    }
    float4* SP = sorted_xyzi + base;
    int32_t* SI = sorted_idx + base;
    // EVERY share writes the sorted copy: table_strip_walks' deferred walk reads it back
    // (table_deferred_walk), and only this work-group's own stores are ordered before those reads
    // by the barrier below -- another share's (possibly on another XCD, whose L2 is not coherent
    // for plain stores) are not.  The shares write identical values, so the duplicates are benign.
    for (int r = tid; r < m; r += blockDim.x) {
        SP[r] = P[idx[r]];
        SI[r] = idx[r];
    }
    __syncthreads();
    SSF_TSTAMP(0);
    int* qlen = reinterpret_cast<int*>(lds + sizeof(lds) - 4);   // last word of the LDS image
    if (tid == 0) *qlen = 0;
    if (m <= kTableStripSoaMax) {
        // the sorted permutation into registers (the strip layout overwrites the sort image),
        // then the strip-major points, the strip table and the deferred queue in the 160 KiB
        const bool soa = m > kTableStripF4Max;                          // uniform
        int own[kStripPerMax];
#pragma unroll
        for (int k = 0; k < kStripPerMax; ++k) {
            const int r = k * kTableThreads + tid;
            own[k] = r < m ? idx[r] : 0;
        }
        __syncthreads();
        float4* F = reinterpret_cast<float4*>(lds);
        float* X = reinterpret_cast<float*>(lds);
        uint16_t* I16 = reinterpret_cast<uint16_t*>(X + 3 * m);
        const int toff = ((soa ? 14 * m : 16 * m) + 15) & ~15;
        StripLds& T = *reinterpret_cast<StripLds*>(lds + toff);
        const int qoff = (toff + (int)sizeof(StripLds) + 15) & ~15;
        int* queue = reinterpret_cast<int*>(lds + qoff);
        const int qcap = ((int)sizeof(lds) - 4 - qoff) / 4;
        auto get = [&](int k, int) {
            float4 p = P[own[k]];
            p.w = __int_as_float(own[k]);
            return p;
        };
#ifdef SSF_TABLE_STAMPS
        int32_t* stamp_out = share == 0 ? SI + m + 1 : nullptr;
        const unsigned long long st0 = tstamp0;
#else
        int32_t* stamp_out = nullptr;
        const unsigned long long st0 = 0;
#endif
#ifdef SSF_TABLE_STAMPS
#define SSF_TSTAMP_BUILD() do { if (tid == 0 && stamp_out) stamp_out[3] = (int32_t)((__builtin_amdgcn_s_memtime() - st0) >> 4); } while (0)
#else
#define SSF_TSTAMP_BUILD() do { } while (0)
#endif
        if (soa) {
            const StripGeo g = strips_build<true, kStripPerMax>(get, m, T, F, X, I16);
            SSF_TSTAMP_BUILD();
            table_strip_walks(P, StripView<true>{F, X, I16, m}, T, g, m, plane_max, base, normal,
                              valid, queue, qcap, qlen, SP, SI, stamp_out, st0, share, nshare);
        } else {
            // 16-B records carry the ring code of every point (bits 16..23 of .w): the pick then
            // runs without the 30-key list (table_pick_walks) unless the frame is tiny or a ring
            // code is out of range (intensities frameFeature never writes)
            bool rows_ok = true;
#pragma unroll
            for (int k = 0; k < kStripPerMax; ++k) {
                const int r = k * kTableThreads + tid;
                if (r < m) rows_ok = rows_ok && row_code(P[own[k]].w) != kRowCodeBad;
            }
            int* rflag = reinterpret_cast<int*>(lds + sizeof(lds) - 8);   // next to qlen, free here
            if (tid == 0) *rflag = 1;
            __syncthreads();
            if (!rows_ok) *rflag = 0;
            __syncthreads();
            rows_ok = *rflag != 0;
            auto getp = [&](int k, int) {
                float4 p = P[own[k]];
                p.w = __int_as_float(own[k] | (int)(row_code(p.w) << 16));
                return p;
            };
            // the pick walks (rows_ok, m > kK) take the narrower strips; table_strip_walks' ring
            // searches (strip_knn_radius) count rings in metres and need W > 1 m
            const StripGeo g = strips_build<false, kStripPerMax>(getp, m, T, F, X, I16,
                                                                 (rows_ok && m > kK) ? kPickStripW : 1.001f);
            SSF_TSTAMP_BUILD();
            // results staged in LDS at their original index and stored coalesced at the end when
            // 13 B per point fit behind the strip image with a queue of m / 4 entries (m <= ~5000):
            // scattered 12-B normal and 1-B validity stores each cost a 64-B write request
            const int soff = ((int)sizeof(lds) - 16 - 13 * m) & ~15;
            // (one work-group per frame only: a share's results are scattered over the frame)
            const bool stage = nshare == 1 && (soff - qoff) / 4 >= m / 4 + 64;   // uniform
            if (rows_ok && m > kK && stage) {
                float* nl = reinterpret_cast<float*>(lds + soff);
                uint8_t* vl = reinterpret_cast<uint8_t*>(lds + soff + 12 * m);
                table_pick_walks(P, StripView<false>{F, X, I16, m}, T, g, m, plane_max, 0, nl, vl,
                                 queue, (soff - qoff) / 4, qlen, stamp_out, st0);
                __syncthreads();
                float* gn = normal + 3 * base;
                uint8_t* gv = valid + base;
                for (int k = tid; k < 3 * m; k += kTableThreads) gn[k] = nl[k];
                for (int k = tid; k < m; k += kTableThreads) gv[k] = vl[k];
            } else if (rows_ok && m > kK)
                table_pick_walks(P, StripView<false>{F, X, I16, m}, T, g, m, plane_max, base, normal, valid,
                                 queue, qcap, qlen, stamp_out, st0, share, nshare);
            else
                table_strip_walks(P, StripView<false>{F, X, I16, m}, T, g, m, plane_max, base, normal,
                                  valid, queue, qcap, qlen, SP, SI, stamp_out, st0, share, nshare);
            // the walks only read F and T: the image leaves as it is (uniform condition)
            if (share == 0 && strip_xyzi && strip_image_frame(m))
                strip_image_store(F, T, g, m, strip_xyzi + base, strip_head + base);
        }
        SSF_TSTAMP(3);
    } else {
        // points from global memory, the permutation in LDS; queue in the (now unused) key region
        int* queue = reinterpret_cast<int*>(lds);
        const PtsF4 v{SP, idx};
        table_walks(P, v, m, plane_max, base, normal, valid, queue, kSortMax, qlen);
    }
}

// Association against an x-sorted last frame: binary search of the query's x, then the same
// outward walk with a 1-element list (ties to the lower original index, as the brute force).
__global__ __launch_bounds__(256) void k_associate_sorted(
    const float4* __restrict__ last, const int64_t* __restrict__ last_off,
    const int32_t* __restrict__ last_count, const float* __restrict__ last_normal,
    const uint8_t* __restrict__ last_valid, const float4* __restrict__ last_sorted,
    const int32_t* __restrict__ last_sidx, const float4* __restrict__ curr,
    const int64_t* __restrict__ curr_off, const int32_t* __restrict__ curr_count,
    const double* __restrict__ pose_rel, CorrRec* __restrict__ corr, int32_t* __restrict__ nn_out) {
    const int p = blockIdx.y;
    const int mc = curr_count[p], ml = last_count[p];
    if ((int)(blockIdx.x * blockDim.x) >= mc || ml <= 10) return;    // uniform (:158)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= mc) return;
    const int64_t lo = last_off[p], co = curr_off[p];
    const float4* SL = last_sorted + lo;
    const int32_t* SI = last_sidx + lo;
    const double q[4] = {pose_rel[7 * p], pose_rel[7 * p + 1], pose_rel[7 * p + 2], pose_rel[7 * p + 3]};
    const double t[3] = {pose_rel[7 * p + 4], pose_rel[7 * p + 5], pose_rel[7 * p + 6]};
    const float4 pc = curr[co + i];
    float4 qs;
    {
        const double v[3] = {(double)pc.x, (double)pc.y, (double)pc.z};
        double r[3];
        quat_rotate(q, v, r);                                          // :74-82
        qs.x = (float)(r[0] + t[0]); qs.y = (float)(r[1] + t[1]); qs.z = (float)(r[2] + t[2]); qs.w = 0.f;
    }
    int lo_i = 0, hi_i = ml;                                            // first x >= qs.x
    while (lo_i < hi_i) {
        const int mid = (lo_i + hi_i) >> 1;
        if (SL[mid].x < qs.x) lo_i = mid + 1; else hi_i = mid;
    }
    float best = __builtin_inff();
    int bi = 0x7fffffff;
    for (int c = lo_i; c < ml; ++c) {
        const float4 pl = SL[c];
        const float dx = qs.x - pl.x;
        if (dx * dx > best) break;
        const float d = l2_simple(qs, pl);
        const int id = SI[c];
        if (lex_less(d, id, best, bi)) { best = d; bi = id; }
    }
    for (int c = lo_i - 1; c >= 0; --c) {
        const float4 pl = SL[c];
        const float dx = qs.x - pl.x;
        if (dx * dx > best) break;
        const float d = l2_simple(qs, pl);
        const int id = SI[c];
        if (lex_less(d, id, best, bi)) { best = d; bi = id; }
    }
    const float4* L = last + lo;
    CorrRec rec;
    const bool ok = last_valid[lo + bi] != 0;
    const float4 pa = L[bi];
    rec.po[0] = pc.x; rec.po[1] = pc.y; rec.po[2] = pc.z; rec.valid = ok ? 1.0f : 0.0f;
    rec.pa[0] = pa.x; rec.pa[1] = pa.y; rec.pa[2] = pa.z; rec.pad0 = 0.f;
    const float* nr = last_normal + 3 * (lo + bi);
    rec.n[0] = nr[0]; rec.n[1] = nr[1]; rec.n[2] = nr[2]; rec.pad1 = 0.f;
    corr[co + i] = rec;
    if (nn_out) nn_out[co + i] = bi;
}

// Same association with the last frame's sorted cloud staged in LDS (x, y, z, original index
// in .w: 16 B per point, dynamic LDS sized by the launch's plane-point bound).  Each
// work-group handles kAssocQ queries of one pair in two phases:
//   1. every query walks outward in x only while dx^2 < R^2 (and dx^2 <= best), R = 1 m.  If
//      the best squared distance found is < R^2 the answer is exact: any closer point has
//      dx^2 < R^2 and was visited.  About 95 % of queries finish here.
//   2. the rest (no point within R: sparse, far regions, where an x-band walk would cover
//      most of the frame) were queued in LDS; after a barrier they are answered 64 at a time by
//      an exhaustive scan split over all waves (disjoint slices, merged in LDS).
// Candidates are compared as (distance, original index), so visit order never changes the result.
constexpr int kAssocThreads = 1024;
constexpr int kAssocQ = 2048;              // queries per work-group (2 per thread)
constexpr int kAssocLdsMax = 6144;         // last-frame plane points staged in LDS (96 KiB)
constexpr int kAssocSoaMax = 12032;        // ... as 12-B SoA points: 141 KiB + queue + reductions
#ifndef SSF_ASSOC_BAND2
#define SSF_ASSOC_BAND2 1.0f
#endif
constexpr float kAssocBand2 = SSF_ASSOC_BAND2;   // phase-1 band: dx^2 < 1 (R = 1 m; 0.5 / 0.7 m measured slower)

SSF_DEV float4 assoc_query_point(const float4& pc, const double q[4], const double t[3]) {
    const double v[3] = {(double)pc.x, (double)pc.y, (double)pc.z};
    double r[3];
    quat_rotate(q, v, r);                                               // :74-82
    float4 qs;
    qs.x = (float)(r[0] + t[0]); qs.y = (float)(r[1] + t[1]); qs.z = (float)(r[2] + t[2]); qs.w = 0.f;
    return qs;
}

// Candidates are kept as a sorted rank bc; the original index (the tie-break key) is read only
// on an exact distance tie, and once at the end.
template <class V>
SSF_DEV bool assoc_better(const V& v, int c, float d, float best, int bc) {
    return d < best || (d == best && (bc < 0 || v.id(c) < v.id(bc)));
}

template <class V>
SSF_DEV void assoc_walk(const V& v, int ml, const float4& qs, float lim, float& best, int& bc,
                        int* visited = nullptr) {
    int lo_i = 0, hi_i = ml;                                            // first x >= qs.x
    while (lo_i < hi_i) {
        const int mid = (lo_i + hi_i) >> 1;
        if (v.pt(mid).x < qs.x) lo_i = mid + 1; else hi_i = mid;
    }
    int c = lo_i;
    for (; c < ml; ++c) {
        const float4 pl = v.pt(c);
        const float dx = qs.x - pl.x;
        const float dx2 = dx * dx;
        if (dx2 > best || dx2 >= lim) break;
        const float d = l2_simple(qs, pl);
        if (assoc_better(v, c, d, best, bc)) { best = d; bc = c; }
    }
    int c2 = lo_i - 1;
    for (; c2 >= 0; --c2) {
        const float4 pl = v.pt(c2);
        const float dx = qs.x - pl.x;
        const float dx2 = dx * dx;
        if (dx2 > best || dx2 >= lim) break;
        const float d = l2_simple(qs, pl);
        if (assoc_better(v, c2, d, best, bc)) { best = d; bc = c2; }
    }
    if (visited) *visited = (c - lo_i) + (lo_i - 1 - c2);
}

SSF_DEV void assoc_finish(const float4* __restrict__ L, int64_t lo, const float* __restrict__ last_normal,
                          const uint8_t* __restrict__ last_valid, const float4& pc, int bi,
                          CorrRec* __restrict__ corr, int32_t* __restrict__ nn_out, int64_t ci) {
    CorrRec rec;
    const bool ok = last_valid[lo + bi] != 0;
    const float4 pa = L[bi];
    rec.po[0] = pc.x; rec.po[1] = pc.y; rec.po[2] = pc.z; rec.valid = ok ? 1.0f : 0.0f;
    rec.pa[0] = pa.x; rec.pa[1] = pa.y; rec.pa[2] = pa.z; rec.pad0 = 0.f;
    const float* nr = last_normal + 3 * (lo + bi);
    rec.n[0] = nr[0]; rec.n[1] = nr[1]; rec.n[2] = nr[2]; rec.pad1 = 0.f;
    corr[ci] = rec;
    if (nn_out) nn_out[ci] = bi;
}

// phases 1 and 2 for one work-group over the sorted last frame v
template <class V>
SSF_DEV void assoc_phases(const V& v, int ml, int mc, int i0, int64_t lo, int64_t co,
                          const double* __restrict__ pose_rel, int p, const float4* __restrict__ curr,
                          const float4* __restrict__ L, const float* __restrict__ last_normal,
                          const uint8_t* __restrict__ last_valid, CorrRec* __restrict__ corr,
                          int32_t* __restrict__ nn_out, int* queue, int* qlen, float* red_d,
                          int* red_i, unsigned long long* stamp1) {
    const double q[4] = {pose_rel[7 * p], pose_rel[7 * p + 1], pose_rel[7 * p + 2], pose_rel[7 * p + 3]};
    const double t[3] = {pose_rel[7 * p + 4], pose_rel[7 * p + 5], pose_rel[7 * p + 6]};
    const int i1 = min(mc, i0 + kAssocQ);
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {           // phase 1: the x band
        const float4 pc = curr[co + i];
        const float4 qs = assoc_query_point(pc, q, t);
        float best = __builtin_inff();
        int bc = -1;
#ifdef SSF_ASSOC_COUNT
        // diagnostic build only: candidates visited by the phase-1 walk into nn_out
        // (negative: the query went on to phase 2)
        int vis = 0;
        assoc_walk(v, ml, qs, kAssocBand2, best, bc, &vis);
#else
        assoc_walk(v, ml, qs, kAssocBand2, best, bc);
#endif
        if (best < kAssocBand2) assoc_finish(L, lo, last_normal, last_valid, pc, v.id(bc), corr, nn_out, co + i);
        else queue[atomicAdd(qlen, 1)] = i;                             // <= kAssocQ entries
#ifdef SSF_ASSOC_COUNT
        if (nn_out) nn_out[co + i] = best < kAssocBand2 ? vis : -1 - vis;
#endif
    }
    __syncthreads();
#ifdef SSF_ASSOC_STAMPS
    *stamp1 = __builtin_amdgcn_s_memtime();
#endif
    // phase 2: the queued queries in groups of 64 (one per lane); for each group all waves scan
    // disjoint slices of the last frame (broadcast LDS reads, 8 in flight, no divergence) and the
    // per-slice (distance, rank) bests are merged in LDS -- ties by original index, so exact
    const int nq = *qlen;
    const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int chunk = (ml + nw - 1) / nw;
    const int c0 = min(ml, w * chunk), c1 = min(ml, c0 + chunk);
    for (int g0 = 0; g0 < nq; g0 += 64) {
        const int k = g0 + lane;
        const bool act = k < nq;
        const int i = queue[act ? k : g0];
        const float4 pc = curr[co + i];
        const float4 qs = assoc_query_point(pc, q, t);
        float best = __builtin_inff();
        int bc = -1;
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            float4 pl[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) pl[u] = v.pt(c + u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float d = l2_simple(qs, pl[u]);
                if (assoc_better(v, c + u, d, best, bc)) { best = d; bc = c + u; }
            }
        }
        for (; c < c1; ++c) {
            const float d = l2_simple(qs, v.pt(c));
            if (assoc_better(v, c, d, best, bc)) { best = d; bc = c; }
        }
        red_d[w * 64 + lane] = best;
        red_i[w * 64 + lane] = bc;
        __syncthreads();
        if (w == 0 && act) {
            for (int u = 1; u < nw; ++u) {
                const float d = red_d[u * 64 + lane];
                const int cu = red_i[u * 64 + lane];
                if (cu >= 0 && assoc_better(v, cu, d, best, bc)) { best = d; bc = cu; }
            }
#ifdef SSF_ASSOC_COUNT
            assoc_finish(L, lo, last_normal, last_valid, pc, v.id(max(bc, 0)), corr, nullptr, co + i);
#else
            assoc_finish(L, lo, last_normal, last_valid, pc, v.id(max(bc, 0)), corr, nn_out, co + i);
#endif
        }
        __syncthreads();
    }
}

// kSoa = false: the last frame staged as 16-B points (index in .w), up to kAssocLdsMax;
// kSoa = true:  as x | y | z float arrays (12 B per point, up to kAssocSoaMax), the original index
//               read from the global permutation on distance ties and for the answer.
template <bool kSoa>
__global__ __launch_bounds__(kAssocThreads) void k_associate_lds(
    const float4* __restrict__ last, const int64_t* __restrict__ last_off,
    const int32_t* __restrict__ last_count, const float* __restrict__ last_normal,
    const uint8_t* __restrict__ last_valid, const float4* __restrict__ last_sorted,
    const int32_t* __restrict__ last_sidx, const float4* __restrict__ curr,
    const int64_t* __restrict__ curr_off, const int32_t* __restrict__ curr_count,
    const double* __restrict__ pose_rel, CorrRec* __restrict__ corr, int32_t* __restrict__ nn_out,
    int lds_cap) {
    extern __shared__ float4 SLl[];                 // [lds_cap] points, then the queue
    float* SX = reinterpret_cast<float*>(SLl);
    int* queue = kSoa ? reinterpret_cast<int*>(SX + 3 * lds_cap) : reinterpret_cast<int*>(SLl + lds_cap);
    __shared__ int qlen;
    __shared__ float red_d[kAssocThreads];          // phase-2 per-slice bests
    __shared__ int red_i[kAssocThreads];
    const int p = blockIdx.y;
    const int mc = curr_count[p], ml = last_count[p];
    const int i0 = blockIdx.x * kAssocQ;
    if (i0 >= mc || ml <= 10) return;                                   // uniform (:158)
    const int64_t lo = last_off[p], co = curr_off[p];
    unsigned long long st1 = 0;
#ifdef SSF_ASSOC_STAMPS
    // diagnostic build only: work-group lifetime (s_memtime) into nn_out[co + i0 .. +3]
    const unsigned long long st0 = __builtin_amdgcn_s_memtime();
#endif
    if (threadIdx.x == 0) qlen = 0;
    const float4* L = last + lo;
    if (ml <= lds_cap) {
        if (kSoa) {
            for (int r = threadIdx.x; r < ml; r += blockDim.x) {
                const float4 v = last_sorted[lo + r];
                SX[r] = v.x; SX[ml + r] = v.y; SX[2 * ml + r] = v.z;
            }
            __syncthreads();
            const PtsSoA v{SX, SX + ml, SX + 2 * ml, nullptr};
            struct View {
                PtsSoA s;
                const int32_t* I;
                SSF_DEV float4 pt(int c) const { return s.pt(c); }
                SSF_DEV int id(int c) const { return I[c]; }
            };
            assoc_phases(View{v, last_sidx + lo}, ml, mc, i0, lo, co, pose_rel, p, curr, L,
                         last_normal, last_valid, corr, nn_out, queue, &qlen, red_d, red_i, &st1);
        } else {
            for (int r = threadIdx.x; r < ml; r += blockDim.x) {
                float4 v = last_sorted[lo + r];
                v.w = __int_as_float(last_sidx[lo + r]);
                SLl[r] = v;
            }
            __syncthreads();
            assoc_phases(PtsF4W{SLl}, ml, mc, i0, lo, co, pose_rel, p, curr, L, last_normal,
                         last_valid, corr, nn_out, queue, &qlen, red_d, red_i, &st1);
        }
    } else {  // a last frame above the caller's plane-point bound (the LDS size): global memory
        __syncthreads();
        assoc_phases(PtsF4{last_sorted + lo, last_sidx + lo}, ml, mc, i0, lo, co, pose_rel, p, curr,
                     L, last_normal, last_valid, corr, nn_out, queue, &qlen, red_d, red_i, &st1);
    }
#ifdef SSF_ASSOC_STAMPS
    __syncthreads();
    if (threadIdx.x == 0 && nn_out) {
        const unsigned long long st2 = __builtin_amdgcn_s_memtime();
        nn_out[co + i0] = qlen;
        nn_out[co + i0 + 1] = (int32_t)((st1 - st0) >> 4);
        nn_out[co + i0 + 2] = (int32_t)((st2 - st0) >> 4);
        nn_out[co + i0 + 3] = qlen;
    }
#else
    (void)st1;
#endif
}

// ------------------------------------------------------------------------------------------
// Association over y-strips.  An x band around a query crosses every LiDAR ring: the 1-m walk
// visits ~60 candidates per query (the ~54 points inside |dx| < the final NN distance are
// unavoidable in x order), and the slowest lane of a wave ~217.  One work-group per pair stages
// the last frame (x-sorted) into LDS partitioned into strips of width W >= 1 m in y, x order
// kept inside each strip (stable partition: per-wave match masks on the strip id + per-wave
// strip counts, chunk by chunk in x order).  A query searches its own strip (binary search in
// x, outward walk while dx^2 + dymin^2 <= best), then the strips above and below, ring by
// ring, while a lower bound of their |dy| can still beat the best: ~8 candidates per query,
// every query exact (no 1-m band, no exhaustive phase).  Lower bounds: inside a searched strip,
// dymin from the strip's actual y extent (fl(qy - yhi) <= fl(qy - py) by monotone rounding, so
// fl(fl(dx^2) + fl(dymin^2)) <= the float distance); for the ring stop, the nominal strip edge
// minus 1 mm (float strip assignment).  Candidates compare as (distance, original index).
// kSoa: the strip-major points as x | y | z float arrays and a u16 original index (configs[4]
// frames); otherwise float4 with the index in .w.  A last frame above the launch's staging
// capacity walks the x-sorted copy in global memory, unbounded (exact, slow, not expected).
#ifndef SSF_ASSOC_COMPACT
#define SSF_ASSOC_COMPACT 1                      // lane-mode association writes compacted records (A/B: 0)
#endif
#ifndef SSF_ASSOC_DEFER
#define SSF_ASSOC_DEFER 0                        // 1: far queries of the lane mode to a wave each (r5u: 256-pair launch 0.135 -> 0.200 ms)
#endif
#ifndef SSF_ASSOC_DEFER_R
#define SSF_ASSOC_DEFER_R 4.0f
#endif
constexpr int kAssocDeferMax = 512;              // deferred queries per work-group (more: the lane goes on)
constexpr float kAssocDeferR = SSF_ASSOC_DEFER_R; // a query still open after this level is deferred
#ifndef SSF_ASSOC_DEFER_G
#define SSF_ASSOC_DEFER_G 64
#endif
constexpr int kAssocDeferG = SSF_ASSOC_DEFER_G;  // lanes per deferred query (a wave at 64)
#ifndef SSF_ASSOC_DEFER_EMPTY
#define SSF_ASSOC_DEFER_EMPTY 0                  // defer only queries with no candidate yet (empty regions)
#endif
// kCoopG > 0 (launches of few pairs: a node's one pair, configs[2]'s chained pairs): one query
// per group of kCoopG lanes instead of one per lane -- the query's strips of each search level
// spread over the group's lanes (one strip per lane), so no lane walks ring after ring alone,
// and (kStripThreads / kCoopG) queries per work-group over ceil(m / that) work-groups per pair
// (each stages the last frame).  The lane mode's nested divergent loops (levels, rings, walks)
// leave a wave at the pace of its slowest lane: SQ counters in the chain, r5w: ~138 LDS
// instructions per wave over ~51 k wave-cycles, 56 % of them waiting.
#ifndef SSF_ASSOC_COOP_G
#define SSF_ASSOC_COOP_G 16
#endif
constexpr int kAssocCoopG = SSF_ASSOC_COOP_G;
constexpr int kAssocCoopPairs = 16;             // launches of at most this many pairs take the group mode
#ifndef SSF_ASSOC_BIG_G
#define SSF_ASSOC_BIG_G 0                        // A/B: group mode with this many lanes for big launches too
#endif
constexpr int kAssocBigG = SSF_ASSOC_BIG_G;
template <bool kSoa, int kCoopG = 0>
__global__ __launch_bounds__(kStripThreads) void k_associate_strips(
    const float4* __restrict__ last, const int64_t* __restrict__ last_off,
    const int32_t* __restrict__ last_count, const float* __restrict__ last_normal,
    const uint8_t* __restrict__ last_valid, const float4* __restrict__ last_sorted,
    const int32_t* __restrict__ last_sidx, const float4* __restrict__ curr,
    const int64_t* __restrict__ curr_off, const int32_t* __restrict__ curr_count,
    const double* __restrict__ pose_rel, CorrRec* __restrict__ corr, int32_t* __restrict__ nn_out,
    int lds_cap, const float4* __restrict__ strip_xyzi, const int32_t* __restrict__ strip_head,
    int32_t* __restrict__ nnv, int32_t* __restrict__ ncompact) {
    extern __shared__ float4 SL[];                  // [ml] strip-major, x-sorted in each strip
    __shared__ StripLds T;
    // Compacted records (round 6): with one work-group per pair in the lane mode, the valid
    // correspondences are written in query order at their ranks, [0, ncompact[p]) of the pair's
    // records (a pair whose records are not compacted gets -1): k_solve then streams them into its
    // LDS with no ballot pass and evaluates them on the way in.  Each query's (1-NN index, valid)
    // goes to nnv first; the ranks need every query's validity.
    const bool compact = kCoopG == 0 && !SSF_ASSOC_DEFER && ncompact && gridDim.y == 1;   // uniform
    __shared__ int cwave[kStripWaves];
#if SSF_ASSOC_DEFER == 2
    // far queries kept by their own wave (no barrier): each wave answers its list in groups of
    // kAssocDeferG lanes after its lane walks (not in the SoA launch: no LDS left there)
    constexpr int kDqW = 32;
    __shared__ int dqw[kSoa ? 1 : kStripWaves][kSoa ? 1 : kDqW];
    __shared__ int dqnw[kSoa ? 1 : kStripWaves];
    if (!kSoa && (threadIdx.x & 63) == 0) dqnw[threadIdx.x >> 6] = 0;
#elif SSF_ASSOC_DEFER
    // far queries, answered a wave each at the end (the SoA launch has ~0.3 KiB of LDS left)
    constexpr int kDq = kSoa ? kAssocDeferMax / 4 : kAssocDeferMax;
    __shared__ int dq[kDq];
    __shared__ int dqn;
    if (threadIdx.x == 0) dqn = 0;                  // (the staging's barriers order it)
#endif
    // gridDim.y work-groups per pair (few pairs in a launch): each stages the whole last frame
    // and answers every gridDim.y-th block of kStripThreads queries
    const int p = blockIdx.x, tid = threadIdx.x;
    const int q0 = tid + (int)blockIdx.y * kStripThreads, qstep = kStripThreads * (int)gridDim.y;
    const int mc = curr_count[p], ml = last_count[p];
    if (mc <= 0 || ml <= 10) {                                          // uniform (:158)
        if (compact && tid == 0) ncompact[p] = 0;
        return;
    }
    constexpr int kQpw = kCoopG > 0 ? kStripThreads / kCoopG : kStripThreads;   // queries per work-group
    if (kCoopG > 0 && (int)blockIdx.y * kQpw >= mc) return;             // uniform: no query here
    const int64_t lo = last_off[p], co = curr_off[p];
    const float4* SP = last_sorted + lo;
    const int32_t* SI = last_sidx + lo;
    const double q[4] = {pose_rel[7 * p], pose_rel[7 * p + 1], pose_rel[7 * p + 2], pose_rel[7 * p + 3]};
    const double t[3] = {pose_rel[7 * p + 4], pose_rel[7 * p + 5], pose_rel[7 * p + 6]};
    const float4* L = last + lo;
#ifdef SSF_STRIPS_STAMPS
    // diagnostic build only: per work-group s_memrealtime (100 MHz) and s_memtime (core clock)
    // at entry, after the staging and after the queries, into nn_out[co + 8 y ..] at the end
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
    unsigned long long rt1 = rt0, mt1 = mt0;
#endif
    if (ml > lds_cap) {                                                 // uniform
        if (compact && tid == 0) ncompact[p] = -1;                      // records in query order
        const PtsF4 g{SP, SI};
        for (int i = q0; i < mc; i += qstep) {
            const float4 pc = curr[co + i];
            const float4 qs = assoc_query_point(pc, q, t);
            float best = __builtin_inff();
            int bc = -1;
            assoc_walk(g, ml, qs, __builtin_inff(), best, bc);
            assoc_finish(L, lo, last_normal, last_valid, pc, g.id(max(bc, 0)), corr, nn_out, co + i);
        }
        return;
    }
    float* SX = reinterpret_cast<float*>(SL);
    uint16_t* SI16 = reinterpret_cast<uint16_t*>(SX + 3 * ml);
    // the plane table's image of this last frame when the caller kept it (a copy: ~4 us of the
    // ~40 us build), otherwise the build
    const StripGeo geo = (!kSoa && strip_xyzi && strip_image_frame(ml) && strip_image_valid(strip_head + lo))
        ? strip_image_load(strip_xyzi + lo, strip_head + lo, ml, SL, T)
        : strips_build<kSoa, kStripPerMax>(
              [&](int, int r) { float4 pt = SP[r]; pt.w = __int_as_float(SI[r]); return pt; }, ml, T, SL, SX, SI16);
    const float y0 = geo.y0, W = geo.W;
    const int ns = geo.ns;
    auto strip_of = [&](float y) { return geo.strip_of(y); };
    const StripView<kSoa> v{SL, SX, SI16, ml};
#ifdef SSF_STRIPS_STAMPS
    rt1 = __builtin_amdgcn_s_memrealtime(); mt1 = __builtin_amdgcn_s_memtime();
#elif !SSF_ASSOC_DEFER
    if (kCoopG == 0 && q0 >= mc && !compact) return;                    // (after the barriers of the build)
#endif
#ifdef SSF_ASSOC_COUNT
    int vis = 0;
#endif
    // one strip: points with dx^2 + dymin^2 <= min(best, lim) (lim = R^2 of the search radius)
    auto search = [&](int sidx, float lim, const float4& qs, float& best, int& bc) __attribute__((always_inline)) {
        const int a = T.start[sidx], b = T.start[sidx + 1];
        if (a >= b) return;
        const float yl = T.ylo[sidx], yh = T.yhi[sidx];
        const float dyl = qs.y < yl ? yl - qs.y : (qs.y > yh ? qs.y - yh : 0.0f);
        const float dy2 = dyl * dyl;
        if (dy2 > fminf(best, lim)) return;
#ifdef SSF_ASSOC_COUNT
        vis += 1 << 16;                                                  // strip searches (high half)
#endif
        int l = a, h = b;                                                // first x >= qs.x
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (v.x(mid) < qs.x) l = mid + 1; else h = mid;
        }
        // the next record is read while the current one is processed (clamped into the strip)
        if (l < b) {
            float4 pn = v.pt(l);
            for (int c = l; c < b; ++c) {
                const float4 pl = pn;
                pn = v.pt(min(c + 1, b - 1));
                const float dx = qs.x - pl.x;
                if (dx * dx + dy2 > fminf(best, lim)) break;
                const float d = l2_simple(qs, pl);
                if (assoc_better(v, c, d, best, bc)) { best = d; bc = c; }
#ifdef SSF_ASSOC_COUNT
                ++vis;
#endif
            }
        }
        if (l > a) {
            float4 pn = v.pt(l - 1);
            for (int c = l - 1; c >= a; --c) {
                const float4 pl = pn;
                pn = v.pt(max(c - 1, a));
                const float dx = qs.x - pl.x;
                if (dx * dx + dy2 > fminf(best, lim)) break;
                const float d = l2_simple(qs, pl);
                if (assoc_better(v, c, d, best, bc)) { best = d; bc = c; }
#ifdef SSF_ASSOC_COUNT
                ++vis;
#endif
            }
        }
    };
    if (kCoopG > 0) {
        // one query per kCoopG-lane group (groups are aligned lane ranges: the reductions stay
        // inside one), the same levels and bounds as the deferred pass below
        const int gl = tid % kCoopG;
        for (int i = (int)blockIdx.y * kQpw + tid / kCoopG; i < mc; i += (int)gridDim.y * kQpw) {   // uniform per group
            const float4 pc = curr[co + i];
            const float4 qs = assoc_query_point(pc, q, t);
            float best = __builtin_inff();
            int bc = -1;
            unsigned long long key = ~0ull;
            for (float R = 2.0f;; R *= 2.0f) {
                const bool unbounded = R > 4096.0f;
                const float lim = unbounded ? __builtin_inff() : R * R;
                const int sa = unbounded ? 0 : strip_of(qs.y - R - W - 1e-3f);
                const int sb = unbounded ? ns - 1 : strip_of(qs.y + R + W + 1e-3f);
                for (int sidx = sa + gl; sidx <= sb; sidx += kCoopG) search(sidx, lim, qs, best, bc);
                unsigned long long k = bc >= 0
                    ? ((unsigned long long)__float_as_uint(best) << 32) | (unsigned)v.id(bc) : ~0ull;
#pragma unroll
                for (int o = kCoopG / 2; o >= 1; o >>= 1) {
                    const unsigned long long x = __shfl_xor(k, o, kWave);
                    k = x < k ? x : k;
                }
                key = k < key ? k : key;
                const float wb = key == ~0ull ? __builtin_inff() : __uint_as_float((unsigned)(key >> 32));
                if (wb <= lim || unbounded) break;
                best = wb; bc = -1;
            }
            if (gl == 0) {
                // no candidate at all (a NaN query, e.g. after a NaN warm start): the lane mode's
                // fallback, sorted rank 0, instead of index -1
                assoc_finish(L, lo, last_normal, last_valid, pc, key == ~0ull ? v.id(0) : (int)(key & 0xffffffffu),
                             corr, nn_out, co + i);
#ifdef SSF_ASSOC_COUNT
                if (nn_out) nn_out[co + i] = vis;
#endif
            }
        }
    }
    for (int i = q0; i < (kCoopG > 0 ? 0 : mc); i += qstep) {
        const float4 pc = curr[co + i];
        const float4 qs = assoc_query_point(pc, q, t);
        float best = __builtin_inff();
        int bc = -1;
#ifdef SSF_ASSOC_COUNT
        vis = 0;
#endif
        // Radius doubling (R = 2, 4, 8, ... m, then unbounded): a level visits, strip ring by
        // strip ring from the query's, every point with dx^2 + dymin^2 <= min(best, R^2).  Once
        // best <= R^2 every point as close as best has been seen (its lower bound is <= its
        // distance <= best <= R^2), so the 1-NN is exact; a query in an empty region (a masked
        // hole, BASELINE configs[2]) therefore walks the points within ~2x its 1-NN distance,
        // not every point within the distance of the first point its own strip happens to hold.
        const int s0 = strip_of(qs.y);
        bool deferred = false;
        for (float R = 2.0f;; R *= 2.0f) {
            const bool unbounded = R > 4096.0f;                          // uniform per lane
            const float lim = unbounded ? __builtin_inff() : R * R;
            search(s0, lim, qs, best, bc);
            bool up = true, dn = true;
            for (int rr = 1; up || dn; ++rr) {
                const float bnd = fminf(best, lim);
                if (up) {
                    const int su = s0 + rr;
                    // every point of strips >= su has y >= y0 + su W (less float slack)
                    const float gap = (y0 + (float)su * W) - qs.y - 1e-3f;
                    if (su >= ns || (gap > 0.0f && gap * gap > bnd)) up = false;
                    else search(su, lim, qs, best, bc);
                }
                if (dn) {
                    const int sd = s0 - rr;
                    const float gap = qs.y - (y0 + (float)(sd + 1) * W) - 1e-3f;
                    if (sd < 0 || (gap > 0.0f && gap * gap > bnd)) dn = false;
                    else search(sd, lim, qs, best, bc);
                }
            }
            if (best <= lim || unbounded) break;
#if SSF_ASSOC_DEFER
            // a far 1-NN: the next levels' ~4 R / W strip searches in a row on one lane set the
            // wave's (and often the launch's) time -- hand the query to the work-group's queue,
            // answered below by a whole wave, one strip per lane
            if (R >= kAssocDeferR && (!SSF_ASSOC_DEFER_EMPTY || !(best < __builtin_inff()))) {
#if SSF_ASSOC_DEFER == 2
                if (!kSoa) {
                    const int wq = tid >> 6;
                    const int slot = atomicAdd(&dqnw[kSoa ? 0 : wq], 1);
                    if (slot < kDqW) { dqw[kSoa ? 0 : wq][kSoa ? 0 : slot] = i; deferred = true; break; }
                }
#else
                const int slot = atomicAdd(&dqn, 1);
                if (slot < kDq) { dq[slot] = i; deferred = true; break; }
#endif
            }
#endif
        }
        if (compact) {
            // the 1-NN's LDS position (its point and index are read back from the strips)
            const int bp = max(bc, 0), bi = v.id(bp);
            nnv[co + i] = last_valid[lo + bi] != 0 ? bp : -1 - bp;      // read back by this thread
            if (nn_out) nn_out[co + i] = bi;
        } else if (!deferred) {
            assoc_finish(L, lo, last_normal, last_valid, pc, v.id(max(bc, 0)), corr, nn_out, co + i);
        }
#ifdef SSF_ASSOC_COUNT
        if (nn_out && !deferred) nn_out[co + i] = vis;
#endif
    }
    if (compact) {
        // query trip k (queries k T + tid, T = kStripThreads: the lane loop's own, so every thread
        // reads back its own nnv entries): ballot + wave counts give the ranks in query order
        const int lane = tid & 63, w = tid >> 6;
        int base = 0;                                                   // uniform
        for (int i0 = 0; i0 < mc; i0 += kStripThreads) {
            const int i = i0 + tid;
            const int e = i < mc ? nnv[co + i] : -1;
            const bool val = e >= 0;
            const uint64_t m = __ballot(val);
            if (lane == 0) cwave[w] = __popcll(m);
            __syncthreads();
            int before = base, tot = 0;
#pragma unroll
            for (int j = 0; j < kStripWaves; ++j) { const int x = cwave[j]; if (j < w) before += x; tot += x; }
            if (val) {
                CorrRec rec;
                const float4 pc = curr[co + i], pa = v.pt(e);                 // pa: L[bi]'s floats
                const float* nr = last_normal + 3 * (lo + v.id(e));
                rec.po[0] = pc.x; rec.po[1] = pc.y; rec.po[2] = pc.z; rec.valid = 1.0f;
                rec.pa[0] = pa.x; rec.pa[1] = pa.y; rec.pa[2] = pa.z; rec.pad0 = 0.f;
                rec.n[0] = nr[0]; rec.n[1] = nr[1]; rec.n[2] = nr[2]; rec.pad1 = 0.f;
                corr[co + before + __popcll(m & lanemask_lt())] = rec;
            }
            base += tot;
            __syncthreads();                                            // cwave is rewritten next trip
        }
        if (tid == 0) ncompact[p] = base;
    }
#if SSF_ASSOC_DEFER
    // Deferred queries, one per wave: each level R searches every strip that can hold a point
    // within R (nominal band [qy - R - W, qy + R + W]), one strip per lane, each lane bounded by
    // min(its best, R^2) and, from the second level on, by the wave's best; then the wave's
    // minimum of (distance, original index).  The same exact 1-NN as the lane walk: at the level
    // where the wave's best is <= R^2, every point at least as close was in a searched strip and
    // within every lane's bound.
#if SSF_ASSOC_DEFER == 2
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");             // this wave's list is complete
    __builtin_amdgcn_wave_barrier();
#ifdef SSF_STRIPS_STAMPS
    const unsigned long long rtl = __builtin_amdgcn_s_memrealtime();
#endif
    if (kCoopG == 0 && !kSoa) {
        constexpr int DG = kAssocDeferG;                                  // lanes per deferred query
        const int wq = tid >> 6, lane = tid % DG;
        const int nq = min(dqnw[kSoa ? 0 : wq], kDqW);
        for (int e = (tid & 63) / DG; e < nq; e += 64 / DG) {
            const int i = dqw[kSoa ? 0 : wq][kSoa ? 0 : e];               // uniform per group
#else
    __syncthreads();
#ifdef SSF_STRIPS_STAMPS
    const unsigned long long rtl = __builtin_amdgcn_s_memrealtime();   // the slowest wave's lane pass
#endif
    if (kCoopG == 0) {
        constexpr int DG = kAssocDeferG;                                  // lanes per deferred query
        const int nq = min(dqn, kDq), lane = tid % DG;
        for (int e = tid / DG; e < nq; e += kStripThreads / DG) {
            const int i = dq[e];                                          // uniform per group
#endif
            const float4 pc = curr[co + i];
            const float4 qs = assoc_query_point(pc, q, t);
            float best = __builtin_inff();
            int bc = -1;
            unsigned long long key = ~0ull;
            for (float R = 2.0f;; R *= 2.0f) {
                const bool unbounded = R > 4096.0f;
                const float lim = unbounded ? __builtin_inff() : R * R;
                const int sa = unbounded ? 0 : strip_of(qs.y - R - W - 1e-3f);
                const int sb = unbounded ? ns - 1 : strip_of(qs.y + R + W + 1e-3f);
                for (int sidx = sa + lane; sidx <= sb; sidx += DG) search(sidx, lim, qs, best, bc);
                unsigned long long k = bc >= 0
                    ? ((unsigned long long)__float_as_uint(best) << 32) | (unsigned)v.id(bc) : ~0ull;
#pragma unroll
                for (int o = DG / 2; o >= 1; o >>= 1) {
                    const unsigned long long x = __shfl_xor(k, o, kWave);
                    k = x < k ? x : k;
                }
                key = k < key ? k : key;
                const float wb = key == ~0ull ? __builtin_inff() : __uint_as_float((unsigned)(key >> 32));
                if (wb <= lim || unbounded) break;
                best = wb; bc = -1;          // the wave's bound (a tie taken later only raises a key)
            }
            if (lane == 0) {
                assoc_finish(L, lo, last_normal, last_valid, pc, key == ~0ull ? v.id(0) : (int)(key & 0xffffffffu),
                             corr, nn_out, co + i);
#ifdef SSF_ASSOC_COUNT
                if (nn_out) nn_out[co + i] = -1;                        // deferred (diagnostic build)
#endif
            }
        }
    }
#endif
#ifdef SSF_STRIPS_STAMPS
    __syncthreads();
    if (tid == 0 && nn_out) {
        const unsigned long long rt2 = __builtin_amdgcn_s_memrealtime(), mt2 = __builtin_amdgcn_s_memtime();
        int32_t* o = nn_out + co + kQpw * blockIdx.y;                // this work-group's own query slots
        o[0] = (int32_t)(rt1 - rt0); o[1] = (int32_t)(rt2 - rt0);
#if SSF_ASSOC_DEFER
#if SSF_ASSOC_DEFER == 1
        o[2] = (int32_t)(rtl - rt0); o[3] = dqn;
#else
        o[2] = (int32_t)(rtl - rt0); o[3] = 0;
#endif
#else
        o[2] = (int32_t)(rt2 - rt0); o[3] = 0;
#endif
        (void)mt1; (void)mt2;
        o[4] = (int32_t)(rt0 & 0x7fffffff); o[5] = __smid();
        o[6] = (int32_t)(strip_xyzi && strip_image_frame(ml) && strip_image_valid(strip_head + lo));
        o[7] = ml;
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Edge features (beyond the reference; oracle/edge_oracle.c states the definitions).
// k_edge_table: one work-group per LAST frame, its edge cloud staged in LDS; per edge point the
// exact 5-NN (packed (distance, index) keys, brute force over the frame's few hundred edges),
// centroid + covariance in double in rank order, cyclic Jacobi, line test.
constexpr int kEdgeK = 5;
constexpr int kEdgeThreads = 1024;
constexpr int kEdgeLdsMax = 8192;          // edges per frame staged in LDS (128 KiB)

SSF_DEV void sym3_eig(double A[9], double V[9]) {       // = orc_sym3_eig, operation for operation
#pragma unroll
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        const double dia = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (!(off > 1e-30 * dia)) break;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int p = k == 2 ? 1 : 0, q = k == 0 ? 1 : 2;
            const double apq = A[3 * p + q];
            if (apq == 0.0) continue;
            const double theta = (A[3 * q + q] - A[3 * p + p]) / (2.0 * apq);
            const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double aip = A[3 * i + p], aiq = A[3 * i + q];
                A[3 * i + p] = c * aip - sn * aiq;
                A[3 * i + q] = sn * aip + c * aiq;
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double api = A[3 * p + i], aqi = A[3 * q + i];
                A[3 * p + i] = c * api - sn * aqi;
                A[3 * q + i] = sn * api + c * aqi;
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double vip = V[3 * i + p], viq = V[3 * i + q];
                V[3 * i + p] = c * vip - sn * viq;
                V[3 * i + q] = sn * vip + c * viq;
            }
        }
    }
}

__global__ __launch_bounds__(kEdgeThreads) void k_edge_table(
    const float4* __restrict__ edges, const int64_t* __restrict__ frame_off,
    const int32_t* __restrict__ count, float max_nn_d2, float line_ratio, float* __restrict__ line,
    uint8_t* __restrict__ valid, int lds_cap) {
    extern __shared__ float4 EL[];
    const int f = blockIdx.x;
    const int m = count[f];
    const int64_t base = frame_off[f];
    const float4* E = edges + base;
    const bool in_lds = m <= lds_cap;                                   // uniform
    if (in_lds)
        for (int r = threadIdx.x; r < m; r += blockDim.x) EL[r] = E[r];
    __syncthreads();
    const float4* P = in_lds ? EL : E;
    for (int a = threadIdx.x; a < m; a += blockDim.x) {
        float* L = line + 6 * (base + a);
        float out[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        uint8_t ok = 0;
        if (m >= kEdgeK) {
            const float4 q = P[a];
            double kk[kEdgeK];
#pragma unroll
            for (int k = 0; k < kEdgeK; ++k) kk[k] = knn_key(__builtin_inff(), 0x7fffffff);
            for (int c = 0; c < m; ++c) {
                // most candidates of a brute-force scan are far: the insertion runs only when
                // some lane's candidate beats its 5th key (keys are exact, so order is kept)
                const double key = knn_key(l2_simple(q, P[c]), c);
                if (key < kk[kEdgeK - 1]) key_insert<kEdgeK>(kk, key);
            }
            double cen[3] = {0.0, 0.0, 0.0};
            float4 nb[kEdgeK];
#pragma unroll
            for (int k = 0; k < kEdgeK; ++k) {
                nb[k] = P[key_index(kk[k])];
                cen[0] += (double)nb[k].x; cen[1] += (double)nb[k].y; cen[2] += (double)nb[k].z;
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) cen[j] = cen[j] / 5.0;
            double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, V[9];
#pragma unroll
            for (int k = 0; k < kEdgeK; ++k) {
                const double v[3] = {(double)nb[k].x - cen[0], (double)nb[k].y - cen[1], (double)nb[k].z - cen[2]};
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c) A[3 * r + c] += v[r] * v[c];
            }
#pragma unroll
            for (int j = 0; j < 9; ++j) A[j] = A[j] / 5.0;
            sym3_eig(A, V);
            const double w[3] = {A[0], A[4], A[8]};
            int i1 = 0;
            if (w[1] > w[i1]) i1 = 1;
            if (w[2] > w[i1]) i1 = 2;
            double l2 = -__builtin_inf();
#pragma unroll
            for (int i = 0; i < 3; ++i) if (i != i1 && w[i] > l2) l2 = w[i];
            double u[3] = {V[i1], V[3 + i1], V[6 + i1]};
            int big = 0;
            if (fabs(u[1]) > fabs(u[big])) big = 1;
            if (fabs(u[2]) > fabs(u[big])) big = 2;
            if (u[big] < 0.0) { u[0] = -u[0]; u[1] = -u[1]; u[2] = -u[2]; }
#pragma unroll
            for (int j = 0; j < 3; ++j) { out[j] = (float)cen[j]; out[3 + j] = (float)u[j]; }
            ok = (key_dist(kk[kEdgeK - 1]) < max_nn_d2) && (w[i1] > (double)line_ratio * l2) ? 1 : 0;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) L[j] = out[j];
        valid[base + a] = ok;
    }
}

// k_edge_associate: one work-group per pair.  Per current edge point, transformToLast (:74-82)
// and the exact 1-NN among the last frame's edges (brute force from LDS, (distance, index)
// order); the correspondence record carries the line (centroid in pa, direction in n) and its
// validity.  (A grid sized by the host's edge bound would launch ~50 mostly empty work-groups
// per pair, each holding the LDS staging size.)
constexpr int kEdgeAssocThreads = 1024;
__global__ __launch_bounds__(kEdgeAssocThreads) void k_edge_associate(
    const float4* __restrict__ last, const int64_t* __restrict__ last_off,
    const int32_t* __restrict__ last_count, const float* __restrict__ line,
    const uint8_t* __restrict__ line_valid, const float4* __restrict__ curr,
    const int64_t* __restrict__ curr_off, const int32_t* __restrict__ curr_count,
    const double* __restrict__ pose_rel, CorrRec* __restrict__ corr, int lds_cap) {
    extern __shared__ float4 LL[];
    const int p = blockIdx.x;
    const int mc = curr_count[p], ml = last_count[p];
    if (mc <= 0) return;                                                // uniform
    const int64_t lo = last_off[p], co = curr_off[p];
    const bool in_lds = ml <= lds_cap;                                  // uniform
    if (in_lds)
        for (int r = threadIdx.x; r < ml; r += blockDim.x) LL[r] = last[lo + r];
    __syncthreads();
    const float4* P = in_lds ? LL : last + lo;
    const double q[4] = {pose_rel[7 * p], pose_rel[7 * p + 1], pose_rel[7 * p + 2], pose_rel[7 * p + 3]};
    const double t[3] = {pose_rel[7 * p + 4], pose_rel[7 * p + 5], pose_rel[7 * p + 6]};
    for (int i = threadIdx.x; i < mc; i += blockDim.x) {
    const float4 pc = curr[co + i];
    const float4 qs = assoc_query_point(pc, q, t);
    float best = __builtin_inff();
    int bi = -1;
    for (int c = 0; c < ml; ++c) {
        const float d = l2_simple(qs, P[c]);
        if (d < best) { best = d; bi = c; }                             // ascending c: ties keep the lower index
    }
    CorrRec rec;
    rec.po[0] = pc.x; rec.po[1] = pc.y; rec.po[2] = pc.z;
    rec.valid = (bi >= 0 && line_valid[lo + bi]) ? 1.0f : 0.0f;
    const float* L = line + 6 * (lo + (bi >= 0 ? bi : 0));
    rec.pa[0] = L[0]; rec.pa[1] = L[1]; rec.pa[2] = L[2]; rec.pad0 = 0.f;
    rec.n[0] = L[3]; rec.n[1] = L[4]; rec.n[2] = L[5]; rec.pad1 = 0.f;
    corr[co + i] = rec;
    }
}

// ------------------------------------------------------------------------------------------
// one wave per SIMD: the per-pair solve is latency-bound (a block reduction and a 6x6 solve per
// iteration), and 256 threads measured 0.083 ms per 256-pair launch against 0.092 at 512 and
// 0.28 at 1024 (round 2c, tools/gpu/r2c_solve3.sh).  For a launch of ONE pair (BASELINE
// configs[1] as written) 512 threads were slower too: 0.083 against 0.073 ms (round 3,
// tools/gpu/r3g.sh; 1024 threads cap the solve at 128 VGPRs and spill).
#ifndef SSF_SOLVE_THREADS
#define SSF_SOLVE_THREADS 256
#endif
constexpr int kSolveThreads = SSF_SOLVE_THREADS;
#ifndef SSF_SOLVE_SPECIALISE
#define SSF_SOLVE_SPECIALISE 1                   // one k_solve instantiation per solver mode (A/B: 0)
#endif
constexpr int kNE = 28;  // 21 (packed upper JtWJ) + 6 (JtWr) + cost

SSF_DEV int pk(int u, int v) {
    if (u > v) { int t = u; u = v; v = t; }
    return u * 6 - (u * (u - 1)) / 2 + (v - u);
}

// All threads: evaluate Huber(0.1)-corrected normal equations at (q, t) over the pair's
// records; result (x2 for the reference's duplicated residual blocks) in ne[] of every thread.
// Valid correspondences of a pair compacted (original order) into LDS once per solve, SoA floats:
// every evaluation of the LM/GN loop then reads LDS instead of re-streaming the 48-byte records.
constexpr int kSolveLdsCap = 4096;
#ifndef SSF_SOLVE_COMPACT1
#define SSF_SOLVE_COMPACT1 1                     // one-pass compaction of the correspondences (A/B: 0)
#endif
#ifndef SSF_SOLVE_CMP_PER
#define SSF_SOLVE_CMP_PER 8
#endif
constexpr int kCmpPer = SSF_SOLVE_CMP_PER;        // records per thread and pass of it
struct CorrLds {
    float po[3][kSolveLdsCap], pa[3][kSolveLdsCap], n[3][kSolveLdsCap];
};

// Eigen Quaterniond::toRotationMatrix (x, y, z, w storage).
SSF_DEV void quat_to_R(const double q[4], double R[9]) {
    const double tx = 2.0 * q[0], ty = 2.0 * q[1], tz = 2.0 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

#ifndef SSF_SOLVE_RSQ
#define SSF_SOLVE_RSQ 1                          // Cholesky pivots by refined v_rsq_f64 (A/B: 0 = sqrt + divide)
#endif
// 1 / sqrt(s) (s > 0, normal): v_rsq_f64 and two Newton steps, r <- r + r (1 - s r^2) / 2; the
// pivot is d = s r (sqrt(s)) and its reciprocal r -- one short chain instead of the f64 sqrt and
// divide expansions on the solve's critical path (every thread runs it)
SSF_DEV double rsq_refined(double s) {
    double r = __builtin_amdgcn_rsq(s);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = __builtin_fma(-s * r, r, 1.0);
        r = __builtin_fma(0.5 * r, e, r);
    }
    return r;
}

// 1 / x (x > 0, normal): v_rcp_f64 and two Newton steps, r <- r + r (1 - x r) -- the Huber
// weight a / |r| of an outlier residual without the f64 divide expansion (within an ulp of it)
SSF_DEV double rcp_refined(double x) {
    double r = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int it = 0; it < 2; ++it) r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
    return r;
}
#ifndef SSF_SOLVE_HUBER_RCP
#define SSF_SOLVE_HUBER_RCP 0                    // 1: Huber weights by refined rcp / rsq (r5l: 0.0857 vs 0.0808 ms, slower)
#endif

// The rotational Jacobian columns carry a factor 2 (the quaternion parameterisation below).
// With SSF_SOLVE_JSCALE it is applied to the block sums instead of every correspondence: every
// product and partial sum of those entries is then exactly 2 or 4 times the unscaled one (a
// power-of-two scaling commutes with rounding), so the sums are bit-identical and each
// correspondence saves three f64 multiplies.  kNeScale folds it into the evaluation's final x2
// (the duplicated residual blocks): packed J^T W J entries (u, v) x4 (u, v < 3) / x2 (u < 3 <= v)
// / x1, J^T W r entries x2 (u < 3), the cost x1 -- each times that 2.
#ifndef SSF_SOLVE_JSCALE
#define SSF_SOLVE_JSCALE 1
#endif
#if SSF_SOLVE_JSCALE
constexpr double kJ2 = 1.0;
__device__ constexpr double kNeScale[kNE] = {8, 8, 8, 4, 4, 4, 8, 8, 4, 4, 4, 8, 4, 4, 4, 2, 2, 2, 2, 2, 2,
                                             4, 4, 4, 2, 2, 2, 2};
#else
constexpr double kJ2 = 2.0;
__device__ constexpr double kNeScale[kNE] = {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
                                             2, 2, 2, 2, 2, 2, 2};
#endif
#ifndef SSF_SOLVE_HF32
#define SSF_SOLVE_HF32 0
#endif
// SSF_SOLVE_HF32: J^T W J (the 21 packed entries) accumulated per thread in packed f32 FMAs
// (v_pk_fma_f32, two entries per instruction at the f32 rate) and added to the f64 sums before
// the block reduction; the gradient J^T W r and the cost stay f64.  A GN / LM fixed point is set
// by the f64 gradient; the f32 Hessian (~1e-7 relative per thread sum) moves the steps, not the
// converged pose.  A/B switch.
typedef float hf2 __attribute__((ext_vector_type(2)));
constexpr int kHF = 11;                          // 21 entries in pk order, as pairs (+1 pad)
SSF_DEV constexpr int pk_u(int e) { return e < 6 ? 0 : e < 11 ? 1 : e < 15 ? 2 : e < 18 ? 3 : e < 20 ? 4 : 5; }
SSF_DEV constexpr int pk_v(int e) {
    return e < 6 ? e : e < 11 ? e - 6 + 1 : e < 15 ? e - 11 + 2 : e < 18 ? e - 15 + 3 : e < 20 ? e - 18 + 4 : 5;
}
SSF_DEV void hess_f32(const float (&wj)[6], const float (&J)[6], hf2 (&H)[kHF]) {
#pragma unroll
    for (int p = 0; p < kHF; ++p) {
        const int e0 = 2 * p, e1 = 2 * p + 1 < 21 ? 2 * p + 1 : 20;
        const hf2 a = {wj[pk_u(e0)], 2 * p + 1 < 21 ? wj[pk_u(e1)] : 0.0f};
        const hf2 b = {J[pk_v(e0)], J[pk_v(e1)]};
        H[p] = __builtin_elementwise_fma(a, b, H[p]);
    }
}

// Per-correspondence residual r = (R po + t - pa) . n (PlaneFeatureCost, :25-43) and its local
// Jacobian [2 (R po x n), n]: the EigenQuaternionParameterization's 4x3 Jacobian composed with
// the autodiff gradient (what the oracle's residual_jac spells out) reduces to that for a unit
// quaternion, so an evaluation costs ~65 f64 operations per correspondence instead of ~140 (same
// values to rounding, explicit FMAs; the per-step poses keep the 1e-5 m / 1e-6 rad bar against
// the oracle).  R is built once per evaluation (wave-uniform).  Huber(0.1) corrector as Ceres:
// rho'(s) = 0.1 / sqrt(s) above s = 0.01 (sqrt(r^2) taken as |r|), rho(s) = 0.2 sqrt(s) - 0.01.
// One correspondence's Huber-weighted contribution (x wgt: 0 for a padding slot) to the
// normal equations ne (21 packed upper J^T W J, 6 J^T W r, cost).
SSF_DEV void accum_corr(const double R[9], const double t[3], const double po[3], const double pa[3],
                        const double nn[3], double wgt, double (&ne)[kNE], hf2 (&H)[kHF]) {
    const double a = 0.1, b = 0.1 * 0.1;
    double u[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) u[k] = __builtin_fma(R[3 * k + 2], po[2], __builtin_fma(R[3 * k + 1], po[1], R[3 * k] * po[0]));
    const double d0 = (u[0] + t[0]) - pa[0], d1 = (u[1] + t[1]) - pa[1], d2 = (u[2] + t[2]) - pa[2];
    const double r = __builtin_fma(d2, nn[2], __builtin_fma(d1, nn[1], d0 * nn[0]));
    double J[6];
    J[0] = kJ2 * __builtin_fma(u[1], nn[2], -u[2] * nn[1]);
    J[1] = kJ2 * __builtin_fma(u[2], nn[0], -u[0] * nn[2]);
    J[2] = kJ2 * __builtin_fma(u[0], nn[1], -u[1] * nn[0]);
    J[3] = nn[0]; J[4] = nn[1]; J[5] = nn[2];
    const double s = r * r;
    double rho0, rho1;
    if (s > b) {
        const double rr = fabs(r);
        rho0 = 2.0 * a * rr - b;
#if SSF_SOLVE_HUBER_RCP
        rho1 = rr < 1e290 ? a * rcp_refined(rr) : a / rr;
#else
        rho1 = a / rr;
#endif
        if (rho1 < DBL_MIN) rho1 = DBL_MIN;
    } else {
        rho0 = s; rho1 = 1.0;
    }
    ne[27] = __builtin_fma(0.5 * wgt, rho0, ne[27]);
    rho1 *= wgt;
#if SSF_SOLVE_HF32
    {
        float jf[6], wf[6];
        const float rf = (float)rho1;
#pragma unroll
        for (int uu = 0; uu < 6; ++uu) { jf[uu] = (float)J[uu]; wf[uu] = rf * jf[uu]; }
        hess_f32(wf, jf, H);
#pragma unroll
        for (int uu = 0; uu < 6; ++uu) ne[21 + uu] = __builtin_fma(rho1 * J[uu], r, ne[21 + uu]);
        return;
    }
#else
    (void)H;
#endif
    int k = 0;
#pragma unroll
    for (int uu = 0; uu < 6; ++uu) {             // explicit FMAs: the file is built without
        const double wj = rho1 * J[uu];          // contraction (bit-exact float stages)
        ne[21 + uu] = __builtin_fma(wj, r, ne[21 + uu]);
#pragma unroll
        for (int v = uu; v < 6; ++v) { ne[k] = __builtin_fma(wj, J[v], ne[k]); ++k; }
    }
}

// Point-to-line block (beyond the reference): e = P (R po + t - c), P = I - u u^T; row k is the
// plane residual with "normal" P row k, so its local Jacobian is [2 (R po x P_k), P_k]; one
// Huber(0.1) block on s = |e|^2 (rho'(s) = 0.1 / sqrt(s) above s = 0.01).
SSF_DEV void accum_edge(const double R[9], const double t[3], const double po[3], const double c[3],
                        const double uu[3], double wgt, double (&ne)[kNE]) {
    const double a = 0.1, b = 0.1 * 0.1;
    double g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) g[k] = __builtin_fma(R[3 * k + 2], po[2], __builtin_fma(R[3 * k + 1], po[1], R[3 * k] * po[0]));
    const double d[3] = {(g[0] + t[0]) - c[0], (g[1] + t[1]) - c[1], (g[2] + t[2]) - c[2]};
    double r[3], J[3][6], s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double nk[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) nk[j] = (j == k ? 1.0 : 0.0) - uu[k] * uu[j];
        r[k] = __builtin_fma(d[2], nk[2], __builtin_fma(d[1], nk[1], d[0] * nk[0]));
        J[k][0] = kJ2 * __builtin_fma(g[1], nk[2], -g[2] * nk[1]);
        J[k][1] = kJ2 * __builtin_fma(g[2], nk[0], -g[0] * nk[2]);
        J[k][2] = kJ2 * __builtin_fma(g[0], nk[1], -g[1] * nk[0]);
        J[k][3] = nk[0]; J[k][4] = nk[1]; J[k][5] = nk[2];
        s = __builtin_fma(r[k], r[k], s);
    }
    double rho0, rho1;
    if (s > b) {
#if SSF_SOLVE_HUBER_RCP
        const double ri = s < 1e290 ? rsq_refined(s) : 1.0 / sqrt(s);
        const double rr = s < 1e290 ? s * ri : sqrt(s);
        rho0 = 2.0 * a * rr - b;
        rho1 = a * ri;
#else
        const double rr = sqrt(s);
        rho0 = 2.0 * a * rr - b;
        rho1 = a / rr;
#endif
        if (rho1 < DBL_MIN) rho1 = DBL_MIN;
    } else {
        rho0 = s; rho1 = 1.0;
    }
    ne[27] = __builtin_fma(0.5 * wgt, rho0, ne[27]);
    rho1 *= wgt;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int m = 0;
#pragma unroll
        for (int uu2 = 0; uu2 < 6; ++uu2) {
            const double wj = rho1 * J[k][uu2];
            ne[21 + uu2] = __builtin_fma(wj, r[k], ne[21 + uu2]);
#pragma unroll
            for (int v = uu2; v < 6; ++v) { ne[m] = __builtin_fma(wj, J[k][v], ne[m]); ++m; }
        }
    }
}

SSF_DEV void evaluate(const CorrRec* __restrict__ rec, int n, const double q[4], const double t[3],
                      double (&ne)[kNE], double* lds, const CorrRec* __restrict__ erec = nullptr,
                      int en = 0) {
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] = 0.0;
    double R[9];
    quat_to_R(q, R);
    hf2 H[kHF];
#pragma unroll
    for (int k = 0; k < kHF; ++k) H[k] = hf2{0.0f, 0.0f};
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const CorrRec c = rec[i];
        if (c.valid == 0.0f) continue;
        const double po[3] = {c.po[0], c.po[1], c.po[2]}, pa[3] = {c.pa[0], c.pa[1], c.pa[2]},
                     nn[3] = {c.n[0], c.n[1], c.n[2]};
        accum_corr(R, t, po, pa, nn, 1.0, ne, H);
    }
#if SSF_SOLVE_HF32
#pragma unroll
    for (int e = 0; e < 21; ++e) ne[e] += (double)H[e >> 1][e & 1];
#endif
    for (int i = threadIdx.x; i < en; i += blockDim.x) {          // edge blocks (en = 0: none)
        const CorrRec c = erec[i];
        if (c.valid == 0.0f) continue;
        const double po[3] = {c.po[0], c.po[1], c.po[2]}, pa[3] = {c.pa[0], c.pa[1], c.pa[2]},
                     uu[3] = {c.n[0], c.n[1], c.n[2]};
        accum_edge(R, t, po, pa, uu, 1.0, ne);
    }
    block_sum_rs<kNE>(ne, lds);
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] *= kNeScale[k];
}

// LDS-resident correspondences, kSolveStep per step (i, i + T, ...; a missing one is a clamped
// duplicate weighted 0): all of a step's loads are in flight before the first is used.
#ifndef SSF_SOLVE_STEP
#define SSF_SOLVE_STEP 2
#endif
constexpr int kSolveStep = SSF_SOLVE_STEP;
#ifndef SSF_SOLVE_QDIRECT
#define SSF_SOLVE_QDIRECT 0                      // A/B: every thread reads the warm start from global memory
#endif
#ifndef SSF_SOLVE_DIRECT
#define SSF_SOLVE_DIRECT 1                       // compacted records: 1 loaded by the first evaluation, 2 copied first (A/B)
#endif
#ifndef SSF_SOLVE_LOADALL
#define SSF_SOLVE_LOADALL 0                      // A/B: first evaluation requests every record of a thread at
                                                 // once (r6zh: 23.2 k vs 15.5 k cycles, 0.070 vs 0.066 ms, slower)
#endif
#ifndef SSF_SOLVE_LDS_PF
#define SSF_SOLVE_LDS_PF 0                       // 1: LDS records of the next step in flight (r6m: 0.0706 vs 0.0674 ms, slower)
#endif
#ifndef SSF_SOLVE_RED
#define SSF_SOLVE_RED 2                          // 0 block_sum_rs; block_sum_db: 1 DPP one barrier, 2 DPP two, 3 shuffles two
#endif
template <int NW>
SSF_DEV void evaluate(const CorrLds& C, int nv, const double q[4], const double t[3],
                      double (&ne)[kNE], double* lds, int nve = 0, int parity = 0) {
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] = 0.0;
    double R[9];
    quat_to_R(q, R);
    const int T = blockDim.x;
    hf2 H[kHF];
#pragma unroll
    for (int k = 0; k < kHF; ++k) H[k] = hf2{0.0f, 0.0f};
#if SSF_SOLVE_LDS_PF
    // the next step's LDS records are read while this step's are evaluated (one wave per SIMD:
    // nothing else hides the LDS latency); clamped reads, a step past nv is never used
    float g[kSolveStep][9];
    if (threadIdx.x < nv) {
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            const int ih = min((int)threadIdx.x + h * T, nv - 1);
#pragma unroll
            for (int d = 0; d < 3; ++d) { g[h][d] = C.po[d][ih]; g[h][3 + d] = C.pa[d][ih]; g[h][6 + d] = C.n[d][ih]; }
        }
    }
#endif
    for (int i = threadIdx.x; i < nv; i += kSolveStep * T) {
        float f[kSolveStep][9];
#if SSF_SOLVE_LDS_PF
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            const int ih = min(i + kSolveStep * T + h * T, nv - 1);
#pragma unroll
            for (int d = 0; d < 9; ++d) f[h][d] = g[h][d];
#pragma unroll
            for (int d = 0; d < 3; ++d) { g[h][d] = C.po[d][ih]; g[h][3 + d] = C.pa[d][ih]; g[h][6 + d] = C.n[d][ih]; }
        }
#else
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            const int ih = min(i + h * T, nv - 1);
#pragma unroll
            for (int d = 0; d < 3; ++d) { f[h][d] = C.po[d][ih]; f[h][3 + d] = C.pa[d][ih]; f[h][6 + d] = C.n[d][ih]; }
        }
#endif
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            const double po[3] = {f[h][0], f[h][1], f[h][2]}, pa[3] = {f[h][3], f[h][4], f[h][5]},
                         nn[3] = {f[h][6], f[h][7], f[h][8]};
            accum_corr(R, t, po, pa, nn, (h == 0 || i + h * T < nv) ? 1.0 : 0.0, ne, H);
        }
    }
#if SSF_SOLVE_HF32
#pragma unroll
    for (int e = 0; e < 21; ++e) ne[e] += (double)H[e >> 1][e & 1];
#endif
    for (int i = nv + threadIdx.x; i < nv + nve; i += T) {        // edge blocks after the planes
        const double po[3] = {C.po[0][i], C.po[1][i], C.po[2][i]}, pa[3] = {C.pa[0][i], C.pa[1][i], C.pa[2][i]},
                     uu[3] = {C.n[0][i], C.n[1][i], C.n[2][i]};
        accum_edge(R, t, po, pa, uu, 1.0, ne);
    }
#if SSF_SOLVE_RED == 0
    (void)parity;
    block_sum_rs<kNE>(ne, lds);
#else
    block_sum_db<kNE, NW, SSF_SOLVE_RED != 3, SSF_SOLVE_RED == 1>(ne, lds, parity);
#endif
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] *= kNeScale[k];
}

// The first evaluation over records the association compacted ([0, nv) of rec, rank order, all
// valid, nv <= kSolveLdsCap): evaluate<NW>()'s loop -- the same records per thread in the same
// order and the same sums -- with each record read from global memory and stored to the LDS
// arrays the later evaluations read (positions i + h T of thread t are read back by thread t
// only: no barrier).  The loads of a step are in flight together; the first evaluation's
// arithmetic overlaps the stream that the ballot compaction used to wait for alone.
template <int NW>
SSF_DEV void evaluate_load(const CorrRec* __restrict__ rec, CorrLds& C, int nv, const double q[4],
                           const double t[3], double (&ne)[kNE], double* lds, int parity) {
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] = 0.0;
    double R[9];
    quat_to_R(q, R);
    const int T = blockDim.x;
    hf2 H[kHF];
#pragma unroll
    for (int k = 0; k < kHF; ++k) H[k] = hf2{0.0f, 0.0f};
#if SSF_SOLVE_LOADALL
    // every record of this thread (<= kSolveLdsCap / T of them) requested at once into registers
    // (one wave per SIMD: 512 VGPRs per lane to spend, and nothing else hides a load's latency),
    // then the same steps in the same order as below; clamped, unconditional loads
    constexpr int kR = kSolveLdsCap / (NW * 64);
    static_assert(kR % kSolveStep == 0, "whole steps");
    float4 a0[kR], a1[kR], a2[kR];
#pragma unroll
    for (int k = 0; k < kR; ++k) {
        const float4* rp = reinterpret_cast<const float4*>(rec + min((int)threadIdx.x + k * T, nv - 1));
        a0[k] = rp[0]; a1[k] = rp[1]; a2[k] = rp[2];
    }
#pragma unroll
    for (int s0 = 0; s0 < kR; s0 += kSolveStep) {
        const int i = (int)threadIdx.x + s0 * T;
        if (i < nv) {
#pragma unroll
            for (int h = 0; h < kSolveStep; ++h) {
                const int ih = i + h * T;
                const int k = s0 + h;
                if (ih < nv) {
                    C.po[0][ih] = a0[k].x; C.po[1][ih] = a0[k].y; C.po[2][ih] = a0[k].z;
                    C.pa[0][ih] = a1[k].x; C.pa[1][ih] = a1[k].y; C.pa[2][ih] = a1[k].z;
                    C.n[0][ih] = a2[k].x; C.n[1][ih] = a2[k].y; C.n[2][ih] = a2[k].z;
                }
                const double po[3] = {a0[k].x, a0[k].y, a0[k].z}, pa[3] = {a1[k].x, a1[k].y, a1[k].z},
                             nn[3] = {a2[k].x, a2[k].y, a2[k].z};
                accum_corr(R, t, po, pa, nn, (h == 0 || ih < nv) ? 1.0 : 0.0, ne, H);
            }
        }
    }
#else
    // one step's records in flight ahead of the step being evaluated (clamped, unconditional
    // loads: a step past nv re-reads record nv - 1 and is never used)
    float4 n0[kSolveStep], n1[kSolveStep], n2[kSolveStep];
#pragma unroll
    for (int h = 0; h < kSolveStep; ++h) {
        const float4* rp = reinterpret_cast<const float4*>(rec + min((int)threadIdx.x + h * T, nv - 1));
        n0[h] = rp[0]; n1[h] = rp[1]; n2[h] = rp[2];
    }
    for (int i = threadIdx.x; i < nv; i += kSolveStep * T) {
        float4 r0[kSolveStep], r1[kSolveStep], r2[kSolveStep];
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            r0[h] = n0[h]; r1[h] = n1[h]; r2[h] = n2[h];
            const float4* rp = reinterpret_cast<const float4*>(rec + min(i + kSolveStep * T + h * T, nv - 1));
            n0[h] = rp[0]; n1[h] = rp[1]; n2[h] = rp[2];
        }
#pragma unroll
        for (int h = 0; h < kSolveStep; ++h) {
            const int ih = i + h * T;
            if (ih < nv) {
                C.po[0][ih] = r0[h].x; C.po[1][ih] = r0[h].y; C.po[2][ih] = r0[h].z;
                C.pa[0][ih] = r1[h].x; C.pa[1][ih] = r1[h].y; C.pa[2][ih] = r1[h].z;
                C.n[0][ih] = r2[h].x; C.n[1][ih] = r2[h].y; C.n[2][ih] = r2[h].z;
            }
            const double po[3] = {r0[h].x, r0[h].y, r0[h].z}, pa[3] = {r1[h].x, r1[h].y, r1[h].z},
                         nn[3] = {r2[h].x, r2[h].y, r2[h].z};
            accum_corr(R, t, po, pa, nn, (h == 0 || ih < nv) ? 1.0 : 0.0, ne, H);
        }
    }
#endif
#if SSF_SOLVE_HF32
#pragma unroll
    for (int e = 0; e < 21; ++e) ne[e] += (double)H[e >> 1][e & 1];
#endif
#if SSF_SOLVE_RED == 0
    (void)parity;
    block_sum_rs<kNE>(ne, lds);
#else
    block_sum_db<kNE, NW, SSF_SOLVE_RED != 3, SSF_SOLVE_RED == 1>(ne, lds, parity);
#endif
#pragma unroll
    for (int k = 0; k < kNE; ++k) ne[k] *= kNeScale[k];
}

// quat_plus for a GN step: |d| = theta < 2^-7 (a step of a converging solve) takes sin(theta) /
// theta and cos(theta) as their Taylor polynomials in theta^2 = |d|^2 -- no sqrt, division, sin or
// cos on the per-iteration critical path every thread runs.  The first omitted terms are below
// 2^-95 (sinc, x2^5 / 11!) and 2^-112 (cos, x2^6 / 12!) of the results, far under one f64 ulp
// (2^-53): the values agree with libm's to an ulp or so, as libm agrees with the oracle's glibc.
// Larger steps take quat_plus itself.  -DSSF_QUAT_PLUS_LIBM restores libm everywhere (A/B).
SSF_DEV void quat_plus_step(const double q[4], const double d[3], double o[4]) {
#ifndef SSF_QUAT_PLUS_LIBM
    const double x2 = __builtin_fma(d[2], d[2], __builtin_fma(d[1], d[1], d[0] * d[0]));
    if (x2 > 0.0 && x2 < 0x1p-14) {
        // Horner in x2: sinc = sum (-x2)^k / (2k + 1)!, k <= 4; cos = sum (-x2)^k / (2k)!, k <= 5
        double sc = 1.0 / 362880.0;
        sc = __builtin_fma(sc, x2, -1.0 / 5040.0);
        sc = __builtin_fma(sc, x2, 1.0 / 120.0);
        sc = __builtin_fma(sc, x2, -1.0 / 6.0);
        sc = __builtin_fma(sc, x2, 1.0);
        double c = -1.0 / 3628800.0;
        c = __builtin_fma(c, x2, 1.0 / 40320.0);
        c = __builtin_fma(c, x2, -1.0 / 720.0);
        c = __builtin_fma(c, x2, 1.0 / 24.0);
        c = __builtin_fma(c, x2, -0.5);
        c = __builtin_fma(c, x2, 1.0);
        const double dq[4] = {sc * d[0], sc * d[1], sc * d[2], c};
        quat_mul(dq, q, o);
        return;
    }
#endif
    quat_plus(q, d, o);
}

SSF_DEV int chol_solve6(double M[6][6], const double b[6], double y[6]) {
    double L[6][6];
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) L[i][j] = 0.0;
    for (int j = 0; j < 6; ++j) {
        double s = M[j][j];
        for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
        if (!(s > 0.0)) return -1;
        L[j][j] = sqrt(s);
        for (int i = j + 1; i < 6; ++i) {
            double v = M[i][j];
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            L[i][j] = v / L[j][j];
        }
    }
    double z[6];
    for (int i = 0; i < 6; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= L[i][k] * z[k];
        z[i] = v / L[i][i];
    }
    for (int i = 5; i >= 0; --i) {
        double v = z[i];
        for (int k = i + 1; k < 6; ++k) v -= L[k][i] * y[k];
        y[i] = v / L[i][i];
    }
    return 0;
}

// Cholesky solve of the packed symmetric normal equations A y = -g (A = ne[0..20] upper packed,
// g = ne[21..26]): 21 + 21 doubles of state, one reciprocal per diagonal instead of a division
// per element (the GN path runs it redundantly on every thread).
#ifndef SSF_SOLVE_CHOL_FMA
#define SSF_SOLVE_CHOL_FMA 1                     // the 6x6 solve's multiply-subtracts as FMAs (A/B: 0)
#endif
// a - b c, as one fused operation (a shorter dependent chain; the step moves by rounding only)
SSF_DEV double msub(double a, double b, double c) {
#if SSF_SOLVE_CHOL_FMA
    return __builtin_fma(-b, c, a);
#else
    return a - b * c;
#endif
}
SSF_DEV int chol_solve_packed(const double (&ne)[kNE], double y[6]) {
    double L[21];                         // L(i, j), j <= i, at pk(j, i)
    double inv[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double s = ne[pk(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) s = msub(s, L[pk(k, j)], L[pk(k, j)]);
        if (!(s > 0.0)) return -1;
#if SSF_SOLVE_RSQ
        const double r = (s > 1e-290 && s < 1e290) ? rsq_refined(s) : 1.0 / sqrt(s);
        const double d = (s > 1e-290 && s < 1e290) ? s * r : sqrt(s);
        inv[j] = r;
#else
        const double d = sqrt(s);
        inv[j] = 1.0 / d;
#endif
        L[pk(j, j)] = d;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double v = ne[pk(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v = msub(v, L[pk(k, i)], L[pk(k, j)]);
            L[pk(j, i)] = v * inv[j];
        }
    }
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double v = -ne[21 + i];
#pragma unroll
        for (int k = 0; k < i; ++k) v = msub(v, L[pk(k, i)], z[k]);
        z[i] = v * inv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double v = z[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) v = msub(v, L[pk(i, k)], y[k]);
        y[i] = v * inv[i];
    }
    return 0;
}

struct SolveShared {
    double q[4], t[3], qc[4], tc[3];
    double s[6];
    double ne[kNE];       // normal equations at the current x
    double radius, dec, mcc;
    int invalid, flag, nlog, done;
};

SSF_DEV void write_log(double* log, int max_iter, int p, int idx, const double q[4],
                       const double t[3], double cost, double status, double radius) {
    if (!log || idx >= max_iter) return;
    double* r = log + ((int64_t)p * max_iter + idx) * 10;
    r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[3] = q[3];
    r[4] = t[0]; r[5] = t[1]; r[6] = t[2];
    r[7] = cost; r[8] = status; r[9] = radius;
}

#ifndef SSF_SOLVE_LM_REG
#define SSF_SOLVE_LM_REG 1                       // LM state in every thread's registers (A/B: 0 = lane-0 step)
#endif
// kEdges: point-to-line blocks (ecorr at ecurr_off / ecurr_count) join every evaluation; they
// are compacted into the same LDS arrays after the planes.
// kMode: the solver this instantiation runs (SSF_SOLVER_GN / SSF_SOLVER_CERES_LM), so each mode's
// register allocation covers its own loop only (the LM state does not weigh on the GN kernel);
// -1 dispatches on the runtime `mode` (A/B: SSF_SOLVE_SPECIALISE=0).
template <bool kEdges, int NT, int kMode>
__global__ __launch_bounds__(NT) void k_solve(const CorrRec* __restrict__ corr,
                                                         const int64_t* __restrict__ curr_off,
                                                         const int32_t* __restrict__ curr_count,
                                                         const int32_t* __restrict__ last_count,
                                                         int mode, int max_iter,
                                                         const double* pose_in,
                                                         const double* pose_abs_in,
                                                         double* pose_rel,
                                                         double* pose_abs,
                                                         double* __restrict__ log,
                                                         int32_t* __restrict__ nlog_out,
                                                         int32_t* __restrict__ ncorr_out,
                                                         const CorrRec* __restrict__ ecorr,
                                                         const int64_t* __restrict__ ecurr_off,
                                                         const int32_t* __restrict__ ecurr_count,
                                                         int32_t* __restrict__ ncorr_edge_out,
                                                         const int32_t* __restrict__ ncompact) {
    __shared__ SolveShared S;
    __shared__ double red[2 * (NT / 64 + 1) * kNE];                   // block_sum_db: two halves
    __shared__ CorrLds C;
#if SSF_SOLVE_COMPACT1
    __shared__ int wtot2[2][NT / 64];
#else
    __shared__ int wtot[NT / 64];
#endif
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = curr_count[p];
    const CorrRec* rec = corr + curr_off[p];
    // records the association already compacted (ncompact[p] >= 0): read with the other per-pair
    // scalars, before the first barrier
    const int ncp = (!kEdges && ncompact) ? ncompact[p] : -1;          // uniform
    const int en = kEdges ? ecurr_count[p] : 0;
    const CorrRec* erec = kEdges ? ecorr + ecurr_off[p] : nullptr;
#ifdef SSF_SOLVE_STAMPS
    // diagnostic build only: s_memtime phase stamps into the last log row (cost/status/radius)
    const unsigned long long st0 = __builtin_amdgcn_s_memtime();
    unsigned long long st1 = st0, st2 = st0;
#endif
#ifdef SSF_SOLVE_STAMPS2
    // diagnostic build only: the GN iterations split into the 6x6 solve + pose update and the
    // evaluation (replacing the compaction / first-evaluation stamps of the log row)
    unsigned long long t_sol = 0, t_ev = 0;
#endif
    if (tid == 0) {
        for (int k = 0; k < 4; ++k) S.q[k] = pose_in[7 * p + k];
        for (int k = 0; k < 3; ++k) S.t[k] = pose_in[7 * p + 4 + k];
        S.nlog = 0; S.done = 0;
    }
    __syncthreads();
    const bool skip = last_count[p] <= 10;                              // :158
    if (!skip) {
        // order-preserving compaction of the valid records into LDS, coalesced: record i goes
        // to thread i % T in trip i / T; per trip a ballot + the wave counts give every valid
        // record its rank.  kPre trips' records are loaded before the first is used (one load
        // latency per kPre trips).
        const int lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
        const int T = blockDim.x;
#if SSF_SOLVE_COMPACT1
        // one pass per kCmpPer x T records: wave w takes a contiguous range of kCmpPer x 64, every
        // load of the pass in flight at once; per 64-record step a ballot, the ranks from the
        // wave's own popcounts and ONE exchange of the wave totals (one barrier per pass; the
        // totals alternate between two LDS rows, so the next pass needs no second barrier)
        auto compact = [&](const CorrRec* __restrict__ src, int cnt, int start) {
            int nv = 0;                                                 // uniform
            for (int i0 = 0, ps = 0; i0 < cnt; i0 += kCmpPer * T, ps ^= 1) {
                const int wb = i0 + w * kCmpPer * 64;
                float4 c0[kCmpPer], c1[kCmpPer], c2[kCmpPer];
#pragma unroll
                for (int j = 0; j < kCmpPer; ++j) {
                    const CorrRec* r = src + min(wb + j * 64 + lane, cnt - 1);   // clamped
                    c0[j] = reinterpret_cast<const float4*>(r)[0];
                    c1[j] = reinterpret_cast<const float4*>(r)[1];
                    c2[j] = reinterpret_cast<const float4*>(r)[2];
                }
                uint64_t m[kCmpPer];
                int wt = 0;
#pragma unroll
                for (int j = 0; j < kCmpPer; ++j) {
                    m[j] = __ballot(wb + j * 64 + lane < cnt && c0[j].w != 0.0f);
                    wt += __popcll(m[j]);
                }
                if (lane == 0) wtot2[ps][w] = wt;
                __syncthreads();
                int before = start + nv, tot = 0;
                for (int j = 0; j < nw; ++j) { const int x = wtot2[ps][j]; if (j < w) before += x; tot += x; }
#pragma unroll
                for (int j = 0; j < kCmpPer; ++j) {
                    const int pos = before + __popcll(m[j] & lanemask_lt());
                    if (((m[j] >> lane) & 1ull) && pos < kSolveLdsCap) {
                        C.po[0][pos] = c0[j].x; C.po[1][pos] = c0[j].y; C.po[2][pos] = c0[j].z;
                        C.pa[0][pos] = c1[j].x; C.pa[1][pos] = c1[j].y; C.pa[2][pos] = c1[j].z;
                        C.n[0][pos] = c2[j].x; C.n[1][pos] = c2[j].y; C.n[2][pos] = c2[j].z;
                    }
                    before += __popcll(m[j]);
                }
                nv += tot;
            }
            __syncthreads();                                            // the LDS records, for every wave
            return nv;
        };
#else
        constexpr int kPre = 2;
        // records [0, cnt) of src appended at LDS position `start`; returns the valid count
        auto compact = [&](const CorrRec* __restrict__ src, int cnt, int start) {
            int nv = 0;                                                 // uniform
            for (int i0 = 0; i0 < cnt; i0 += kPre * T) {
                CorrRec c[kPre];
#pragma unroll
                for (int k = 0; k < kPre; ++k) c[k] = src[min(i0 + k * T + tid, cnt - 1)];   // clamped
#pragma unroll
                for (int k = 0; k < kPre; ++k) {
                    const bool v = i0 + k * T + tid < cnt && c[k].valid != 0.0f;
                    const uint64_t m = __ballot(v);
                    if (lane == 0) wtot[w] = __popcll(m);
                    __syncthreads();
                    int before = start + nv, tot = 0;
                    for (int j = 0; j < nw; ++j) { const int x = wtot[j]; if (j < w) before += x; tot += x; }
                    const int pos = before + __popcll(m & lanemask_lt());
                    if (v && pos < kSolveLdsCap) {
#pragma unroll
                        for (int d = 0; d < 3; ++d) { C.po[d][pos] = c[k].po[d]; C.pa[d][pos] = c[k].pa[d]; C.n[d][pos] = c[k].n[d]; }
                    }
                    nv += tot;
                    __syncthreads();                                    // wtot is rewritten next trip
                }
            }
            return nv;
        };
#endif
        // compacted records: [0, ncp) in rank order, streamed into LDS by the first evaluation
        // itself (evaluate_load: the same per-thread order and sums as evaluate() from LDS), no
        // ballot pass
        const int nv = ncp >= 0 ? ncp : compact(rec, n, 0);
        const int nve = kEdges ? compact(erec, en, nv) : 0;
        const bool in_lds = nv + nve <= kSolveLdsCap;                  // uniform
#ifdef SSF_SOLVE_STAMPS
        st1 = __builtin_amdgcn_s_memtime();
#endif
        if (tid == 0 && ncorr_out) ncorr_out[p] = nv;
        if (kEdges && tid == 0 && ncorr_edge_out) ncorr_edge_out[p] = nve;
        int par = 0;                                                    // block_sum_dpp's LDS half
        // (compacted records beyond the LDS: every record of [0, nv) is valid)
        const int nglob = ncp >= 0 ? nv : n;
        auto eval_at = [&](const double* qq, const double* tt, double (&ne_)[kNE]) {
            if (in_lds) evaluate<NT / 64>(C, nv, qq, tt, ne_, red, nve, par);
            else evaluate(rec, nglob, qq, tt, ne_, red, erec, en);
            par ^= 1;
        };
        double ne[kNE];
        double q[4], t[3];
#if SSF_SOLVE_QDIRECT
        for (int k = 0; k < 4; ++k) q[k] = pose_in[7 * p + k];                 // (A/B) uniform loads
        for (int k = 0; k < 3; ++k) t[k] = pose_in[7 * p + 4 + k];
#else
        for (int k = 0; k < 4; ++k) q[k] = S.q[k];
        for (int k = 0; k < 3; ++k) t[k] = S.t[k];
#endif
        if (ncp >= 0 && in_lds && SSF_SOLVE_DIRECT == 1) {
            evaluate_load<NT / 64>(rec, C, nv, q, t, ne, red, par);
            par ^= 1;
        } else {
            if (ncp >= 0 && in_lds) {
                // (A/B, SSF_SOLVE_DIRECT=2) a plain copy of the compacted records into LDS, four
                // per thread in flight: thread t writes the positions t + k T it reads itself
                const int T = blockDim.x;
                for (int i0 = tid; i0 < nv; i0 += 4 * T) {
                    float4 a[4][3];
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        const float4* rp = reinterpret_cast<const float4*>(rec + min(i0 + h * T, nv - 1));
                        a[h][0] = rp[0]; a[h][1] = rp[1]; a[h][2] = rp[2];
                    }
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        const int ih = i0 + h * T;
                        if (ih < nv) {
                            C.po[0][ih] = a[h][0].x; C.po[1][ih] = a[h][0].y; C.po[2][ih] = a[h][0].z;
                            C.pa[0][ih] = a[h][1].x; C.pa[1][ih] = a[h][1].y; C.pa[2][ih] = a[h][1].z;
                            C.n[0][ih] = a[h][2].x; C.n[1][ih] = a[h][2].y; C.n[2][ih] = a[h][2].z;
                        }
                    }
                }
            }
            eval_at(q, t, ne);
        }
#ifdef SSF_SOLVE_STAMPS
        st2 = __builtin_amdgcn_s_memtime();
#endif
#if !SSF_SOLVE_LM_REG
        if (tid == 0) {
            for (int k = 0; k < kNE; ++k) S.ne[k] = ne[k];
            for (int u = 0; u < 6; ++u) S.s[u] = 1.0 / (1.0 + sqrt(ne[pk(u, u)]));
            S.radius = 1e4; S.dec = 2.0; S.invalid = 0;
        }
        __syncthreads();
#endif
        if ((kMode >= 0 ? kMode : mode) == SSF_SOLVER_GN) {
            // every thread holds the same sums after the block reduction, so every thread runs
            // the same 6x6 solve on the same bits and carries the same pose: no lane-0 step, no
            // LDS broadcast, no extra barrier per iteration (thread 0 alone writes the log)
            int nl = 0;
            for (int it = 0; it < max_iter; ++it) {
                double y[6];
#ifdef SSF_SOLVE_STAMPS2
                const unsigned long long sa = __builtin_amdgcn_s_memtime();
#endif
                if (chol_solve_packed(ne, y) != 0) {                         // uniform
                    if (tid == 0) write_log(log, max_iter, p, nl, q, t, ne[27], 2, 0);
                    ++nl;
                    break;
                }
                double qn[4];
                quat_plus_step(q, y, qn);
                for (int k = 0; k < 4; ++k) q[k] = qn[k];
                t[0] += y[3]; t[1] += y[4]; t[2] += y[5];
#ifdef SSF_SOLVE_STAMPS2
                const unsigned long long sb = __builtin_amdgcn_s_memtime();
#endif
                eval_at(q, t, ne);
#ifdef SSF_SOLVE_STAMPS2
                const unsigned long long sc = __builtin_amdgcn_s_memtime();
                t_sol += sb - sa; t_ev += sc - sb;
#endif
                if (tid == 0) write_log(log, max_iter, p, nl, q, t, ne[27], 6, 0);
                ++nl;
            }

            if (tid == 0) {
                for (int k = 0; k < 4; ++k) S.q[k] = q[k];
                for (int k = 0; k < 3; ++k) S.t[k] = t[k];
                S.nlog = nl;
            }
            __syncthreads();
        } else {
#if SSF_SOLVE_LM_REG
            // every thread carries the LM state (accepted pose and normal equations, scaling,
            // radius) in registers and runs the same step on the same bits, as the GN path does:
            // no lane-0 section that the other 255 threads wait on at two barriers per iteration,
            // no LDS round trips on the serial chain, the 6x6 solve by rsq pivots
            double qa[4], ta[3], na[kNE], sc[6];
            for (int k = 0; k < 4; ++k) qa[k] = q[k];
            for (int k = 0; k < 3; ++k) ta[k] = t[k];
#pragma unroll
            for (int k = 0; k < kNE; ++k) na[k] = ne[k];
#pragma unroll
            for (int u = 0; u < 6; ++u) sc[u] = 1.0 / (1.0 + sqrt(ne[pk(u, u)]));
            double radius = 1e4, dec = 2.0;
            int invalid = 0, nl = 0;
            for (int it = 1; it <= max_iter; ++it) {
                // LevenbergMarquardtStrategy::ComputeStep on the Jacobi-scaled system: m holds
                // M = As + diag(clamp(As_uu)) / radius packed, and gs, so chol_solve_packed
                // solves M y = -gs
                double As[21], m[kNE], y[6];
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    m[21 + u] = sc[u] * na[21 + u];
#pragma unroll
                    for (int v = u; v < 6; ++v) As[pk(u, v)] = sc[u] * na[pk(u, v)] * sc[v];
                }
#pragma unroll
                for (int k = 0; k < 21; ++k) m[k] = As[k];
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    double d = As[pk(u, u)];
                    if (d < 1e-6) d = 1e-6;
                    if (d > 1e32) d = 1e32;
                    m[pk(u, u)] += d / radius;
                }
                const bool ok = chol_solve_packed(m, y) == 0;             // uniform
                double mcc = 0.0;
                if (ok) {
                    double yg = 0.0, yAy = 0.0;
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        yg += y[u] * m[21 + u];
                        double Ay = 0.0;
#pragma unroll
                        for (int v = 0; v < 6; ++v) Ay += As[pk(u, v)] * y[v];
                        yAy += y[u] * Ay;
                    }
                    mcc = -(yg + 0.5 * yAy);
                }
                if (!ok || !(mcc > 0.0)) {
                    radius /= dec; dec *= 2.0;
                    if (tid == 0) write_log(log, max_iter, p, nl, qa, ta, na[27], 2, radius);
                    ++nl;
                    if (++invalid > 5) break;
                    continue;
                }
                invalid = 0;
                double delta[6], qc[4], tc[3];
#pragma unroll
                for (int u = 0; u < 6; ++u) delta[u] = y[u] * sc[u];
                quat_plus_step(qa, delta, qc);
                tc[0] = ta[0] + delta[3]; tc[1] = ta[1] + delta[4]; tc[2] = ta[2] + delta[5];
                eval_at(qc, tc, ne);
                double xn = 0.0, sn = 0.0;
                for (int u = 0; u < 4; ++u) { xn += qa[u] * qa[u]; sn += (qa[u] - qc[u]) * (qa[u] - qc[u]); }
                for (int u = 0; u < 3; ++u) { xn += ta[u] * ta[u]; sn += (ta[u] - tc[u]) * (ta[u] - tc[u]); }
                xn = sqrt(xn); sn = sqrt(sn);
                const double dcost = na[27] - ne[27];
                if (!(sn > (xn + 1e-8) * 1e-8)) {                       // ParameterToleranceReached
                    if (tid == 0) write_log(log, max_iter, p, nl, qa, ta, na[27], 3, radius);
                    ++nl;
                    break;
                }
                if (!(fabs(dcost) > 1e-6 * na[27])) {                   // FunctionToleranceReached
                    if (tid == 0) write_log(log, max_iter, p, nl, qa, ta, na[27], 4, radius);
                    ++nl;
                    break;
                }
                const double rho = dcost / mcc;
                if (rho > 1e-3) {                                       // accept
                    for (int k = 0; k < 4; ++k) qa[k] = qc[k];
                    for (int k = 0; k < 3; ++k) ta[k] = tc[k];
#pragma unroll
                    for (int k = 0; k < kNE; ++k) na[k] = ne[k];
                    const double f = 2.0 * rho - 1.0;
                    double den = 1.0 - f * f * f;
                    if (den < 1.0 / 3.0) den = 1.0 / 3.0;
                    radius = radius / den;
                    if (radius > 1e16) radius = 1e16;
                    dec = 2.0;
                    const double mg[3] = {-ne[21], -ne[22], -ne[23]};
                    double qg[4], gm = 0.0;
                    quat_plus(qa, mg, qg);
                    for (int u = 0; u < 4; ++u) gm = fmax(gm, fabs(qa[u] - qg[u]));
                    for (int u = 3; u < 6; ++u) gm = fmax(gm, fabs(ne[21 + u]));
                    const bool conv = gm <= 1e-10;                      // GradientToleranceReached
                    if (tid == 0) write_log(log, max_iter, p, nl, qa, ta, na[27], conv ? 5 : 1, radius);
                    ++nl;
                    if (conv) break;
                } else {                                                // reject
                    radius /= dec; dec *= 2.0;
                    if (tid == 0) write_log(log, max_iter, p, nl, qa, ta, na[27], 0, radius);
                    ++nl;
                }
            }
            if (tid == 0) {
                for (int k = 0; k < 4; ++k) S.q[k] = qa[k];
                for (int k = 0; k < 3; ++k) S.t[k] = ta[k];
                S.nlog = nl;
            }
#else
            for (int it = 1; it <= max_iter; ++it) {
                if (tid == 0) {
                    // LevenbergMarquardtStrategy::ComputeStep on the Jacobi-scaled system
                    double As[6][6], gs[6], M[6][6], bb[6], y[6];
                    for (int u = 0; u < 6; ++u) {
                        gs[u] = S.s[u] * S.ne[21 + u];
                        for (int v = 0; v < 6; ++v) As[u][v] = S.s[u] * S.ne[pk(u, v)] * S.s[v];
                    }
                    for (int u = 0; u < 6; ++u) {
                        double d = As[u][u];
                        if (d < 1e-6) d = 1e-6;
                        if (d > 1e32) d = 1e32;
                        for (int v = 0; v < 6; ++v) M[u][v] = As[u][v];
                        M[u][u] += d / S.radius;
                        bb[u] = -gs[u];
                    }
                    const bool ok = chol_solve6(M, bb, y) == 0;
                    double mcc = 0.0;
                    if (ok) {
                        double yg = 0.0, yAy = 0.0;
                        for (int u = 0; u < 6; ++u) {
                            yg += y[u] * gs[u];
                            double Ay = 0.0;
                            for (int v = 0; v < 6; ++v) Ay += As[u][v] * y[v];
                            yAy += y[u] * Ay;
                        }
                        mcc = -(yg + 0.5 * yAy);
                    }
                    if (!ok || !(mcc > 0.0)) {
                        S.radius /= S.dec; S.dec *= 2.0;
                        write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 2, S.radius);
                        S.flag = 0;
                        if (++S.invalid > 5) S.done = 1;
                    } else {
                        S.invalid = 0;
                        double delta[6];
                        for (int u = 0; u < 6; ++u) delta[u] = y[u] * S.s[u];
                        quat_plus(S.q, delta, S.qc);
                        S.tc[0] = S.t[0] + delta[3]; S.tc[1] = S.t[1] + delta[4]; S.tc[2] = S.t[2] + delta[5];
                        S.mcc = mcc;
                        S.flag = 1;
                    }
                }
                __syncthreads();
                if (S.done) break;
                if (!S.flag) continue;
                double qc[4], tc[3];
                for (int k = 0; k < 4; ++k) qc[k] = S.qc[k];
                for (int k = 0; k < 3; ++k) tc[k] = S.tc[k];
                eval_at(qc, tc, ne);
                if (tid == 0) {
                    double xn = 0.0, sn = 0.0;
                    for (int u = 0; u < 4; ++u) { xn += S.q[u] * S.q[u]; sn += (S.q[u] - S.qc[u]) * (S.q[u] - S.qc[u]); }
                    for (int u = 0; u < 3; ++u) { xn += S.t[u] * S.t[u]; sn += (S.t[u] - S.tc[u]) * (S.t[u] - S.tc[u]); }
                    xn = sqrt(xn); sn = sqrt(sn);
                    const double dcost = S.ne[27] - ne[27];
                    if (!(sn > (xn + 1e-8) * 1e-8)) {                   // ParameterToleranceReached
                        write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 3, S.radius);
                        S.done = 1;
                    } else if (!(fabs(dcost) > 1e-6 * S.ne[27])) {      // FunctionToleranceReached
                        write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 4, S.radius);
                        S.done = 1;
                    } else {
                        const double rho = dcost / S.mcc;
                        if (rho > 1e-3) {                               // accept
                            for (int k = 0; k < 4; ++k) S.q[k] = S.qc[k];
                            for (int k = 0; k < 3; ++k) S.t[k] = S.tc[k];
                            for (int k = 0; k < kNE; ++k) S.ne[k] = ne[k];
                            const double f = 2.0 * rho - 1.0;
                            double den = 1.0 - f * f * f;
                            if (den < 1.0 / 3.0) den = 1.0 / 3.0;
                            S.radius = S.radius / den;
                            if (S.radius > 1e16) S.radius = 1e16;
                            S.dec = 2.0;
                            const double mg[3] = {-ne[21], -ne[22], -ne[23]};
                            double qg[4], gm = 0.0;
                            quat_plus(S.q, mg, qg);
                            for (int u = 0; u < 4; ++u) gm = fmax(gm, fabs(S.q[u] - qg[u]));
                            for (int u = 3; u < 6; ++u) gm = fmax(gm, fabs(ne[21 + u]));
                            if (gm <= 1e-10) {
                                write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 5, S.radius);
                                S.done = 1;
                            } else {
                                write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 1, S.radius);
                            }
                        } else {                                        // reject
                            S.radius /= S.dec; S.dec *= 2.0;
                            write_log(log, max_iter, p, S.nlog++, S.q, S.t, S.ne[27], 0, S.radius);
                        }
                    }
                }
                __syncthreads();
                if (S.done) break;
            }
#endif
        }
    } else if (tid == 0) {
        if (ncorr_out) ncorr_out[p] = -1;
        if (kEdges && ncorr_edge_out) ncorr_edge_out[p] = -1;
    }
    if (tid == 0) {
#ifdef SSF_SOLVE_STAMPS
        if (log) {
            double* r = log + ((int64_t)p * max_iter + max_iter - 1) * 10;
#ifdef SSF_SOLVE_STAMPS2
            r[7] = (double)t_sol; r[8] = (double)t_ev;
#else
            r[7] = (double)(st1 - st0); r[8] = (double)(st2 - st1);
#endif
            r[9] = (double)(__builtin_amdgcn_s_memtime() - st2);
        }
#endif
        for (int k = 0; k < 4; ++k) pose_rel[7 * p + k] = S.q[k];
        for (int k = 0; k < 3; ++k) pose_rel[7 * p + 4 + k] = S.t[k];
        if (nlog_out) nlog_out[p] = S.nlog;
        if (pose_abs) {                                                 // :87-90
            double q0l[4], t0l[3], q0c[4], r[3];
            for (int k = 0; k < 4; ++k) q0l[k] = pose_abs_in[7 * p + k];
            for (int k = 0; k < 3; ++k) t0l[k] = pose_abs_in[7 * p + 4 + k];
            quat_mul(q0l, S.q, q0c);
            quat_rotate(q0l, S.t, r);
            for (int k = 0; k < 4; ++k) pose_abs[7 * p + k] = q0c[k];
            for (int k = 0; k < 3; ++k) pose_abs[7 * p + 4 + k] = t0l[k] + r[k];
        }
    }
}

__global__ void k_accumulate(int n, const double* __restrict__ rel, const double* __restrict__ start,
                             double* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double q[4] = {0, 0, 0, 1}, t[3] = {0, 0, 0};
    if (start) {
        for (int k = 0; k < 4; ++k) q[k] = start[k];
        for (int k = 0; k < 3; ++k) t[k] = start[4 + k];
    }
    for (int i = 0; i < n; ++i) {
        const double* r = rel + 7 * i;
        double qn[4], rt[3];
        quat_mul(q, r, qn);
        quat_rotate(q, r + 4, rt);
        for (int k = 0; k < 3; ++k) t[k] = t[k] + rt[k];
        for (int k = 0; k < 4; ++k) q[k] = qn[k];
        for (int k = 0; k < 4; ++k) out[7 * i + k] = q[k];
        for (int k = 0; k < 3; ++k) out[7 * i + 4 + k] = t[k];
    }
}

__global__ __launch_bounds__(256) void k_strip_invalidate(const int64_t* __restrict__ frame_off,
                                                          const int32_t* __restrict__ count, int n_frames,
                                                          int32_t* __restrict__ strip_head) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f < n_frames && strip_image_frame(count[f])) strip_head[frame_off[f] + 3 * kStripMax + 4] = 0;
}

hipError_t launch_plane_table(hipStream_t s, const ssf_config& cfg, int n_frames,
                              const float4* plane, const int64_t* frame_off, const int32_t* count,
                              int64_t max_m, float* normal, uint8_t* valid, float4* sorted_xyzi,
                              int32_t* sorted_idx, float4* strip_xyzi, int32_t* strip_head) {
    if (n_frames <= 0 || max_m <= 0) return hipSuccess;
    if (max_m <= kSortMax && sorted_xyzi && sorted_idx) {
        // few frames (a node's one frame, configs[2]'s 32): up to 8 work-groups per frame share
        // its queries (each sorts and builds the strips itself), so the launch spreads over the
        // chip instead of n_frames CUs; 256 frames and more keep one work-group per frame
        const int qsplit = (int)std::max<int64_t>(1, std::min<int64_t>({SSF_TABLE_MAX_SPLIT, 256 / n_frames,
                                                             max_m / 256}));
        kmark(s, "k_plane_table_sorted");
        hipLaunchKernelGGL(k_plane_table_sorted, dim3(n_frames, qsplit), dim3(kTableThreads), 0, s, plane,
                           frame_off, count, cfg.plane_max, normal, valid, sorted_xyzi, sorted_idx,
                           strip_head ? strip_xyzi : nullptr, strip_head);
    } else {
        const int bx = (int)((max_m + 255) / 256);
        kmark(s, "k_plane_table");
        hipLaunchKernelGGL(k_plane_table, dim3(bx, n_frames), dim3(256), 0, s, plane, frame_off,
                           count, cfg.plane_max, normal, valid);
        if (strip_head)                     // no image from this launch: no frame may look imaged
            hipLaunchKernelGGL(k_strip_invalidate, dim3((n_frames + 255) / 256), dim3(256), 0, s,
                               frame_off, count, n_frames, strip_head);
    }
    return hipGetLastError();
}

hipError_t launch_register(hipStream_t s, const ssf_config& cfg, int n_pairs, const float4* last,
                           const int64_t* last_off, const int32_t* last_count,
                           const float* last_normal, const uint8_t* last_valid,
                           const float4* last_sorted, const int32_t* last_sidx, const float4* curr,
                           const int64_t* curr_off, const int32_t* curr_count, int64_t max_m,
                           CorrRec* corr, double* pose_rel, double* pose_abs, double* log,
                           int32_t* nlog, int32_t* ncorr, int32_t* nn, const EdgeReg* edge,
                           const float4* last_strip_xyzi, const int32_t* last_strip_head,
                           const double* pose_in, const double* pose_abs_in, int32_t* nnv,
                           int32_t* ncompact) {
    if (n_pairs <= 0) return hipSuccess;
    // warm starts / start poses read from pose_in / pose_abs_in (default: in place), results
    // written to pose_rel / pose_abs: a chain reads pair k - 1's output slot directly
    const double* pin = pose_in ? pose_in : pose_rel;
    const double* ain = pose_abs_in ? pose_abs_in : pose_abs;
    // compacted records (k_associate_strips' lane mode with one work-group per pair, planes only):
    // the association writes the counts, the solve reads them; otherwise neither sees them
    int32_t* ncp = nullptr;
    if (max_m > 0) {
        const int bx = (int)((max_m + 255) / 256);
#ifndef SSF_ASSOC_XBAND
        if (max_m <= kSortMax && last_sorted && last_sidx) {
            const bool soa = max_m > kAssocStripF4Max;
            const int cap = (int)std::min<int64_t>(max_m, soa ? kAssocStripSoaMax : kAssocStripF4Max);
            const size_t lds = soa ? (size_t)cap * 14 + 16 : (size_t)cap * sizeof(float4);
            // few pairs (a node's one pair, configs[2]'s chained pairs): up to 8 work-groups per
            // pair, each staging the last frame and taking a share of the queries, so the launch
            // spreads over ~256 CUs instead of n_pairs
            const bool coop = kAssocCoopG > 0 && n_pairs <= kAssocCoopPairs;
            constexpr int kQpwCoop = kAssocCoopG > 0 ? kStripThreads / kAssocCoopG : kStripThreads;
            // big launches: one work-group per pair, the lane mode (or SSF_ASSOC_BIG_G-lane groups, A/B)
            const bool bigc = !coop && kAssocBigG > 0;
            // (group mode: every work-group stages the whole last frame, so the split is capped at
            // ~4 launch-filling waves of work-groups; the query loop strides over gridDim.y)
            const int qsplit = coop ? (int)std::min<int64_t>((max_m + kQpwCoop - 1) / kQpwCoop,
                                                             std::max(8, 1024 / n_pairs))
                                    : (int)std::max<int64_t>(1, std::min<int64_t>({8, 256 / n_pairs,
                                                             (max_m + kStripThreads - 1) / kStripThreads}));
            if (!coop && !bigc && qsplit == 1 && nnv && ncompact && !edge && !SSF_ASSOC_DEFER && SSF_ASSOC_COMPACT)
                ncp = ncompact;
            kmark(s, coop ? "k_associate_strips_coop" : soa ? "k_associate_strips_soa" : "k_associate_strips");
            hipLaunchKernelGGL(coop ? (soa ? k_associate_strips<true, kAssocCoopG> : k_associate_strips<false, kAssocCoopG>)
                                    : bigc ? (soa ? k_associate_strips<true, kAssocBigG> : k_associate_strips<false, kAssocBigG>)
                                    : (soa ? k_associate_strips<true> : k_associate_strips<false>),
                               dim3(n_pairs, qsplit), dim3(kStripThreads), lds, s, last, last_off, last_count,
                               last_normal, last_valid, last_sorted, last_sidx, curr, curr_off,
                               curr_count, pin, corr, nn, cap,
                               last_strip_head ? last_strip_xyzi : nullptr, last_strip_head,
                               ncp ? nnv : nullptr, ncp);
        } else
#endif
        if (max_m <= kAssocSoaMax && last_sorted && last_sidx) {
            const int qx = (int)((max_m + kAssocQ - 1) / kAssocQ);
            const bool soa = max_m > kAssocLdsMax;
            kmark(s, soa ? "k_associate_lds_soa" : "k_associate_lds");
            const size_t lds = (size_t)max_m * (soa ? 12 : sizeof(float4)) + kAssocQ * sizeof(int);
            hipLaunchKernelGGL(soa ? k_associate_lds<true> : k_associate_lds<false>,
                               dim3(qx, n_pairs), dim3(kAssocThreads), lds, s, last, last_off,
                               last_count, last_normal, last_valid, last_sorted, last_sidx, curr,
                               curr_off, curr_count, pin, corr, nn, (int)max_m);
        } else if (max_m <= kSortMax && last_sorted && last_sidx) {
            kmark(s, "k_associate_sorted");
            hipLaunchKernelGGL(k_associate_sorted, dim3(bx, n_pairs), dim3(256), 0, s, last, last_off,
                               last_count, last_normal, last_valid, last_sorted, last_sidx, curr,
                               curr_off, curr_count, pin, corr, nn);
        } else {
            kmark(s, "k_associate");
            hipLaunchKernelGGL(k_associate, dim3(bx, n_pairs), dim3(256), 0, s, last, last_off,
                               last_count, last_normal, last_valid, curr, curr_off, curr_count,
                               pin, corr, nn);
        }
    }
    if (edge && edge->max_m > 0) {
        const int cap = (int)std::min<int64_t>(edge->max_m, kEdgeLdsMax);
        kmark(s, "k_edge_associate");
        hipLaunchKernelGGL(k_edge_associate, dim3(n_pairs), dim3(kEdgeAssocThreads), (size_t)cap * sizeof(float4),
                           s, edge->last, edge->last_off, edge->last_count, edge->line,
                           edge->line_valid, edge->curr, edge->curr_off, edge->curr_count, pin,
                           edge->corr, cap);
    }
    kmark(s, "k_solve");
#if SSF_SOLVE_SPECIALISE
#define SSF_SOLVE_LAUNCH(E, NT, ...)                                                               \
    hipLaunchKernelGGL((cfg.solver == SSF_SOLVER_GN ? k_solve<E, NT, SSF_SOLVER_GN> : k_solve<E, NT, SSF_SOLVER_CERES_LM>), \
                       dim3(n_pairs), dim3(NT), 0, s, corr, curr_off, curr_count, \
                       last_count, cfg.solver, cfg.max_iter, pin, ain, pose_rel, pose_abs, log, nlog, ncorr, \
                       __VA_ARGS__, ncp)
#else
#define SSF_SOLVE_LAUNCH(E, NT, ...)                                                               \
    hipLaunchKernelGGL((k_solve<E, NT, -1>), dim3(n_pairs), dim3(NT), 0, s, corr, curr_off, curr_count, \
                       last_count, cfg.solver, cfg.max_iter, pin, ain, pose_rel, pose_abs, log, nlog, ncorr, \
                       __VA_ARGS__, ncp)
#endif
    if (edge)
        SSF_SOLVE_LAUNCH(true, kSolveThreads, edge->corr, edge->curr_off, edge->curr_count, edge->ncorr);
    else
        SSF_SOLVE_LAUNCH(false, kSolveThreads, (const CorrRec*)nullptr, (const int64_t*)nullptr,
                         (const int32_t*)nullptr, (int32_t*)nullptr);
#undef SSF_SOLVE_LAUNCH
    return hipGetLastError();
}

hipError_t launch_edge_table(hipStream_t s, const ssf_edge_config& ec, int n_frames,
                             const float4* edges, const int64_t* frame_off, const int32_t* count,
                             int64_t max_m, float* line, uint8_t* valid) {
    if (n_frames <= 0 || max_m <= 0) return hipSuccess;
    const int cap = (int)std::min<int64_t>(max_m, kEdgeLdsMax);
    kmark(s, "k_edge_table");
    hipLaunchKernelGGL(k_edge_table, dim3(n_frames), dim3(kEdgeThreads), (size_t)cap * sizeof(float4),
                       s, edges, frame_off, count, ec.max_nn_d2, ec.line_ratio, line, valid, cap);
    return hipGetLastError();
}

hipError_t launch_accumulate(hipStream_t s, int n, const double* rel, const double* start,
                             double* abs_out) {
    if (n <= 0) return hipSuccess;
    kmark(s, "k_accumulate");
    hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(64), 0, s, n, rel, start, abs_out);
    return hipGetLastError();
}

}  // namespace ssf
