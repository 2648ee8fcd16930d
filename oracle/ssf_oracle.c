/*
 * ssf_oracle.c -- CPU restatement of the SSF-SLAM front-end hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ssf_oracle.h for the parity-pinning status).
 * Each function cites the reference line(s) it restates.  Build:
 *   gcc -O2 -ffp-contract=off -fno-fast-math -fPIC -shared  (oracle/Makefile)
 */
#include "ssf_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================== */
/* Profiles: src/frameFeature.cpp:141-152 and src/lidarOdometry_onlyPC.cpp:313-319 */
int orc_profile_get(int32_t n_rows, orc_profile* p) {
    memset(p, 0, sizeof(*p));
    p->n_rows = n_rows;
    if (n_rows == 16) {
        p->plane_min = 0.05f; p->plane_span = 3; p->row_start = 0; p->row_end = 0;
        p->plane_max = 0.15f;
        return 0;
    }
    if (n_rows == 64) {
        p->plane_min = 0.005f; p->plane_span = 25; p->row_start = 5; p->row_end = 5;
        p->plane_max = 0.05f;
        return 0;
    }
    return -1;
}

/* ======================================================================== */
/* frameFeature.cpp:57-72 -- vertical angle -> scan row.
 * `float angle = atan(point.z / sqrt(point.x * point.x + point.y * point.y)) * 180 / M_PI;`
 * with float members.  Which atan / sqrt that names is C++ overload resolution over what the
 * TU's headers declare at global scope (header.h:8-35: ROS, tf, PCL, Ceres, GTSAM):
 *  - libstdc++'s <math.h> wrapper (any of those headers including <math.h>, e.g. tf's
 *    LinearMath/Scalar.h, ros/time.h) adds `using std::atan; using std::sqrt;`, so the float
 *    overloads win (exact match over promotion): sqrtf, a float divide, atanf, then `* 180` is a
 *    FLOAT multiply (int 180 -> 180.0f) and `/ M_PI` a double divide, stored to float.  This is
 *    ORC_RING_CHAIN_FLOAT, the default.
 *  - with only the C declarations, the chain is double from the sqrt on: ORC_RING_CHAIN_DOUBLE.
 * glibc's atanf / atan are the ones evaluated (this container's glibc; the device table is built
 * by the same host libm).  The `||` guards at :59 and :64 are always true and are omitted. */
static int32_t g_ring_chain = ORC_RING_CHAIN_FLOAT;
int32_t orc_set_ring_chain(int32_t chain) {
    int32_t prev = g_ring_chain;
    g_ring_chain = chain == ORC_RING_CHAIN_DOUBLE ? ORC_RING_CHAIN_DOUBLE : ORC_RING_CHAIN_FLOAT;
    return prev;
}
int32_t orc_get_ring_chain(void) { return g_ring_chain; }

float orc_ring_angle(float x, float y, float z, int32_t chain) {
    float r2 = x * x + y * y;                                   /* float members: a float sum */
    if (chain == ORC_RING_CHAIN_DOUBLE)
        return (float)(atan((double)z / sqrt((double)r2)) * 180.0 / M_PI);
    float deg = atanf(z / sqrtf(r2)) * 180.0f;                  /* std::atan(float) * 180 */
    return (float)((double)deg / M_PI);                         /* float / double, to float */
}

/* The row of a float angle, with the C++ promotions of the reference's expressions:
 *   :60  (angle + 15) / 2 + 0.5   float + int, float / int (float), then + double
 *   :66  (2 - angle) * 3.0 + 0.5  int - float is a FLOAT subtraction, then double
 *   :68  (-8.83 - angle) * 2.0    double - float (double) */
int32_t orc_ring_id_of_angle(float angle, int32_t n_rows) {
    int32_t id = -1;
    if (angle != angle) return -1;     /* 0/0: int(NaN) is INT_MIN on x86 -> no row either way */
    if (n_rows == 16) {
        double v = (double)((angle + 15.0f) / 2.0f) + 0.5;                 /* :60 */
        id = v > -2147483648.0 && v < 2147483647.0 ? (int32_t)v : -1;
    } else if (n_rows == 64) {
        if ((double)angle >= -8.83) {                                      /* :65 */
            double v = (double)(2.0f - angle) * 3.0 + 0.5;                 /* :66 */
            id = v > -2147483648.0 && v < 2147483647.0 ? (int32_t)v : -1;
        } else {
            double v = (-8.83 - (double)angle) * 2.0 + 0.5;                /* :68 */
            id = v > -2147483648.0 && v < 2147483647.0 ? n_rows / 2 + (int32_t)v : -1;
        }
    }
    if (id > -1 && id < n_rows) return id;                               /* :73 */
    return -1;
}

int32_t orc_ring_id_chain(float x, float y, float z, int32_t n_rows, int32_t chain) {
    return orc_ring_id_of_angle(orc_ring_angle(x, y, z, chain), n_rows);
}
int32_t orc_ring_id(float x, float y, float z, int32_t n_rows) {
    return orc_ring_id_chain(x, y, z, n_rows, g_ring_chain);
}
int32_t orc_ring_id_ratio_d(double ratio, int32_t n_rows) {
    if (ratio != ratio) return -1;
    return orc_ring_id_of_angle((float)(atan(ratio) * 180.0 / M_PI), n_rows);
}

int64_t orc_ring_changes_f32(float lo, float hi, int32_t n_rows, float* at, int32_t* id, int64_t cap) {
    /* walk the floats of [lo, hi] in increasing order through their order-preserving keys */
    uint32_t b;
    memcpy(&b, &lo, 4);
    uint32_t k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    memcpy(&b, &hi, 4);
    const uint32_t kh = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    int32_t prev = -2;
    int64_t n = 0;
    for (;; ++k) {
        const uint32_t fb = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
        float r;
        memcpy(&r, &fb, 4);
        const int32_t v = orc_ring_id_chain(1.0f, 0.0f, r, n_rows, ORC_RING_CHAIN_FLOAT);
        if (v != prev) {
            if (n < cap) { at[n] = r; id[n] = v; }
            ++n;
            prev = v;
        }
        if (k == kh) break;
    }
    return n;
}

/* frameFeature.cpp:45-81 -- stable append per row, intensity = indexInRow + id/100.0 */
int64_t orc_bin(const float* pts, int64_t n, int64_t stride, int32_t n_rows, float* rxyzi,
                int64_t* ring_off, int64_t* src_idx, int32_t* ring_of_input) {
    int64_t* cnt = (int64_t*)calloc((size_t)n_rows, sizeof(int64_t));
    int32_t* rid = ring_of_input ? ring_of_input : (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        const float* p = pts + i * stride;
        int32_t id = orc_ring_id(p[0], p[1], p[2], n_rows);
        rid[i] = id;
        if (id >= 0) cnt[id]++;
    }
    ring_off[0] = 0;
    for (int32_t r = 0; r < n_rows; ++r) ring_off[r + 1] = ring_off[r] + cnt[r];
    memset(cnt, 0, sizeof(int64_t) * (size_t)n_rows);
    for (int64_t i = 0; i < n; ++i) {
        int32_t id = rid[i];
        if (id < 0) continue;
        const float* p = pts + i * stride;
        int64_t idx_in_row = cnt[id]++;
        int64_t o = ring_off[id] + idx_in_row;
        rxyzi[4 * o + 0] = p[0];
        rxyzi[4 * o + 1] = p[1];
        rxyzi[4 * o + 2] = p[2];
        rxyzi[4 * o + 3] = (float)((double)idx_in_row + (double)id / 100.0); /* :77 */
        if (src_idx) src_idx[o] = i;
    }
    int64_t kept = ring_off[n_rows];
    if (!ring_of_input) free(rid);
    free(cnt);
    return kept;
}

/* frameFeature.cpp:84-107 -- 11-tap curvature, float, left-to-right, no FMA. */
void orc_curvature(const float* rxyzi, const int64_t* ring_off, int32_t n_rows, int32_t row_start,
                   int32_t row_end, float* curv) {
    memset(curv, 0, sizeof(float) * (size_t)ring_off[n_rows]);
    for (int32_t r = row_start; r < n_rows - row_end; ++r) {
        const float* row = rxyzi + 4 * ring_off[r];
        int64_t size = ring_off[r + 1] - ring_off[r];
        for (int64_t j = 5; j < size - 5; ++j) {
            float d[3];
            for (int c = 0; c < 3; ++c) {
                float s = row[4 * (j - 5) + c] + row[4 * (j - 4) + c];
                s = s + row[4 * (j - 3) + c];
                s = s + row[4 * (j - 2) + c];
                s = s + row[4 * (j - 1) + c];
                s = s - 10.0f * row[4 * j + c];
                s = s + row[4 * (j + 1) + c];
                s = s + row[4 * (j + 2) + c];
                s = s + row[4 * (j + 3) + c];
                s = s + row[4 * (j + 4) + c];
                s = s + row[4 * (j + 5) + c];
                d[c] = s;
            }
            float v = d[0] * d[0] + d[1] * d[1];
            v = v + d[2] * d[2];
            curv[ring_off[r] + j] = v;                                   /* :105 */
        }
    }
}

/* frameFeature.cpp:110-123 -- greedy spacing selection, row-major output. */
int64_t orc_select(const float* rxyzi, const float* curv, const int64_t* ring_off, int32_t n_rows,
                   int32_t row_start, int32_t row_end, float plane_min, int32_t plane_span,
                   float* plane_xyzi, int64_t* sel_idx) {
    int64_t m = 0;
    for (int32_t r = row_start; r < n_rows - row_end; ++r) {
        int64_t size = ring_off[r + 1] - ring_off[r];
        int64_t jstart = 0;
        for (int64_t j = 0; j < size; ++j) {
            int64_t o = ring_off[r] + j;
            if (j >= jstart && curv[o] < plane_min) {
                memcpy(plane_xyzi + 4 * m, rxyzi + 4 * o, 4 * sizeof(float));
                if (sel_idx) sel_idx[m] = o;
                m++;
                jstart = j + plane_span;
            }
        }
    }
    return m;
}

int64_t orc_extract_planes(const float* pts, int64_t n, int64_t stride, int32_t n_rows,
                           float* plane_xyzi) {
    orc_profile p;
    if (orc_profile_get(n_rows, &p) != 0) return -1;
    float* rxyzi = (float*)malloc(sizeof(float) * 4 * (size_t)(n > 0 ? n : 1));
    float* curv = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_rows + 1));
    orc_bin(pts, n, stride, n_rows, rxyzi, off, NULL, NULL);
    orc_curvature(rxyzi, off, n_rows, p.row_start, p.row_end, curv);
    int64_t m = orc_select(rxyzi, curv, off, n_rows, p.row_start, p.row_end, p.plane_min,
                           p.plane_span, plane_xyzi, NULL);
    free(rxyzi); free(curv); free(off);
    return m;
}

/* ======================================================================== */
/* Exact k-NN by brute force, (d2, index) ascending.  d2 = ((dx*dx)+dy*dy)+dz*dz in float,
 * the FLANN L2_Simple accumulation behind PCL KdTreeFLANN (lidarOdometry_onlyPC.cpp:155-173).
 * FLANN's tie order is traversal dependent (parity unpinned on ties); ties here go to the
 * lower index, the same rule as the HIP kernels. */
void orc_knn(const float* cloud, int64_t m, const float q[3], int32_t k, int32_t* idx, float* d2) {
    int32_t cnt = 0;
    for (int64_t j = 0; j < m; ++j) {
        float dx = q[0] - cloud[4 * j + 0];
        float dy = q[1] - cloud[4 * j + 1];
        float dz = q[2] - cloud[4 * j + 2];
        float d = dx * dx + dy * dy;
        d = d + dz * dz;
        if (cnt == k && !(d < d2[k - 1])) continue;
        int32_t pos = cnt < k ? cnt : k - 1;
        while (pos > 0 && d < d2[pos - 1]) {
            d2[pos] = d2[pos - 1];
            idx[pos] = idx[pos - 1];
            pos--;
        }
        d2[pos] = d;
        idx[pos] = (int32_t)j;
        if (cnt < k) cnt++;
    }
    for (int32_t r = cnt; r < k; ++r) { idx[r] = -1; d2[r] = INFINITY; }
}

/* The same exact k-NN through an x-sorted index (the CPU baseline's stand-in for the kd-tree;
 * brute force made the baseline O(M^2)).  Candidates are visited outward from the query's x
 * and ranked by (d2, index) lexicographically, so the list is identical to orc_knn's whatever
 * the visit order.  A walk stops once dx*dx exceeds the k-th distance: d2 >= dx*dx holds in
 * float because each addition of a non-negative term rounds monotonically. */
typedef struct { float x; int32_t i; } orc_xkey;

static int xkey_cmp(const void* a, const void* b) {
    const orc_xkey* u = (const orc_xkey*)a;
    const orc_xkey* v = (const orc_xkey*)b;
    if (u->x < v->x) return -1;
    if (u->x > v->x) return 1;
    return (u->i > v->i) - (u->i < v->i);
}

orc_xindex* orc_xindex_build(const float* cloud, int64_t m) {
    orc_xindex* X = (orc_xindex*)malloc(sizeof(orc_xindex));
    orc_xkey* k = (orc_xkey*)malloc(sizeof(orc_xkey) * (size_t)(m > 0 ? m : 1));
    for (int64_t j = 0; j < m; ++j) { k[j].x = cloud[4 * j]; k[j].i = (int32_t)j; }
    qsort(k, (size_t)m, sizeof(orc_xkey), xkey_cmp);
    X->cloud = cloud;
    X->m = m;
    X->xs = (float*)malloc(sizeof(float) * (size_t)(m > 0 ? m : 1));
    X->order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
    for (int64_t j = 0; j < m; ++j) { X->xs[j] = k[j].x; X->order[j] = k[j].i; }
    free(k);
    return X;
}

void orc_xindex_free(orc_xindex* X) {
    if (!X) return;
    free(X->xs); free(X->order); free(X);
}

static int lexless(float da, int32_t ia, float db, int32_t ib) {
    return da < db || (da == db && ia < ib);
}

static void xknn_visit(const orc_xindex* X, int64_t c, const float q[3], int32_t k, int32_t* idx,
                       float* d2, int32_t* cnt) {
    const int32_t j = X->order[c];
    const float* p = X->cloud + 4 * (int64_t)j;
    float dx = q[0] - p[0];
    float dy = q[1] - p[1];
    float dz = q[2] - p[2];
    float d = dx * dx + dy * dy;
    d = d + dz * dz;
    if (*cnt == k && !lexless(d, j, d2[k - 1], idx[k - 1])) return;
    int32_t pos = *cnt < k ? *cnt : k - 1;
    while (pos > 0 && lexless(d, j, d2[pos - 1], idx[pos - 1])) {
        d2[pos] = d2[pos - 1];
        idx[pos] = idx[pos - 1];
        pos--;
    }
    d2[pos] = d;
    idx[pos] = j;
    if (*cnt < k) (*cnt)++;
}

void orc_xindex_knn(const orc_xindex* X, const float q[3], int32_t k, int32_t* idx, float* d2) {
    int32_t cnt = 0;
    int64_t lo = 0, hi = X->m;                       /* first sorted x >= q.x */
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (X->xs[mid] < q[0]) lo = mid + 1; else hi = mid;
    }
    for (int64_t c = lo; c < X->m; ++c) {
        float dx = q[0] - X->xs[c];
        if (cnt == k && dx * dx > d2[k - 1]) break;
        xknn_visit(X, c, q, k, idx, d2, &cnt);
    }
    for (int64_t c = lo - 1; c >= 0; --c) {
        float dx = q[0] - X->xs[c];
        if (cnt == k && dx * dx > d2[k - 1]) break;
        xknn_visit(X, c, q, k, idx, d2, &cnt);
    }
    for (int32_t r = cnt; r < k; ++r) { idx[r] = -1; d2[r] = INFINITY; }
}

/* Eigen ColPivHouseholderQR<Matrix<float,5,3>>::solve(-1) restated (Eigen 3.3
 * ColPivHouseholder.h computeInPlace / _solve_impl, Householder.h makeHouseholder /
 * applyHouseholderOnTheLeft), reductions in index order.  Eigen's SIMD reduction order is
 * not reproducible without Eigen (unpinned, ~1 ulp); the HIP kernel runs this exact
 * sequence, so oracle and GPU agree bit for bit. */
static float sqnorm_f(const float* v, int n) {
    float s = 0.0f;
    for (int i = 0; i < n; ++i) s = s + v[i] * v[i];
    return s;
}

static void qr_solve_5x3(const float A[5][3], float x[3]) {
    float m[3][5]; /* column-major m[col][row] */
    for (int r = 0; r < 5; ++r)
        for (int c = 0; c < 3; ++c) m[c][r] = A[r][c];
    float hc[3] = {0, 0, 0};
    int tr[3];
    float nu[3], nd[3];
    for (int k = 0; k < 3; ++k) { nd[k] = sqrtf(sqnorm_f(m[k], 5)); nu[k] = nd[k]; }
    float mx = nu[0];
    for (int k = 1; k < 3; ++k) if (nu[k] > mx) mx = nu[k];
    float th = mx * FLT_EPSILON;
    th = (th * th) / 5.0f;
    const float ndt = sqrtf(FLT_EPSILON);
    int nz = 3;
    for (int k = 0; k < 3; ++k) {
        int bi = k;
        float bv = nu[k];
        for (int j = k + 1; j < 3; ++j) if (nu[j] > bv) { bv = nu[j]; bi = j; }
        float bsq = bv * bv;
        if (nz == 3 && bsq < th * (float)(5 - k)) nz = k;
        tr[k] = bi;
        if (k != bi) {
            for (int r = 0; r < 5; ++r) { float t = m[k][r]; m[k][r] = m[bi][r]; m[bi][r] = t; }
            float t = nu[k]; nu[k] = nu[bi]; nu[bi] = t;
            t = nd[k]; nd[k] = nd[bi]; nd[bi] = t;
        }
        /* makeHouseholderInPlace on m[k][k..4] */
        int L = 5 - k;
        float* v = &m[k][k];
        float tail = sqnorm_f(v + 1, L - 1);
        float c0 = v[0], beta, tau;
        if (tail <= FLT_MIN) {
            tau = 0.0f; beta = c0;
            for (int i = 1; i < L; ++i) v[i] = 0.0f;
        } else {
            beta = sqrtf(c0 * c0 + tail);
            if (c0 >= 0.0f) beta = -beta;
            float den = c0 - beta;
            for (int i = 1; i < L; ++i) v[i] = v[i] / den;
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        v[0] = beta;
        /* applyHouseholderOnTheLeft on rows k..4, cols k+1..2 */
        if (tau != 0.0f) {
            for (int c = k + 1; c < 3; ++c) {
                float tmp = 0.0f;
                for (int i = 1; i < L; ++i) tmp = tmp + v[i] * m[c][k + i];
                tmp = tmp + m[c][k];
                m[c][k] = m[c][k] - tau * tmp;
                for (int i = 1; i < L; ++i) m[c][k + i] = m[c][k + i] - (tau * v[i]) * tmp;
            }
        }
        /* norm downdate (LAPACK xGEQPF) */
        for (int j = k + 1; j < 3; ++j) {
            if (nu[j] != 0.0f) {
                float t = fabsf(m[j][k]) / nu[j];
                t = (1.0f + t) * (1.0f - t);
                if (t < 0.0f) t = 0.0f;
                float rr = nu[j] / nd[j];
                float t2 = t * (rr * rr);
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
    for (int k = 0; k < 3; ++k) { int t = perm[k]; perm[k] = perm[tr[k]]; perm[tr[k]] = t; }
    x[0] = x[1] = x[2] = 0.0f;
    if (nz == 0) return;
    float c[5] = {-1.0f, -1.0f, -1.0f, -1.0f, -1.0f};
    for (int k = 0; k < nz; ++k) {
        float tau = hc[k];
        int L = 5 - k;
        if (L == 1) {
            c[k] = c[k] * (1.0f - tau);
        } else if (tau != 0.0f) {
            const float* v = &m[k][k];
            float tmp = 0.0f;
            for (int i = 1; i < L; ++i) tmp = tmp + v[i] * c[k + i];
            tmp = tmp + c[k];
            c[k] = c[k] - tau * tmp;
            for (int i = 1; i < L; ++i) c[k + i] = c[k + i] - (tau * v[i]) * tmp;
        }
    }
    for (int i = nz - 1; i >= 0; --i) {
        if (c[i] != 0.0f) {
            c[i] = c[i] / m[i][i];
            for (int s = 0; s < i; ++s) c[s] = c[s] - c[i] * m[i][s];
        }
    }
    for (int i = 0; i < nz; ++i) x[perm[i]] = c[i];
}

/* lidarOdometry_onlyPC.cpp:173-232 evaluated once per last-frame point a (everything there
 * depends only on the last frame and a).  normal[3a..], valid[a]; pick5 the 5 indices used;
 * gate_rank = n (the rank whose d2 is gated < 1). */
void orc_plane_table(const float* last, int64_t m, float plane_max, float* normal, int32_t* valid,
                     int32_t* pick5, int32_t* gate_rank) {
    int32_t idx[30];
    float d2[30];
    orc_xindex* X = orc_xindex_build(last, m);
    for (int64_t a = 0; a < m; ++a) {
        float q[3] = {last[4 * a], last[4 * a + 1], last[4 * a + 2]};
        orc_xindex_knn(X, q, 30, idx, d2);
        int32_t K = m < 30 ? (int32_t)m : 30;
        float nrm[3] = {0, 0, 0};
        int32_t ok = 0;
        int32_t v5[5] = {-1, -1, -1, -1, -1};
        int32_t n = 5;
        if (K >= 5) {                                                      /* :177 */
            int32_t prow = -1, vr[2], nvr = 0;
            for (int32_t ik = 0; ik < K; ++ik) {                            /* :180-198 */
                float f = last[4 * idx[ik] + 3];
                int32_t ii = (int32_t)f;
                int32_t row = (int32_t)(100.0 * ((double)(f - (float)ii) + 0.002));
                if (ik == 0) prow = row;
                if (ik < 5) {
                    v5[ik] = idx[ik];
                } else if (row != prow && row >= 0 && row <= 63) {
                    vr[nvr++] = idx[ik];
                    n = ik;
                    if (nvr >= 2) break;
                }
            }
            if (nvr == 1) v5[4] = vr[0];                                   /* :199-205 */
            if (nvr == 2) { v5[3] = vr[0]; v5[4] = vr[1]; }
            if (d2[n] < 1.0f) {                                            /* :207 */
                float A[5][3];
                for (int j = 0; j < 5; ++j)
                    for (int c = 0; c < 3; ++c) A[j][c] = last[4 * v5[j] + c];
                qr_solve_5x3(A, nrm);                                      /* :219 */
                float z = nrm[0] * nrm[0] + nrm[1] * nrm[1];
                z = z + nrm[2] * nrm[2];
                if (z > 0.0f) {                                            /* :220 normalize */
                    float s = sqrtf(z);
                    nrm[0] = nrm[0] / s; nrm[1] = nrm[1] / s; nrm[2] = nrm[2] / s;
                }
                ok = 1;
                for (int k = 0; k < 4; ++k) {                              /* :222-232 */
                    double vx = (double)(A[k][0] - A[k + 1][0]);
                    double vy = (double)(A[k][1] - A[k + 1][1]);
                    double vz = (double)(A[k][2] - A[k + 1][2]);
                    double dd = (double)nrm[0] * vx + (double)nrm[1] * vy;
                    dd = dd + (double)nrm[2] * vz;
                    if (fabs(dd) > (double)plane_max) { ok = 0; break; }
                }
            }
        }
        normal[3 * a] = nrm[0]; normal[3 * a + 1] = nrm[1]; normal[3 * a + 2] = nrm[2];
        valid[a] = ok;
        if (pick5) for (int j = 0; j < 5; ++j) pick5[5 * a + j] = v5[j];
        if (gate_rank) gate_rank[a] = n;
    }
    orc_xindex_free(X);
}

/* Eigen Quaterniond * Vector3d (_transformVector): uv = 2 (qv x v); v + w uv + qv x uv. */
static void quat_rotate(const double q[4], const double v[3], double out[3]) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] = uv[0] + uv[0]; uv[1] = uv[1] + uv[1]; uv[2] = uv[2] + uv[2];
    double cr[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2],
                    q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; ++i) out[i] = (v[i] + q[3] * uv[i]) + cr[i];
}

/* transformToLast (lidarOdometry_onlyPC.cpp:74-82) -- double math, stored to float. */
void orc_transform_point(const double q[4], const double t[3], const float p[3], float out[3]) {
    double v[3] = {(double)p[0], (double)p[1], (double)p[2]}, r[3];
    quat_rotate(q, v, r);
    for (int i = 0; i < 3; ++i) out[i] = (float)(r[i] + t[i]);
}

/* 1-NN association, lidarOdometry_onlyPC.cpp:161-169 (unbounded distance). */
void orc_correspond(const float* last, int64_t m_last, const float* curr, int64_t m_curr,
                    const double q[4], const double t[3], int32_t* nn) {
    orc_xindex* X = orc_xindex_build(last, m_last);
    for (int64_t i = 0; i < m_curr; ++i) {
        float p[3] = {curr[4 * i], curr[4 * i + 1], curr[4 * i + 2]}, s[3];
        orc_transform_point(q, t, p, s);
        int32_t idx;
        float d2;
        orc_xindex_knn(X, s, 1, &idx, &d2);
        nn[i] = idx;
    }
    orc_xindex_free(X);
}

/* Eigen quaternion product a*b, (x,y,z,w) storage. */
static void quat_mul(const double a[4], const double b[4], double o[4]) {
    double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

/* ceres::EigenQuaternionParameterization::Plus: [cos|d|, sin|d|/|d| d] * q */
static void quat_plus(const double q[4], const double d[3], double o[4]) {
    double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (nd > 0.0) {
        double s = sin(nd) / nd;
        double dq[4] = {s * d[0], s * d[1], s * d[2], cos(nd)};
        quat_mul(dq, q, o);
    } else {
        memcpy(o, q, 4 * sizeof(double));
    }
}

/* Residual + local Jacobian of PlaneFeatureCost (lidarOdometry_onlyPC.cpp:25-43) composed with
 * the EigenQuaternionParameterization 4x3 Jacobian.  J[0..2] rotation (local), J[3..5] = n. */
static double residual_jac(const double q[4], const double t[3], const double po[3],
                           const double pa[3], const double n[3], double J[6]) {
    double f[3];
    quat_rotate(q, po, f);
    double d0 = (f[0] + t[0]) - pa[0], d1 = (f[1] + t[1]) - pa[1], d2 = (f[2] + t[2]) - pa[2];
    double r = d0 * n[0] + d1 * n[1];
    r = r + d2 * n[2];
    if (J) {
        const double x = q[0], y = q[1], z = q[2], w = q[3];
        /* ambient gradient of n.(p + 2w(qv x p) + 2 qv x (qv x p)) */
        double u[3] = {y * po[2] - z * po[1], z * po[0] - x * po[2], x * po[1] - y * po[0]}; /* qv x p */
        double pxn[3] = {po[1] * n[2] - po[2] * n[1], po[2] * n[0] - po[0] * n[2],
                         po[0] * n[1] - po[1] * n[0]};
        double uxn[3] = {u[1] * n[2] - u[2] * n[1], u[2] * n[0] - u[0] * n[2],
                         u[0] * n[1] - u[1] * n[0]};
        double nxq[3] = {n[1] * z - n[2] * y, n[2] * x - n[0] * z, n[0] * y - n[1] * x};
        double pnq[3] = {po[1] * nxq[2] - po[2] * nxq[1], po[2] * nxq[0] - po[0] * nxq[2],
                         po[0] * nxq[1] - po[1] * nxq[0]};
        double g[4];
        for (int i = 0; i < 3; ++i) g[i] = 2.0 * w * pxn[i] + 2.0 * uxn[i] + 2.0 * pnq[i];
        g[3] = 2.0 * (n[0] * u[0] + n[1] * u[1] + n[2] * u[2]);
        /* Jplus rows (x,y,z,w): [w z -y; -z w x; y -x w; -x -y -z] */
        J[0] = g[0] * w - g[1] * z + g[2] * y - g[3] * x;
        J[1] = g[0] * z + g[1] * w - g[2] * x - g[3] * y;
        J[2] = -g[0] * y + g[1] * x + g[2] * w - g[3] * z;
        J[3] = n[0]; J[4] = n[1]; J[5] = n[2];
    }
    return r;
}

typedef struct { double A[21]; double g[6]; double cost; } ne_t; /* packed upper, row-major */

/* Huber(0.1) (lidarOdometry_onlyPC.cpp:239): rho(s) and rho'(s), Ceres HuberLoss. */
static void huber(double s, double* rho0, double* rho1) {
    const double a = 0.1, b = 0.1 * 0.1;
    if (s > b) {
        double rr = sqrt(s);
        *rho0 = 2.0 * a * rr - b;
        *rho1 = a / rr;
        if (*rho1 < DBL_MIN) *rho1 = DBL_MIN;
    } else {
        *rho0 = s; *rho1 = 1.0;
    }
}

/* Evaluate Huber(0.1)-corrected cost / normal equations at (q, t).  Every residual block is
 * inserted twice by the reference (the i_opt loop, lidarOdometry_onlyPC.cpp:160), hence dup=2.
 * Edge blocks (beyond the reference, see orc_edge_table): the 3-vector point-to-line residual
 * e = P (R po + t - c), P = I - u u^T, one Huber block on s = |e|^2; row k is the plane
 * residual with "normal" P row k, so residual_jac gives its value and local Jacobian. */
static void evaluate(const float* po, const float* pa, const float* nrm, int64_t c,
                     const float* epo, const float* ec, const float* eu, int64_t ce,
                     const double q[4], const double t[3], int need_jac, ne_t* out) {
    memset(out, 0, sizeof(*out));
    for (int64_t i = 0; i < c; ++i) {
        double p0[3] = {po[3 * i], po[3 * i + 1], po[3 * i + 2]};
        double p1[3] = {pa[3 * i], pa[3 * i + 1], pa[3 * i + 2]};
        double nn[3] = {nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]};
        double J[6];
        double r = residual_jac(q, t, p0, p1, nn, need_jac ? J : NULL);
        double rho0, rho1;
        huber(r * r, &rho0, &rho1);
        out->cost += 0.5 * rho0;
        if (need_jac) {
            int k = 0;
            for (int u = 0; u < 6; ++u) {
                out->g[u] += rho1 * J[u] * r;
                for (int v = u; v < 6; ++v) out->A[k++] += rho1 * J[u] * J[v];
            }
        }
    }
    for (int64_t i = 0; i < ce; ++i) {
        double p0[3] = {epo[3 * i], epo[3 * i + 1], epo[3 * i + 2]};
        double cc[3] = {ec[3 * i], ec[3 * i + 1], ec[3 * i + 2]};
        double uu[3] = {eu[3 * i], eu[3 * i + 1], eu[3 * i + 2]};
        double r[3], J[3][6], s = 0.0;
        for (int k = 0; k < 3; ++k) {
            double nk[3];
            for (int j = 0; j < 3; ++j) nk[j] = (j == k ? 1.0 : 0.0) - uu[k] * uu[j];
            r[k] = residual_jac(q, t, p0, cc, nk, need_jac ? J[k] : NULL);
            s += r[k] * r[k];
        }
        double rho0, rho1;
        huber(s, &rho0, &rho1);
        out->cost += 0.5 * rho0;
        if (need_jac) {
            for (int k = 0; k < 3; ++k) {
                int m = 0;
                for (int u = 0; u < 6; ++u) {
                    out->g[u] += rho1 * J[k][u] * r[k];
                    for (int v = u; v < 6; ++v) out->A[m++] += rho1 * J[k][u] * J[k][v];
                }
            }
        }
    }
    out->cost *= 2.0;
    for (int k = 0; k < 21; ++k) out->A[k] *= 2.0;
    for (int k = 0; k < 6; ++k) out->g[k] *= 2.0;
}

static inline int pk(int u, int v) { /* packed upper index, u <= v */
    if (u > v) { int t = u; u = v; v = t; }
    return u * 6 - (u * (u - 1)) / 2 + (v - u);
}

/* Solve M y = b for SPD M (6x6, full) by Cholesky; returns 0 on success. */
static int chol_solve6(double M[6][6], const double b[6], double y[6]) {
    double L[6][6];
    memset(L, 0, sizeof(L));
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

static void log_rec(double* log, int32_t* n_log, const double q[4], const double t[3], double cost,
                    double status, double radius) {
    if (log) {
        double* r = log + ORC_LOG_STRIDE * (*n_log);
        r[0] = q[0]; r[1] = q[1]; r[2] = q[2]; r[3] = q[3];
        r[4] = t[0]; r[5] = t[1]; r[6] = t[2];
        r[7] = cost; r[8] = status; r[9] = radius;
    }
    (*n_log)++;
}

/* ceres::Solve restated (Ceres 1.14 TrustRegionMinimizer + LevenbergMarquardtStrategy,
 * DENSE_QR replaced by Cholesky of the damped normal equations), lidarOdometry_onlyPC.cpp:244-252.
 * Log status: 1 accepted, 0 rejected, 2 invalid step, 3 parameter tol, 4 function tol,
 * 5 gradient tol, 6 GN step. */
int32_t orc_solve2(const float* po, const float* pa, const float* nrm, int64_t c,
                   const float* epo, const float* ec, const float* eu, int64_t ce, int32_t mode,
                   int32_t max_iter, const double q_init[4], const double t_init[3], double q_out[4],
                   double t_out[3], double* log, int32_t* n_log) {
    double q[4], t[3];
    memcpy(q, q_init, sizeof(q)); memcpy(t, t_init, sizeof(t));
    int32_t nl = 0;
    ne_t ne, cand;
    evaluate(po, pa, nrm, c, epo, ec, eu, ce, q, t, 1, &ne);
    if (mode == ORC_MODE_GN) {
        for (int32_t it = 0; it < max_iter; ++it) {
            double M[6][6], b[6], y[6];
            for (int u = 0; u < 6; ++u) {
                b[u] = -ne.g[u];
                for (int v = 0; v < 6; ++v) M[u][v] = ne.A[pk(u, v)];
            }
            if (chol_solve6(M, b, y) != 0) { log_rec(log, &nl, q, t, ne.cost, 2, 0); break; }
            double qn[4];
            quat_plus(q, y, qn);
            memcpy(q, qn, sizeof(q));
            t[0] += y[3]; t[1] += y[4]; t[2] += y[5];
            evaluate(po, pa, nrm, c, epo, ec, eu, ce, q, t, 1, &ne);
            log_rec(log, &nl, q, t, ne.cost, 6, 0);
        }
    } else {
        double s[6];
        for (int u = 0; u < 6; ++u) s[u] = 1.0 / (1.0 + sqrt(ne.A[pk(u, u)]));
        double radius = 1e4, dec = 2.0;
        int invalid = 0;
        for (int32_t it = 1; it <= max_iter; ++it) {
            double As[6][6], gs[6], y[6];
            for (int u = 0; u < 6; ++u) {
                gs[u] = s[u] * ne.g[u];
                for (int v = 0; v < 6; ++v) As[u][v] = s[u] * ne.A[pk(u, v)] * s[v];
            }
            double M[6][6], bb[6];
            for (int u = 0; u < 6; ++u) {
                double d = As[u][u];
                if (d < 1e-6) d = 1e-6;
                if (d > 1e32) d = 1e32;
                for (int v = 0; v < 6; ++v) M[u][v] = As[u][v];
                M[u][u] += d / radius;
                bb[u] = -gs[u];
            }
            int ok = chol_solve6(M, bb, y) == 0;
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
                radius /= dec; dec *= 2.0;
                log_rec(log, &nl, q, t, ne.cost, 2, radius);
                if (++invalid > 5) break;
                continue;
            }
            invalid = 0;
            double delta[6];
            for (int u = 0; u < 6; ++u) delta[u] = y[u] * s[u];
            double qc[4], tc[3];
            quat_plus(q, delta, qc);
            tc[0] = t[0] + delta[3]; tc[1] = t[1] + delta[4]; tc[2] = t[2] + delta[5];
            evaluate(po, pa, nrm, c, epo, ec, eu, ce, qc, tc, 1, &cand);
            double xn = 0.0, sn = 0.0;
            for (int u = 0; u < 4; ++u) { xn += q[u] * q[u]; sn += (q[u] - qc[u]) * (q[u] - qc[u]); }
            for (int u = 0; u < 3; ++u) { xn += t[u] * t[u]; sn += (t[u] - tc[u]) * (t[u] - tc[u]); }
            xn = sqrt(xn); sn = sqrt(sn);
            if (!(sn > (xn + 1e-8) * 1e-8)) { log_rec(log, &nl, q, t, ne.cost, 3, radius); break; }
            double dcost = ne.cost - cand.cost;
            if (!(fabs(dcost) > 1e-6 * ne.cost)) { log_rec(log, &nl, q, t, ne.cost, 4, radius); break; }
            double rho = dcost / mcc;
            if (rho > 1e-3) {
                memcpy(q, qc, sizeof(q)); memcpy(t, tc, sizeof(t));
                ne = cand;
                double f = 2.0 * rho - 1.0;
                double den = 1.0 - f * f * f;
                if (den < 1.0 / 3.0) den = 1.0 / 3.0;
                radius = radius / den;
                if (radius > 1e16) radius = 1e16;
                dec = 2.0;
                /* gradient max-norm: |x - Plus(x, -g)|_inf <= 1e-10 */
                double mg[3] = {-ne.g[0], -ne.g[1], -ne.g[2]}, qg[4], gm = 0.0;
                quat_plus(q, mg, qg);
                for (int u = 0; u < 4; ++u) gm = fmax(gm, fabs(q[u] - qg[u]));
                for (int u = 3; u < 6; ++u) gm = fmax(gm, fabs(ne.g[u]));
                if (gm <= 1e-10) { log_rec(log, &nl, q, t, ne.cost, 5, radius); break; }
                log_rec(log, &nl, q, t, ne.cost, 1, radius);
            } else {
                radius /= dec; dec *= 2.0;
                log_rec(log, &nl, q, t, ne.cost, 0, radius);
            }
        }
    }
    memcpy(q_out, q, sizeof(q)); memcpy(t_out, t, sizeof(t));
    if (n_log) *n_log = nl;
    return 0;
}

int32_t orc_solve(const float* po, const float* pa, const float* nrm, int64_t c, int32_t mode,
                  int32_t max_iter, const double q_init[4], const double t_init[3], double q_out[4],
                  double t_out[3], double* log, int32_t* n_log) {
    return orc_solve2(po, pa, nrm, c, NULL, NULL, NULL, 0, mode, max_iter, q_init, t_init, q_out,
                      t_out, log, n_log);
}

int64_t orc_register_pair(const float* last, int64_t m_last, const float* curr, int64_t m_curr,
                          float plane_max, int32_t mode, int32_t max_iter, const double q_init[4],
                          const double t_init[3], double q_out[4], double t_out[3], double* log,
                          int32_t* n_log) {
    if (n_log) *n_log = 0;
    if (m_last <= 10) {                                                    /* :158 */
        memcpy(q_out, q_init, 4 * sizeof(double)); memcpy(t_out, t_init, 3 * sizeof(double));
        return -1;
    }
    size_t ml = (size_t)m_last, mc = (size_t)(m_curr > 0 ? m_curr : 1);
    float* normal = (float*)malloc(sizeof(float) * 3 * ml);
    int32_t* valid = (int32_t*)malloc(sizeof(int32_t) * ml);
    int32_t* nn = (int32_t*)malloc(sizeof(int32_t) * mc);
    float* po = (float*)malloc(sizeof(float) * 3 * mc);
    float* pa = (float*)malloc(sizeof(float) * 3 * mc);
    float* nr = (float*)malloc(sizeof(float) * 3 * mc);
    orc_plane_table(last, m_last, plane_max, normal, valid, NULL, NULL);
    orc_correspond(last, m_last, curr, m_curr, q_init, t_init, nn);
    int64_t c = 0;
    for (int64_t i = 0; i < m_curr; ++i) {
        int32_t a = nn[i];
        if (a < 0 || !valid[a]) continue;
        for (int k = 0; k < 3; ++k) {
            po[3 * c + k] = curr[4 * i + k];
            pa[3 * c + k] = last[4 * a + k];
            nr[3 * c + k] = normal[3 * a + k];
        }
        c++;
    }
    orc_solve(po, pa, nr, c, mode, max_iter, q_init, t_init, q_out, t_out, log, n_log);
    free(normal); free(valid); free(nn); free(po); free(pa); free(nr);
    return c;
}

/* publishResult accumulation: lidarOdometry_onlyPC.cpp:87-90 / lidarOdometry.cpp:80-83 */
void orc_accumulate(const double q0l[4], const double t0l[3], const double qlc[4],
                    const double tlc[3], double q0c[4], double t0c[3]) {
    double r[3];
    quat_rotate(q0l, tlc, r);
    double q[4];
    quat_mul(q0l, qlc, q);
    for (int i = 0; i < 3; ++i) t0c[i] = t0l[i] + r[i];
    memcpy(q0c, q, sizeof(q));
}

/* ======================================================================== */
/* numpy legacy RandomState (MT19937, init_genrand seeding, 53-bit random_sample). */
void orc_mt_seed(orc_mt19937* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->pos = 624;
}

static uint32_t mt_next(orc_mt19937* s) {
    if (s->pos >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->pos = 0;
    }
    uint32_t y = s->mt[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double orc_mt_random_sample(orc_mt19937* s) {
    uint32_t a = mt_next(s) >> 5, b = mt_next(s) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

/* 6x6 Cholesky of covariance (lower) -> precision Cholesky U = L^{-T} (upper), scipy
 * linalg.cholesky + solve_triangular(L, I).T as in sklearn _compute_precision_cholesky. */
static int prec_chol6(const double C[36], double U[36], double* logdet) {
    double L[36];
    memset(L, 0, sizeof(L));
    for (int j = 0; j < 6; ++j) {
        double s = C[j * 6 + j];
        for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
        if (!(s > 0.0)) return -1;
        L[j * 6 + j] = sqrt(s);
        for (int i = j + 1; i < 6; ++i) {
            double v = C[i * 6 + j];
            for (int k = 0; k < j; ++k) v -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = v / L[j * 6 + j];
        }
    }
    double Li[36]; /* inverse of L (lower) */
    memset(Li, 0, sizeof(Li));
    for (int c = 0; c < 6; ++c) {
        for (int i = c; i < 6; ++i) {
            double v = (i == c) ? 1.0 : 0.0;
            for (int k = c; k < i; ++k) v -= L[i * 6 + k] * Li[k * 6 + c];
            Li[i * 6 + c] = v / L[i * 6 + i];
        }
    }
    double ld = 0.0;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) U[i * 6 + j] = Li[j * 6 + i];
    for (int i = 0; i < 6; ++i) ld += log(U[i * 6 + i]);
    *logdet = ld;
    return 0;
}

typedef struct { double w[2], mu[12], U[72], logdet[2], logw[2]; } gmm_par;

/* M-step / _initialize from responsibilities given as per-point resp0 (resp1 = 1 - resp0 for
 * one-hot init; general resp via r0/r1 arrays). sklearn _estimate_gaussian_parameters. */
static int gmm_mstep(const double* X, int64_t n, const double* r0, const double* r1, int init,
                     gmm_par* P) {
    const double eps10 = 10.0 * DBL_EPSILON;
    for (int k = 0; k < 2; ++k) {
        const double* r = k == 0 ? r0 : r1;
        double nk = 0.0, sx[6] = {0};
        for (int64_t i = 0; i < n; ++i) {
            nk += r[i];
            for (int d = 0; d < 6; ++d) sx[d] += r[i] * X[6 * i + d];
        }
        nk += eps10;
        double* mu = P->mu + 6 * k;
        for (int d = 0; d < 6; ++d) mu[d] = sx[d] / nk;
        double C[36] = {0};
        for (int64_t i = 0; i < n; ++i) {
            double df[6];
            for (int d = 0; d < 6; ++d) df[d] = X[6 * i + d] - mu[d];
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) C[a * 6 + b] += r[i] * df[a] * df[b];
        }
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 6; ++b) { C[a * 6 + b] /= nk; C[b * 6 + a] = C[a * 6 + b]; }
        for (int a = 0; a < 6; ++a) C[a * 6 + a] += 1e-6;
        if (prec_chol6(C, P->U + 36 * k, &P->logdet[k]) != 0) return -1;
        P->w[k] = nk;
    }
    if (init) {
        P->w[0] /= (double)n; P->w[1] /= (double)n;
    } else {
        double s = P->w[0] + P->w[1];
        P->w[0] /= s; P->w[1] /= s;
    }
    P->logw[0] = log(P->w[0]); P->logw[1] = log(P->w[1]);
    return 0;
}

/* weighted log prob of point x for component k (sklearn _estimate_log_gaussian_prob). */
static double gmm_wlp(const double* x, const gmm_par* P, int k) {
    const double* U = P->U + 36 * k;
    const double* mu = P->mu + 6 * k;
    double lp = 0.0;
    for (int j = 0; j < 6; ++j) {
        double y = 0.0;
        for (int i = 0; i <= j; ++i) y += (x[i] - mu[i]) * U[i * 6 + j];
        lp += y * y;
    }
    return -0.5 * (6.0 * log(2.0 * M_PI) + lp) + P->logdet[k] + P->logw[k];
}

/* scipy 1.15 logsumexp over two terms: max + log1p(sum of the others / m) + log(m). */
static double lse2(double a, double b) {
    double mx = a > b ? a : b;
    if (a == b) return log1p(0.0) + log(2.0) + mx;
    double mn = a > b ? b : a;
    return log1p(exp(mn - mx)) + mx;
}

/* GaussianMixture(n_components=2).fit_predict  (PointCloudOdometry_noSeg.py:97-101), sklearn 1.7.2. */
int32_t orc_gmm_labels(const double* X, int64_t n, const double draws[3], uint8_t* labels,
                       double* info, double* means_out) {
    if (n < 2) return -1;
    size_t N = (size_t)n;
    double* Xc = (double*)malloc(sizeof(double) * 6 * N);
    double* xsq = (double*)malloc(sizeof(double) * N);
    double* dist = (double*)malloc(sizeof(double) * N);
    int32_t* lab = (int32_t*)malloc(sizeof(int32_t) * N);
    int32_t* lab_old = (int32_t*)malloc(sizeof(int32_t) * N);
    double* r0 = (double*)malloc(sizeof(double) * N);
    double* r1 = (double*)malloc(sizeof(double) * N);
    /* KMeans.fit: X_mean, tol = mean(var(X)) * 1e-4 */
    double mean[6] = {0}, var[6] = {0};
    for (size_t i = 0; i < N; ++i)
        for (int d = 0; d < 6; ++d) mean[d] += X[6 * i + d];
    for (int d = 0; d < 6; ++d) mean[d] /= (double)n;
    for (size_t i = 0; i < N; ++i)
        for (int d = 0; d < 6; ++d) { double v = X[6 * i + d] - mean[d]; var[d] += v * v; }
    double tol = 0.0;
    for (int d = 0; d < 6; ++d) tol += var[d] / (double)n;
    tol = tol / 6.0 * 1e-4;
    for (size_t i = 0; i < N; ++i) {
        double s = 0.0;
        for (int d = 0; d < 6; ++d) { Xc[6 * i + d] = X[6 * i + d] - mean[d]; s += Xc[6 * i + d] * Xc[6 * i + d]; }
        xsq[i] = s;
    }
    /* k-means++ (_kmeans_plusplus): choice(n, p=1/n) -> searchsorted(cdf, u, 'right') */
    int64_t c0 = n - 1;
    {
        double p = 1.0 / (double)n, cs = 0.0;
        double* cdf = dist;
        for (size_t i = 0; i < N; ++i) { cs += p; cdf[i] = cs; }
        double last = cdf[N - 1];
        for (size_t i = 0; i < N; ++i) cdf[i] /= last;
        for (size_t i = 0; i < N; ++i) if (cdf[i] > draws[0]) { c0 = (int64_t)i; break; }
    }
    double cen[12];
    memcpy(cen, Xc + 6 * c0, 6 * sizeof(double));
    double cn0 = 0.0;
    for (int d = 0; d < 6; ++d) cn0 += cen[d] * cen[d];
    double pot = 0.0;
    for (size_t i = 0; i < N; ++i) {
        double dt = 0.0;
        for (int d = 0; d < 6; ++d) dt += cen[d] * Xc[6 * i + d];
        double v = (-2.0 * dt + cn0) + xsq[i];
        dist[i] = v > 0.0 ? v : 0.0;
        pot += dist[i];
    }
    int64_t cand[2];
    for (int j = 0; j < 2; ++j) {
        double rv = draws[1 + j] * pot, cs = 0.0;
        cand[j] = n - 1;
        for (size_t i = 0; i < N; ++i) { cs += dist[i]; if (cs >= rv) { cand[j] = (int64_t)i; break; } }
    }
    double cpot[2];
    for (int j = 0; j < 2; ++j) {
        const double* cc = Xc + 6 * cand[j];
        double ccn = 0.0, s = 0.0;
        for (int d = 0; d < 6; ++d) ccn += cc[d] * cc[d];
        for (size_t i = 0; i < N; ++i) {
            double dt = 0.0;
            for (int d = 0; d < 6; ++d) dt += cc[d] * Xc[6 * i + d];
            double v = (-2.0 * dt + ccn) + xsq[i];
            v = v > 0.0 ? v : 0.0;
            s += v < dist[i] ? v : dist[i];
        }
        cpot[j] = s;
    }
    int best = cpot[1] < cpot[0] ? 1 : 0;
    int64_t c1 = cand[best];
    memcpy(cen + 6, Xc + 6 * c1, 6 * sizeof(double));
    /* Lloyd (_kmeans_single_lloyd, max_iter 300) */
    for (size_t i = 0; i < N; ++i) lab_old[i] = -1;
    int strict = 0, kit = 0;
    for (int it = 0; it < 300; ++it) {
        kit = it + 1;
        double csn[2] = {0, 0}, sums[12] = {0}, wsum[2] = {0, 0};
        for (int k = 0; k < 2; ++k) for (int d = 0; d < 6; ++d) csn[k] += cen[6 * k + d] * cen[6 * k + d];
        for (size_t i = 0; i < N; ++i) {
            double v[2];
            for (int k = 0; k < 2; ++k) {
                double dt = 0.0;
                for (int d = 0; d < 6; ++d) dt += Xc[6 * i + d] * cen[6 * k + d];
                v[k] = -2.0 * dt + csn[k];
            }
            int l = v[1] < v[0] ? 1 : 0;
            lab[i] = l;
            wsum[l] += 1.0;
            for (int d = 0; d < 6; ++d) sums[6 * l + d] += Xc[6 * i + d];
        }
        double shift = 0.0, newc[12];
        for (int k = 0; k < 2; ++k) {
            double sh = 0.0;
            for (int d = 0; d < 6; ++d) {
                newc[6 * k + d] = wsum[k] > 0.0 ? sums[6 * k + d] * (1.0 / wsum[k]) : cen[6 * k + d];
                double df = newc[6 * k + d] - cen[6 * k + d];
                sh += df * df;
            }
            sh = sqrt(sh); /* _center_shift: euclidean norm, then (center_shift**2).sum() */
            shift += sh * sh;
        }
        memcpy(cen, newc, sizeof(newc));
        int same = 1;
        for (size_t i = 0; i < N; ++i) if (lab[i] != lab_old[i]) { same = 0; break; }
        if (same) { strict = 1; break; }
        if (shift <= tol) break;
        memcpy(lab_old, lab, sizeof(int32_t) * N);
    }
    if (!strict) {
        double csn[2] = {0, 0};
        for (int k = 0; k < 2; ++k) for (int d = 0; d < 6; ++d) csn[k] += cen[6 * k + d] * cen[6 * k + d];
        for (size_t i = 0; i < N; ++i) {
            double v[2];
            for (int k = 0; k < 2; ++k) {
                double dt = 0.0;
                for (int d = 0; d < 6; ++d) dt += Xc[6 * i + d] * cen[6 * k + d];
                v[k] = -2.0 * dt + csn[k];
            }
            lab[i] = v[1] < v[0] ? 1 : 0;
        }
    }
    /* GMM init from one-hot resp (GaussianMixture._initialize) */
    for (size_t i = 0; i < N; ++i) { r0[i] = lab[i] == 0 ? 1.0 : 0.0; r1[i] = 1.0 - r0[i]; }
    gmm_par P;
    int32_t rc = 0;
    if (gmm_mstep(X, n, r0, r1, 1, &P) != 0) { rc = -4; goto done; }
    double lb = -INFINITY;
    int emit = 0, conv = 0;
    for (int it = 1; it <= 100; ++it) {
        emit = it;
        double prev = lb, slse = 0.0;
        for (size_t i = 0; i < N; ++i) {
            double a0 = gmm_wlp(X + 6 * i, &P, 0), a1 = gmm_wlp(X + 6 * i, &P, 1);
            double l = lse2(a0, a1);
            slse += l;
            r0[i] = exp(a0 - l);
            r1[i] = exp(a1 - l);
        }
        lb = slse / (double)n;
        if (gmm_mstep(X, n, r0, r1, 0, &P) != 0) { rc = -4; goto done; }
        if (fabs(lb - prev) < 1e-3) { conv = 1; break; }
    }
    int64_t n1 = 0;
    for (size_t i = 0; i < N; ++i) {
        double a0 = gmm_wlp(X + 6 * i, &P, 0), a1 = gmm_wlp(X + 6 * i, &P, 1);
        labels[i] = a1 > a0 ? 1 : 0;
        n1 += labels[i];
    }
    /* Counter(all_label).most_common(1): ties -> first label seen */
    int bg;
    if (n1 * 2 > n) bg = 1;
    else if (n1 * 2 < n) bg = 0;
    else bg = labels[0];
    if (info) {
        info[0] = kit; info[1] = emit; info[2] = conv; info[3] = (double)c0; info[4] = (double)c1;
        info[5] = bg; info[6] = (double)(bg ? n1 : n - n1); info[7] = lb;
    }
    if (means_out) memcpy(means_out, P.mu, sizeof(P.mu));
done:
    free(Xc); free(xsq); free(dist); free(lab); free(lab_old); free(r0); free(r1);
    return rc;
}

/* 3x3 SVD by one-sided Jacobi (f64), singular values descending (LAPACK convention). */
void orc_svd3(const double A[9], double U[9], double S[3], double Vt[9]) {
    double a[3][3], v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) a[i][j] = A[i * 3 + j];
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 2; ++p) {
            for (int q = p + 1; q < 3; ++q) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int i = 0; i < 3; ++i) {
                    alpha += a[i][p] * a[i][p]; beta += a[i][q] * a[i][q]; gamma += a[i][p] * a[i][q];
                }
                if (fabs(gamma) <= 1e-300) continue;
                double rel = fabs(gamma) / sqrt(alpha * beta);
                if (rel > off) off = rel;
                if (rel < 1e-17) continue;
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 3; ++i) {
                    double x = a[i][p], y = a[i][q];
                    a[i][p] = c * x - s * y; a[i][q] = s * x + c * y;
                    x = v[i][p]; y = v[i][q];
                    v[i][p] = c * x - s * y; v[i][q] = s * x + c * y;
                }
            }
        }
        if (off < 1e-16) break;
    }
    double sv[3];
    int ord[3] = {0, 1, 2};
    for (int j = 0; j < 3; ++j) sv[j] = sqrt(a[0][j] * a[0][j] + a[1][j] * a[1][j] + a[2][j] * a[2][j]);
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    double u[3][3];
    for (int k = 0; k < 3; ++k) {
        int j = ord[k];
        S[k] = sv[j];
        for (int i = 0; i < 3; ++i) {
            u[i][k] = sv[j] > 0 ? a[i][j] / sv[j] : 0.0;
            Vt[k * 3 + i] = v[i][j];
        }
    }
    if (!(S[2] > 1e-12 * S[0])) { /* rank-deficient H (coplanar points): right-handed u3, v3 */
        u[0][2] = u[1][0] * u[2][1] - u[2][0] * u[1][1];
        u[1][2] = u[2][0] * u[0][1] - u[0][0] * u[2][1];
        u[2][2] = u[0][0] * u[1][1] - u[1][0] * u[0][1];
        Vt[6] = Vt[1] * Vt[5] - Vt[2] * Vt[4];
        Vt[7] = Vt[2] * Vt[3] - Vt[0] * Vt[5];
        Vt[8] = Vt[0] * Vt[4] - Vt[1] * Vt[3];
    }
    for (int i = 0; i < 3; ++i) for (int k = 0; k < 3; ++k) U[i * 3 + k] = u[i][k];
}

static double det3(const double R[9]) {
    return R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
           R[2] * (R[3] * R[7] - R[4] * R[6]);
}

/* slove_RT_by_SVD (PointCloudOdometry_noSeg.py:19-37), restricted to mask rows. */
int32_t orc_kabsch(const double* src, const double* dst, int64_t n, const uint8_t* mask,
                   int32_t reflection, double R[9], double t[3]) {
    double ms[3] = {0}, md[3] = {0};
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        for (int d = 0; d < 3; ++d) { ms[d] += src[3 * i + d]; md[d] += dst[3 * i + d]; }
        cnt++;
    }
    if (cnt == 0) return -1;
    for (int d = 0; d < 3; ++d) { ms[d] /= (double)cnt; md[d] /= (double)cnt; }
    double H[9] = {0};
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        double a[3], b[3];
        for (int d = 0; d < 3; ++d) { a[d] = src[3 * i + d] - ms[d]; b[d] = dst[3 * i + d] - md[d]; }
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) H[r * 3 + c] += a[r] * b[c];
    }
    double U[9], S[3], Vt[9];
    orc_svd3(H, U, S, Vt);
    for (int r = 0; r < 3; ++r)           /* R = Vt.T @ U.T */
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += Vt[k * 3 + r] * U[c * 3 + k];
            R[r * 3 + c] = s;
        }
    int32_t rc = 0;
    if (det3(R) < 0) {                    /* :30-33 (reference: TypeError from `&`) */
        if (!reflection) rc = -2;
        for (int k = 0; k < 3; ++k) Vt[2 * 3 + k] *= -1.0;
        if (reflection) {
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < 3; ++k) s += Vt[k * 3 + r] * U[c * 3 + k];
                    R[r * 3 + c] = s;
                }
        }
    }
    for (int r = 0; r < 3; ++r) t[r] = -(R[r * 3] * ms[0] + R[r * 3 + 1] * ms[1] + R[r * 3 + 2] * ms[2]) + md[r];
    return rc;
}

/* pyquaternion Quaternion(matrix=R): allclose(R R^T, I, 1e-5, 1e-8) then trace method on m = R^T. */
int32_t orc_quat_from_R(const double R[9], double q[4]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += R[i * 3 + k] * R[j * 3 + k];
            double e = (i == j) ? 1.0 : 0.0;
            if (!(fabs(s - e) <= 1e-8 + 1e-5 * fabs(e))) return -3;
        }
    double m[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) m[i][j] = R[j * 3 + i];
    double t, w, x, y, z;
    if (m[2][2] < 0) {
        if (m[0][0] > m[1][1]) {
            t = 1 + m[0][0] - m[1][1] - m[2][2];
            w = m[1][2] - m[2][1]; x = t; y = m[0][1] + m[1][0]; z = m[2][0] + m[0][2];
        } else {
            t = 1 - m[0][0] + m[1][1] - m[2][2];
            w = m[2][0] - m[0][2]; x = m[0][1] + m[1][0]; y = t; z = m[1][2] + m[2][1];
        }
    } else {
        if (m[0][0] < -m[1][1]) {
            t = 1 - m[0][0] - m[1][1] + m[2][2];
            w = m[0][1] - m[1][0]; x = m[2][0] + m[0][2]; y = m[1][2] + m[2][1]; z = t;
        } else {
            t = 1 + m[0][0] + m[1][1] + m[2][2];
            w = t; x = m[1][2] - m[2][1]; y = m[2][0] - m[0][2]; z = m[0][1] - m[1][0];
        }
    }
    double f = 0.5 / sqrt(t);
    q[0] = x * f; q[1] = y * f; q[2] = z * f; q[3] = w * f;
    return 0;
}

/* The ASF block's float32 tail (main_sju_occ_ros.py:273-284): the network flow is
 * float32, so `target = points[bg] + move_gt[bg]` (:273) and every line of slove_RT_by_SVD
 * (:455-473) run on float32 arrays.  Restated step by step:
 *   - src = f32(pos + flow), dst = pos (the numpy f32 add of :273-274);
 *   - src.mean(axis=0): numpy's add.reduce over axis 0 of a C-ordered (n, 3) array accumulates
 *     row after row into the f32 output, starting from the first row (no pairwise summation on
 *     that axis); _mean then divides by the intp count (f64 loop, stored to f32: out=ret);
 *   - centred f32 arrays (:461-462);
 *   - H = src.T @ dst (:463) is an OpenBLAS sgemm whose summation order is not pinned: the exact
 *     f32 products are summed in f64 here (measured 2e-7 from the fixture's R, tests);
 *   - svd (LAPACK sgesdd on f32 H, unpinned) -> the f64 Jacobi SVD, R rounded to f32;
 *   - det(R) < 0 as in orc_kabsch (:467-470);
 *   - t = -R @ src_mean.T + dst_mean.T (:472): the 3-term f32 product rounded once, then the f32
 *     add.
 * R and t are returned as the f32 values (in doubles).  q: pyquaternion on the f32 R (recalled,
 * parity unpinned): allclose(dot(R, R^T), I) with the dot in f32, the trace-method
 * terms in f32, the 0.5 / sqrt(t) scale in f64.  Returns 0, -1 (no rows), -2 (reflection,
 * reflection == 0) or -3 (not orthogonal); q is zero unless 0 is returned. */
int32_t orc_kabsch_f32(const float* pos, const float* flow, int64_t n, const uint8_t* mask,
                       int32_t reflection, double R_out[9], double t_out[3], double q[4]) {
    float ss[3] = {0, 0, 0}, sd[3] = {0, 0, 0};
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        for (int d = 0; d < 3; ++d) {
            const float s = pos[3 * i + d] + flow[3 * i + d];
            const float p = pos[3 * i + d];
            if (cnt == 0) { ss[d] = s; sd[d] = p; }
            else { ss[d] = ss[d] + s; sd[d] = sd[d] + p; }
        }
        cnt++;
    }
    for (int k = 0; k < 4; ++k) q[k] = 0.0;
    if (cnt == 0) return -1;
    float ms[3], md[3];
    for (int d = 0; d < 3; ++d) {
        ms[d] = (float)((double)ss[d] / (double)cnt);
        md[d] = (float)((double)sd[d] / (double)cnt);
    }
    double H[9] = {0};
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        float a[3], b[3];
        for (int d = 0; d < 3; ++d) {
            a[d] = (pos[3 * i + d] + flow[3 * i + d]) - ms[d];
            b[d] = pos[3 * i + d] - md[d];
        }
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) H[r * 3 + c] += (double)a[r] * (double)b[c];
    }
    double U[9], S[3], Vt[9], R[9];
    orc_svd3(H, U, S, Vt);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += Vt[k * 3 + r] * U[c * 3 + k];
            R[r * 3 + c] = s;
        }
    int32_t rc = 0;
    if (det3(R) < 0) {
        if (!reflection) rc = -2;
        for (int k = 0; k < 3; ++k) Vt[2 * 3 + k] *= -1.0;
        if (reflection)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < 3; ++k) s += Vt[k * 3 + r] * U[c * 3 + k];
                    R[r * 3 + c] = s;
                }
    }
    float R32[9], t32[3];
    for (int k = 0; k < 9; ++k) R32[k] = (float)R[k];
    for (int r = 0; r < 3; ++r) {
        const double dot = (double)R32[r * 3] * ms[0] + (double)R32[r * 3 + 1] * ms[1] + (double)R32[r * 3 + 2] * ms[2];
        t32[r] = (float)(-dot) + md[r];
    }
    for (int k = 0; k < 9; ++k) R_out[k] = R32[k];
    for (int r = 0; r < 3; ++r) t_out[r] = t32[r];
    if (rc != 0) return rc;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const float s = (R32[i * 3] * R32[j * 3] + R32[i * 3 + 1] * R32[j * 3 + 1]) + R32[i * 3 + 2] * R32[j * 3 + 2];
            const double e = (i == j) ? 1.0 : 0.0;
            if (!(fabs((double)s - e) <= 1e-8 + 1e-5 * fabs(e))) return -3;
        }
    float m[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) m[i][j] = R32[j * 3 + i];
    float t, w, x, y, z;
    if (m[2][2] < 0) {
        if (m[0][0] > m[1][1]) {
            t = ((1.0f + m[0][0]) - m[1][1]) - m[2][2];
            w = m[1][2] - m[2][1]; x = t; y = m[0][1] + m[1][0]; z = m[2][0] + m[0][2];
        } else {
            t = ((1.0f - m[0][0]) + m[1][1]) - m[2][2];
            w = m[2][0] - m[0][2]; x = m[0][1] + m[1][0]; y = t; z = m[1][2] + m[2][1];
        }
    } else {
        if (m[0][0] < -m[1][1]) {
            t = ((1.0f - m[0][0]) - m[1][1]) + m[2][2];
            w = m[0][1] - m[1][0]; x = m[2][0] + m[0][2]; y = m[1][2] + m[2][1]; z = t;
        } else {
            t = ((1.0f + m[0][0]) + m[1][1]) + m[2][2];
            w = t; x = m[1][2] - m[2][1]; y = m[2][0] - m[0][2]; z = m[0][1] - m[1][0];
        }
    }
    const double f = 0.5 / sqrt((double)t);
    q[0] = (double)x * f; q[1] = (double)y * f; q[2] = (double)z * f; q[3] = (double)w * f;
    return 0;
}
