/* edge_oracle.c -- CPU restatement of the EDGE features and point-to-line residuals.
 *
 * TEST INFRASTRUCTURE ONLY (see ssf_oracle.c).  Beyond the reference: SSF-SLAM's frameFeature is
 * planar only (src/frameFeature.cpp:110-123) and lidarOdometry_onlyPC is point-to-plane only
 * (:25-43); the north_star asks for edge extraction and point-to-line residuals, so these
 * definitions are the build's own (parity UNPINNED: nothing in the reference pins them), written
 * to mirror the reference's planar rules and LOAM's edge step:
 *   selection   per row in [rowStart, R - rowEnd), greedy in index order: j >= jstart and
 *               curvature > edge_min (curvature as :84-107, 0 outside [5, size-5)) -> emit,
 *               jstart = j + edge_span  (the mirror image of :110-123)
 *   edge table  per last-frame edge point a: exact 5-NN among the last frame's edges ((d2, index)
 *               order, L2_Simple float distances), gate d2[4] < max_nn_d2; centroid c and
 *               covariance of the 5 points in double (rank order); cyclic Jacobi eigen
 *               decomposition; valid iff gate && lambda1 > line_ratio * lambda2; u = the unit
 *               eigenvector of lambda1, sign fixed so its largest-|.| component is positive
 *   residual    curr edge point p -> transformToLast (:74-82) -> exact 1-NN a among the last
 *               edges; if valid[a]: e = (I - u u^T)(R p + t - c), one Huber(0.1) block on |e|^2,
 *               inserted twice like every residual of the :160 loop
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ssf_oracle.h"

int64_t orc_select_edges(const float* rxyzi, const float* curv, const int64_t* ring_off,
                         int32_t n_rows, int32_t row_start, int32_t row_end, float edge_min,
                         int32_t edge_span, float* edge_xyzi) {
    int64_t m = 0;
    for (int32_t r = row_start; r < n_rows - row_end; ++r) {
        int64_t size = ring_off[r + 1] - ring_off[r];
        int64_t jstart = 0;
        for (int64_t j = 0; j < size; ++j) {
            int64_t o = ring_off[r] + j;
            if (j >= jstart && curv[o] > edge_min) {
                memcpy(edge_xyzi + 4 * m, rxyzi + 4 * o, 4 * sizeof(float));
                m++;
                jstart = j + edge_span;
            }
        }
    }
    return m;
}

int64_t orc_extract_features(const float* pts, int64_t n, int64_t stride, int32_t n_rows,
                             float edge_min, int32_t edge_span, float* plane_xyzi,
                             float* edge_xyzi, int64_t* m_edge) {
    orc_profile p;
    if (orc_profile_get(n_rows, &p) != 0) return -1;
    size_t nn = (size_t)(n > 0 ? n : 1);
    float* rxyzi = (float*)malloc(sizeof(float) * 4 * nn);
    float* curv = (float*)malloc(sizeof(float) * nn);
    int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_rows + 1));
    orc_bin(pts, n, stride, n_rows, rxyzi, off, NULL, NULL);
    orc_curvature(rxyzi, off, n_rows, p.row_start, p.row_end, curv);
    int64_t m = orc_select(rxyzi, curv, off, n_rows, p.row_start, p.row_end, p.plane_min,
                           p.plane_span, plane_xyzi, NULL);
    *m_edge = orc_select_edges(rxyzi, curv, off, n_rows, p.row_start, p.row_end, edge_min,
                               edge_span, edge_xyzi);
    free(rxyzi); free(curv); free(off);
    return m;
}

/* Cyclic Jacobi on a symmetric 3x3 (row-major, in place): eigenvalues on the diagonal, the
 * eigenvectors in the columns of V.  Fixed pair order (0,1), (0,2), (1,2), at most 32 sweeps. */
void orc_sym3_eig(double A[9], double V[9]) {
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    static const int P[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int sweep = 0; sweep < 32; ++sweep) {
        double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        double dia = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (!(off > 1e-30 * dia)) break;
        for (int k = 0; k < 3; ++k) {
            int p = P[k][0], q = P[k][1];
            double apq = A[3 * p + q];
            if (apq == 0.0) continue;
            double theta = (A[3 * q + q] - A[3 * p + p]) / (2.0 * apq);
            double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
            for (int i = 0; i < 3; ++i) {
                double aip = A[3 * i + p], aiq = A[3 * i + q];
                A[3 * i + p] = c * aip - s * aiq;
                A[3 * i + q] = s * aip + c * aiq;
            }
            for (int i = 0; i < 3; ++i) {
                double api = A[3 * p + i], aqi = A[3 * q + i];
                A[3 * p + i] = c * api - s * aqi;
                A[3 * q + i] = s * api + c * aqi;
            }
            for (int i = 0; i < 3; ++i) {
                double vip = V[3 * i + p], viq = V[3 * i + q];
                V[3 * i + p] = c * vip - s * viq;
                V[3 * i + q] = s * vip + c * viq;
            }
        }
    }
}

/* line[6 m]: centroid c (3), direction u (3) per last-frame edge point; valid[m]. */
void orc_edge_table(const float* edges, int64_t m, float max_nn_d2, float line_ratio,
                    float* line, int32_t* valid) {
    for (int64_t a = 0; a < m; ++a) {
        float* L = line + 6 * a;
        memset(L, 0, 6 * sizeof(float));
        valid[a] = 0;
        if (m < 5) continue;
        float q[3] = {edges[4 * a], edges[4 * a + 1], edges[4 * a + 2]}, d2[5];
        int32_t idx[5];
        orc_knn(edges, m, q, 5, idx, d2);
        double c[3] = {0, 0, 0};
        for (int k = 0; k < 5; ++k)
            for (int j = 0; j < 3; ++j) c[j] += (double)edges[4 * idx[k] + j];
        for (int j = 0; j < 3; ++j) c[j] = c[j] / 5.0;
        double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, V[9];
        for (int k = 0; k < 5; ++k) {
            double v[3];
            for (int j = 0; j < 3; ++j) v[j] = (double)edges[4 * idx[k] + j] - c[j];
            for (int r = 0; r < 3; ++r)
                for (int s = 0; s < 3; ++s) A[3 * r + s] += v[r] * v[s];
        }
        for (int j = 0; j < 9; ++j) A[j] = A[j] / 5.0;
        orc_sym3_eig(A, V);
        double w[3] = {A[0], A[4], A[8]};
        int i1 = 0;                                        /* largest, ties to the lower index */
        for (int i = 1; i < 3; ++i) if (w[i] > w[i1]) i1 = i;
        double l2 = -INFINITY;
        for (int i = 0; i < 3; ++i) if (i != i1 && w[i] > l2) l2 = w[i];
        double u[3] = {V[i1], V[3 + i1], V[6 + i1]};
        int big = 0;
        for (int j = 1; j < 3; ++j) if (fabs(u[j]) > fabs(u[big])) big = j;
        if (u[big] < 0.0) for (int j = 0; j < 3; ++j) u[j] = -u[j];
        for (int j = 0; j < 3; ++j) { L[j] = (float)c[j]; L[3 + j] = (float)u[j]; }
        valid[a] = (d2[4] < max_nn_d2) && (w[i1] > (double)line_ratio * l2);
    }
}

/* frameRegistration with planes (exactly orc_register_pair) plus edge blocks.
 * Returns plane correspondences; *n_edge_corr the edge correspondences. */
int64_t orc_register_pair_edges(const float* last, int64_t m_last, const float* curr,
                                int64_t m_curr, const float* last_e, int64_t me_last,
                                const float* curr_e, int64_t me_curr, float plane_max,
                                float max_nn_d2, float line_ratio, int32_t mode, int32_t max_iter,
                                const double q_init[4], const double t_init[3], double q_out[4],
                                double t_out[3], double* log, int32_t* n_log,
                                int64_t* n_edge_corr) {
    if (n_log) *n_log = 0;
    *n_edge_corr = 0;
    if (m_last <= 10) {                                                    /* :158 */
        memcpy(q_out, q_init, 4 * sizeof(double)); memcpy(t_out, t_init, 3 * sizeof(double));
        return -1;
    }
    size_t ml = (size_t)m_last, mc = (size_t)(m_curr > 0 ? m_curr : 1);
    size_t el = (size_t)(me_last > 0 ? me_last : 1), ecn = (size_t)(me_curr > 0 ? me_curr : 1);
    float* normal = (float*)malloc(sizeof(float) * 3 * ml);
    int32_t* valid = (int32_t*)malloc(sizeof(int32_t) * ml);
    int32_t* nn = (int32_t*)malloc(sizeof(int32_t) * mc);
    float* po = (float*)malloc(sizeof(float) * 3 * mc);
    float* pa = (float*)malloc(sizeof(float) * 3 * mc);
    float* nr = (float*)malloc(sizeof(float) * 3 * mc);
    float* line = (float*)malloc(sizeof(float) * 6 * el);
    int32_t* lvalid = (int32_t*)malloc(sizeof(int32_t) * el);
    int32_t* enn = (int32_t*)malloc(sizeof(int32_t) * ecn);
    float* epo = (float*)malloc(sizeof(float) * 3 * ecn);
    float* ec = (float*)malloc(sizeof(float) * 3 * ecn);
    float* eu = (float*)malloc(sizeof(float) * 3 * ecn);
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
    int64_t ce = 0;
    if (me_last > 0 && me_curr > 0) {
        orc_edge_table(last_e, me_last, max_nn_d2, line_ratio, line, lvalid);
        orc_correspond(last_e, me_last, curr_e, me_curr, q_init, t_init, enn);
        for (int64_t i = 0; i < me_curr; ++i) {
            int32_t a = enn[i];
            if (a < 0 || !lvalid[a]) continue;
            for (int k = 0; k < 3; ++k) {
                epo[3 * ce + k] = curr_e[4 * i + k];
                ec[3 * ce + k] = line[6 * a + k];
                eu[3 * ce + k] = line[6 * a + 3 + k];
            }
            ce++;
        }
    }
    orc_solve2(po, pa, nr, c, epo, ec, eu, ce, mode, max_iter, q_init, t_init, q_out, t_out, log,
               n_log);
    *n_edge_corr = ce;
    free(normal); free(valid); free(nn); free(po); free(pa); free(nr);
    free(line); free(lvalid); free(enn); free(epo); free(ec); free(eu);
    return c;
}
