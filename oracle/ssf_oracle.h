/*
 * ssf_oracle.h -- CPU restatement of the SSF-SLAM LiDAR front-end hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (ssf-slam_amd/) may link,
 * load or call this library: it is the parity checker used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - Python half (GMM mask, Kabsch, quaternion): PINNED.  Golden vectors in
 *     tests/golden/ were produced by importing the reference's own
 *     scripts/PointCloudOdometry_noSeg.py (ROS modules stubbed) and the sklearn
 *     1.7.2 GaussianMixture it calls; tests/test_oracle_golden.py checks this
 *     restatement against them.
 *   - C++ half (frameFeature.cpp, lidarOdometry_onlyPC.cpp): PARITY UNPINNED
 *     against the reference binary.  The reference needs ROS/PCL/Eigen/Ceres,
 *     none of which exist in this image, so it cannot be built; it holds no
 *     golden vectors or tests.  The restatement follows the source line by line
 *     (citations per function) and is pinned only by hand-checkable
 *     known-answer tests.
 *
 * Floating point: build with -O2 -ffp-contract=off (no FMA contraction), the
 * same as the HIP kernels, so float stages are bit-comparable.
 */
#ifndef SSF_ORACLE_H
#define SSF_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Parameter blocks selected by N_SCAN_ROW (src/frameFeature.cpp:141-152,
 * src/lidarOdometry_onlyPC.cpp:313-319). */
typedef struct {
    int32_t n_rows;      /* 16 or 64                                   */
    float plane_min;     /* curvature threshold, 0.05 / 0.005           */
    int32_t plane_span;  /* greedy spacing, 3 / 25                      */
    int32_t row_start;   /* rowIndexStart, 0 / 5                        */
    int32_t row_end;     /* rowIndexEnd, 0 / 5                          */
    float plane_max;     /* coplanarity gate, 0.15 / 0.05               */
} orc_profile;

int orc_profile_get(int32_t n_rows, orc_profile* out);

/* ---- frameFeature (src/frameFeature.cpp:45-123) ---- */
/* The two evaluations C++ overload resolution allows for frameFeature.cpp:57:
 *   ORC_RING_CHAIN_FLOAT   std::atan(float) / std::sqrt(float) visible at global scope (libstdc++'s
 *                          <math.h> wrapper, pulled in by header.h:8-35's ROS / tf / PCL headers):
 *                          (float)((double)(atanf(z / sqrtf(r2)) * 180.0f) / M_PI)  -- the default
 *   ORC_RING_CHAIN_DOUBLE  only ::atan(double) / ::sqrt(double):
 *                          (float)(atan((double)z / sqrt((double)r2)) * 180.0 / M_PI)
 * r2 = x*x + y*y is a float sum in both.  orc_ring_id uses the process-wide chain
 * (orc_set_ring_chain, default FLOAT); the _chain variants take it explicitly. */
enum { ORC_RING_CHAIN_FLOAT = 0, ORC_RING_CHAIN_DOUBLE = 1 };
int32_t orc_set_ring_chain(int32_t chain);     /* returns the previous chain */
int32_t orc_get_ring_chain(void);
float orc_ring_angle(float x, float y, float z, int32_t chain);
int32_t orc_ring_id_chain(float x, float y, float z, int32_t n_rows, int32_t chain);
int32_t orc_ring_id(float x, float y, float z, int32_t n_rows);
int32_t orc_ring_id_of_angle(float angle, int32_t n_rows);
/* the double chain's id of a double ratio z / sqrt(r2) (thresholds of the device table) */
int32_t orc_ring_id_ratio_d(double ratio, int32_t n_rows);
/* Exhaustive scan of EVERY float ratio r in [lo, hi] (points (1, 0, r): the float chain's ratio is
 * r itself): records each change of the float chain's id as (first float of the new id, new id),
 * up to cap entries; returns the number of changes (may exceed cap). */
int64_t orc_ring_changes_f32(float lo, float hi, int32_t n_rows, float* at, int32_t* id, int64_t cap);
/* Stable per-ring partition.  pts has stride `stride` floats (xyz at 0..2).
 * rxyzi: ring-ordered kept points (x,y,z,intensity) -- capacity n*4 floats.
 * ring_off[n_rows+1]: exclusive prefix of per-ring counts.
 * src_idx[kept]: input index of each ring-ordered point.
 * ring_of_input[n]: ring id per input point (-1 = dropped).
 * returns number of kept points. */
int64_t orc_bin(const float* pts, int64_t n, int64_t stride, int32_t n_rows, float* rxyzi,
                int64_t* ring_off, int64_t* src_idx, int32_t* ring_of_input);
void orc_curvature(const float* rxyzi, const int64_t* ring_off, int32_t n_rows, int32_t row_start,
                   int32_t row_end, float* curv);
int64_t orc_select(const float* rxyzi, const float* curv, const int64_t* ring_off, int32_t n_rows,
                   int32_t row_start, int32_t row_end, float plane_min, int32_t plane_span,
                   float* plane_xyzi, int64_t* sel_idx);
/* bin + curvature + select in one call; plane_xyzi capacity n*4 floats. */
int64_t orc_extract_planes(const float* pts, int64_t n, int64_t stride, int32_t n_rows,
                           float* plane_xyzi);

/* ---- lidarOdometry_onlyPC (src/lidarOdometry_onlyPC.cpp:74-82,147-252) ---- */
void orc_knn(const float* cloud_xyzi, int64_t m, const float q[3], int32_t k, int32_t* idx,
             float* d2);
/* The same k-NN lists through an x-sorted index (plane table and association use it). */
typedef struct { const float* cloud; int64_t m; float* xs; int32_t* order; } orc_xindex;
orc_xindex* orc_xindex_build(const float* cloud_xyzi, int64_t m);
void orc_xindex_free(orc_xindex* X);
void orc_xindex_knn(const orc_xindex* X, const float q[3], int32_t k, int32_t* idx, float* d2);
void orc_plane_table(const float* last_xyzi, int64_t m, float plane_max, float* normal,
                     int32_t* valid, int32_t* pick5, int32_t* gate_rank);
void orc_transform_point(const double q[4], const double t[3], const float p[3], float out[3]);
void orc_correspond(const float* last_xyzi, int64_t m_last, const float* curr_xyzi, int64_t m_curr,
                    const double q[4], const double t[3], int32_t* nn);

/* per-iteration log record: q(4,xyzw) t(3) cost accepted radius = 10 doubles */
#define ORC_LOG_STRIDE 10
enum { ORC_MODE_CERES_LM = 0, ORC_MODE_GN = 1 };
int32_t orc_solve(const float* po, const float* pa, const float* nrm, int64_t c, int32_t mode,
                  int32_t max_iter, const double q_init[4], const double t_init[3], double q_out[4],
                  double t_out[3], double* log, int32_t* n_log);
/* Full frameRegistration(): table + 1-NN + solve.  Returns number of correspondences used
 * (-1 when the last frame has <= 10 points: pose returned unchanged). */
int64_t orc_register_pair(const float* last_xyzi, int64_t m_last, const float* curr_xyzi,
                          int64_t m_curr, float plane_max, int32_t mode, int32_t max_iter,
                          const double q_init[4], const double t_init[3], double q_out[4],
                          double t_out[3], double* log, int32_t* n_log);
int32_t orc_solve2(const float* po, const float* pa, const float* nrm, int64_t c,
                   const float* epo, const float* ec, const float* eu, int64_t ce, int32_t mode,
                   int32_t max_iter, const double q_init[4], const double t_init[3], double q_out[4],
                   double t_out[3], double* log, int32_t* n_log);
/* edge_oracle.c: edge features + point-to-line residuals (beyond the reference, parity unpinned) */
int64_t orc_select_edges(const float* rxyzi, const float* curv, const int64_t* ring_off,
                         int32_t n_rows, int32_t row_start, int32_t row_end, float edge_min,
                         int32_t edge_span, float* edge_xyzi);
int64_t orc_extract_features(const float* pts, int64_t n, int64_t stride, int32_t n_rows,
                             float edge_min, int32_t edge_span, float* plane_xyzi,
                             float* edge_xyzi, int64_t* m_edge);
void orc_sym3_eig(double A[9], double V[9]);
void orc_edge_table(const float* edges, int64_t m, float max_nn_d2, float line_ratio,
                    float* line, int32_t* valid);
int64_t orc_register_pair_edges(const float* last, int64_t m_last, const float* curr,
                                int64_t m_curr, const float* last_e, int64_t me_last,
                                const float* curr_e, int64_t me_curr, float plane_max,
                                float max_nn_d2, float line_ratio, int32_t mode, int32_t max_iter,
                                const double q_init[4], const double t_init[3], double q_out[4],
                                double t_out[3], double* log, int32_t* n_log,
                                int64_t* n_edge_corr);
void orc_accumulate(const double q0l[4], const double t0l[3], const double qlc[4],
                    const double tlc[3], double q0c[4], double t0c[3]);

/* ---- PointCloudOdometry_noSeg.py mask + Kabsch ---- */
typedef struct { uint32_t mt[624]; int32_t pos; } orc_mt19937;
void orc_mt_seed(orc_mt19937* s, uint32_t seed);
double orc_mt_random_sample(orc_mt19937* s);
/* GMM(2) on X (n x 6, [flow, xyz]) with sklearn 1.7.2 semantics; draws[3] = the three
 * RandomState doubles consumed by k-means++ (choice, uniform(2)).  labels[n] (0/1).
 * info[8] = {kmeans_iter, em_iter, converged, center0, center1, bg_label, n_bg, lower_bound} */
int32_t orc_gmm_labels(const double* X, int64_t n, const double draws[3], uint8_t* labels,
                       double* info, double* means /* 12, nullable */);
/* slove_RT_by_SVD(src, dst) over rows with mask[i] != 0 (mask nullable = all).
 * reflection: 0 -> return -2 on det<0 (reference raises), 1 -> Vt[2]*=-1 fix.  R row-major. */
int32_t orc_kabsch(const double* src, const double* dst, int64_t n, const uint8_t* mask,
                   int32_t reflection, double R[9], double t[3]);
/* pyquaternion Quaternion(matrix=R) trace method -> q (x,y,z,w); -3 if not orthogonal */
int32_t orc_quat_from_R(const double R[9], double q[4]);
/* slove_RT_by_SVD + Quaternion on float32 arrays (the ASF block, main_sju_occ_ros.py:273-284):
 * src = pos + flow in f32, dst = pos, mask rows only; R, t are the f32 results */
int32_t orc_kabsch_f32(const float* pos, const float* flow, int64_t n, const uint8_t* mask,
                       int32_t reflection, double R[9], double t[3], double q[4]);
void orc_svd3(const double A[9], double U[9], double S[3], double Vt[9]);

/* ---- mapOptmization loop closure, oracle/loop_oracle.c ---- */
/* pcl::VoxelGrid<PointXYZI> (leaf cube), xyzi n x 4 -> centroids m x 4 in voxel order; returns m */
int64_t orc_voxel_grid(const float* xyzi, int64_t n, float leaf, float* out);
enum { ORC_ICP_NOT_CONVERGED = 0, ORC_ICP_ITERATIONS = 1, ORC_ICP_TRANSFORM = 2, ORC_ICP_ABS_MSE = 3,
       ORC_ICP_REL_MSE = 4, ORC_ICP_NO_CORRESPONDENCES = 5 };
typedef struct { int32_t max_iter; float max_corr_dist; double trans_eps; double fit_eps; } orc_icp_params;
typedef struct { float T[16]; double fitness; int32_t converged; int32_t iterations; int32_t state;
                 int32_t n_corr; } orc_icp_result;
/* pcl::IterativeClosestPoint<PointXYZI, PointXYZI>: T row-major 4x4 float (final transformation) */
int32_t orc_icp(const float* src, int64_t ns, const float* tgt, int64_t nt, const orc_icp_params* p,
                const float guess[16], orc_icp_result* r);

#ifdef __cplusplus
}
#endif
#endif
