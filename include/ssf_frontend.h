/*
 * ssf_frontend.h -- C ABI of the MI355X (gfx950) SSF-SLAM LiDAR front-end.
 *
 * This is the drop-in boundary for the reference's hot path.  Every entry point names the
 * reference interface it replaces (file:line under YQChen8/SSF-SLAM).  Plain pointers and
 * sizes only: no C++ types, no exceptions, no torch types cross this boundary.
 *
 * Conventions
 *   - Pointers prefixed d_ are DEVICE pointers (hipMalloc'd / torch CUDA tensors) owned by the
 *     caller; pointers prefixed h_ are host pointers.  `stream` is a hipStream_t (NULL = the
 *     default stream).  All work is enqueued on `stream`; nothing synchronises unless stated.
 *   - A batch of F frames is stored back to back: frame f occupies points
 *     [d_frame_off[f], d_frame_off[f+1]) of the point arrays (int64 offsets, device).  Per-frame
 *     outputs that are point-shaped (plane clouds, ring-ordered clouds) use the SAME offsets:
 *     frame f's plane points start at d_frame_off[f] and d_plane_count[f] of them are valid.
 *   - Points are float32 x,y,z with a stride of `point_stride` floats (3 for the PointCloud2
 *     point_step 12 layout published by PointCloudOdometry*.py:84-92, 4 or 8 for padded PCL
 *     layouts).  Plane clouds are float32 x,y,z,intensity (16 B), intensity encoding
 *     indexInRow + row/100 exactly as src/frameFeature.cpp:77.
 *   - Poses are 7 doubles: q (x,y,z,w) then t (x,y,z) -- the para_q / para_t layout of
 *     src/lidarOdometry_onlyPC.cpp:62-63.
 *   - Return 0 on success, <0 on error; ssf_last_error() describes the last error of a context.
 *     HIP errors are mapped to SSF_E_HIP.  One context per host thread/stream (calls on a
 *     context are not thread-safe, different contexts are independent).
 */
#ifndef SSF_FRONTEND_H
#define SSF_FRONTEND_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define SSF_ABI_VERSION 2

enum {
    SSF_OK = 0,
    SSF_E_ARG = -1,       /* bad argument / shape                                  */
    SSF_E_HIP = -2,       /* HIP runtime error                                     */
    SSF_E_NOMEM = -3,     /* device allocation failed                              */
    SSF_E_CAPACITY = -4,  /* output capacity too small                             */
    SSF_E_NODEV = -5      /* no gfx950 device                                      */
};

enum { SSF_SOLVER_CERES_LM = 0, SSF_SOLVER_GN = 1 };
enum { SSF_MASK_GMM = 0, SSF_MASK_GT = 1, SSF_MASK_GIVEN = 2 };
/* The evaluation of src/frameFeature.cpp:57 `atan(point.z / sqrt(x*x + y*y)) * 180 / M_PI` on
 * float members.  C++ overload resolution allows exactly two:
 *   SSF_RING_CHAIN_FLOAT   the float overloads std::atan(float) / std::sqrt(float) are visible at
 *                          global scope -- libstdc++'s <math.h> wrapper does `using std::atan;
 *                          using std::sqrt;`, and include/header.h:8-35 (ROS, tf, PCL, Ceres)
 *                          includes <math.h>: ratio z / sqrtf(r2), atanf, `* 180` in float,
 *                          `/ M_PI` in double, stored to float.  The default.
 *   SSF_RING_CHAIN_DOUBLE  only the C ::sqrt(double) / ::atan(double): the ratio and the angle
 *                          in double, stored to float.
 * The host libm (glibc) evaluates atanf / atan once per context into a step table; the device
 * never evaluates atan. */
enum { SSF_RING_CHAIN_FLOAT = 0, SSF_RING_CHAIN_DOUBLE = 1 };

/* Runtime replacement of the compile-time N_SCAN_ROW parameter blocks
 * (include/header.h:37-38, src/frameFeature.cpp:141-152, src/lidarOdometry_onlyPC.cpp:313-319). */
typedef struct {
    int32_t n_rows;       /* 16 or 64                                              */
    float plane_min;      /* curvature threshold (planeMin)                        */
    int32_t plane_span;   /* greedy spacing (planeSpan)                            */
    int32_t row_start;    /* rowIndexStart                                         */
    int32_t row_end;      /* rowIndexEnd                                           */
    float plane_max;      /* coplanarity gate (planeMax)                           */
    int32_t solver;       /* SSF_SOLVER_CERES_LM (reference) or SSF_SOLVER_GN      */
    int32_t max_iter;     /* 8 (ceres::Solver::Options max_num_iterations) or 10   */
    int32_t ring_chain;   /* SSF_RING_CHAIN_FLOAT (default) or SSF_RING_CHAIN_DOUBLE  */
} ssf_config;

typedef struct ssf_ctx ssf_ctx;

int32_t ssf_abi_version(void);
/* Fill `out` with the reference's parameter block for n_rows (16 or 64). */
int32_t ssf_config_default(int32_t n_rows, ssf_config* out);
/* Create a context bound to HIP device `device`. */
int32_t ssf_create(int32_t device, const ssf_config* cfg, ssf_ctx** out);
void ssf_destroy(ssf_ctx* ctx);
const char* ssf_last_error(const ssf_ctx* ctx);
/* Pre-size device scratch so later calls never allocate (graph-capture friendly). */
int32_t ssf_reserve(ssf_ctx* ctx, int32_t max_frames, int64_t max_points_per_frame);

/* Kernel timing (no reference counterpart: the reference has no timers).  While
 * enabled, every kernel this context launches is bracketed by HIP events on its stream; on a
 * stream no other stream competes with, each interval is that kernel's duration.
 * ssf_profile_read synchronises on the recorded events and returns, per kernel name, the
 * launches and total milliseconds recorded since the previous read (then clears them). */
typedef struct {
    char name[48];
    int32_t launches;
    double total_ms;
} ssf_kernel_time;
int32_t ssf_profile_enable(ssf_ctx* ctx, int32_t on);
int32_t ssf_profile_read(ssf_ctx* ctx, ssf_kernel_time* out, int32_t cap, int32_t* n_out);

/* ---------------------------------------------------------------------------------------
 * frameFeature: replaces cloudHandler() (src/frameFeature.cpp:35-139) -- ring binning
 * (:45-81), 11-tap curvature (:84-107) and greedy planar selection (:110-123) -- for a batch
 * of frames.  The VoxelGrid at :125-127 is dead work in the reference (its output is
 * discarded) and is not performed.
 *   d_pts           F frames of xyz (stride point_stride floats), offsets d_frame_off[F+1]
 *   total_points    host copy of d_frame_off[F] (extent of every point-shaped array)
 *   max_frame_points  host upper bound of points in any frame (grid sizing)
 *   d_plane_xyzi    out, plane points x,y,z,intensity (16 B) at frame offsets
 *   d_plane_count   out [F] int32, number of plane points per frame
 *   d_ring_xyzi     out, nullable: ring-ordered kept points (x,y,z,intensity) at frame offsets
 *   d_ring_off      out, nullable: [F*(n_rows+1)] int32 per-frame row offsets (frame relative)
 *   d_curv          out, nullable: curvature per ring-ordered point (0 where not computed)
 */
int32_t ssf_extract_planes_batch(ssf_ctx* ctx, void* stream, int32_t n_frames,
                                 const float* d_pts, int32_t point_stride,
                                 const int64_t* d_frame_off, int64_t total_points,
                                 int64_t max_frame_points,
                                 float* d_plane_xyzi, int32_t* d_plane_count,
                                 float* d_ring_xyzi, int32_t* d_ring_off, float* d_curv);

/* Beyond the reference (BASELINE configs[2] "mask applied before features"; parity unpinned,
 * off unless called): the same extraction on the points whose d_keep byte is non-zero -- e.g.
 * the background mask of ssf_mask_pose_batch at the same offsets.  Dropped points are treated as
 * if they were not in the cloud (the reference's frameFeature always receives every point,
 * scripts/PointCloudOdometry_noSeg.py:92-94), so the result equals ssf_extract_planes_batch on
 * the stably compacted cloud. */
int32_t ssf_extract_planes_batch_masked(ssf_ctx* ctx, void* stream, int32_t n_frames,
                                        const float* d_pts, int32_t point_stride,
                                        const int64_t* d_frame_off, int64_t total_points,
                                        int64_t max_frame_points, const uint8_t* d_keep,
                                        float* d_plane_xyzi, int32_t* d_plane_count,
                                        float* d_ring_xyzi, int32_t* d_ring_off, float* d_curv);
/* Single-frame form with the SURVEY §8(b) signature: synchronises, returns the plane count in
 * *h_out_m; SSF_E_CAPACITY if more than out_cap points were selected. */
int32_t ssf_extract_planes(ssf_ctx* ctx, void* stream, const float* d_pts, int64_t n,
                           int32_t point_step_bytes, int32_t xyz_offset_bytes,
                           float* d_out_xyzi, int64_t* h_out_m, int64_t out_cap);

/* ---------------------------------------------------------------------------------------
 * Plane table for frames that will serve as the LAST frame of a registration pair: for every
 * plane point a, the 30-NN ring-diverse 5-point pick, the 5x3 least-squares plane and the
 * coplanarity gate of src/lidarOdometry_onlyPC.cpp:173-232 (which depend only on the last
 * frame and a, so they are computed once per frame instead of once per correspondence x2).
 *   d_normal  out float32 x3 per plane point (frame offsets), d_valid out uint8 per point.
 *   d_sorted_xyzi / d_sorted_idx  out (nullable): the frame's plane points sorted by (x, index)
 *             and the permutation, the search index the k-NN walks use; pass them back to
 *             ssf_register_batch when this frame is the last frame.  When they are NULL, or
 *             max_plane_points exceeds SSF_SORTED_MAX, both calls fall back to brute-force k-NN.
 *             Use the same max_plane_points bound for a frame's table and its registration.
 *   d_strip_xyzi / d_strip_head  out (nullable, both or neither; needs the sorted buffers):
 *             float32 x4 and int32 per plane point (frame offsets).  The table's y-strip image of
 *             the frame (the association's search structure), kept so that ssf_register_batch
 *             stages it instead of rebuilding it when this frame is the last frame.  Frames of
 *             773..6144 plane points carry an image; others are rebuilt as before.
 */
#define SSF_SORTED_MAX 16384
int32_t ssf_plane_table_batch(ssf_ctx* ctx, void* stream, int32_t n_frames,
                              const float* d_plane_xyzi, const int64_t* d_frame_off,
                              const int32_t* d_plane_count, int64_t max_plane_points,
                              float* d_normal, uint8_t* d_valid, float* d_sorted_xyzi,
                              int32_t* d_sorted_idx, float* d_strip_xyzi, int32_t* d_strip_head);

/* ---------------------------------------------------------------------------------------
 * lidarOdometry_onlyPC: replaces frameRegistration() (src/lidarOdometry_onlyPC.cpp:147-252)
 * plus the pose accumulation of publishResult() (:87-90) for P independent pairs.
 *   last / curr      plane clouds (x,y,z,intensity) with their own offsets + counts
 *   d_last_normal/valid/sorted_*  plane table + search index of the last frames
 *                        (ssf_plane_table_batch); the sorted arrays are nullable (brute force)
 *   curr_total_points    host copy of d_curr_off[P] (correspondence scratch extent)
 *   max_plane_points     host upper bound of plane points in any frame (grid sizing)
 *   d_pose_rel [P*7] in: warm start q_last_curr/t_last_curr (the previous pair's solution,
 *                    :164,251-252); out: the solution.  Last frames with <= 10 points leave
 *                    it unchanged (:158).
 *   d_pose_abs [P*7] nullable; in: q_0_last,t_0_last; out: q_0_curr,t_0_curr (:87-90).
 *   d_log      nullable [P*max_iter*10] doubles per iteration: q(4) t(3) cost status radius
 *   d_nlog     nullable [P] iterations logged;  d_ncorr nullable [P] correspondences used
 *              (-1 when skipped);  d_nn nullable: per curr point 1-NN index into last.
 *   d_last_strip_xyzi / d_last_strip_head  nullable (both or neither): the strip image the
 *              last frames' ssf_plane_table_batch call wrote (same max_plane_points).  The results
 *              are identical with or without it; with it the association skips its strip build.
 */
int32_t ssf_register_batch(ssf_ctx* ctx, void* stream, int32_t n_pairs,
                           const float* d_last_xyzi, const int64_t* d_last_off,
                           const int32_t* d_last_count, const float* d_last_normal,
                           const uint8_t* d_last_valid, const float* d_last_sorted_xyzi,
                           const int32_t* d_last_sorted_idx, const float* d_curr_xyzi,
                           const int64_t* d_curr_off, const int32_t* d_curr_count,
                           int64_t curr_total_points, int64_t max_plane_points,
                           double* d_pose_rel, double* d_pose_abs,
                           double* d_log, int32_t* d_nlog, int32_t* d_ncorr, int32_t* d_nn,
                           const float* d_last_strip_xyzi, const int32_t* d_last_strip_head);

/* A sequence's consecutive pairs in one call (lidarOdometry_onlyPC's frame loop over a sequence:
 * every pair is warm-started from the previous pair's solution, src/lidarOdometry_onlyPC.cpp:164,
 * 251-252).  Frames 0..n_pairs of ONE plane batch (d_off / d_count: n_pairs + 2 / n_pairs + 1
 * entries, the table / search index / strip image of ssf_plane_table_batch on the same batch);
 * pair k registers frame k + 1 (curr) against frame k (last).
 *   d_pose_init [7]          warm start of pair 0 (q xyzw, t)
 *   d_pose_seq [n_pairs*7]   out: pair k's solution (the warm start of pair k + 1)
 *   d_pose_abs_init [7] / d_pose_abs_seq [n_pairs*7]  nullable (both or neither): the pose of
 *                            frame 0, and out the pose of frame k + 1 (:87-90)
 *   d_ncorr [n_pairs]        nullable: correspondences per pair (-1 when skipped, :158)
 * Results are identical to n_pairs ssf_register_batch calls of one pair each with the warm start
 * copied between them; the links read the previous output in place (no copy launches). */
int32_t ssf_register_chain(ssf_ctx* ctx, void* stream, int32_t n_pairs, const float* d_xyzi,
                           const int64_t* d_off, const int32_t* d_count, const float* d_normal,
                           const uint8_t* d_valid, const float* d_sorted_xyzi,
                           const int32_t* d_sorted_idx, int64_t total_points,
                           int64_t max_plane_points, const double* d_pose_init,
                           double* d_pose_seq, const double* d_pose_abs_init,
                           double* d_pose_abs_seq, int32_t* d_ncorr,
                           const float* d_strip_xyzi, const int32_t* d_strip_head);

/* Single-pair form with the SURVEY §8(b) signature: frameRegistration() on the globals
 * lastFramePlanePtr / currFramePlanePtr / para_q / para_t (src/lidarOdometry_onlyPC.cpp:51-71,
 * 147-252).  The plane clouds are device float4 (x, y, z, intensity) as frameFeature publishes
 * them; the warm start h_q_init (x,y,z,w) / h_t_init is the previous pair's solution (:164,
 * 251-252) and the solution comes back in h_q_out / h_t_out.  The last frame's plane table and
 * search index are built inside the call (ctx scratch).  A last frame with <= 10 points adds no
 * residual (:158): the warm start is returned unchanged, rc 0, log->n_corr = -1.  Synchronous.
 * log (nullable): per LM/GN iteration the pose after it, the Ceres cost, a status code and the
 * trust-region radius. */
enum {
    SSF_STEP_REJECTED = 0,        /* LM step computed, rho <= 1e-3, radius shrunk            */
    SSF_STEP_ACCEPTED = 1,        /* LM step accepted                                        */
    SSF_STEP_INVALID = 2,         /* LM/GN linear solve failed or non-positive model decrease */
    SSF_STEP_PARAM_TOL = 3,       /* ParameterToleranceReached (|dx| <= 1e-8 (|x| + 1e-8))   */
    SSF_STEP_FUNC_TOL = 4,        /* FunctionToleranceReached (|dcost| <= 1e-6 cost)         */
    SSF_STEP_GRAD_TOL = 5,        /* GradientToleranceReached (max-norm <= 1e-10)            */
    SSF_STEP_GN = 6               /* undamped Gauss-Newton step (SSF_SOLVER_GN)              */
};
typedef struct {
    double q[4];       /* pose after the iteration, q x,y,z,w                          */
    double t[3];
    double cost;       /* Ceres cost 1/2 sum rho(r^2) over the duplicated blocks        */
    int32_t status;    /* SSF_STEP_*                                                    */
    int32_t pad;
    double radius;     /* trust-region radius after the iteration (0 in GN mode)         */
} ssf_step;
typedef struct {
    int32_t cap;       /* in: capacity of steps[] (cfg.max_iter holds a full log)        */
    int32_t n_steps;   /* out: iterations logged                                        */
    int32_t n_corr;    /* out: valid correspondences (-1: skipped, :158)                */
    int32_t pad;
    ssf_step* steps;   /* caller-owned host array of cap entries                        */
} ssf_step_log;
int32_t ssf_register_pair(ssf_ctx* ctx, void* stream, const float* d_last_xyzi, int64_t m_last,
                          const float* d_curr_xyzi, int64_t m_curr, const double* h_q_init,
                          const double* h_t_init, double* h_q_out, double* h_t_out,
                          ssf_step_log* log);

/* ---------------------------------------------------------------------------------------
 * Edge features + point-to-line residuals: BEYOND THE REFERENCE.  SSF-SLAM's frameFeature is
 * planar only (src/frameFeature.cpp:110-123) and its registration point-to-plane only
 * (src/lidarOdometry_onlyPC.cpp:25-43); the north_star asks for edge extraction and
 * point-to-line terms, so these entry points are the build's own extension, off unless called,
 * with parity unpinned (definitions restated in oracle/edge_oracle.c):
 *   selection   per row in [row_start, n_rows - row_end), greedy in index order: curvature (the
 *               :84-107 value) > edge_min and j >= jstart -> select, jstart = j + edge_span
 *   line table  per LAST-frame edge point: exact 5-NN among that frame's edges, centroid and
 *               covariance (double), Jacobi eigen-decomposition; valid iff the 5th squared
 *               distance < max_nn_d2 and lambda1 > line_ratio * lambda2; direction u = the
 *               principal eigenvector (largest-|.| component positive)
 *   residual    e = (I - u u^T)(R p + t - c) for the 1-NN last edge of the transformed current
 *               edge point, one Huber(0.1) block on |e|^2, doubled like every :160 block
 */
typedef struct {
    float edge_min;       /* curvature threshold, m^2 (1.0)                                     */
    int32_t edge_span;    /* greedy spacing in a row (10 for 64 rows, 3 for 16)                 */
    float line_ratio;     /* lambda1 > line_ratio * lambda2 (3.0)                               */
    float max_nn_d2;      /* 5th-NN squared distance gate (1.0)                                 */
} ssf_edge_config;
int32_t ssf_edge_config_default(int32_t n_rows, ssf_edge_config* out);
int32_t ssf_set_edge_config(ssf_ctx* ctx, const ssf_edge_config* cfg);
/* ssf_extract_planes_batch(_masked) plus the edge cloud: d_edge_xyzi (x,y,z,intensity, frame
 * offsets, capacity = the points) and d_edge_count [F].  d_keep nullable. */
int32_t ssf_extract_features_batch(ssf_ctx* ctx, void* stream, int32_t n_frames,
                                   const float* d_pts, int32_t point_stride,
                                   const int64_t* d_frame_off, int64_t total_points,
                                   int64_t max_frame_points, const uint8_t* d_keep,
                                   float* d_plane_xyzi, int32_t* d_plane_count,
                                   float* d_edge_xyzi, int32_t* d_edge_count);
/* Line table of frames that will be LAST frames: d_line 6 floats per edge point (centroid x,y,z,
 * direction x,y,z) and d_line_valid u8, at the frame offsets. */
int32_t ssf_edge_table_batch(ssf_ctx* ctx, void* stream, int32_t n_frames,
                             const float* d_edge_xyzi, const int64_t* d_frame_off,
                             const int32_t* d_edge_count, int64_t max_edge_points,
                             float* d_line, uint8_t* d_line_valid);
/* ssf_register_batch with point-to-line blocks added to every pair's problem (same LM/GN loop,
 * same pose / log outputs).  Edge clouds at their own offsets; d_ncorr_edge nullable [P]; the
 * strip image as in ssf_register_batch. */
int32_t ssf_register_batch_edges(ssf_ctx* ctx, void* stream, int32_t n_pairs,
                                 const float* d_last_xyzi, const int64_t* d_last_off,
                                 const int32_t* d_last_count, const float* d_last_normal,
                                 const uint8_t* d_last_valid, const float* d_last_sorted_xyzi,
                                 const int32_t* d_last_sorted_idx, const float* d_curr_xyzi,
                                 const int64_t* d_curr_off, const int32_t* d_curr_count,
                                 int64_t curr_total_points, int64_t max_plane_points,
                                 const float* d_last_edge_xyzi, const int64_t* d_last_edge_off,
                                 const int32_t* d_last_edge_count, const float* d_last_line,
                                 const uint8_t* d_last_line_valid, const float* d_curr_edge_xyzi,
                                 const int64_t* d_curr_edge_off, const int32_t* d_curr_edge_count,
                                 int64_t curr_edge_total, int64_t max_edge_points,
                                 double* d_pose_rel, double* d_pose_abs, double* d_log,
                                 int32_t* d_nlog, int32_t* d_ncorr, int32_t* d_ncorr_edge,
                                 const float* d_last_strip_xyzi, const int32_t* d_last_strip_head);

/* ---------------------------------------------------------------------------------------
 * PointCloudOdometry{,_noSeg}.py: replaces the dynamic-point mask + slove_RT_by_SVD + Quaternion
 * block (scripts/PointCloudOdometry_noSeg.py:97-125, scripts/PointCloudOdometry.py:91-101 and the
 * identical ASF block main_sju_occ_ros.py:256-284) for F frames.
 *   d_pts / d_flow      packed float32 xyz (stride 3) per point: pos1 and the scene flow (gt).
 *   h_frame_off [F+1]   host copy of the offsets (frame sizes drive the RandomState choice()).
 *   mode SSF_MASK_GMM:  GaussianMixture(n_components=2).fit_predict([flow, xyz]) (sklearn 1.7.2
 *                       semantics), background = most common label;  h_draws [F*3] (host,
 *                       nullable) are the three numpy RandomState doubles its k-means++ init
 *                       consumes per frame; NULL draws them from the context RNG (ssf_rng_seed).
 *        SSF_MASK_GT:   background = d_mask_in == 0 (s_fg_mask, PointCloudOdometry.py:91).
 *        SSF_MASK_GIVEN: background = d_mask_in != 0.
 *   Kabsch on background rows: slove_RT_by_SVD(points + flow, points) (:114-118).
 *   reflection 0: det<0 -> status SSF_POSE_REFLECTION (the reference raises TypeError at :33);
 *              1: flip Vt[2] (the evident intent of :32-33).
 *   d_bg_mask  out, nullable: uint8 per point, 1 = background.
 *   d_out      out [F*SSF_POSE_OUT_STRIDE] doubles, see SSF_POSE_OUT_* below.
 *   A frame of more than 2^32 / 12 points (2^32 / 24 for the f64 form) fails with SSF_E_ARG
 *   before any launch: the kernel addresses a frame with 32-bit byte offsets.
 */
#define SSF_POSE_OUT_STRIDE 32
enum {
    SSF_POSE_OUT_T = 0,        /* t (3)                  -- para_t_q[0:3]                    */
    SSF_POSE_OUT_Q = 3,        /* q x,y,z,w (4)          -- para_t_q[3:7]                    */
    SSF_POSE_OUT_R = 7,        /* R row-major (9)                                            */
    SSF_POSE_OUT_STATUS = 16,  /* 0 ok, <0 SSF_POSE_* error                                  */
    SSF_POSE_OUT_NBG = 17,     /* background point count                                     */
    SSF_POSE_OUT_BGLABEL = 18, /* GMM label taken as background                              */
    SSF_POSE_OUT_KM_ITER = 19, /* KMeans n_iter_                                             */
    SSF_POSE_OUT_EM_ITER = 20, /* GaussianMixture n_iter_                                    */
    SSF_POSE_OUT_CONVERGED = 21,
    SSF_POSE_OUT_CENTER0 = 22, /* k-means++ chosen indices                                   */
    SSF_POSE_OUT_CENTER1 = 23,
    SSF_POSE_OUT_LOWER_BOUND = 24,
    SSF_POSE_OUT_PASSES = 25   /* algorithmic bytes / (24 B x points): full-pass equivalents */
};
enum { SSF_POSE_EMPTY = -1, SSF_POSE_REFLECTION = -2, SSF_POSE_NOT_ORTHOGONAL = -3,
       SSF_POSE_GMM_FAILED = -4, SSF_POSE_SYNC_FAILED = -5 };
int32_t ssf_mask_pose_batch(ssf_ctx* ctx, void* stream, int32_t n_frames, const float* d_pts,
                            const float* d_flow, const int64_t* d_frame_off,
                            const int64_t* h_frame_off, int32_t mode, const uint8_t* d_mask_in,
                            const double* h_draws, int32_t reflection, uint8_t* d_bg_mask,
                            double* d_out);
/* The same block on float64 pos / flow (the reference's own dtype when the npz arrays or the
 * ASF network output arrive as float64, PointCloudOdometry_noSeg.py:97-118): every load is exact,
 * so R / t carry no float32 rounding of the inputs.  Otherwise identical to ssf_mask_pose_batch
 * (same modes, draws, outputs and status codes); 48 B per point per pass instead of 24. */
int32_t ssf_mask_pose_batch_f64(ssf_ctx* ctx, void* stream, int32_t n_frames, const double* d_pts,
                                const double* d_flow, const int64_t* d_frame_off,
                                const int64_t* h_frame_off, int32_t mode, const uint8_t* d_mask_in,
                                const double* h_draws, int32_t reflection, uint8_t* d_bg_mask,
                                double* d_out);
/* slove_RT_by_SVD + Quaternion(matrix=R) on FLOAT32 arrays, per frame, as numpy runs them when
 * the inputs are float32: the ASF block on the network's float32 flow
 * (scripts/ActiveSceneFlow/main_sju_occ_ros.py:273-284, slove_RT_by_SVD :455-473).
 * Replaces the f64 tail that ssf_mask_pose_batch computes (the reference's behaviour on float64
 * inputs) with the reference's float32 arithmetic: f32 src = dst + flow, row-order f32 means,
 * f32 centring, R and t rounded to f32 (oracle/ssf_oracle.c orc_kabsch_f32 restates each step).
 *   source rows: d_flow != NULL -> f32(d_dst + d_flow) (target = points + move_gt, :273), with
 *                d_src ignored; d_flow == NULL -> d_src (slove_RT_by_SVD(src, dst) directly).
 *   d_mask   nullable uint8 per point: rows with mask != 0 (the background of ssf_mask_pose_batch's
 *            d_bg_mask); NULL = every row.
 *   after_mask 1: d_out holds ssf_mask_pose_batch's results for these frames (same stream, before
 *            this call); T, Q, R, NBG and STATUS are replaced, the fit fields kept, and frames with
 *            SSF_POSE_GMM_FAILED / SSF_POSE_SYNC_FAILED left as they are.  0: d_out is written whole.
 *   d_out    [F * SSF_POSE_OUT_STRIDE] doubles (SSF_POSE_OUT_* below); R / t hold float32 values.
 * Asynchronous on stream.  One work-group per frame; the two means are serial in row order. */
int32_t ssf_kabsch_f32_batch(ssf_ctx* ctx, void* stream, int32_t n_frames, const float* d_src,
                             const float* d_dst, const float* d_flow, const int64_t* d_frame_off,
                             const uint8_t* d_mask, int32_t reflection, int32_t after_mask,
                             double* d_out);
/* Work-groups per frame of the GMM fit in ssf_mask_pose_batch (no reference counterpart;
 * results do not depend on it beyond f64 summation order): 0 = automatic (as many as keep the
 * chip full: ~256 / frames, at most 32; 1 for 256 frames and more), 1..32 = fixed.  Memory: a
 * launch with G > 1 keeps frames x G x 104 KiB of exchange slots in the context (grown on
 * demand, never shrunk): a fixed 32 on a 256-frame batch is ~850 MB.  With more
 * than one, a frame's points are cut into contiguous parts whose per-pass sums are exchanged
 * in global memory; a partner that never arrives gives status SSF_POSE_SYNC_FAILED. */
int32_t ssf_set_mask_split(ssf_ctx* ctx, int32_t parts_per_frame);
/* Frame scheduling of the next ssf_mask_pose_batch / _f64 launches (no reference counterpart: a
 * frame's result does not depend on when it runs, so every schedule gives the same outputs).
 *   d_order  nullable device int32 [n_order], a permutation of 0 .. n_order - 1 (caller-owned; it
 *            must stay valid until the launches that read it have run): the k-th frame dispatched
 *            is d_order[k].  Longest-first by the previous step's SSF_POSE_OUT_PASSES of the same
 *            sequences starts the slow frames first and shortens a launch's straggler tail.  A
 *            launch of n_frames != n_order fails with SSF_E_ARG; an entry out of range is skipped.
 *   queue    > 0 (frames on one work-group each): at most `queue` work-groups, each taking the
 *            next frame when its own is done (a frame queue: a slow frame holds one CU while the
 *            others drain the batch); 0 = one work-group per frame. */
int32_t ssf_set_mask_schedule(ssf_ctx* ctx, const int32_t* d_order, int32_t n_order, int32_t queue);
/* Seed the context's numpy-legacy RandomState (MT19937) -- the `np.random.seed(s)` the reference
 * never calls; every GMM frame then consumes 3 doubles in frame order, as the reference's global
 * RandomState does across frames. */
int32_t ssf_rng_seed(ssf_ctx* ctx, uint32_t seed);

/* ---------------------------------------------------------------------------------------
 * lidarOdometry.cpp (SSF path): frameRegistration() (src/lidarOdometry.cpp:145-159) ingests
 * [t, q] and publishResult() (:80-83) accumulates.  Batched prefix product over a sequence of
 * n relative poses (7 doubles each, q xyzw + t): d_abs[i] = d_abs[i-1] * d_rel[i], seeded with
 * h_start (nullable = identity).  One device thread walks the chain (it is inherently serial).
 */
int32_t ssf_accumulate_sequence(ssf_ctx* ctx, void* stream, int32_t n, const double* d_rel,
                                const double* h_start, double* d_abs);

/* ---------------------------------------------------------------------------------------
 * mapOptmization loop closure.
 *
 * ssf_voxel_grid_batch replaces pcl::VoxelGrid<PointXYZI>::filter as downSizeFilterICP
 * (leaf 0.1, src/mapOptmization.cpp:214-217, 461) and downSizeFilterMap (leaf 0.4, :406-409,
 * 462) use it: per cloud, the centroid (x, y, z, intensity) of every occupied cube, in voxel
 * index order.  d_xyzi: float4 points of n_clouds clouds at d_off / h_off (int64, n_clouds + 1);
 * d_out: float4 at the SAME offsets (a cloud's output never exceeds its input);
 * d_out_count: int32 per cloud.  Asynchronous on stream.
 */
int32_t ssf_voxel_grid_batch(ssf_ctx* ctx, void* stream, int32_t n_clouds, const float* d_xyzi,
                             const int64_t* d_off, const int64_t* h_off, float leaf,
                             float* d_out, int32_t* d_out_count);

/* ssf_icp_batch replaces pcl::IterativeClosestPoint<PointXYZI, PointXYZI>::align +
 * hasConverged + getFitnessScore + getFinalTransformation as addLoopFactor() uses them
 * (src/mapOptmization.cpp:224-238): n_prob independent (source, target) problems, float4
 * clouds at int64 offsets (device + host copies).  h_guess: n_prob row-major 4x4 float initial
 * transforms (nullable = identity).  h_out (host, n_prob * SSF_ICP_OUT_STRIDE doubles): the
 * final transformation (16, row-major, float values), fitness score, converged, iterations,
 * convergence state (SSF_ICP_*), correspondences of the last iteration.  Synchronous: the
 * iteration loop runs on device; the host only polls the per-problem done flags. */
typedef struct {
    int32_t max_iter;       /* setMaximumIterations (100)                              */
    float max_corr_dist;    /* setMaxCorrespondenceDistance (50)                       */
    double trans_eps;       /* setTransformationEpsilon (1e-6)                         */
    double fit_eps;         /* setEuclideanFitnessEpsilon (1e-6)                       */
} ssf_icp_params;
#define SSF_ICP_OUT_STRIDE 24
enum {
    SSF_ICP_OUT_T = 0, SSF_ICP_OUT_FITNESS = 16, SSF_ICP_OUT_CONVERGED = 17,
    SSF_ICP_OUT_ITERATIONS = 18, SSF_ICP_OUT_STATE = 19, SSF_ICP_OUT_NCORR = 20
};
enum {  /* pcl::registration::DefaultConvergenceCriteria::ConvergenceState */
    SSF_ICP_NOT_CONVERGED = 0, SSF_ICP_ITERATIONS = 1, SSF_ICP_TRANSFORM = 2, SSF_ICP_ABS_MSE = 3,
    SSF_ICP_REL_MSE = 4, SSF_ICP_NO_CORRESPONDENCES = 5
};
int32_t ssf_icp_params_default(ssf_icp_params* out);
int32_t ssf_icp_batch(ssf_ctx* ctx, void* stream, int32_t n_prob, const float* d_src,
                      const int64_t* d_src_off, const int64_t* h_src_off, const float* d_tgt,
                      const int64_t* d_tgt_off, const int64_t* h_tgt_off,
                      const ssf_icp_params* params, const float* h_guess, double* h_out);

#ifdef __cplusplus
}
#endif
#endif
