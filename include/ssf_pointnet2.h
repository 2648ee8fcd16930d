/*
 * ssf_pointnet2.h -- C ABI of the point-set operators of the TFlow scene-flow network
 *  on MI355X (gfx950).
 *
 * The reference imports these operators as `lib.pointnet2_utils` (the "pointutils" module of
 * scripts/ActiveSceneFlow/utils/utils.py:7 and utils/soflow.py:7), a CUDA extension that is not
 * vendored in the repository.  Each entry point below replaces one of its functions, with the
 * semantics of the reference's own torch restatement of that operator (cited per function).
 *
 * Conventions
 *   - d_ pointers are DEVICE pointers owned by the caller; `stream` is a hipStream_t (NULL = the
 *     default stream).  Every call is asynchronous on `stream` and stateless (no context).
 *   - Coordinates are [B, N, 3] float32 (the extension's "xyz_t" layout) unless stated;
 *     features are [B, C, N] float32; indices are int32.
 *   - Return 0 on success, <0 on error; ssf_pn2_last_error() describes the calling thread's
 *     last error.  Indices outside their range read as 0 and set *d_bad (device int32) to 1.
 */
#ifndef SSF_POINTNET2_H
#define SSF_POINTNET2_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define SSF_PN2_OK 0
#define SSF_PN2_E_ARG (-1)
#define SSF_PN2_E_HIP (-2)
#define SSF_PN2_KNN_MAX 32
#define SSF_PN2_UPSAMPLE_MAX_SPARSE 4096

const char* ssf_pn2_last_error(void);

/* pointutils.furthest_point_sample(xyz_t, npoint) (utils/utils.py:226; torch restatement
 * farthest_point_sample, :68-89): d_xyz [b, n, 3] -> d_idx [b, npoint].  The first centroid is
 * d_start[i] (nullable = 0, the extension's choice; the torch restatement draws it with
 * torch.randint).  Squared distances in f32 ((dx^2 + dy^2) + dz^2), running minimum, argmax with
 * ties to the lowest index (torch.max).  d_temp: b * n floats of scratch, needed when n > 16384
 * (nullable otherwise). */
int32_t ssf_pn2_furthest_point_sample(void* stream, int32_t b, int32_t n, int32_t npoint,
                                      const float* d_xyz, const int32_t* d_start, float* d_temp,
                                      int32_t* d_idx);

/* pointutils.knn(k, query, ref) (utils/utils.py:229,291,397,604; soflow.py:1461; torch
 * restatement knn_point, :92-108): for each of the s_q points of d_query [b, s_q, 3], the k
 * (<= 32) nearest of the n points of d_ref [b, n, 3], ascending by f32 squared distance, ties
 * to the lower index.  d_dist [b, s_q, k] = sqrt(squared distance) (:108), d_idx [b, s_q, k]. */
int32_t ssf_pn2_knn(void* stream, int32_t b, int32_t s_q, int32_t n, int32_t k,
                    const float* d_query, const float* d_ref, float* d_dist, int32_t* d_idx);

/* pointutils.three_nn(unknown, known) (utils/utils.py:560,658; soflow.py:1459): knn with k = 3,
 * d_dist / d_idx [b, n, 3]. */
int32_t ssf_pn2_three_nn(void* stream, int32_t b, int32_t n, int32_t m, const float* d_unknown,
                         const float* d_known, float* d_dist, int32_t* d_idx);

/* pointutils.gather_operation(features, idx) (utils/utils.py:228) with g = S indices per batch
 * element ([b, c, n] x [b, g] -> [b, c, g]), and pointutils.grouping_operation(features, idx)
 * (:231,233; soflow.py:30,1462,1472) with g = S * K ([b, c, n] x [b, S, K] -> [b, c, S, K]).
 * Torch restatements: index_points (utils.py:48-65), index_points_group (soflow.py:21-32). */
int32_t ssf_pn2_gather(void* stream, int32_t b, int32_t c, int32_t n, int32_t g,
                       const float* d_feat, const int32_t* d_idx, float* d_out, int32_t* d_bad);

/* The grouping block of PointNetSetAbstraction.forward (utils/utils.py:228-234) in one call:
 * out [b, 3 + c, s, k] = cat(grouping(xyz, idx) - new_xyz[..., None], grouping(feat, idx)),
 * with d_xyz [b, 3, n] (n <= 36864), d_new_xyz [b, 3, s], d_feat [b, c, n] (nullable when
 * c = 0), d_idx [b, s, k]. */
int32_t ssf_pn2_group_relative(void* stream, int32_t b, int32_t n, int32_t s, int32_t k, int32_t c,
                               const float* d_xyz, const float* d_new_xyz, const float* d_feat,
                               const int32_t* d_idx, float* d_out, int32_t* d_bad);

/* pointutils.three_interpolate(features [b, c, m], idx [b, n, 3], weight [b, n, 3]) ->
 * [b, c, n]: w0 f[i0] + w1 f[i1] + w2 f[i2] (the weighted 3-NN sum of
 * PointNetFeaturePropogation, utils/utils.py:658-663). */
int32_t ssf_pn2_three_interpolate(void* stream, int32_t b, int32_t c, int32_t m, int32_t n,
                                  const float* d_feat, const int32_t* d_idx, const float* d_weight,
                                  float* d_out, int32_t* d_bad);

/* UpsampleFlow.forward(xyz, sparse_xyz, sparse_flow, k) (utils/soflow.py:1442-1470), fused:
 * d_xyz [b, 3, n], d_sparse_xyz [b, 3, s] (s <= 4096), d_sparse_feat [b, c, s] -> d_out
 * [b, c, n]: k (<= 16) nearest sparse points (three_nn for k = 3), inverse Euclidean distances
 * (clamped at 1e-10) normalised to sum 1, weighted feature sum clamped to [-100, 100]. */
int32_t ssf_pn2_upsample_flow(void* stream, int32_t b, int32_t n, int32_t s, int32_t c, int32_t k,
                              const float* d_xyz, const float* d_sparse_xyz,
                              const float* d_sparse_feat, float* d_out);

#ifdef __cplusplus
}
#endif
#endif
