// ssf_internal.hpp -- host-side context and kernel-launch declarations (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/ssf_frontend.h"

namespace ssf {

// Device scratch owned by a context: grown on demand, never shrunk.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr; bytes = 0;
        }
        size_t want = need + need / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) { p = nullptr; return e; }
        bytes = want;
        return hipSuccess;
    }
    template <typename T> T* as() const { return static_cast<T*>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; }
};

// Kernel timing (ssf_profile_enable): a launcher calls kmark(stream, "k_name") right before
// each kernel it launches; the ABI entry that owns those launches closes the last interval.
// With timing off (the default) kmark is one thread-local load and a branch.
void kmark(hipStream_t s, const char* name);

#ifndef SSF_BIN_CHUNK
#define SSF_BIN_CHUNK 2048
#endif
constexpr int kBinChunk = SSF_BIN_CHUNK;   // points per binning work-group (2048: 8 points per
                                           // thread; 4096 measured 11-12 % slower binning)
constexpr int kMaxRows = 64;
#ifndef SSF_MASK_MAX_SPLIT
#define SSF_MASK_MAX_SPLIT 32
#endif
constexpr int kMaskMaxSplit = SSF_MASK_MAX_SPLIT;   // work-groups per frame of the GMM fit at most
// candidate flag bytes of a batch (k_bin_curv -> k_select, one per ring position, per frame
// 64-byte aligned) and the curvature fix-up lists (per-frame counts, then ring positions at the
// frame offsets)
size_t flag_bytes(int64_t total, int n_frames);
size_t fix_bytes(int64_t total, int n_frames);

// Per-correspondence record written by the association kernel, read by the solver.
struct alignas(16) CorrRec {
    float po[3]; float valid;   // current-frame point (untransformed), 1 if the plane is valid
    float pa[3]; float pad0;    // last-frame 1-NN point
    float n[3];  float pad1;    // plane normal (float, as matX0)
};

// ---- launchers (features.hip) ----
// Edge selection of launch_extract_planes (beyond the reference; nullptr = planes only):
// the per-row selection slots in ctx scratch, the compacted edge cloud (float4 x, y, z,
// intensity at the frame offsets) and per-frame counts out (the candidates ride in bit 1 of
// the planar flag bytes).
struct EdgeSel {
    float min_curv;
    int span;
    int32_t* sel;
    float4* out;
    int32_t* count;
};
// Scratch of the single-read feature stage (k_feat_chunk / k_feat_select, frames of at most
// 128 chunks): per-(chunk, row) counts -> row bases, u16 chunk positions per own-tile slot, the
// chunks' candidate / unresolved bit planes, and (debug outputs only) chunk-major curvature.
struct FeatScratch {
    const void* rtab;   // the ring-id table (build_ring_table), device copy
    int32_t* cnt;       // feat_cnt_bytes
    uint16_t* gidx;     // feat_idx_bytes
    uint64_t* gbits;    // feat_bits_bytes
    float* curv_cm;     // total floats (debug), else nullptr
    uint8_t* irr;       // feat_irr_bytes: per (frame, chunk) block, 1 = not a regular window
    uint8_t* lmap;      // feat_lmap_bytes: per regular block, row -> lane (64 B)
};
size_t feat_idx_bytes(int64_t total, int n_frames);
size_t feat_bits_bytes(int n_frames, int64_t max_pts);
size_t feat_cnt_bytes(int n_frames, int64_t max_pts);
size_t feat_irr_bytes(int n_frames, int64_t max_pts);
size_t feat_lmap_bytes(int n_frames, int64_t max_pts);
bool feat_single_read(int64_t max_pts);
// host: the ring-id table of n_rows (16 / 64) and ring_chain (SSF_RING_CHAIN_*) into out
// (ring_table_bytes); 0 or a negative code
int build_ring_table(int n_rows, int chain, void* out_host);
size_t ring_table_bytes();
hipError_t launch_extract_planes(hipStream_t s, const ssf_config& cfg, int n_frames,
                                 const float* pts, int stride, const int64_t* frame_off,
                                 int64_t max_pts, const uint8_t* keep, int8_t* rid, int32_t* hist,
                                 int32_t* ring_off, int32_t* ring_idx, float4* ring_xyzi,
                                 float* curv, uint8_t* flags, void* fix, int32_t* sel, float4* plane,
                                 int32_t* plane_count, const EdgeSel* edge = nullptr,
                                 const FeatScratch* fs = nullptr);

// ---- launchers (registration.hip) ----
hipError_t launch_plane_table(hipStream_t s, const ssf_config& cfg, int n_frames,
                              const float4* plane, const int64_t* frame_off, const int32_t* count,
                              int64_t max_m, float* normal, uint8_t* valid, float4* sorted_xyzi,
                              int32_t* sorted_idx, float4* strip_xyzi = nullptr,
                              int32_t* strip_head = nullptr);
// Point-to-line blocks of launch_register (beyond the reference; nullptr = planes only): the
// edge clouds, the last frames' line table (6 floats per edge: centroid, direction) and the
// correspondence scratch / per-pair counts.
struct EdgeReg {
    const float4* last;
    const int64_t* last_off;
    const int32_t* last_count;
    const float* line;
    const uint8_t* line_valid;
    const float4* curr;
    const int64_t* curr_off;
    const int32_t* curr_count;
    int64_t max_m;
    CorrRec* corr;
    int32_t* ncorr;
};
hipError_t launch_register(hipStream_t s, const ssf_config& cfg, int n_pairs, const float4* last,
                           const int64_t* last_off, const int32_t* last_count,
                           const float* last_normal, const uint8_t* last_valid,
                           const float4* last_sorted, const int32_t* last_sidx, const float4* curr,
                           const int64_t* curr_off, const int32_t* curr_count, int64_t max_m,
                           CorrRec* corr, double* pose_rel, double* pose_abs, double* log,
                           int32_t* nlog, int32_t* ncorr, int32_t* nn,
                           const EdgeReg* edge = nullptr, const float4* last_strip_xyzi = nullptr,
                           const int32_t* last_strip_head = nullptr, const double* pose_in = nullptr,
                           const double* pose_abs_in = nullptr, int32_t* nnv = nullptr,
                           int32_t* ncompact = nullptr);
// (nnv [>= the current frames' total points] and ncompact [>= n_pairs]: scratch that lets the
// lane-mode association hand the solve compacted records; nullptr = records in query order)
hipError_t launch_edge_table(hipStream_t s, const ssf_edge_config& ec, int n_frames,
                             const float4* edges, const int64_t* frame_off, const int32_t* count,
                             int64_t max_m, float* line, uint8_t* valid);
hipError_t launch_accumulate(hipStream_t s, int n, const double* rel, const double* start,
                             double* abs_out);

// ---- launchers (mask_pose.hip) ----
// G > 1 cuts every frame into G parts on G work-groups (sync: ticket + per-frame arrival
// counters, mask_sync_bytes; parts: exchange slots, mask_parts_bytes); slots = resident
// work-groups of k_mask_pose on the device (mask_pose_slots).  order (nullable): the dispatch
// order of the frames (a device permutation); queue > 0 (G == 1): at most `queue` work-groups
// taking frame tickets in order (the frame queue; sync holds the ticket).
hipError_t launch_mask_pose(hipStream_t s, int n_frames, const float* pts, const float* flow,
                            const int64_t* frame_off, int mode, const uint8_t* mask_in,
                            const double* draws, uint2* lloyd_rec, int reflection, uint8_t* bg_mask,
                            double* out, int G, int slots, uint32_t* sync, double* parts,
                            const int32_t* order = nullptr, int queue = 0);
hipError_t launch_mask_pose(hipStream_t s, int n_frames, const double* pts, const double* flow,
                            const int64_t* frame_off, int mode, const uint8_t* mask_in,
                            const double* draws, uint2* lloyd_rec, int reflection, uint8_t* bg_mask,
                            double* out, int G, int slots, uint32_t* sync, double* parts,
                            const int32_t* order = nullptr, int queue = 0);
int mask_pose_slots(int device);
// ---- launcher (kabsch_f32.hip): the float32 slove_RT_by_SVD + Quaternion tail per frame; source
// rows = dst + flow (f32) when flow is given, else src; keep_failures: leave frames whose status
// is SSF_POSE_GMM_FAILED / SSF_POSE_SYNC_FAILED (a k_mask_pose output) untouched.
hipError_t launch_kabsch_f32(hipStream_t s, int n_frames, const float* src, const float* dst,
                             const float* flow, const int64_t* frame_off, const uint8_t* mask,
                             int reflection, int keep_failures, double* out);
size_t mask_sync_bytes(int n_frames);
size_t mask_parts_bytes(int n_frames, int G);

// ---- launchers (loop.hip) ----
struct IcpState {             // one per ICP problem, device-resident across iterations
    float fin[16];            // final transformation (row-major, float as PCL's Matrix4f)
    double prev_mse;
    double fitness;
    int32_t it, done, state, converged, n_corr, pad;
};
typedef ssf_icp_params IcpParams;
size_t vg_scratch_bytes(int n_clouds, int64_t n);
hipError_t launch_voxel_grid(hipStream_t s, int n_clouds, const float4* pts, const int64_t* off,
                             int64_t n, int64_t max_pts, float leaf, void* scratch, float4* out,
                             int32_t* out_count);
hipError_t launch_icp_init(hipStream_t s, int n_prob, const float4* src, const int64_t* soff,
                           int64_t max_ns, const float* guess, float4* cur, IcpState* st,
                           unsigned long long* key);
hipError_t launch_icp_iteration(hipStream_t s, int n_prob, float4* cur, const int64_t* soff,
                                int64_t max_ns, const float4* tgt, const int64_t* toff,
                                int64_t max_nt, const IcpParams& prm, IcpState* st,
                                unsigned long long* key);
hipError_t launch_icp_fitness(hipStream_t s, int n_prob, const float4* src, const int64_t* soff,
                              int64_t total_ns, int64_t max_ns, const float4* tgt,
                              const int64_t* toff, int64_t max_nt, IcpState* st,
                              unsigned long long* key);

}  // namespace ssf
