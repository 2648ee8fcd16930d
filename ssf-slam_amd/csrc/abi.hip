// abi.hip -- extern "C" entry points of libssf_frontend.so (include/ssf_frontend.h).
//
// Host side of the boundary: argument checks, per-context device scratch (grown on demand,
// never shrunk; ssf_reserve pre-sizes it), the numpy-legacy RandomState used by the GMM
// k-means++ init, and kernel launches on the caller's stream.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "ssf_internal.hpp"

using ssf::DevBuf;

// Kernel timing (ssf_profile_enable): events recorded on the launching stream right before each
// kernel and at the end of the ABI call; consecutive events bracket one kernel.  On a stream
// that no other stream competes with, that is the kernel's own duration.
struct KTimer {
    bool on = false;
    struct Mark { hipEvent_t ev; const char* name; };   // name == nullptr closes an ABI call
    std::vector<Mark> marks;
    std::vector<hipEvent_t> pool;                       // events reused after every read
    static constexpr size_t kMaxMarks = 1 << 14;
    void mark(hipStream_t s, const char* name) {
        if (marks.size() >= kMaxMarks) return;          // unread backlog: stop recording
        if (marks.size() == pool.size()) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) return;
            pool.push_back(e);
        }
        hipEvent_t e = pool[marks.size()];
        if (hipEventRecord(e, s) != hipSuccess) return;
        marks.push_back({e, name});
    }
    void release() {
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
        pool.clear(); marks.clear();
    }
};

struct ssf_ctx {
    int device = 0;
    ssf_config cfg{};
    std::string err;
    // frameFeature scratch
    DevBuf rid, hist, ring_off, ring_xyzi /* ring index */, sel, sel_cnt /* candidate flags */, fix, plane1, off1, cnt1;
    // single-read feature stage: per-(chunk, row) counts, u16 chunk positions, bit planes,
    // chunk-major curvature (debug outputs only)
    DevBuf fcnt, fidx, fbits, fcurv, rtab, firr, flmap;
    bool rtab_ready = false;
    // registration scratch
    DevBuf corr;
    DevBuf cidx;                       // compacted-record scratch: per query (index, valid), per pair count
    // ssf_register_pair: offsets, counts, the last frame's plane table + search index, pose, log
    DevBuf pair;
    // mask: k-means++ draws staged per launch through a ring of slots, so launches on different
    // streams (e.g. consecutive batches overlapping their slow frames) never share a buffer
    struct DrawSlot {
        DevBuf d;
        DevBuf rec;                    // Lloyd label/bound records (8 B) + relabel queue (4 B) per point
        DevBuf sync, parts;            // frame split: ticket + arrival counters, exchange slots
        double* h = nullptr;           // pinned staging
        int64_t hcap = 0;
        hipEvent_t copied = nullptr;   // this slot's H2D finished: the staging may be rewritten
        hipEvent_t used = nullptr;     // the kernel that read this slot finished
    };
    static constexpr int kDrawSlots = 4;
    // edge features (beyond the reference): selection scratch, correspondence records
    ssf_edge_config ecfg{};
    DevBuf esel, ecorr;
    int mask_split = 0;                // ssf_set_mask_split: 0 = automatic
    const int32_t* mask_order = nullptr;   // ssf_set_mask_schedule
    int mask_order_n = 0, mask_queue = 0;
    int mask_slots = -1;               // resident k_mask_pose work-groups (queried once)
    DrawSlot dslot[kDrawSlots];
    int dnext = 0;
    DevBuf start1;
    // loop closure (loop.hip): voxel-grid sort scratch; ICP transformed source, 1-NN keys,
    // per-problem state and guesses
    DevBuf vg, icp_cur, icp_key, icp_st, icp_guess;
    // host RandomState (MT19937, numpy legacy seeding)
    uint32_t mt[624];
    int mt_pos = 625;
    std::map<int64_t, std::vector<double>> cdf_cache;  // choice(n, p=1/n) cumulative table
    KTimer prof;
};

namespace {
thread_local KTimer* t_prof = nullptr;   // the timer of the ABI call running on this thread

// Scope of one ABI call: its launches mark into the context's timer when timing is on.
struct ProfScope {
    KTimer* prev;
    KTimer* mine;
    hipStream_t s;
    ProfScope(ssf_ctx* c, void* stream)
        : prev(t_prof), mine(c && c->prof.on ? &c->prof : nullptr), s((hipStream_t)stream) {
        if (mine) t_prof = mine;
    }
    ~ProfScope() {
        if (mine) { mine->mark(s, nullptr); t_prof = prev; }
    }
};
}  // namespace

void ssf::kmark(hipStream_t s, const char* name) {
    if (t_prof) t_prof->mark(s, name);
}

namespace {

int32_t fail(ssf_ctx* c, int32_t code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int32_t hip_fail(ssf_ctx* c, hipError_t e, const char* where) {
    if (c) c->err = std::string(where) + ": " + hipGetErrorString(e);
    return SSF_E_HIP;
}

#define SSF_TRY_HIP(ctx, expr, where)                              \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return hip_fail((ctx), _e, (where)); \
    } while (0)

void mt_seed(ssf_ctx* c, uint32_t seed) {
    c->mt[0] = seed;
    for (int i = 1; i < 624; ++i) c->mt[i] = 1812433253u * (c->mt[i - 1] ^ (c->mt[i - 1] >> 30)) + (uint32_t)i;
    c->mt_pos = 624;
}

uint32_t mt_next(ssf_ctx* c) {
    if (c->mt_pos >= 624) {
        if (c->mt_pos > 624) mt_seed(c, 5489u);
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (c->mt[i] & 0x80000000u) | (c->mt[(i + 1) % 624] & 0x7fffffffu);
            c->mt[i] = c->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        c->mt_pos = 0;
    }
    uint32_t y = c->mt[c->mt_pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double mt_random_sample(ssf_ctx* c) {
    uint32_t a = mt_next(c) >> 5, b = mt_next(c) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// numpy RandomState.choice(n, p=ones/n): cdf = cumsum(p); cdf /= cdf[-1];
// searchsorted(cdf, u, side='right')  (sklearn _kmeans_plusplus first centre).
int64_t choice_uniform(ssf_ctx* c, int64_t n, double u) {
    auto it = c->cdf_cache.find(n);
    if (it == c->cdf_cache.end()) {
        if (c->cdf_cache.size() > 8) c->cdf_cache.clear();
        std::vector<double> cdf((size_t)n);
        const double p = 1.0 / (double)n;
        double s = 0.0;
        for (int64_t i = 0; i < n; ++i) { s += p; cdf[(size_t)i] = s; }
        const double last = cdf[(size_t)n - 1];
        for (auto& v : cdf) v /= last;
        it = c->cdf_cache.emplace(n, std::move(cdf)).first;
    }
    const auto& cdf = it->second;
    auto pos = std::upper_bound(cdf.begin(), cdf.end(), u);
    int64_t idx = (int64_t)(pos - cdf.begin());
    return idx < n ? idx : n - 1;
}

bool valid_cfg(const ssf_config& c) {
    return (c.n_rows == 16 || c.n_rows == 64) && c.plane_span >= 2 && c.row_start >= 0 &&
           c.row_end >= 0 && c.max_iter >= 0 && c.max_iter <= 64 &&
           (c.solver == SSF_SOLVER_CERES_LM || c.solver == SSF_SOLVER_GN) &&
           (c.ring_chain == SSF_RING_CHAIN_FLOAT || c.ring_chain == SSF_RING_CHAIN_DOUBLE);
}

}  // namespace

extern "C" {

int32_t ssf_abi_version(void) { return SSF_ABI_VERSION; }

int32_t ssf_config_default(int32_t n_rows, ssf_config* out) {
    if (!out) return SSF_E_ARG;
    std::memset(out, 0, sizeof(*out));
    out->n_rows = n_rows;
    out->solver = SSF_SOLVER_CERES_LM;
    out->max_iter = 8;                          // lidarOdometry_onlyPC.cpp:246
    out->ring_chain = SSF_RING_CHAIN_FLOAT;     // frameFeature.cpp:57 under libstdc++
    if (n_rows == 16) {                         // frameFeature.cpp:143-146, onlyPC:314-316
        out->plane_min = 0.05f; out->plane_span = 3; out->plane_max = 0.15f;
        return SSF_OK;
    }
    if (n_rows == 64) {                         // frameFeature.cpp:147-152, onlyPC:317-319
        out->plane_min = 0.005f; out->plane_span = 25; out->row_start = 5; out->row_end = 5;
        out->plane_max = 0.05f;
        return SSF_OK;
    }
    return SSF_E_ARG;
}

int32_t ssf_create(int32_t device, const ssf_config* cfg, ssf_ctx** out) {
    if (!out || !cfg || !valid_cfg(*cfg)) return SSF_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SSF_E_NODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SSF_E_NODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SSF_E_NODEV;
    ssf_ctx* c = new (std::nothrow) ssf_ctx();
    if (!c) return SSF_E_NOMEM;
    c->device = device;
    c->cfg = *cfg;
    ssf_edge_config_default(cfg->n_rows, &c->ecfg);
    *out = c;
    return SSF_OK;
}

void ssf_destroy(ssf_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    DevBuf* bufs[] = {&c->rid, &c->hist, &c->ring_off, &c->ring_xyzi, &c->sel, &c->sel_cnt, &c->fix,
                      &c->plane1, &c->off1, &c->cnt1, &c->corr, &c->cidx, &c->pair, &c->start1, &c->vg,
                      &c->icp_cur, &c->icp_key, &c->icp_st, &c->icp_guess, &c->esel,
                      &c->ecorr, &c->fcnt, &c->fidx, &c->fbits, &c->fcurv, &c->rtab, &c->firr, &c->flmap};
    for (auto& ds : c->dslot) {
        if (ds.used) { (void)hipEventSynchronize(ds.used); (void)hipEventDestroy(ds.used); }
        if (ds.copied) { (void)hipEventSynchronize(ds.copied); (void)hipEventDestroy(ds.copied); }
        if (ds.h) (void)hipHostFree(ds.h);
        ds.d.release();
        ds.rec.release();
        ds.sync.release();
        ds.parts.release();
    }
    for (DevBuf* b : bufs) b->release();
    if (!c->prof.marks.empty()) (void)hipEventSynchronize(c->prof.marks.back().ev);
    c->prof.release();
    delete c;
}

int32_t ssf_profile_enable(ssf_ctx* c, int32_t on) {
    if (!c) return SSF_E_ARG;
    c->prof.on = on != 0;
    return SSF_OK;
}

int32_t ssf_profile_read(ssf_ctx* c, ssf_kernel_time* out, int32_t cap, int32_t* n_out) {
    if (!c || !n_out || cap < 0 || (cap > 0 && !out)) return SSF_E_ARG;
    *n_out = 0;
    KTimer& P = c->prof;
    if (P.marks.empty()) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    for (const auto& m : P.marks) SSF_TRY_HIP(c, hipEventSynchronize(m.ev), "profile sync");
    int n = 0;
    for (size_t i = 0; i + 1 < P.marks.size(); ++i) {
        const char* nm = P.marks[i].name;
        if (!nm) continue;                               // between two ABI calls: no kernel
        float ms = 0.0f;
        SSF_TRY_HIP(c, hipEventElapsedTime(&ms, P.marks[i].ev, P.marks[i + 1].ev), "profile elapsed");
        int k = 0;
        while (k < n && std::strncmp(out[k].name, nm, sizeof(out[k].name)) != 0) ++k;
        if (k == n) {
            if (n == cap) continue;
            std::memset(&out[k], 0, sizeof(out[k]));
            std::strncpy(out[k].name, nm, sizeof(out[k].name) - 1);
            ++n;
        }
        out[k].launches += 1;
        out[k].total_ms += ms;
    }
    P.marks.clear();
    *n_out = n;
    return SSF_OK;
}

const char* ssf_last_error(const ssf_ctx* c) { return c ? c->err.c_str() : "null context"; }

int32_t ssf_set_mask_schedule(ssf_ctx* c, const int32_t* d_order, int32_t n_order, int32_t queue) {
    if (!c) return SSF_E_ARG;
    if (queue < 0 || (d_order && n_order <= 0)) return fail(c, SSF_E_ARG, "set_mask_schedule: bad arguments");
    c->mask_order = d_order;
    c->mask_order_n = d_order ? n_order : 0;
    c->mask_queue = queue;
    return SSF_OK;
}

int32_t ssf_set_mask_split(ssf_ctx* c, int32_t parts_per_frame) {
    if (!c || parts_per_frame < 0 || parts_per_frame > ssf::kMaskMaxSplit) return SSF_E_ARG;
    c->mask_split = parts_per_frame;
    return SSF_OK;
}

int32_t ssf_edge_config_default(int32_t n_rows, ssf_edge_config* out) {
    if (!out || (n_rows != 16 && n_rows != 64)) return SSF_E_ARG;
    out->edge_min = 1.0f;
    out->edge_span = n_rows == 64 ? 10 : 3;
    out->line_ratio = 3.0f;
    out->max_nn_d2 = 1.0f;
    return SSF_OK;
}

int32_t ssf_set_edge_config(ssf_ctx* c, const ssf_edge_config* ec) {
    if (!c || !ec || ec->edge_span < 1 || !(ec->line_ratio >= 1.0f) || !(ec->max_nn_d2 > 0.0f))
        return c ? fail(c, SSF_E_ARG, "set_edge_config: bad arguments") : SSF_E_ARG;
    c->ecfg = *ec;
    return SSF_OK;
}

int32_t ssf_rng_seed(ssf_ctx* c, uint32_t seed) {
    if (!c) return SSF_E_ARG;
    mt_seed(c, seed);
    return SSF_OK;
}

static int32_t ensure_features(ssf_ctx* c, int32_t n_frames, int64_t total, int64_t max_pts) {
    const int R = c->cfg.n_rows;
    const int64_t n_chunks = (max_pts + ssf::kBinChunk - 1) / ssf::kBinChunk;
    SSF_TRY_HIP(c, c->rid.ensure((size_t)std::max<int64_t>(total, 1)), "alloc rid");
    SSF_TRY_HIP(c, c->hist.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(n_frames * n_chunks * R, 1)), "alloc hist");
    SSF_TRY_HIP(c, c->ring_off.ensure(sizeof(int32_t) * (size_t)n_frames * (R + 1)), "alloc ring_off");
    // ring index (input index per ring position), per-row selection slots (indexInRow at ring
    // positions, k_select), candidate flag bytes, curvature fix-up list
    SSF_TRY_HIP(c, c->ring_xyzi.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(total, 1)), "alloc ring index");
    SSF_TRY_HIP(c, c->sel.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(total, 1)), "alloc sel");
    SSF_TRY_HIP(c, c->sel_cnt.ensure(ssf::flag_bytes(total, n_frames)), "alloc cand flags");
    SSF_TRY_HIP(c, c->fix.ensure(ssf::fix_bytes(total, n_frames)), "alloc curvature fix-up list");
    if (!c->rtab_ready) {                           // every feature path looks ring ids up in it
        std::vector<char> h(ssf::ring_table_bytes());
        const int rc = ssf::build_ring_table(R, c->cfg.ring_chain, h.data());
        if (rc) return fail(c, SSF_E_ARG, "ring-id table: build failed (" + std::to_string(rc) + ")");
        SSF_TRY_HIP(c, c->rtab.ensure(h.size()), "alloc ring table");
        SSF_TRY_HIP(c, hipMemcpy(c->rtab.p, h.data(), h.size(), hipMemcpyHostToDevice), "H2D ring table");
        c->rtab_ready = true;
    }
    if (ssf::feat_single_read(max_pts)) {
        SSF_TRY_HIP(c, c->fcnt.ensure(ssf::feat_cnt_bytes(n_frames, max_pts)), "alloc feature counts");
        SSF_TRY_HIP(c, c->fidx.ensure(ssf::feat_idx_bytes(total, n_frames)), "alloc feature index");
        SSF_TRY_HIP(c, c->fbits.ensure(ssf::feat_bits_bytes(n_frames, max_pts)), "alloc feature bits");
        SSF_TRY_HIP(c, c->firr.ensure(ssf::feat_irr_bytes(n_frames, max_pts)), "alloc feature block flags");
        SSF_TRY_HIP(c, c->flmap.ensure(ssf::feat_lmap_bytes(n_frames, max_pts)), "alloc feature lane maps");
    }
    return SSF_OK;
}

int32_t ssf_reserve(ssf_ctx* c, int32_t max_frames, int64_t max_points_per_frame) {
    if (!c || max_frames < 0 || max_points_per_frame < 0) return SSF_E_ARG;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    const int64_t total = (int64_t)max_frames * max_points_per_frame;
    int32_t rc = ensure_features(c, max_frames, total, max_points_per_frame);
    if (rc) return rc;
    SSF_TRY_HIP(c, c->corr.ensure(sizeof(ssf::CorrRec) * (size_t)std::max<int64_t>(total, 1)), "alloc corr");
    SSF_TRY_HIP(c, c->cidx.ensure(sizeof(int32_t) * ((size_t)std::max<int64_t>(total, 1) + (size_t)max_frames)),
                "alloc corr index");
    for (auto& ds : c->dslot) {
        SSF_TRY_HIP(c, ds.d.ensure(sizeof(double) * 3 * (size_t)std::max(max_frames, 1)), "alloc draws");
        SSF_TRY_HIP(c, ds.rec.ensure(sizeof(uint2) * (size_t)(total + 2 * (int64_t)max_frames + 2) + sizeof(uint32_t) * (size_t)(total + 64 * (int64_t)max_frames)), "alloc lloyd records");
        SSF_TRY_HIP(c, ds.sync.ensure(ssf::mask_sync_bytes(std::max(max_frames, 1)) + 16), "alloc mask sync");
        // exchange slots of the automatic split for max_frames (a fixed split grows them on demand)
        if (c->mask_slots < 0) c->mask_slots = ssf::mask_pose_slots(c->device);
        const int g_auto = std::max(1, std::min(ssf::kMaskMaxSplit, c->mask_slots > 0 ? c->mask_slots / std::max(max_frames, 1) : 1));
        const size_t pb = ssf::mask_parts_bytes(std::max(max_frames, 1), g_auto);
        if (pb) SSF_TRY_HIP(c, ds.parts.ensure(pb), "alloc mask parts");
    }
    return SSF_OK;
}

static int32_t extract_planes_impl(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_pts,
                                   int32_t point_stride, const int64_t* d_frame_off,
                                   int64_t total_points, int64_t max_frame_points,
                                   const uint8_t* d_keep, float* d_plane_xyzi,
                                   int32_t* d_plane_count, float* d_ring_xyzi, int32_t* d_ring_off,
                                   float* d_curv, float* d_edge_xyzi = nullptr,
                                   int32_t* d_edge_count = nullptr) {
    if (!c) return SSF_E_ARG;
    if (n_frames < 0 || point_stride < 3 || total_points < 0 || max_frame_points < 0 ||
        (n_frames > 0 && (!d_pts || !d_frame_off || !d_plane_xyzi || !d_plane_count)))
        return fail(c, SSF_E_ARG, "extract_planes_batch: bad arguments");
    if (max_frame_points >= ((int64_t)1 << 24))
        return fail(c, SSF_E_ARG, "extract_planes_batch: frames of at most 16777215 points (24-bit ring positions)");
    if (n_frames == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    int32_t rc = ensure_features(c, n_frames, total_points, max_frame_points);
    if (rc) return rc;
    ssf::EdgeSel es{};
    const bool edges = d_edge_xyzi != nullptr;
    if (edges) {
        SSF_TRY_HIP(c, c->esel.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(total_points, 1)), "alloc esel");
        es = ssf::EdgeSel{c->ecfg.edge_min, c->ecfg.edge_span,
                          c->esel.as<int32_t>(), reinterpret_cast<float4*>(d_edge_xyzi), d_edge_count};
    }
    float4* ring4 = reinterpret_cast<float4*>(d_ring_xyzi);   // debug output only (nullable)
    if ((ring4 || d_curv) && ssf::feat_single_read(max_frame_points))
        SSF_TRY_HIP(c, c->fcurv.ensure(sizeof(float) * (size_t)std::max<int64_t>(total_points, 1)), "alloc chunk curvature");
    ssf::FeatScratch fs{c->rtab.p, c->fcnt.as<int32_t>(), c->fidx.as<uint16_t>(), c->fbits.as<uint64_t>(),
                        c->fcurv.as<float>(), c->firr.as<uint8_t>(), c->flmap.as<uint8_t>()};
    ProfScope prof(c, stream);
    int32_t* roff = d_ring_off ? d_ring_off : c->ring_off.as<int32_t>();
    hipError_t e = ssf::launch_extract_planes(
        (hipStream_t)stream, c->cfg, n_frames, d_pts, point_stride, d_frame_off, max_frame_points,
        d_keep, c->rid.as<int8_t>(), c->hist.as<int32_t>(), roff, c->ring_xyzi.as<int32_t>(), ring4,
        d_curv, c->sel_cnt.as<uint8_t>(), c->fix.p, c->sel.as<int32_t>(),
        reinterpret_cast<float4*>(d_plane_xyzi), d_plane_count, edges ? &es : nullptr, &fs);
    if (e != hipSuccess) return hip_fail(c, e, "extract_planes launch");
    return SSF_OK;
}

int32_t ssf_extract_planes_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_pts,
                                 int32_t point_stride, const int64_t* d_frame_off,
                                 int64_t total_points, int64_t max_frame_points,
                                 float* d_plane_xyzi, int32_t* d_plane_count, float* d_ring_xyzi,
                                 int32_t* d_ring_off, float* d_curv) {
    return extract_planes_impl(c, stream, n_frames, d_pts, point_stride, d_frame_off, total_points,
                               max_frame_points, nullptr, d_plane_xyzi, d_plane_count, d_ring_xyzi,
                               d_ring_off, d_curv);
}

int32_t ssf_extract_planes_batch_masked(ssf_ctx* c, void* stream, int32_t n_frames,
                                        const float* d_pts, int32_t point_stride,
                                        const int64_t* d_frame_off, int64_t total_points,
                                        int64_t max_frame_points, const uint8_t* d_keep,
                                        float* d_plane_xyzi, int32_t* d_plane_count,
                                        float* d_ring_xyzi, int32_t* d_ring_off, float* d_curv) {
    if (c && n_frames > 0 && !d_keep) return fail(c, SSF_E_ARG, "extract_planes_batch_masked: null keep mask");
    return extract_planes_impl(c, stream, n_frames, d_pts, point_stride, d_frame_off, total_points,
                               max_frame_points, d_keep, d_plane_xyzi, d_plane_count, d_ring_xyzi,
                               d_ring_off, d_curv);
}

int32_t ssf_extract_features_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_pts,
                                   int32_t point_stride, const int64_t* d_frame_off,
                                   int64_t total_points, int64_t max_frame_points,
                                   const uint8_t* d_keep, float* d_plane_xyzi,
                                   int32_t* d_plane_count, float* d_edge_xyzi,
                                   int32_t* d_edge_count) {
    if (c && n_frames > 0 && (!d_edge_xyzi || !d_edge_count))
        return fail(c, SSF_E_ARG, "extract_features_batch: null edge outputs");
    return extract_planes_impl(c, stream, n_frames, d_pts, point_stride, d_frame_off, total_points,
                               max_frame_points, d_keep, d_plane_xyzi, d_plane_count, nullptr,
                               nullptr, nullptr, d_edge_xyzi, d_edge_count);
}

int32_t ssf_edge_table_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_edge_xyzi,
                             const int64_t* d_frame_off, const int32_t* d_edge_count,
                             int64_t max_edge_points, float* d_line, uint8_t* d_line_valid) {
    if (!c) return SSF_E_ARG;
    if (n_frames < 0 || max_edge_points < 0 ||
        (n_frames > 0 && (!d_edge_xyzi || !d_frame_off || !d_edge_count || !d_line || !d_line_valid)))
        return fail(c, SSF_E_ARG, "edge_table_batch: bad arguments");
    if (n_frames == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_edge_table((hipStream_t)stream, c->ecfg, n_frames,
                                         reinterpret_cast<const float4*>(d_edge_xyzi), d_frame_off,
                                         d_edge_count, max_edge_points, d_line, d_line_valid);
    if (e != hipSuccess) return hip_fail(c, e, "edge_table launch");
    return SSF_OK;
}

int32_t ssf_extract_planes(ssf_ctx* c, void* stream, const float* d_pts, int64_t n,
                           int32_t point_step_bytes, int32_t xyz_offset_bytes, float* d_out_xyzi,
                           int64_t* h_out_m, int64_t out_cap) {
    if (!c) return SSF_E_ARG;
    if (n < 0 || !h_out_m || point_step_bytes < 12 || point_step_bytes % 4 || xyz_offset_bytes < 0 ||
        xyz_offset_bytes % 4 || xyz_offset_bytes + 12 > point_step_bytes || (n > 0 && (!d_pts || !d_out_xyzi)))
        return fail(c, SSF_E_ARG, "extract_planes: bad arguments");
    *h_out_m = 0;
    if (n == 0) return SSF_OK;
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->off1.ensure(2 * sizeof(int64_t)), "alloc off1");
    SSF_TRY_HIP(c, c->cnt1.ensure(sizeof(int32_t)), "alloc cnt1");
    SSF_TRY_HIP(c, c->plane1.ensure(sizeof(float4) * (size_t)n), "alloc plane1");
    const int64_t off[2] = {0, n};
    SSF_TRY_HIP(c, hipMemcpyAsync(c->off1.p, off, sizeof(off), hipMemcpyHostToDevice, s), "H2D off");
    const float* base = reinterpret_cast<const float*>(reinterpret_cast<const char*>(d_pts) + xyz_offset_bytes);
    int32_t rc = ssf_extract_planes_batch(c, stream, 1, base, point_step_bytes / 4, c->off1.as<int64_t>(), n, n,
                                          c->plane1.as<float>(), c->cnt1.as<int32_t>(), nullptr, nullptr, nullptr);
    if (rc) return rc;
    int32_t m = 0;
    SSF_TRY_HIP(c, hipMemcpyAsync(&m, c->cnt1.p, sizeof(m), hipMemcpyDeviceToHost, s), "D2H count");
    SSF_TRY_HIP(c, hipStreamSynchronize(s), "sync");
    *h_out_m = m;
    if (m > out_cap) return fail(c, SSF_E_CAPACITY, "extract_planes: " + std::to_string(m) + " plane points exceed out_cap");
    if (m > 0)
        SSF_TRY_HIP(c, hipMemcpyAsync(d_out_xyzi, c->plane1.p, sizeof(float4) * (size_t)m, hipMemcpyDeviceToDevice, s), "D2D planes");
    return SSF_OK;
}

int32_t ssf_plane_table_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_plane_xyzi,
                              const int64_t* d_frame_off, const int32_t* d_plane_count,
                              int64_t max_plane_points, float* d_normal, uint8_t* d_valid,
                              float* d_sorted_xyzi, int32_t* d_sorted_idx, float* d_strip_xyzi,
                              int32_t* d_strip_head) {
    if (!c) return SSF_E_ARG;
    if (n_frames < 0 || max_plane_points < 0 ||
        (n_frames > 0 && (!d_plane_xyzi || !d_frame_off || !d_plane_count || !d_normal || !d_valid)))
        return fail(c, SSF_E_ARG, "plane_table_batch: bad arguments");
    if (!d_strip_xyzi != !d_strip_head || (d_strip_xyzi && (!d_sorted_xyzi || !d_sorted_idx)))
        return fail(c, SSF_E_ARG, "plane_table_batch: the strip image needs both strip buffers and the sorted buffers");
    if (n_frames == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_plane_table((hipStream_t)stream, c->cfg, n_frames,
                                           reinterpret_cast<const float4*>(d_plane_xyzi), d_frame_off,
                                           d_plane_count, max_plane_points, d_normal, d_valid,
                                           reinterpret_cast<float4*>(d_sorted_xyzi), d_sorted_idx,
                                           reinterpret_cast<float4*>(d_strip_xyzi), d_strip_head);
    if (e != hipSuccess) return hip_fail(c, e, "plane_table launch");
    return SSF_OK;
}

int32_t ssf_register_batch(ssf_ctx* c, void* stream, int32_t n_pairs, const float* d_last_xyzi,
                           const int64_t* d_last_off, const int32_t* d_last_count,
                           const float* d_last_normal, const uint8_t* d_last_valid,
                           const float* d_last_sorted_xyzi, const int32_t* d_last_sorted_idx,
                           const float* d_curr_xyzi, const int64_t* d_curr_off,
                           const int32_t* d_curr_count, int64_t curr_total_points,
                           int64_t max_plane_points, double* d_pose_rel, double* d_pose_abs,
                           double* d_log, int32_t* d_nlog, int32_t* d_ncorr, int32_t* d_nn,
                           const float* d_last_strip_xyzi, const int32_t* d_last_strip_head) {
    if (!c) return SSF_E_ARG;
    if (n_pairs < 0 || curr_total_points < 0 || max_plane_points < 0 ||
        (n_pairs > 0 && (!d_last_xyzi || !d_last_off || !d_last_count || !d_last_normal ||
                         !d_last_valid || !d_curr_xyzi || !d_curr_off || !d_curr_count || !d_pose_rel)))
        return fail(c, SSF_E_ARG, "register_batch: bad arguments");
    if (!d_last_strip_xyzi != !d_last_strip_head ||
        (d_last_strip_xyzi && (!d_last_sorted_xyzi || !d_last_sorted_idx)))
        return fail(c, SSF_E_ARG, "register_batch: the strip image needs both strip buffers and the sorted buffers");
    if (n_pairs == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->corr.ensure(sizeof(ssf::CorrRec) * (size_t)std::max<int64_t>(curr_total_points, 1)), "alloc corr");
    const size_t nq = (size_t)std::max<int64_t>(curr_total_points, 1);
    SSF_TRY_HIP(c, c->cidx.ensure(sizeof(int32_t) * (nq + (size_t)n_pairs)), "alloc corr index");
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_register(
        (hipStream_t)stream, c->cfg, n_pairs, reinterpret_cast<const float4*>(d_last_xyzi), d_last_off,
        d_last_count, d_last_normal, d_last_valid, reinterpret_cast<const float4*>(d_last_sorted_xyzi),
        d_last_sorted_idx, reinterpret_cast<const float4*>(d_curr_xyzi), d_curr_off,
        d_curr_count, max_plane_points, c->corr.as<ssf::CorrRec>(), d_pose_rel, d_pose_abs, d_log,
        d_nlog, d_ncorr, d_nn, nullptr, reinterpret_cast<const float4*>(d_last_strip_xyzi),
        d_last_strip_head, nullptr, nullptr, c->cidx.as<int32_t>(), c->cidx.as<int32_t>() + nq);
    if (e != hipSuccess) return hip_fail(c, e, "register launch");
    return SSF_OK;
}

int32_t ssf_register_chain(ssf_ctx* c, void* stream, int32_t n_pairs, const float* d_xyzi,
                           const int64_t* d_off, const int32_t* d_count, const float* d_normal,
                           const uint8_t* d_valid, const float* d_sorted_xyzi,
                           const int32_t* d_sorted_idx, int64_t total_points,
                           int64_t max_plane_points, const double* d_pose_init,
                           double* d_pose_seq, const double* d_pose_abs_init,
                           double* d_pose_abs_seq, int32_t* d_ncorr,
                           const float* d_strip_xyzi, const int32_t* d_strip_head) {
    if (!c) return SSF_E_ARG;
    if (n_pairs < 0 || total_points < 0 || max_plane_points < 0 ||
        (n_pairs > 0 && (!d_xyzi || !d_off || !d_count || !d_normal || !d_valid || !d_pose_init ||
                         !d_pose_seq)) ||
        (!d_pose_abs_init != !d_pose_abs_seq))
        return fail(c, SSF_E_ARG, "register_chain: bad arguments");
    if (!d_strip_xyzi != !d_strip_head || (d_strip_xyzi && (!d_sorted_xyzi || !d_sorted_idx)))
        return fail(c, SSF_E_ARG, "register_chain: the strip image needs both strip buffers and the sorted buffers");
    if (n_pairs == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->corr.ensure(sizeof(ssf::CorrRec) * (size_t)std::max<int64_t>(total_points, 1)), "alloc corr");
    ProfScope prof(c, stream);
    // pair k = (frame k, frame k + 1) of the same arrays: its warm start is pair k - 1's output
    // slot (lidarOdometry_onlyPC.cpp:164,251-252), read in place by the association and the
    // solve -- no copy between the links, two launches per pair, all enqueued here
    const float4* X = reinterpret_cast<const float4*>(d_xyzi);
    for (int k = 0; k < n_pairs; ++k) {
        hipError_t e = ssf::launch_register(
            (hipStream_t)stream, c->cfg, 1, X, d_off + k, d_count + k, d_normal, d_valid,
            reinterpret_cast<const float4*>(d_sorted_xyzi), d_sorted_idx, X, d_off + k + 1,
            d_count + k + 1, max_plane_points, c->corr.as<ssf::CorrRec>(), d_pose_seq + 7 * k,
            d_pose_abs_seq ? d_pose_abs_seq + 7 * k : nullptr, nullptr, nullptr,
            d_ncorr ? d_ncorr + k : nullptr, nullptr, nullptr,
            reinterpret_cast<const float4*>(d_strip_xyzi), d_strip_head,
            k == 0 ? d_pose_init : d_pose_seq + 7 * (k - 1),
            d_pose_abs_seq ? (k == 0 ? d_pose_abs_init : d_pose_abs_seq + 7 * (k - 1)) : nullptr);
        if (e != hipSuccess) return hip_fail(c, e, "register_chain launch");
    }
    return SSF_OK;
}

int32_t ssf_register_batch_edges(ssf_ctx* c, void* stream, int32_t n_pairs,
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
                                 const float* d_last_strip_xyzi, const int32_t* d_last_strip_head) {
    if (!c) return SSF_E_ARG;
    if (!d_last_strip_xyzi != !d_last_strip_head ||
        (d_last_strip_xyzi && (!d_last_sorted_xyzi || !d_last_sorted_idx)))
        return fail(c, SSF_E_ARG, "register_batch_edges: the strip image needs both strip buffers and the sorted buffers");
    if (n_pairs < 0 || curr_total_points < 0 || max_plane_points < 0 || curr_edge_total < 0 ||
        max_edge_points < 0 ||
        (n_pairs > 0 && (!d_last_xyzi || !d_last_off || !d_last_count || !d_last_normal ||
                         !d_last_valid || !d_curr_xyzi || !d_curr_off || !d_curr_count || !d_pose_rel ||
                         !d_last_edge_xyzi || !d_last_edge_off || !d_last_edge_count || !d_last_line ||
                         !d_last_line_valid || !d_curr_edge_xyzi || !d_curr_edge_off || !d_curr_edge_count)))
        return fail(c, SSF_E_ARG, "register_batch_edges: bad arguments");
    if (n_pairs == 0) return SSF_OK;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->corr.ensure(sizeof(ssf::CorrRec) * (size_t)std::max<int64_t>(curr_total_points, 1)), "alloc corr");
    SSF_TRY_HIP(c, c->ecorr.ensure(sizeof(ssf::CorrRec) * (size_t)std::max<int64_t>(curr_edge_total, 1)), "alloc edge corr");
    if (max_edge_points == 0) {
        // no edge point anywhere: the edge records are never read, but their counts are
        SSF_TRY_HIP(c, hipMemsetAsync(c->ecorr.p, 0, sizeof(ssf::CorrRec), (hipStream_t)stream), "zero ecorr");
    }
    ProfScope prof(c, stream);
    const ssf::EdgeReg er{reinterpret_cast<const float4*>(d_last_edge_xyzi), d_last_edge_off,
                          d_last_edge_count, d_last_line, d_last_line_valid,
                          reinterpret_cast<const float4*>(d_curr_edge_xyzi), d_curr_edge_off,
                          d_curr_edge_count, max_edge_points, c->ecorr.as<ssf::CorrRec>(), d_ncorr_edge};
    hipError_t e = ssf::launch_register(
        (hipStream_t)stream, c->cfg, n_pairs, reinterpret_cast<const float4*>(d_last_xyzi), d_last_off,
        d_last_count, d_last_normal, d_last_valid, reinterpret_cast<const float4*>(d_last_sorted_xyzi),
        d_last_sorted_idx, reinterpret_cast<const float4*>(d_curr_xyzi), d_curr_off,
        d_curr_count, max_plane_points, c->corr.as<ssf::CorrRec>(), d_pose_rel, d_pose_abs, d_log,
        d_nlog, d_ncorr, nullptr, &er, reinterpret_cast<const float4*>(d_last_strip_xyzi),
        d_last_strip_head);
    if (e != hipSuccess) return hip_fail(c, e, "register_edges launch");
    return SSF_OK;
}

int32_t ssf_register_pair(ssf_ctx* c, void* stream, const float* d_last_xyzi, int64_t m_last,
                          const float* d_curr_xyzi, int64_t m_curr, const double* h_q_init,
                          const double* h_t_init, double* h_q_out, double* h_t_out,
                          ssf_step_log* log) {
    if (!c) return SSF_E_ARG;
    if (m_last < 0 || m_curr < 0 || m_last > INT32_MAX || m_curr > INT32_MAX || !h_q_init ||
        !h_t_init || !h_q_out || !h_t_out || (m_last > 0 && !d_last_xyzi) ||
        (m_curr > 0 && !d_curr_xyzi) || (log && log->cap > 0 && !log->steps))
        return fail(c, SSF_E_ARG, "register_pair: bad arguments");
    double pose[7] = {h_q_init[0], h_q_init[1], h_q_init[2], h_q_init[3], h_t_init[0], h_t_init[1], h_t_init[2]};
    if (log) { log->n_steps = 0; log->n_corr = -1; }
    if (m_last <= 10 || m_curr == 0) {             // :158 -- no residuals, the warm start stands
        for (int k = 0; k < 4; ++k) h_q_out[k] = pose[k];
        for (int k = 0; k < 3; ++k) h_t_out[k] = pose[4 + k];
        if (log && m_last > 10) log->n_corr = 0;
        return SSF_OK;
    }
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    const int max_iter = c->cfg.max_iter;
    const int64_t mx = std::max(m_last, m_curr);
    // scratch layout (8-byte aligned pieces): offsets, counts, pose, log doubles, nlog/ncorr,
    // normals, valid, sorted cloud (16 B aligned), sorted index
    auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t o_off = 0, o_cnt = al(o_off + 4 * sizeof(int64_t)), o_pose = al(o_cnt + 4 * sizeof(int32_t));
    const size_t o_log = al(o_pose + 7 * sizeof(double));
    const size_t o_nl = al(o_log + (size_t)std::max(max_iter, 1) * 10 * sizeof(double));
    const size_t o_nrm = al(o_nl + 2 * sizeof(int32_t));
    const size_t o_val = al(o_nrm + 3 * sizeof(float) * (size_t)m_last);
    const size_t o_srt = al(o_val + (size_t)m_last);
    const size_t o_sid = al(o_srt + sizeof(float4) * (size_t)m_last);
    const size_t o_sim = al(o_sid + sizeof(int32_t) * (size_t)m_last);
    const size_t o_shd = al(o_sim + sizeof(float4) * (size_t)m_last);
    const size_t bytes = al(o_shd + sizeof(int32_t) * (size_t)m_last);
    SSF_TRY_HIP(c, c->pair.ensure(bytes), "alloc pair scratch");
    char* P = c->pair.as<char>();
    int64_t* d_off = reinterpret_cast<int64_t*>(P + o_off);     // [0, m_last] and [0, m_curr]
    int32_t* d_cnt = reinterpret_cast<int32_t*>(P + o_cnt);
    double* d_pose = reinterpret_cast<double*>(P + o_pose);
    double* d_log = reinterpret_cast<double*>(P + o_log);
    int32_t* d_nl = reinterpret_cast<int32_t*>(P + o_nl);
    float* d_nrm = reinterpret_cast<float*>(P + o_nrm);
    uint8_t* d_val = reinterpret_cast<uint8_t*>(P + o_val);
    float* d_srt = reinterpret_cast<float*>(P + o_srt);
    int32_t* d_sid = reinterpret_cast<int32_t*>(P + o_sid);
    float* d_sim = reinterpret_cast<float*>(P + o_sim);        // the table's strip image
    int32_t* d_shd = reinterpret_cast<int32_t*>(P + o_shd);
    struct { int64_t off[4]; int32_t cnt[4]; double pose[7]; } h;
    h.off[0] = 0; h.off[1] = m_last; h.off[2] = 0; h.off[3] = m_curr;
    h.cnt[0] = (int32_t)m_last; h.cnt[1] = (int32_t)m_curr; h.cnt[2] = h.cnt[3] = 0;
    for (int k = 0; k < 7; ++k) h.pose[k] = pose[k];
    SSF_TRY_HIP(c, hipMemcpyAsync(d_off, h.off, sizeof(h.off), hipMemcpyHostToDevice, s), "H2D off");
    SSF_TRY_HIP(c, hipMemcpyAsync(d_cnt, h.cnt, sizeof(h.cnt), hipMemcpyHostToDevice, s), "H2D counts");
    SSF_TRY_HIP(c, hipMemcpyAsync(d_pose, h.pose, sizeof(h.pose), hipMemcpyHostToDevice, s), "H2D pose");
    int32_t rc = ssf_plane_table_batch(c, stream, 1, d_last_xyzi, d_off, d_cnt, mx, d_nrm, d_val, d_srt, d_sid,
                                       d_sim, d_shd);
    if (rc) return rc;
    rc = ssf_register_batch(c, stream, 1, d_last_xyzi, d_off, d_cnt, d_nrm, d_val, d_srt, d_sid,
                            d_curr_xyzi, d_off + 2, d_cnt + 1, m_curr, mx, d_pose, nullptr,
                            d_log, d_nl, d_nl + 1, nullptr, d_sim, d_shd);
    if (rc) return rc;
    std::vector<double> hl((size_t)std::max(max_iter, 1) * 10);
    int32_t hn[2] = {0, 0};
    SSF_TRY_HIP(c, hipMemcpyAsync(h.pose, d_pose, sizeof(h.pose), hipMemcpyDeviceToHost, s), "D2H pose");
    SSF_TRY_HIP(c, hipMemcpyAsync(hn, d_nl, sizeof(hn), hipMemcpyDeviceToHost, s), "D2H nlog");
    if (log && log->cap > 0)
        SSF_TRY_HIP(c, hipMemcpyAsync(hl.data(), d_log, sizeof(double) * hl.size(), hipMemcpyDeviceToHost, s), "D2H log");
    SSF_TRY_HIP(c, hipStreamSynchronize(s), "sync");
    for (int k = 0; k < 4; ++k) h_q_out[k] = h.pose[k];
    for (int k = 0; k < 3; ++k) h_t_out[k] = h.pose[4 + k];
    if (log) {
        log->n_corr = hn[1];
        const int n = std::min(std::min(hn[0], max_iter), std::max(log->cap, 0));
        for (int i = 0; i < n; ++i) {
            const double* r = &hl[(size_t)i * 10];
            ssf_step& st = log->steps[i];
            for (int k = 0; k < 4; ++k) st.q[k] = r[k];
            for (int k = 0; k < 3; ++k) st.t[k] = r[4 + k];
            st.cost = r[7];
            st.status = (int32_t)r[8];
            st.pad = 0;
            st.radius = r[9];
        }
        log->n_steps = n;
    }
    return SSF_OK;
}

}  // extern "C"

template <class T>
static int32_t mask_pose_batch(ssf_ctx* c, void* stream, int32_t n_frames, const T* d_pts,
                            const T* d_flow, const int64_t* d_frame_off,
                            const int64_t* h_frame_off, int32_t mode, const uint8_t* d_mask_in,
                            const double* h_draws, int32_t reflection, uint8_t* d_bg_mask,
                            double* d_out) {
    if (!c) return SSF_E_ARG;
    if (n_frames < 0 || mode < SSF_MASK_GMM || mode > SSF_MASK_GIVEN ||
        (n_frames > 0 && (!d_pts || !d_flow || !d_frame_off || !h_frame_off || !d_out)) ||
        (mode != SSF_MASK_GMM && !d_mask_in))
        return fail(c, SSF_E_ARG, "mask_pose_batch: bad arguments");
    if (n_frames == 0) return SSF_OK;
    if (c->mask_order && c->mask_order_n != n_frames)
        return fail(c, SSF_E_ARG, "mask_pose_batch: the frame order (ssf_set_mask_schedule) has another length");
    const int64_t total = h_frame_off[n_frames];
    for (int f = 0; f < n_frames; ++f) {
        if (h_frame_off[f + 1] < h_frame_off[f]) return fail(c, SSF_E_ARG, "mask_pose_batch: offsets not monotone");
        // the streaming loops address a frame with 32-bit byte offsets (mask_pose.hip load3_off)
        if (h_frame_off[f + 1] - h_frame_off[f] > (int64_t)(0xFFFFFFFFu / (3 * sizeof(T))))
            return fail(c, SSF_E_ARG, "mask_pose_batch: a frame above 2^32 / (3 sizeof(T)) points");
    }
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    ssf_ctx::DrawSlot& ds = c->dslot[c->dnext];
    c->dnext = (c->dnext + 1) % ssf_ctx::kDrawSlots;
    const size_t need = 3 * (size_t)n_frames;
    if (!ds.copied) {
        SSF_TRY_HIP(c, hipEventCreateWithFlags(&ds.copied, hipEventDisableTiming), "draws event");
        SSF_TRY_HIP(c, hipEventCreateWithFlags(&ds.used, hipEventDisableTiming), "draws event");
    } else {
        SSF_TRY_HIP(c, hipEventSynchronize(ds.copied), "draws event");   // staging reusable
    }
    const size_t rec_need = mode == SSF_MASK_GMM ? sizeof(uint2) * (size_t)(total + 2 * (int64_t)n_frames + 2) + sizeof(uint32_t) * (size_t)(total + 64 * (int64_t)n_frames) : 0;
    // parts per frame: fixed, or automatic -- enough to fill the resident work-group slots
    if (c->mask_slots < 0) c->mask_slots = ssf::mask_pose_slots(c->device);
    int G = c->mask_split;
    // automatic: as many parts as keep the resident slots busy.  A fixed split is honoured as
    // set (frames x G may exceed the slots: work-groups then take several tickets); its exchange
    // scratch grows with it (mask_parts_bytes: frames x G x 104 KiB, see ssf_set_mask_split)
    if (G <= 0) G = c->mask_slots > 0 ? c->mask_slots / n_frames : 1;
    G = std::max(1, std::min(G, ssf::kMaskMaxSplit));
    if (mode != SSF_MASK_GMM) G = 1;
    const bool queued = G == 1 && c->mask_queue > 0 && c->mask_queue < n_frames;
    const size_t sync_need = (G > 1 || queued) ? ssf::mask_sync_bytes(n_frames) + 16 : 0;
    const size_t parts_need = G > 1 ? ssf::mask_parts_bytes(n_frames, G) : 0;
    if (ds.d.bytes < sizeof(double) * need || ds.rec.bytes < rec_need || ds.sync.bytes < sync_need ||
        ds.parts.bytes < parts_need) {                                    // growing frees the old buffer
        SSF_TRY_HIP(c, hipEventSynchronize(ds.used), "draws event");
        SSF_TRY_HIP(c, ds.d.ensure(sizeof(double) * need), "alloc draws");
        if (rec_need) SSF_TRY_HIP(c, ds.rec.ensure(rec_need), "alloc lloyd records");
        if (sync_need) SSF_TRY_HIP(c, ds.sync.ensure(sync_need), "alloc mask sync");
        if (parts_need) SSF_TRY_HIP(c, ds.parts.ensure(parts_need), "alloc mask parts");
    } else {
        SSF_TRY_HIP(c, hipStreamWaitEvent(s, ds.used, 0), "draws wait");   // device-side: no host stall
    }
    if (ds.hcap < (int64_t)need) {
        if (ds.h) SSF_TRY_HIP(c, hipHostFree(ds.h), "free pinned");
        ds.h = nullptr; ds.hcap = 0;
        SSF_TRY_HIP(c, hipHostMalloc((void**)&ds.h, sizeof(double) * need), "pinned draws");
        ds.hcap = (int64_t)need;
    }
    std::memset(ds.h, 0, sizeof(double) * need);
    if (mode == SSF_MASK_GMM) {
        for (int f = 0; f < n_frames; ++f) {
            const int64_t nf = h_frame_off[f + 1] - h_frame_off[f];
            double u0, u1, u2;
            if (h_draws) { u0 = h_draws[3 * f]; u1 = h_draws[3 * f + 1]; u2 = h_draws[3 * f + 2]; }
            else { u0 = mt_random_sample(c); u1 = mt_random_sample(c); u2 = mt_random_sample(c); }
            ds.h[3 * f] = nf > 0 ? (double)choice_uniform(c, nf, u0) : 0.0;
            ds.h[3 * f + 1] = u1;
            ds.h[3 * f + 2] = u2;
        }
    }
    SSF_TRY_HIP(c, hipMemcpyAsync(ds.d.p, ds.h, sizeof(double) * need, hipMemcpyHostToDevice, s), "H2D draws");
    SSF_TRY_HIP(c, hipEventRecord(ds.copied, s), "draws record");
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_mask_pose(s, n_frames, d_pts, d_flow, d_frame_off, mode, d_mask_in,
                                         ds.d.as<double>(), ds.rec.as<uint2>(), reflection, d_bg_mask, d_out,
                                         G, c->mask_slots, ds.sync.as<uint32_t>(), ds.parts.as<double>(),
                                         c->mask_order, queued ? c->mask_queue : 0);
    if (e == hipSuccess) e = hipEventRecord(ds.used, s);
    if (e != hipSuccess) return hip_fail(c, e, "mask_pose launch");
    return SSF_OK;
}

extern "C" {

int32_t ssf_mask_pose_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_pts,
                            const float* d_flow, const int64_t* d_frame_off,
                            const int64_t* h_frame_off, int32_t mode, const uint8_t* d_mask_in,
                            const double* h_draws, int32_t reflection, uint8_t* d_bg_mask,
                            double* d_out) {
    return mask_pose_batch(c, stream, n_frames, d_pts, d_flow, d_frame_off, h_frame_off, mode,
                           d_mask_in, h_draws, reflection, d_bg_mask, d_out);
}

int32_t ssf_mask_pose_batch_f64(ssf_ctx* c, void* stream, int32_t n_frames, const double* d_pts,
                                const double* d_flow, const int64_t* d_frame_off,
                                const int64_t* h_frame_off, int32_t mode, const uint8_t* d_mask_in,
                                const double* h_draws, int32_t reflection, uint8_t* d_bg_mask,
                                double* d_out) {
    return mask_pose_batch(c, stream, n_frames, d_pts, d_flow, d_frame_off, h_frame_off, mode,
                           d_mask_in, h_draws, reflection, d_bg_mask, d_out);
}

int32_t ssf_kabsch_f32_batch(ssf_ctx* c, void* stream, int32_t n_frames, const float* d_src,
                             const float* d_dst, const float* d_flow, const int64_t* d_frame_off,
                             const uint8_t* d_mask, int32_t reflection, int32_t after_mask,
                             double* d_out) {
    if (!c) return SSF_E_ARG;
    if (n_frames < 0 || (n_frames > 0 && (!d_dst || (!d_flow && !d_src) || !d_frame_off || !d_out)))
        return fail(c, SSF_E_ARG, "kabsch_f32_batch: bad arguments");
    if (n_frames == 0) return SSF_OK;
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_kabsch_f32(s, n_frames, d_src, d_dst, d_flow, d_frame_off, d_mask,
                                          reflection ? 1 : 0, after_mask ? 1 : 0, d_out);
    if (e != hipSuccess) return hip_fail(c, e, "kabsch_f32 launch");
    return SSF_OK;
}

int32_t ssf_accumulate_sequence(ssf_ctx* c, void* stream, int32_t n, const double* d_rel,
                                const double* h_start, double* d_abs) {
    if (!c) return SSF_E_ARG;
    if (n < 0 || (n > 0 && (!d_rel || !d_abs))) return fail(c, SSF_E_ARG, "accumulate: bad arguments");
    if (n == 0) return SSF_OK;
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    const double* d_start = nullptr;
    if (h_start) {
        SSF_TRY_HIP(c, c->start1.ensure(sizeof(double) * 8), "alloc start");
        SSF_TRY_HIP(c, hipMemcpyAsync(c->start1.p, h_start, sizeof(double) * 7, hipMemcpyHostToDevice, s), "H2D start");
        d_start = c->start1.as<double>();
    }
    ProfScope prof(c, stream);
    hipError_t e = ssf::launch_accumulate(s, n, d_rel, d_start, d_abs);
    if (e != hipSuccess) return hip_fail(c, e, "accumulate launch");
    if (h_start) SSF_TRY_HIP(c, hipStreamSynchronize(s), "sync start");
    return SSF_OK;
}

int32_t ssf_voxel_grid_batch(ssf_ctx* c, void* stream, int32_t n_clouds, const float* d_xyzi,
                             const int64_t* d_off, const int64_t* h_off, float leaf,
                             float* d_out, int32_t* d_out_count) {
    if (!c) return SSF_E_ARG;
    if (n_clouds < 0 || !(leaf > 0.0f) ||
        (n_clouds > 0 && (!d_xyzi || !d_off || !h_off || !d_out || !d_out_count)))
        return fail(c, SSF_E_ARG, "voxel_grid_batch: bad arguments");
    if (n_clouds == 0) return SSF_OK;
    int64_t max_pts = 0;
    for (int k = 0; k < n_clouds; ++k) {
        const int64_t m = h_off[k + 1] - h_off[k];
        if (m < 0) return fail(c, SSF_E_ARG, "voxel_grid_batch: offsets not monotone");
        if (m > (int64_t)INT32_MAX) return fail(c, SSF_E_ARG, "voxel_grid_batch: cloud too large");
        max_pts = std::max(max_pts, m);
    }
    if (h_off[0] != 0) return fail(c, SSF_E_ARG, "voxel_grid_batch: offsets must start at 0");
    const int64_t n = h_off[n_clouds];
    if (n > (int64_t)INT32_MAX) return fail(c, SSF_E_ARG, "voxel_grid_batch: too many points");
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->vg.ensure(ssf::vg_scratch_bytes(n_clouds, n)), "alloc voxel scratch");
    hipError_t e = ssf::launch_voxel_grid(s, n_clouds, reinterpret_cast<const float4*>(d_xyzi), d_off, n,
                                          max_pts, leaf, c->vg.p, reinterpret_cast<float4*>(d_out),
                                          d_out_count);
    if (e != hipSuccess) return hip_fail(c, e, "voxel_grid launch");
    return SSF_OK;
}

int32_t ssf_icp_params_default(ssf_icp_params* out) {
    if (!out) return SSF_E_ARG;
    out->max_iter = 100;            // mapOptmization.cpp:225-228
    out->max_corr_dist = 50.0f;
    out->trans_eps = 1e-6;
    out->fit_eps = 1e-6;
    return SSF_OK;
}

int32_t ssf_icp_batch(ssf_ctx* c, void* stream, int32_t n_prob, const float* d_src,
                      const int64_t* d_src_off, const int64_t* h_src_off, const float* d_tgt,
                      const int64_t* d_tgt_off, const int64_t* h_tgt_off,
                      const ssf_icp_params* prm, const float* h_guess, double* h_out) {
    if (!c) return SSF_E_ARG;
    if (n_prob < 0 || !prm || prm->max_iter < 0 || !(prm->max_corr_dist >= 0.0f) ||
        (n_prob > 0 && (!d_src || !d_src_off || !h_src_off || !d_tgt || !d_tgt_off || !h_tgt_off || !h_out)))
        return fail(c, SSF_E_ARG, "icp_batch: bad arguments");
    if (n_prob == 0) return SSF_OK;
    int64_t max_ns = 0, max_nt = 0;
    for (int k = 0; k < n_prob; ++k) {
        const int64_t a = h_src_off[k + 1] - h_src_off[k], b = h_tgt_off[k + 1] - h_tgt_off[k];
        if (a < 0 || b < 0) return fail(c, SSF_E_ARG, "icp_batch: offsets not monotone");
        if (b > (int64_t)INT32_MAX) return fail(c, SSF_E_ARG, "icp_batch: target too large");
        max_ns = std::max(max_ns, a); max_nt = std::max(max_nt, b);
    }
    const int64_t s0 = h_src_off[0], total_ns = h_src_off[n_prob] - s0;
    hipStream_t s = (hipStream_t)stream;
    SSF_TRY_HIP(c, hipSetDevice(c->device), "hipSetDevice");
    SSF_TRY_HIP(c, c->icp_cur.ensure(sizeof(float4) * (size_t)std::max<int64_t>(h_src_off[n_prob], 1)), "alloc icp");
    SSF_TRY_HIP(c, c->icp_key.ensure(sizeof(unsigned long long) * (size_t)std::max<int64_t>(h_src_off[n_prob], 1)), "alloc icp");
    SSF_TRY_HIP(c, c->icp_st.ensure(sizeof(ssf::IcpState) * (size_t)n_prob), "alloc icp");
    SSF_TRY_HIP(c, c->icp_guess.ensure(sizeof(float) * 16 * (size_t)n_prob), "alloc icp");
    std::vector<float> g(16 * (size_t)n_prob, 0.0f);
    for (int k = 0; k < n_prob; ++k)
        for (int i = 0; i < 16; ++i) g[16 * k + i] = h_guess ? h_guess[16 * k + i] : (i % 5 == 0 ? 1.0f : 0.0f);
    SSF_TRY_HIP(c, hipMemcpyAsync(c->icp_guess.p, g.data(), sizeof(float) * g.size(), hipMemcpyHostToDevice, s), "H2D guess");
    const float4* src = reinterpret_cast<const float4*>(d_src);
    const float4* tgt = reinterpret_cast<const float4*>(d_tgt);
    float4* cur = c->icp_cur.as<float4>();
    unsigned long long* key = c->icp_key.as<unsigned long long>();
    ssf::IcpState* st = c->icp_st.as<ssf::IcpState>();
    hipError_t e = ssf::launch_icp_init(s, n_prob, src, d_src_off, max_ns, c->icp_guess.as<float>(), cur, st, key);
    if (e != hipSuccess) return hip_fail(c, e, "icp init");
    // the iteration loop runs on device: every launch is skipped by problems already done; the
    // host polls the done flags every 8 iterations and stops once all problems have converged
    std::vector<ssf::IcpState> hs((size_t)n_prob);
    for (int it = 0; it < prm->max_iter; ++it) {
        e = ssf::launch_icp_iteration(s, n_prob, cur, d_src_off, max_ns, tgt, d_tgt_off, max_nt, *prm, st, key);
        if (e != hipSuccess) return hip_fail(c, e, "icp iteration");
        if ((it & 7) == 7 || it + 1 == prm->max_iter) {
            SSF_TRY_HIP(c, hipMemcpyAsync(hs.data(), st, sizeof(ssf::IcpState) * hs.size(), hipMemcpyDeviceToHost, s), "D2H icp state");
            SSF_TRY_HIP(c, hipStreamSynchronize(s), "icp sync");
            bool all = true;
            for (const auto& x : hs) all = all && x.done;
            if (all) break;
        }
    }
    (void)s0; (void)total_ns;
    e = ssf::launch_icp_fitness(s, n_prob, src, d_src_off, h_src_off[n_prob], max_ns, tgt, d_tgt_off, max_nt, st, key);
    if (e != hipSuccess) return hip_fail(c, e, "icp fitness");
    SSF_TRY_HIP(c, hipMemcpyAsync(hs.data(), st, sizeof(ssf::IcpState) * hs.size(), hipMemcpyDeviceToHost, s), "D2H icp state");
    SSF_TRY_HIP(c, hipStreamSynchronize(s), "icp sync");
    for (int k = 0; k < n_prob; ++k) {
        double* o = h_out + (size_t)k * SSF_ICP_OUT_STRIDE;
        for (int i = 0; i < SSF_ICP_OUT_STRIDE; ++i) o[i] = 0.0;
        for (int i = 0; i < 16; ++i) o[SSF_ICP_OUT_T + i] = hs[k].fin[i];
        o[SSF_ICP_OUT_FITNESS] = hs[k].fitness;
        o[SSF_ICP_OUT_CONVERGED] = hs[k].converged;
        o[SSF_ICP_OUT_ITERATIONS] = hs[k].it;
        o[SSF_ICP_OUT_STATE] = hs[k].state;
        o[SSF_ICP_OUT_NCORR] = hs[k].n_corr;
    }
    return SSF_OK;
}

}  // extern "C"
