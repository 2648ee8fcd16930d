// frame_registration.cpp -- the INTEGRATION.md bindings as a compiled host program: the body of
// frameFeature's cloudHandler() (src/frameFeature.cpp:35-139) and lidarOdometry_onlyPC's
// frameRegistration() (src/lidarOdometry_onlyPC.cpp:147-252) on the C ABI, without ROS.
//
//   frame_registration LAST.bin CURR.bin [gn]
//
// Each .bin is a raw float32 x,y,z cloud (the PointCloud2 point_step-12 payload published by
// PointCloudOdometry*.py:84-92).  Prints one JSON line: plane counts, the solved q (x,y,z,w) /
// t from an identity warm start, and the per-iteration step log.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ssf_frontend.h"

static std::vector<float> read_cloud(const char* path) {
    std::vector<float> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    std::fseek(f, 0, SEEK_END);
    const long bytes = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize((size_t)bytes / sizeof(float));
    if (std::fread(v.data(), sizeof(float), v.size(), f) != v.size()) v.clear();
    std::fclose(f);
    return v;
}

#define CHECK(call)                                                                    \
    do {                                                                               \
        const int32_t rc_ = (call);                                                    \
        if (rc_ != SSF_OK) {                                                           \
            std::fprintf(stderr, "%s -> %d: %s\n", #call, rc_, ssf_last_error(ctx));   \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s LAST.bin CURR.bin [gn]\n", argv[0]);
        return 2;
    }
    ssf_config cfg;
    ssf_config_default(64, &cfg);                     // N_SCAN_ROW 64 parameter blocks
    if (argc > 3 && std::strcmp(argv[3], "gn") == 0) { cfg.solver = SSF_SOLVER_GN; cfg.max_iter = 10; }
    ssf_ctx* ctx = nullptr;
    if (ssf_create(0, &cfg, &ctx) != SSF_OK) {
        std::fprintf(stderr, "ssf_create failed (no gfx950 device?)\n");
        return 1;
    }
    float* d_plane[2] = {nullptr, nullptr};
    int64_t m[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {                     // cloudHandler(): one call per message
        const std::vector<float> h = read_cloud(argv[1 + k]);
        const int64_t n = (int64_t)(h.size() / 3);
        if (n == 0) { std::fprintf(stderr, "empty cloud %s\n", argv[1 + k]); return 1; }
        float* d_pts = nullptr;
        if (hipMalloc((void**)&d_pts, h.size() * sizeof(float)) != hipSuccess ||
            hipMalloc((void**)&d_plane[k], (size_t)n * 4 * sizeof(float)) != hipSuccess) return 1;
        if (hipMemcpy(d_pts, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 1;
        CHECK(ssf_extract_planes(ctx, nullptr, d_pts, n, 12, 0, d_plane[k], &m[k], n));
        (void)hipFree(d_pts);
    }
    // frameRegistration(): warm start para_q / para_t (identity for the first pair)
    double q_init[4] = {0, 0, 0, 1}, t_init[3] = {0, 0, 0}, q[4], t[3];
    std::vector<ssf_step> steps(cfg.max_iter);
    ssf_step_log log;
    log.cap = cfg.max_iter;
    log.steps = steps.data();
    CHECK(ssf_register_pair(ctx, nullptr, d_plane[0], m[0], d_plane[1], m[1], q_init, t_init, q, t, &log));
    std::printf("{\"m_last\": %lld, \"m_curr\": %lld, \"n_corr\": %d, \"q\": [%.17g, %.17g, %.17g, %.17g], "
                "\"t\": [%.17g, %.17g, %.17g], \"steps\": [",
                (long long)m[0], (long long)m[1], log.n_corr, q[0], q[1], q[2], q[3], t[0], t[1], t[2]);
    for (int i = 0; i < log.n_steps; ++i)
        std::printf("%s{\"status\": %d, \"cost\": %.17g}", i ? ", " : "", steps[i].status, steps[i].cost);
    std::printf("]}\n");
    (void)hipFree(d_plane[0]);
    (void)hipFree(d_plane[1]);
    ssf_destroy(ctx);
    return 0;
}
