// synth.hip -- batched ray-cast of the synthetic 64/16-beam scans of ssf/synth.py on the GPU.
//
// Bench / test DATA generator, not part of the front-end (libssf_synth.so, its own library):
// bench.py needs 256 sequences x (warmup + steps + 1) frames resident in HBM, and the torch
// eager form of synth.scan costs ~8 ms per frame (its slab tests materialise [rays, boxes, 3]
// f64 tensors, and its per-scan noise comes from a CPU generator).  Here one thread casts one
// ray against the sequence's whole scene held in LDS, with the formulas of synth.scan in the same
// f64 order; the range noise and the jitter come from a counter-based hash of (seed, ray) instead
// of torch's CPU generator, so the scans are the same scenes and sensor, with other noise draws.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

// per-sequence parameter record, doubles (layout shared with ssf/synth.py scan_batch):
//   [0, 9) R, [9, 12) p (sensor pose of the frame), [12, 21) R2, [21, 24) p2 (frame + 1),
//   [24] az0, then boxes (6 each), poles (4 each), cars (6 each: AABB at this frame),
//   car velocities (3 each)
constexpr int kHdr = 25;
constexpr int kMaxObj = 1024;   // doubles of scene objects staged in LDS

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// uniform in (0, 1): 53 random bits, never 0
__device__ __forceinline__ double u01(uint64_t key) {
    return ((double)(mix64(key) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

__global__ __launch_bounds__(256) void k_synth_scan(int n_rows, int n_az, const double* __restrict__ elev,
                                                    const double* __restrict__ prm, int rec,
                                                    int n_box, int n_pole, int n_car,
                                                    const uint64_t* __restrict__ seeds, int layout,
                                                    float* __restrict__ pos, float* __restrict__ flow,
                                                    double* __restrict__ key) {
    __shared__ double P[kHdr + kMaxObj];
    const int s = blockIdx.y;
    const double* src = prm + (size_t)s * rec;
    for (int k = threadIdx.x; k < rec; k += blockDim.x) P[k] = src[k];
    __syncthreads();
    const int64_t n = (int64_t)n_rows * n_az;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // layout 0: azimuth-major (index a * n_rows + r, a spinning sensor's firing order);
    // layout 1: channel-major (index r * n_az + a, as CARLA's ray-cast LiDAR stores a sweep)
    const int a = layout ? (int)(i % n_az) : (int)(i / n_rows);
    const int r = layout ? (int)(i / n_az) : (int)(i - (int64_t)a * n_rows);
    const double* R = P;
    const double* p = P + 9;
    const double* R2 = P + 12;
    const double* p2 = P + 21;
    const double az = P[24] + 2.0 * 3.14159265358979323846 * (double)a / (double)n_az;
    const double el = elev[r];
    const double ce = cos(el), se = sin(el);
    const double ds[3] = {ce * cos(az), ce * sin(az), se};
    double dw[3];
    for (int j = 0; j < 3; ++j) dw[j] = (R[3 * j] * ds[0] + R[3 * j + 1] * ds[1]) + R[3 * j + 2] * ds[2];
    double t = 100.0;
    if (dw[2] < -1e-9) t = fmin(t, (-2.5 - p[2]) / dw[2]);
    double inv[3];
    for (int k = 0; k < 3; ++k) inv[k] = 1.0 / (fabs(dw[k]) < 1e-12 ? 1e-12 : dw[k]);
    auto slab = [&](const double* b) {
        double tmin = -INFINITY, tmax = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const double lo = (b[k] - p[k]) * inv[k], hi = (b[3 + k] - p[k]) * inv[k];
            tmin = fmax(tmin, fmin(lo, hi));
            tmax = fmin(tmax, fmax(lo, hi));
        }
        const bool hit = tmax >= tmin && tmax > 0.5;
        return hit ? (tmin > 0.5 ? tmin : tmax) : INFINITY;
    };
    const double* box = P + kHdr;
    const double* pole = box + 6 * n_box;
    const double* car = pole + 4 * n_pole;
    const double* carv = car + 6 * n_car;
    double tb = INFINITY;
    for (int b = 0; b < n_box; ++b) tb = fmin(tb, slab(box + 6 * b));
    double tp = INFINITY;
    for (int q = 0; q < n_pole; ++q) {
        const double* c = pole + 4 * q;
        const double ox = p[0] - c[0], oy = p[1] - c[1];
        const double A = dw[0] * dw[0] + dw[1] * dw[1];
        const double B = 2.0 * (ox * dw[0] + oy * dw[1]);
        const double C = ox * ox + oy * oy - c[2] * c[2];
        const double disc = B * B - 4.0 * A * C;
        const double tt = (-B - sqrt(fmax(disc, 0.0))) / (2.0 * A);
        const double z = p[2] + tt * dw[2];
        if (disc > 0.0 && tt > 0.5 && z > -2.5 && z < -2.5 + c[3]) tp = fmin(tp, tt);
    }
    double tc = INFINITY;
    int ic = -1;
    for (int c = 0; c < n_car; ++c) {
        const double tt = slab(car + 6 * c);
        if (tt < tc) { tc = tt; ic = c; }      // first minimum, as torch's min
    }
    const double ts = fmin(t, fmin(tb, tp));
    const bool car_hit = tc < ts;
    // the ray's return: an object (box, pole, car), the ground plane (the road, z = -2.5), or
    // none within the 100 m range (the dome)
    const bool object_hit = car_hit || fmin(tb, tp) < t;
    // a ground return on the road (the street between the sidewalks, |y| < kRoadHalf in the world)
    // is removed (rm_road); sidewalks and the ground between and behind the buildings stay
    const bool ground_hit = !object_hit && t < 100.0;
    const bool road_hit = ground_hit && fabs(p[1] + t * dw[1]) < 6.0;
    t = car_hit ? tc : ts;
    const int mover = car_hit ? ic : -1;
    const uint64_t hk = seeds[s] ^ ((uint64_t)i << 2);
    // CARLA-like frames (ssf/synth.py layout "carla"): no point for a ray without a return and
    // for road points (rm_road); the survivors get a uniform selection key (random drop-off)
    if (key) key[(size_t)s * n + i] = (object_hit || (ground_hit && !road_hit)) ? u01(hk ^ 0x5bd1e995ull) : 2.0;
    const uint64_t key_ = hk;
    const double u1 = u01(key_), u2 = u01(key_ + 1);
    const double noise = 0.01 * (sqrt(-2.0 * log(u1)) * cos(2.0 * 3.14159265358979323846 * u2));
    t = fmin(t, 100.0) + noise;
    double p1[3];
    for (int k = 0; k < 3; ++k) p1[k] = ds[k] * t + 1e-4 * (u01(key_ + 2 + (uint64_t)k * 0x10000000000ull) - 0.5);
    double W[3];
    for (int j = 0; j < 3; ++j) W[j] = ((R[3 * j] * p1[0] + R[3 * j + 1] * p1[1]) + R[3 * j + 2] * p1[2]) + p[j];
    if (mover >= 0)
        for (int k = 0; k < 3; ++k) W[k] += carv[3 * mover + k];
    float pf[3];
    for (int k = 0; k < 3; ++k) pf[k] = (float)p1[k];
    float* po = pos + ((size_t)s * n + i) * 3;
    float* fo = flow + ((size_t)s * n + i) * 3;
    for (int k = 0; k < 3; ++k) {
        // pos2 = (W - p2) @ R2, i.e. R2^T (W - p2)
        const double d0 = W[0] - p2[0], d1 = W[1] - p2[1], d2 = W[2] - p2[2];
        const double q = (d0 * R2[k] + d1 * R2[3 + k]) + d2 * R2[6 + k];
        po[k] = pf[k];
        fo[k] = (float)(q - (double)pf[k]);
    }
}

}  // namespace

extern "C" {

// One frame for each of S sequences: rays n_rows x n_az,
// parameter records prm[S][rec] on the device (layout above), seeds[S] (device), outputs
// pos / flow [S * n_rows * n_az][3] f32 on the device.  Returns a hipError_t.
// layout 0 / 1: azimuth- / channel-major rays; d_key (nullable) [S * n_rows * n_az] f64: per ray a
// uniform key in (0, 1) when it returns from an object or off-road ground (not the road |y| < 6 m,
// not the 100 m dome), else 2.
int ssf_synth_scan_batch(void* stream, int32_t n_seq, int32_t n_rows, int32_t n_az, const double* d_elev,
                         const double* d_prm, int32_t rec, int32_t n_box, int32_t n_pole, int32_t n_car,
                         const uint64_t* d_seeds, int32_t layout, float* d_pos, float* d_flow,
                         double* d_key) {
    if (n_seq <= 0) return 0;
    if (rec - kHdr > kMaxObj || rec < kHdr + 6 * n_box + 4 * n_pole + 9 * n_car) return (int)hipErrorInvalidValue;
    const int64_t n = (int64_t)n_rows * n_az;
    dim3 grid((unsigned)((n + 255) / 256), (unsigned)n_seq);
    hipLaunchKernelGGL(k_synth_scan, grid, dim3(256), 0, (hipStream_t)stream, n_rows, n_az, d_elev, d_prm,
                       rec, n_box, n_pole, n_car, d_seeds, layout, d_pos, d_flow, d_key);
    return (int)hipGetLastError();
}

}  // extern "C"
