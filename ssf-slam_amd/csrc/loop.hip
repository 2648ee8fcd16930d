// loop.hip -- the loop-closure registration of mapOptmization (src/mapOptmization.cpp:201-236,
// SURVEY.md §8(f) row 3) on gfx950, batched over independent clouds / problems:
//
//   voxel grid   pcl::VoxelGrid<PointXYZI> (downSizeFilterICP, leaf 0.1 m, :214-217 and
//                downSizeFilterMap 0.4 m, :406-409): per-cloud bounds (one work-group per cloud),
//                64-bit (cloud, voxel) keys, a stable hipCUB radix sort of (key, point), run
//                heads + scan, and one thread per voxel summing its run in input order (float,
//                as PCL's Eigen::VectorXf centroid) -- bit-exact with the oracle.
//   ICP          pcl::IterativeClosestPoint<PointXYZI, PointXYZI> (:224-236): per iteration
//                (a) exact 1-NN of every transformed source point against its target cloud,
//                brute force over target tiles staged in LDS, the (distance, index) pairs packed
//                into u64 keys merged with atomicMin (lexicographic = FLANN L2_Simple distance,
//                ties to the lower index); (b) one work-group per problem: correspondences
//                within the 50 m gate, double means and 3x3 cross-covariance (block sums), the
//                Umeyama rotation from a Jacobi SVD on one lane, the float incremental and final
//                transforms, PCL's DefaultConvergenceCriteria, and the in-place float transform
//                of the source.  Converged problems skip every later launch.  getFitnessScore
//                is one more 1-NN pass of the original source through the final transform.
#include "ssf_device.hpp"
#include "ssf_internal.hpp"
#include "svd3.hpp"

#include <float.h>
#include <hipcub/hipcub.hpp>

namespace ssf {

// ---------------------------------------------------------------------------------------------
// voxel grid
struct VgCloud {
    int minb[3];
    int mul[3];
    int overflow;   // PCL's "leaf size is too small": the cloud passes through unchanged
    int pad;
};

__global__ __launch_bounds__(256) void k_vg_bounds(const float4* __restrict__ pts,
                                                   const int64_t* __restrict__ off, float inv,
                                                   VgCloud* __restrict__ vc) {
    __shared__ float red[6][4];
    const int c = blockIdx.x;
    const int64_t b = off[c], e = off[c + 1];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
        const float4 p = pts[i];
        mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
        mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
    }
#pragma unroll
    for (int d = 0; d < 3; ++d)
        for (int o = 32; o > 0; o >>= 1) {
            mn[d] = fminf(mn[d], __shfl_xor(mn[d], o, 64));
            mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o, 64));
        }
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0)
        for (int d = 0; d < 3; ++d) { red[d][w] = mn[d]; red[3 + d][w] = mx[d]; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k)
            for (int d = 0; d < 3; ++d) { mn[d] = fminf(mn[d], red[d][k]); mx[d] = fmaxf(mx[d], red[3 + d][k]); }
        for (int d = 0; d < 3; ++d) { mn[d] = fminf(mn[d], red[d][0]); mx[d] = fmaxf(mx[d], red[3 + d][0]); }
        VgCloud v;
        const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
        const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
        const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
        v.overflow = (e <= b) || (dx * dy * dz > (int64_t)INT32_MAX);
        int divb[3];
        for (int d = 0; d < 3; ++d) {
            v.minb[d] = (int)floorf(mn[d] * inv);
            divb[d] = (int)floorf(mx[d] * inv) - v.minb[d] + 1;
        }
        v.mul[0] = 1; v.mul[1] = divb[0]; v.mul[2] = v.overflow ? 0 : divb[0] * divb[1];
        v.pad = 0;
        vc[c] = v;
    }
}

// key = cloud << 32 | voxel index (< 2^31); an overflowing cloud keys every point on its own
__global__ __launch_bounds__(256) void k_vg_keys(const float4* __restrict__ pts,
                                                 const int64_t* __restrict__ off, int n_clouds,
                                                 float inv, const VgCloud* __restrict__ vc,
                                                 uint64_t* __restrict__ key, int32_t* __restrict__ val) {
    const int c = blockIdx.y;
    const int64_t b = off[c], e = off[c + 1];
    const int64_t i = b + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e) return;
    const VgCloud v = vc[c];
    const float4 p = pts[i];
    int64_t idx;
    if (v.overflow) {
        idx = i - b;
    } else {
        idx = (int64_t)((int)floorf(p.x * inv) - v.minb[0]) * v.mul[0] +
              (int64_t)((int)floorf(p.y * inv) - v.minb[1]) * v.mul[1] +
              (int64_t)((int)floorf(p.z * inv) - v.minb[2]) * v.mul[2];
    }
    key[i] = ((uint64_t)c << 32) | (uint64_t)idx;
    val[i] = (int32_t)(i - b);
}

__global__ __launch_bounds__(256) void k_vg_heads(const uint64_t* __restrict__ key, int64_t n,
                                                  int32_t* __restrict__ head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

// one thread per voxel (its run head): the centroid summed in input order, PCL's float
// ((0 + p0) + p1) + ... / count.  vid = exclusive scan of the heads; cloud c's sorted elements
// start at off[c], so its first voxel id is vid[off[c]].
__global__ __launch_bounds__(256) void k_vg_reduce(const float4* __restrict__ pts,
                                                   const int64_t* __restrict__ off, int n_clouds,
                                                   const uint64_t* __restrict__ key,
                                                   const int32_t* __restrict__ val,
                                                   const int32_t* __restrict__ head,
                                                   const int32_t* __restrict__ vid, int64_t n,
                                                   float4* __restrict__ out,
                                                   int32_t* __restrict__ out_count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = (int)(key[i] >> 32);
    const int64_t b = off[c];
    const int first = vid[b];
    if (i == off[c + 1] - 1) out_count[c] = vid[i] + head[i] - first;   // the cloud's last element
    if (!head[i]) return;
    int64_t j = i;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    do {
        const float4 p = pts[b + val[j]];
        s0 = s0 + p.x; s1 = s1 + p.y; s2 = s2 + p.z; s3 = s3 + p.w;
        ++j;
    } while (j < n && !head[j]);
    const float cnt = (float)(j - i);
    out[b + (vid[i] - first)] = make_float4(s0 / cnt, s1 / cnt, s2 / cnt, s3 / cnt);
}

size_t vg_temp_bytes(int64_t n) {
    size_t sort_b = 0, scan_b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    return sort_b > scan_b ? sort_b : scan_b;
}

// scratch layout (bytes, 256-aligned pieces): VgCloud[n_clouds], key[2n] u64, val[2n] i32,
// head[n] i32, vid[n] i32, cub temp
size_t vg_scratch_bytes(int n_clouds, int64_t n) {
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    return al(sizeof(VgCloud) * (size_t)n_clouds) + 2 * al(sizeof(uint64_t) * (size_t)n) +
           2 * al(sizeof(int32_t) * (size_t)n) + 2 * al(sizeof(int32_t) * (size_t)n) + al(vg_temp_bytes(n));
}

hipError_t launch_voxel_grid(hipStream_t s, int n_clouds, const float4* pts, const int64_t* off,
                             int64_t n, int64_t max_pts, float leaf, void* scratch,
                             float4* out, int32_t* out_count) {
    if (n_clouds <= 0) return hipSuccess;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    char* p = static_cast<char*>(scratch);
    VgCloud* vc = reinterpret_cast<VgCloud*>(p); p += al(sizeof(VgCloud) * (size_t)n_clouds);
    uint64_t* k0 = reinterpret_cast<uint64_t*>(p); p += al(sizeof(uint64_t) * (size_t)n);
    uint64_t* k1 = reinterpret_cast<uint64_t*>(p); p += al(sizeof(uint64_t) * (size_t)n);
    int32_t* v0 = reinterpret_cast<int32_t*>(p); p += al(sizeof(int32_t) * (size_t)n);
    int32_t* v1 = reinterpret_cast<int32_t*>(p); p += al(sizeof(int32_t) * (size_t)n);
    int32_t* head = reinterpret_cast<int32_t*>(p); p += al(sizeof(int32_t) * (size_t)n);
    int32_t* vid = reinterpret_cast<int32_t*>(p); p += al(sizeof(int32_t) * (size_t)n);
    void* tmp = p;
    size_t tmp_b = vg_temp_bytes(n);
    const float inv = 1.0f / leaf;                       // inverse_leaf_size_ (Array4f)
    hipLaunchKernelGGL(k_vg_bounds, dim3(n_clouds), dim3(256), 0, s, pts, off, inv, vc);
    hipError_t e = hipMemsetAsync(out_count, 0, sizeof(int32_t) * (size_t)n_clouds, s);
    if (e != hipSuccess) return e;
    if (n <= 0) return hipGetLastError();
    const int gx = (int)((max_pts + 255) / 256);
    if (gx > 0)
        hipLaunchKernelGGL(k_vg_keys, dim3(gx, n_clouds), dim3(256), 0, s, pts, off, n_clouds, inv, vc, k0, v0);
    int end_bit = 32;
    while ((1ll << (end_bit - 32)) < (long long)n_clouds) ++end_bit;
    e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_b, k0, k1, v0, v1, (int)n, 0, end_bit, s);
    if (e != hipSuccess) return e;
    const int g = (int)((n + 255) / 256);
    hipLaunchKernelGGL(k_vg_heads, dim3(g), dim3(256), 0, s, k1, n, head);
    tmp_b = vg_temp_bytes(n);
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, head, vid, (int)n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_vg_reduce, dim3(g), dim3(256), 0, s, pts, off, n_clouds, k1, v1, head, vid, n,
                       out, out_count);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ICP
constexpr int kIcpNnThreads = 256;
constexpr int kIcpTgtTile = 2048;        // target points per 1-NN work-group (32 KiB of LDS)
constexpr int kIcpStepThreads = 1024;

SSF_DEV uint64_t nn_key(float d2, int j) { return ((uint64_t)__float_as_uint(d2) << 32) | (uint32_t)j; }

// (a) 1-NN: grid (source tiles, target tiles, problems); each work-group stages one target tile
// and merges its per-source best into key[i] with a u64 atomicMin.  from_original: the
// original source through the final transform (getFitnessScore) instead of the current cloud.
__global__ __launch_bounds__(kIcpNnThreads) void k_icp_nn(const float4* __restrict__ cur,
                                                          const float4* __restrict__ src,
                                                          const int64_t* __restrict__ soff,
                                                          const float4* __restrict__ tgt,
                                                          const int64_t* __restrict__ toff,
                                                          const IcpState* __restrict__ st,
                                                          int from_original,
                                                          unsigned long long* __restrict__ key) {
    __shared__ float4 tile[kIcpTgtTile];
    const int p = blockIdx.z;
    if (!from_original && st[p].done) return;                       // uniform
    const int64_t sb = soff[p], ns = soff[p + 1] - sb;
    const int64_t tb = toff[p], nt = toff[p + 1] - tb;
    const int64_t t0 = (int64_t)blockIdx.y * kIcpTgtTile;
    if (t0 >= nt) return;
    const int tn = (int)min((int64_t)kIcpTgtTile, nt - t0);
    for (int k = threadIdx.x; k < tn; k += blockDim.x) tile[k] = tgt[tb + t0 + k];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    float q[3];
    if (from_original) {
        const float4 a = src[sb + i];
        const float* T = st[p].fin;
        for (int r = 0; r < 3; ++r) q[r] = ((T[4 * r] * a.x + T[4 * r + 1] * a.y) + T[4 * r + 2] * a.z) + T[4 * r + 3];
    } else {
        const float4 a = cur[sb + i];
        q[0] = a.x; q[1] = a.y; q[2] = a.z;
    }
    float bd = __builtin_inff();
    int bj = 0x7fffffff;
    for (int k = 0; k < tn; ++k) {
        const float4 t = tile[k];
        const float dx = q[0] - t.x, dy = q[1] - t.y, dz = q[2] - t.z;
        float d = dx * dx + dy * dy;
        d = d + dz * dz;
        if (d < bd) { bd = d; bj = (int)t0 + k; }                 // ties: the lower index first
    }
    if (bj != 0x7fffffff) atomicMin(&key[sb + i], (unsigned long long)nn_key(bd, bj));
}

// x' = ((r00 x + r01 y) + r02 z) + t0 (Eigen Matrix4f * Vector4f, pcl::transformPointCloud)
SSF_DEV float4 tf4(const float* T, const float4& a) {
    float4 o = a;
    o.x = ((T[0] * a.x + T[1] * a.y) + T[2] * a.z) + T[3];
    o.y = ((T[4] * a.x + T[5] * a.y) + T[6] * a.z) + T[7];
    o.z = ((T[8] * a.x + T[9] * a.y) + T[10] * a.z) + T[11];
    return o;
}

// (b) one work-group per problem: correspondences, Umeyama, transforms, convergence, and the
// source moved by the increment; the keys are reset for the next iteration.
__global__ __launch_bounds__(kIcpStepThreads) void k_icp_step(float4* __restrict__ cur,
                                                              const int64_t* __restrict__ soff,
                                                              const float4* __restrict__ tgt,
                                                              const int64_t* __restrict__ toff,
                                                              IcpParams prm,
                                                              IcpState* __restrict__ st,
                                                              unsigned long long* __restrict__ key) {
    __shared__ double red[(kIcpStepThreads / 64) * 16];
    __shared__ float inc_s[16];
    __shared__ int done_s;
    const int p = blockIdx.x;
    if (st[p].done) return;
    const int64_t sb = soff[p], ns = soff[p + 1] - sb, tb = toff[p];
    const double max_d2 = (double)prm.max_corr_dist * (double)prm.max_corr_dist;
    // pass 1: count, sum d2, sums of source and target points over the correspondences
    double a[8];
    for (int k = 0; k < 8; ++k) a[k] = 0.0;
    for (int64_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const unsigned long long kk = key[sb + i];
        const float d2 = __uint_as_float((uint32_t)(kk >> 32));
        if (kk == ~0ull || (double)d2 > max_d2) continue;
        const float4 s = cur[sb + i], t = tgt[tb + (int64_t)(uint32_t)(kk & 0xffffffffu)];
        a[0] += 1.0; a[1] += (double)d2;
        a[2] += s.x; a[3] += s.y; a[4] += s.z; a[5] += t.x; a[6] += t.y; a[7] += t.z;
    }
    block_sum<8>(a, red);
    const double c = a[0];
    if (c < 3.0) {                                                  // NO_CORRESPONDENCES
        if (threadIdx.x == 0) { st[p].done = 1; st[p].converged = 0; st[p].state = 5; st[p].n_corr = (int)c; }
        return;
    }
    const double sm[3] = {a[2] / c, a[3] / c, a[4] / c}, dm[3] = {a[5] / c, a[6] / c, a[7] / c};
    // pass 2: sigma = sum (t - dm)(s - sm)^T
    double h[9];
    for (int k = 0; k < 9; ++k) h[k] = 0.0;
    for (int64_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const unsigned long long kk = key[sb + i];
        const float d2 = __uint_as_float((uint32_t)(kk >> 32));
        if (kk == ~0ull || (double)d2 > max_d2) continue;
        const float4 s = cur[sb + i], t = tgt[tb + (int64_t)(uint32_t)(kk & 0xffffffffu)];
        const double sv[3] = {s.x - sm[0], s.y - sm[1], s.z - sm[2]};
        const double tv[3] = {t.x - dm[0], t.y - dm[1], t.z - dm[2]};
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) h[3 * r + q] += tv[r] * sv[q];
    }
    block_sum<9>(h, red);
    if (threadIdx.x == 0) {
        IcpState& S = st[p];
        double H[9], U[9], Sv[3], Vt[9];
        for (int k = 0; k < 9; ++k) H[k] = h[k] / c;
        svd3(H, U, Sv, Vt);
        const double du = U[0] * (U[4] * U[8] - U[5] * U[7]) - U[1] * (U[3] * U[8] - U[5] * U[6]) + U[2] * (U[3] * U[7] - U[4] * U[6]);
        const double dv = Vt[0] * (Vt[4] * Vt[8] - Vt[5] * Vt[7]) - Vt[1] * (Vt[3] * Vt[8] - Vt[5] * Vt[6]) + Vt[2] * (Vt[3] * Vt[7] - Vt[4] * Vt[6]);
        const double s3 = du * dv < 0 ? -1.0 : 1.0;
        double R[9];
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q)
                R[3 * r + q] = U[3 * r] * Vt[q] + U[3 * r + 1] * Vt[3 + q] + s3 * U[3 * r + 2] * Vt[6 + q];
        float inc[16];
        for (int k = 0; k < 16; ++k) inc[k] = 0.f;
        for (int r = 0; r < 3; ++r) {
            for (int q = 0; q < 3; ++q) inc[4 * r + q] = (float)R[3 * r + q];
            inc[4 * r + 3] = (float)(dm[r] - (R[3 * r] * sm[0] + R[3 * r + 1] * sm[1] + R[3 * r + 2] * sm[2]));
        }
        inc[15] = 1.f;
        float fin[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                fin[4 * i + j] = ((inc[4 * i] * S.fin[j] + inc[4 * i + 1] * S.fin[4 + j]) + inc[4 * i + 2] * S.fin[8 + j]) +
                                 inc[4 * i + 3] * S.fin[12 + j];
        for (int k = 0; k < 16; ++k) { S.fin[k] = fin[k]; inc_s[k] = inc[k]; }
        S.it += 1;
        S.n_corr = (int)c;
        // DefaultConvergenceCriteria::hasConverged (PCL 1.10, max_iterations_similar_transforms 0)
        int dn = 0, state = 0;
        if (S.it >= prm.max_iter) { dn = 1; state = 1; }
        else {
            const double cos_a = 0.5 * ((double)inc[0] + (double)inc[5] + (double)inc[10] - 1.0);
            const double tr2 = (double)inc[3] * inc[3] + (double)inc[7] * inc[7] + (double)inc[11] * inc[11];
            const double mse = a[1] / c;
            if (cos_a >= 1.0 - prm.trans_eps && tr2 <= prm.trans_eps) { dn = 1; state = 2; }
            else if (fabs(mse - S.prev_mse) < 1e-12) { dn = 1; state = 3; }
            else if (fabs(mse - S.prev_mse) / S.prev_mse < prm.fit_eps) { dn = 1; state = 4; }
            S.prev_mse = mse;
        }
        S.state = state;
        S.converged = dn;
        done_s = dn;
    }
    __syncthreads();
    const float* inc = inc_s;
    for (int64_t i = threadIdx.x; i < ns; i += blockDim.x) {
        cur[sb + i] = tf4(inc, cur[sb + i]);
        key[sb + i] = ~0ull;
    }
    if (threadIdx.x == 0 && done_s) st[p].done = 1;
}

// prepare: the guess into the final transform, the source through the guess, keys reset
__global__ __launch_bounds__(256) void k_icp_init(const float4* __restrict__ src,
                                                  const int64_t* __restrict__ soff,
                                                  const float* __restrict__ guess,
                                                  float4* __restrict__ cur, IcpState* __restrict__ st,
                                                  unsigned long long* __restrict__ key) {
    const int p = blockIdx.y;
    const int64_t sb = soff[p], ns = soff[p + 1] - sb;
    const float* G = guess + 16 * p;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        IcpState& S = st[p];
        for (int k = 0; k < 16; ++k) S.fin[k] = G[k];
        S.prev_mse = DBL_MAX;
        S.it = 0; S.done = 0; S.state = 0; S.converged = 0; S.n_corr = 0;
        S.fitness = DBL_MAX;
    }
    bool ident = true;
    for (int k = 0; k < 16; ++k) ident = ident && (G[k] == ((k % 5 == 0) ? 1.f : 0.f));
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns) return;
    cur[sb + i] = ident ? src[sb + i] : tf4(G, src[sb + i]);     // computeTransformation: guess
    key[sb + i] = ~0ull;
}

// getFitnessScore(): mean of the 1-NN squared distances (all within DBL_MAX)
__global__ __launch_bounds__(kIcpStepThreads) void k_icp_fitness(const int64_t* __restrict__ soff,
                                                                 IcpState* __restrict__ st,
                                                                 const unsigned long long* __restrict__ key) {
    __shared__ double red[(kIcpStepThreads / 64) * 2];
    const int p = blockIdx.x;
    const int64_t sb = soff[p], ns = soff[p + 1] - sb;
    double a[2] = {0.0, 0.0};
    for (int64_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const unsigned long long kk = key[sb + i];
        if (kk == ~0ull) continue;
        a[0] += 1.0; a[1] += (double)__uint_as_float((uint32_t)(kk >> 32));
    }
    block_sum<2>(a, red);
    if (threadIdx.x == 0) st[p].fitness = a[0] > 0 ? a[1] / a[0] : DBL_MAX;
}

__global__ __launch_bounds__(256) void k_icp_reset_keys(const int64_t* __restrict__ soff, int64_t n,
                                                        unsigned long long* __restrict__ key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[soff[0] + i] = ~0ull;
}

hipError_t launch_icp_init(hipStream_t s, int n_prob, const float4* src, const int64_t* soff,
                           int64_t max_ns, const float* guess, float4* cur, IcpState* st,
                           unsigned long long* key) {
    const int gx = (int)((max_ns + 255) / 256);
    hipLaunchKernelGGL(k_icp_init, dim3(gx > 0 ? gx : 1, n_prob), dim3(256), 0, s, src, soff, guess, cur, st, key);
    return hipGetLastError();
}

hipError_t launch_icp_iteration(hipStream_t s, int n_prob, float4* cur, const int64_t* soff,
                                int64_t max_ns, const float4* tgt, const int64_t* toff,
                                int64_t max_nt, const IcpParams& prm, IcpState* st,
                                unsigned long long* key) {
    const int gx = (int)((max_ns + kIcpNnThreads - 1) / kIcpNnThreads);
    const int gy = (int)((max_nt + kIcpTgtTile - 1) / kIcpTgtTile);
    if (gx > 0 && gy > 0)
        hipLaunchKernelGGL(k_icp_nn, dim3(gx, gy, n_prob), dim3(kIcpNnThreads), 0, s, cur, nullptr, soff, tgt,
                           toff, st, 0, key);
    hipLaunchKernelGGL(k_icp_step, dim3(n_prob), dim3(kIcpStepThreads), 0, s, cur, soff, tgt, toff, prm, st, key);
    return hipGetLastError();
}

hipError_t launch_icp_fitness(hipStream_t s, int n_prob, const float4* src, const int64_t* soff,
                              int64_t total_ns, int64_t max_ns, const float4* tgt,
                              const int64_t* toff, int64_t max_nt, IcpState* st,
                              unsigned long long* key) {
    if (total_ns > 0)
        hipLaunchKernelGGL(k_icp_reset_keys, dim3((int)((total_ns + 255) / 256)), dim3(256), 0, s, soff, total_ns, key);
    const int gx = (int)((max_ns + kIcpNnThreads - 1) / kIcpNnThreads);
    const int gy = (int)((max_nt + kIcpTgtTile - 1) / kIcpTgtTile);
    if (gx > 0 && gy > 0)
        hipLaunchKernelGGL(k_icp_nn, dim3(gx, gy, n_prob), dim3(kIcpNnThreads), 0, s, nullptr, src, soff, tgt,
                           toff, st, 1, key);
    hipLaunchKernelGGL(k_icp_fitness, dim3(n_prob), dim3(kIcpStepThreads), 0, s, soff, st, key);
    return hipGetLastError();
}

}  // namespace ssf
