// Probe: re-read bandwidth of a working set that does / does not fit the 256 MiB Infinity
// Cache.  256 work-groups (one per CU), each streams its contiguous slice of an S-byte buffer R
// times with 16-B loads (the mask kernel's pass pattern: every pass re-reads the frame).
// Prints S, R and GB/s (S * R / kernel time).  Decides whether splitting frames so that the
// frames in flight fit the L3 pays.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(768) void stream(const float4* __restrict__ buf, size_t n4, int reps,
                                              float* __restrict__ sink) {
    const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const size_t b = blockIdx.x * per, e = b + per < n4 ? b + per : n4;
    float acc = 0.f;
    for (int r = 0; r < reps; ++r) {
        for (size_t i = b + threadIdx.x; i < e; i += 4 * blockDim.x) {
            float4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = buf[i + k * blockDim.x < e ? i + k * blockDim.x : i];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        __syncthreads();
    }
    if (acc == 12345.f) sink[blockIdx.x] = acc;
}

int main() {
    const size_t MB = 1 << 20;
    std::vector<size_t> sizes = {64 * MB, 128 * MB, 184 * MB, 224 * MB, 320 * MB, 737 * MB, 2048 * MB};
    float4* d = nullptr;
    float* sink = nullptr;
    hipMalloc(&d, sizes.back());
    hipMalloc(&sink, 4096);
    hipMemset(d, 0, sizes.back());
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int grid : {256, 1024}) {
        for (size_t S : sizes) {
            const int reps = 8;
            const size_t n4 = S / 16;
            hipLaunchKernelGGL(stream, dim3(grid), dim3(768), 0, 0, d, n4, 1, sink);   // warm
            hipEventRecord(a);
            hipLaunchKernelGGL(stream, dim3(grid), dim3(768), 0, 0, d, n4, reps, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0.f;
            hipEventElapsedTime(&ms, a, b);
            printf("{\"grid\": %d, \"mib\": %zu, \"reps\": %d, \"ms\": %.3f, \"gbs\": %.1f}\n", grid, S / MB,
                   reps, ms, (double)S * reps / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
