// Probe: LDS layout written by one global_load_lds_dwordx3 wave-instruction on gfx950
// (lane stride 12 or 16 bytes?).  Source floats are 0,1,2,...; the LDS image (2 KiB, pre-filled
// with -1) is dumped to global memory.  Used once to pick the streaming layout in mask_pose.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(const float* __restrict__ src, float* __restrict__ dump) {
    __shared__ __attribute__((aligned(16))) float buf[512];
    for (int i = threadIdx.x; i < 512; i += 64) buf[i] = -1.0f;
    __syncthreads();
    const float* g = src + 3 * threadIdx.x;
    const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&buf[0]);
    unsigned keep;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx3 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) dump[i] = buf[i];
}

int main() {
    float h[256], out[512];
    for (int i = 0; i < 256; ++i) h[i] = (float)i;
    float *ds, *dd;
    hipMalloc(&ds, sizeof(h)); hipMalloc(&dd, sizeof(out));
    hipMemcpy(ds, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, ds, dd);
    hipMemcpy(out, dd, sizeof(out), hipMemcpyDeviceToHost);
    int first_neg = -1;
    for (int i = 0; i < 512; ++i) if (out[i] < 0 && first_neg < 0) first_neg = i;
    printf("first -1 at float %d\n", first_neg);
    for (int i = 0; i < 24; ++i) printf("%g ", out[i]);
    printf("\n");
    return 0;
}
