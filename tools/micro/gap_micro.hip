// Launch gaps around a large kernel (round 5: every fill launch sits between two ~5.4 us
// gaps in the kernel trace, while back-to-back small kernels start with none).  Small
// kernel A, kernel B (variants: grid, block, LDS per workgroup, VGPRs, a spin of fixed
// length), small kernel C, repeated; run under rocprofv3 --kernel-trace and read the gaps
// (tools/micro/gap_report.py).  Diagnostic tool, not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/gap_micro.hip -o tools/micro/bin/gap_micro
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>

__global__ void small_kernel(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// spins ~`ticks` of s_memrealtime (100 MHz) so every variant lasts about as long
template <int LDS, int REGS>
__global__ void big_kernel(int* p, int ticks) {
    __shared__ int lds[LDS > 0 ? LDS / 4 : 1];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int acc[REGS];
#pragma unroll
    for (int i = 0; i < REGS; ++i) acc[i] = threadIdx.x + i;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) {
#pragma unroll
        for (int i = 0; i < REGS; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(acc[i]));
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < REGS; ++i) s += acc[i];
    if (LDS > 0) {
        lds[threadIdx.x % (LDS / 4)] = s;
        __syncthreads();
        s += lds[(threadIdx.x + 1) % (LDS / 4)];
    }
    if (s == 0x7fffffff) p[1] = s;
}

// ev: 0 none, 1 hipEventRecord around the big kernel, 2 hipExtLaunchKernelGGL's own
// start/stop events (recorded by the dispatch packet); on a created stream
template <int LDS, int REGS>
void run(const char* name, int grid, int block, int* d, int ev, hipStream_t st) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL(small_kernel, dim3(64), dim3(256), 0, st, d);
        if (ev == 1) hipEventRecord(e0, st);
        if (ev == 2)
            hipExtLaunchKernelGGL((big_kernel<LDS, REGS>), dim3(grid), dim3(block), 0, st, e0, e1, 0, d, 20000);
        else
            hipLaunchKernelGGL((big_kernel<LDS, REGS>), dim3(grid), dim3(block), 0, st, d, 20000);   // 200 us
        if (ev == 1) hipEventRecord(e1, st);
        hipLaunchKernelGGL(small_kernel, dim3(64), dim3(256), 0, st, d);
    }
    hipStreamSynchronize(st);
    float ms = 0.f;
    if (ev) hipEventElapsedTime(&ms, e0, e1);
    printf("%s grid %d block %d LDS %d regs %d events %d: last big kernel %.3f ms by its events\n", name, grid, block,
           LDS, REGS, ev, ms);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    int* d;
    hipMalloc(&d, 64);
    hipMemset(d, 0, 64);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    run<90624, 200>("null stream", 256, 320, d, 0, 0);
    run<90624, 200>("stream", 256, 320, d, 0, st);
    run<0, 8>("stream", 256, 320, d, 0, st);
    run<90624, 200>("stream+events", 256, 320, d, 1, st);
    run<0, 8>("stream+events", 256, 320, d, 1, st);
    run<90624, 200>("stream+ext events", 256, 320, d, 2, st);
    hipStreamDestroy(st);
    hipFree(d);
    return 0;
}
