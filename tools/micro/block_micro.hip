// Cycles of the generated 32-step block asm (tools/gen_block_asm.py) in a loop,
// one wave: full, without the bottom-row stores, without the top-row reads, bare.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../anyseq_amd/csrc/anyseq_block_asm.inc"

template <int V>
__global__ void k(int iters, uint64_t pm, unsigned long long* out, int* sink) {
    __shared__ __attribute__((aligned(16))) int ring[64];
    __shared__ __attribute__((aligned(16))) int pub[64 * 4 + 64];
    const int lane = threadIdx.x & 63;
    ring[lane] = lane * 3;
    __syncthreads();
    int cur = lane, dg = lane * 2, tf = 5;
    uint32_t ra = (uint32_t)(size_t)(__attribute__((address_space(3))) int*)ring;
    uint32_t pa = (uint32_t)(size_t)(__attribute__((address_space(3))) int*)pub + (V == 4 || V == 0 ? 4 * lane : 0);
    uint32_t sw[8];
    for (int i = 0; i < 8; ++i) sw[i] = 0x41434754u + lane + i;
    int q = 0x41 + (lane & 3), wm = 4, wx = 1;
    uint64_t sv;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define ARGS : [cur] "+v"(cur), [dg] "+v"(dg), [tf] "+v"(tf), [sv] "=&s"(sv) \
             : [ra] "v"(ra), [pa] "v"(pa), [pm] "s"(pm), [s0] "v"(sw[0]), [s1] "v"(sw[1]), [s2] "v"(sw[2]), \
               [s3] "v"(sw[3]), [s4] "v"(sw[4]), [s5] "v"(sw[5]), [s6] "v"(sw[6]), [s7] "v"(sw[7]), [q] "v"(q), \
               [wm] "v"(wm), [wx] "v"(wx) : ANYSEQ_BLOCK_ASM_CLOBBERS, "memory"
        if (V == 0) asm volatile(ANYSEQ_BLOCK_ASM_G ARGS);
        if (V == 1) asm volatile(ANYSEQ_BLOCK_ASM_G_NOST ARGS);
        if (V == 2) asm volatile(ANYSEQ_BLOCK_ASM_G_NORD ARGS);
        if (V == 3) asm volatile(ANYSEQ_BLOCK_ASM_G_NONE ARGS);
        if (V == 4) asm volatile(ANYSEQ_BLOCK_ASM_G_ALLST ARGS);
        if (V == 5) asm volatile(ANYSEQ_BLOCK_ASM_G_EXONLY ARGS);
        if (V == 6) asm volatile(ANYSEQ_BLOCK_ASM_G_EXEC ARGS);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = cur + dg + tf;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

const char* names[] = {"full: b128 reads + shift register + 1 b32 store", "no stores", "no reads", "bare steps",
                       "stores by all lanes, no exec switch", "exec switches only",
                       "lane-63 b128 stores under exec"};
template <int V>
void run(uint64_t pm) {
    unsigned long long* d; int* s;
    hipMalloc(&d, 8); hipMalloc(&s, 4 * 64);
    const int iters = 1000;
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, iters, pm, d, s);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, iters, pm, d, s);
    unsigned long long h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-40s pm=%016llx: %.1f cycles per 32-step block (%.2f per step)\n", names[V], (unsigned long long)pm,
           (double)h / iters, (double)h / iters / 32);
    hipFree(d); hipFree(s);
}
int main() {
    run<0>(1ull << 63); run<0>(0); run<1>(0); run<2>(1ull << 63); run<2>(0); run<3>(0); run<4>(0);
    run<5>(1ull << 63); run<6>(1ull << 63);
    return 0;
}
