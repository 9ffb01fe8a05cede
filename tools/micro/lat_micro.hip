// Latency of the dependency chains that can carry the fill step's lane-to-lane
// dependency (one wave, cycles per chain link, s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

template <int T>
__global__ void k(int iters, unsigned long long* out, int* sink) {
    int a = threadIdx.x, b = threadIdx.x * 7, x = threadIdx.x * 3, y = threadIdx.x ^ 5;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        // 16 links per asm block
        if (T == 0) asm volatile(R16("v_max_i32 %0, %0, %2\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 1) asm volatile(R16("v_max_i32_dpp %0, %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 2) asm volatile(R16("v_max_i32_dpp %0, %0, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 3) asm volatile(R16("s_nop 1\nv_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 4) asm volatile(R16("v_max3_i32 %1, %0, %2, %3\ns_nop 1\nv_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 5) asm volatile(R16("v_max_i32 %1, %0, %2\ns_nop 1\nv_max_i32_dpp %0, %1, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 6) asm volatile(R16("v_max_i32_dpp %0, %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 7) asm volatile(R16("v_max_i32_dpp %0, %0, %2 row_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 0\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 8) asm volatile(R16("v_max_i32_dpp %0, %0, %2 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        // 4 independent chains interleaved, each link = max3 + dpp-fused max
        if (T == 9) asm volatile(R4("v_max_i32_dpp %0, %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %1, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                     "v_max_i32_dpp %0, %0, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_max_i32_dpp %1, %1, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                                 : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 10) asm volatile(R16("v_permlane32_swap_b32 %0, %1\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
        if (T == 11) asm volatile(R16("v_max_i32 %0, %0, %2\nv_max_i32 %1, %1, %2\n") : "+v"(a), "+v"(b) : "v"(x), "v"(y));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = a + b;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

const char* names[] = {"v_max chain", "v_max_dpp wave_shr chain", "v_max_dpp row_shr chain", "nop1+mov_dpp wave_shr chain",
                       "max3 -> nop1 -> mov_dpp link", "max -> nop1 -> max_dpp link", "v_max_dpp wave_shr (bc0)",
                       "v_max_dpp row_shr + nop0", "v_max_dpp quad_perm", "2 chains max_dpp interleaved (per link)",
                       "v_permlane32_swap", "2 indep v_max chains (per instr)"};

template <int T>
void run() {
    unsigned long long* d; int* s;
    hipMalloc(&d, 8); hipMalloc(&s, 4 * 64);
    const int iters = 2000;
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64), 0, 0, iters, d, s);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64), 0, 0, iters, d, s);
    unsigned long long h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    const double links = (T == 9 ? 8.0 : (T == 11 ? 32.0 : 16.0)) * iters;
    printf("%-42s %.2f cycles per link\n", names[T], (double)h / links);
    hipFree(d); hipFree(s);
}

int main() {
    run<0>(); run<1>(); run<2>(); run<3>(); run<4>(); run<5>(); run<6>(); run<7>(); run<8>(); run<9>(); run<10>(); run<11>();
    return 0;
}
