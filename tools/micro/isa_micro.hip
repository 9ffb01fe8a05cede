// Issue cost of the VALU forms the fill step uses, one wave per SIMD (1 WG of
// 64*W threads, W waves): independent streams (throughput) and dependent chains
// (latency).  Prints cycles per instruction per wave (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define IND(op) \
    asm volatile(REP8(op " %0, %8, %9\n" op " %1, %8, %9\n" op " %2, %8, %9\n" op " %3, %8, %9\n" \
                      op " %4, %8, %9\n" op " %5, %8, %9\n" op " %6, %8, %9\n" op " %7, %8, %9\n") \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));

template <int T>
__global__ void k(int iters, unsigned long long* out, int* sink) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int x = threadIdx.x * 3, y = threadIdx.x ^ 5;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (T == 0) IND("v_add_u32")                       // 64 independent adds
        if (T == 1) IND("v_max_i32")
        if (T == 2) asm volatile(REP8("v_max3_i32 %0, %8, %9, %0\nv_max3_i32 %1, %8, %9, %1\nv_max3_i32 %2, %8, %9, %2\nv_max3_i32 %3, %8, %9, %3\n"
                                      "v_max3_i32 %4, %8, %9, %4\nv_max3_i32 %5, %8, %9, %5\nv_max3_i32 %6, %8, %9, %6\nv_max3_i32 %7, %8, %9, %7\n")
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
        if (T == 3) asm volatile(REP8("v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                      "v_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                      "v_mov_b32_dpp %4, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %5, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                      "v_mov_b32_dpp %6, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %7, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
        if (T == 4) asm volatile(REP8("v_cmp_eq_u32_sdwa vcc, %8, %9 src0_sel:DWORD src1_sel:BYTE_1\nv_cndmask_b32 %0, %8, %9, vcc\n"
                                      "v_cmp_eq_u32_sdwa vcc, %8, %9 src0_sel:DWORD src1_sel:BYTE_2\nv_cndmask_b32 %1, %8, %9, vcc\n"
                                      "v_cmp_eq_u32_sdwa vcc, %8, %9 src0_sel:DWORD src1_sel:BYTE_3\nv_cndmask_b32 %2, %8, %9, vcc\n"
                                      "v_cmp_eq_u32_sdwa vcc, %8, %9 src0_sel:DWORD src1_sel:BYTE_0\nv_cndmask_b32 %3, %8, %9, vcc\n")
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y) : "vcc");
        // dependent chains
        if (T == 5) asm volatile(REP8("v_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\n"
                                      "v_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\nv_add_u32 %0, %0, %1\n")
                                 : "+v"(a0) : "v"(x));
        if (T == 6) asm volatile(REP8("v_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\n"
                                      "v_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\nv_max3_i32 %0, %0, %1, %2\n")
                                 : "+v"(a0) : "v"(x), "v"(y));
        // dpp <- max3 chain (the step's critical path): max3 then dpp of its result, s_nop 1 hazard pad
        if (T == 7) asm volatile(REP8("v_max3_i32 %0, %1, %2, %3\ns_nop 1\nv_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                      "v_max3_i32 %0, %1, %2, %3\ns_nop 1\nv_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                                 : "+v"(a0), "+v"(a1) : "v"(x), "v"(y));
        // same chain, two independent copies interleaved (fills the nops)
        if (T == 8) asm volatile(REP8("v_max3_i32 %0, %1, %4, %5\nv_max3_i32 %2, %3, %4, %5\ns_nop 0\nv_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
                                      "v_mov_b32_dpp %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y));
        if (T == 9) asm volatile(REP8("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:DWORD src1_sel:BYTE_1\nv_cmp_eq_u32_sdwa s[100:101], %0, %1 src0_sel:DWORD src1_sel:BYTE_2\n"
                                      "v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:DWORD src1_sel:BYTE_1\nv_cmp_eq_u32_sdwa s[100:101], %0, %1 src0_sel:DWORD src1_sel:BYTE_2\n"
                                      "v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:DWORD src1_sel:BYTE_1\nv_cmp_eq_u32_sdwa s[100:101], %0, %1 src0_sel:DWORD src1_sel:BYTE_2\n"
                                      "v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:DWORD src1_sel:BYTE_1\nv_cmp_eq_u32_sdwa s[100:101], %0, %1 src0_sel:DWORD src1_sel:BYTE_2\n")
                                 : : "v"(x), "v"(y) : "vcc", "s100", "s101");
        if (T == 10) asm volatile(REP8("v_mov_b32 %0, %8\nv_mov_b32 %1, %8\nv_mov_b32 %2, %8\nv_mov_b32 %3, %8\n"
                                      "v_mov_b32 %4, %9\nv_mov_b32 %5, %9\nv_mov_b32 %6, %9\nv_mov_b32 %7, %9\n")
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
        if (T == 11) asm volatile(REP8("v_add_u32_sdwa %0, %0, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
                                       "v_add_u32_sdwa %1, %1, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n"
                                       "v_add_u32_sdwa %2, %2, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3\n"
                                       "v_add_u32_sdwa %3, %3, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n"
                                       "v_add_u32_sdwa %4, %4, sext(%9) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
                                       "v_add_u32_sdwa %5, %5, sext(%9) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n"
                                       "v_add_u32_sdwa %6, %6, sext(%9) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3\n"
                                       "v_add_u32_sdwa %7, %7, sext(%9) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n")
                                  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
        if (T == 12) asm volatile(REP8("v_perm_b32 %0, %8, %9, %0\nv_perm_b32 %1, %8, %9, %1\nv_perm_b32 %2, %8, %9, %2\nv_perm_b32 %3, %8, %9, %3\n"
                                       "v_perm_b32 %4, %8, %9, %4\nv_perm_b32 %5, %8, %9, %5\nv_perm_b32 %6, %8, %9, %6\nv_perm_b32 %7, %8, %9, %7\n")
                                  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
        // the affine step's mix without dependencies: 2 dpp, 2 max3, 2 add, 1 max, 1 sdwa add per 8
        if (T == 13) asm volatile(REP8("v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_max3_i32 %1, %8, %9, %1\n"
                                       "v_add_u32 %2, %8, %9\nv_add_u32_sdwa %3, %3, sext(%8) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
                                       "v_mov_b32_dpp %4, %9 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_max3_i32 %5, %8, %9, %5\n"
                                       "v_add_u32 %6, %8, %9\nv_max_i32 %7, %8, %9\n")
                                  : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

const char* names[] = {"v_add indep", "v_max indep", "v_max3 indep", "v_mov_dpp indep", "cmp_sdwa+cndmask pairs",
                       "v_add dep chain", "v_max3 dep chain", "max3->nop1->dpp chain", "2x max3/dpp chains",
                       "cmp_sdwa indep", "v_mov indep", "v_add_sdwa(byte sext) indep", "v_perm indep",
                       "affine step mix indep"};

template <int T>
void run(int waves) {
    unsigned long long* d; int* s;
    hipMalloc(&d, 8 * 1024); hipMalloc(&s, 4 * 1024 * 256);
    const int iters = 1000;
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves), 0, 0, iters, d, s);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves), 0, 0, iters, d, s);
    unsigned long long h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    const int per = (T == 7) ? 16 : (T == 8 ? 32 : 64);
    printf("%-26s waves/WG=%d: %.2f cycles per instr per wave\n", names[T], waves, (double)h / (iters * (double)per));
    hipFree(d); hipFree(s);
}

template <int T>
void run_all() { run<T>(1); run<T>(4); run<T>(8); }

int main() {
    run_all<0>(); run_all<1>(); run_all<2>(); run_all<3>(); run_all<4>(); run_all<5>(); run_all<6>(); run_all<7>();
    run_all<8>(); run_all<9>(); run_all<10>(); run_all<11>(); run_all<12>(); run_all<13>();
    return 0;
}
