// Which VALU mixes two waves of one SIMD can issue side by side (verdict round 4, item 4).
// Independent streams of 32 instructions per pass (8 accumulators), one workgroup of 4
// waves (one per SIMD) or 8 (two per SIMD); cycles per instruction per wave and per SIMD.
// Diagnostic tool, not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/coissue_micro.hip -o tools/micro/bin/coissue_micro
#include <hip/hip_runtime.h>

#include <cstdio>

#define ADD(r) "v_add_u32_e32 " r ", %8, " r "\n"
#define ADD64(r) "v_add_u32_e64 " r ", %8, " r "\n"
#define DPP(r) "v_mov_b32_dpp " r ", %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define DPPADD(r) "v_add_u32_dpp " r ", %8, " r " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define SDWA(r) "v_add_u32_sdwa " r ", " r ", sext(%9) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define MAX3(r) "v_max3_i32 " r ", %8, %9, " r "\n"
#define MAX(r) "v_max_i32_e32 " r ", %8, " r "\n"
#define PERM(r) "v_perm_b32 " r ", %8, %9, " r "\n"
#define OP2(op) "v_" op " %0, %8, %0\n" "v_" op " %1, %8, %1\n" "v_" op " %2, %8, %2\n" "v_" op " %3, %8, %3\n" \
                "v_" op " %4, %8, %4\n" "v_" op " %5, %8, %5\n" "v_" op " %6, %8, %6\n" "v_" op " %7, %8, %7\n"
#define OPXY(op) "v_" op " %0, %8, %9\n" "v_" op " %1, %8, %9\n" "v_" op " %2, %8, %9\n" "v_" op " %3, %8, %9\n" \
                 "v_" op " %4, %8, %9\n" "v_" op " %5, %8, %9\n" "v_" op " %6, %8, %9\n" "v_" op " %7, %8, %9\n"
#define OP3(op) "v_" op " %0, %8, %9, %0\n" "v_" op " %1, %8, %9, %1\n" "v_" op " %2, %8, %9, %2\n" \
                "v_" op " %3, %8, %9, %3\n" "v_" op " %4, %8, %9, %4\n" "v_" op " %5, %8, %9, %5\n" \
                "v_" op " %6, %8, %9, %6\n" "v_" op " %7, %8, %9, %7\n"

// 8 instructions over the 8 accumulators; X = the op of slot 0 (the others plain adds)
#define ROW(X, Y) X("%0") ADD("%1") ADD("%2") ADD("%3") Y("%4") ADD("%5") ADD("%6") ADD("%7")
#define ALL(X) X("%0") X("%1") X("%2") X("%3") X("%4") X("%5") X("%6") X("%7")
#define NONE(r)

#define KERNEL(NAME, BODY)                                                                                  \
    __global__ void NAME(int iters, unsigned long long* out, int* sink) {                                  \
        int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, \
            a7 = a0 + 7;                                                                                     \
        const int x = threadIdx.x * 3, y = threadIdx.x ^ 5;                                                  \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                          \
        for (int i = 0; i < iters; ++i)                                                                      \
            asm volatile(BODY BODY BODY BODY                                                                 \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)    \
                         : "v"(x), "v"(y));                                                                  \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                          \
        sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                 \
        if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;                                        \
    }

KERNEL(k_add, ALL(ADD))
KERNEL(k_add64, ALL(ADD64))
KERNEL(k_dpp, ALL(DPP))
KERNEL(k_dppadd, ALL(DPPADD))
KERNEL(k_sdwa, ALL(SDWA))
KERNEL(k_max3, ALL(MAX3))
KERNEL(k_max, ALL(MAX))
KERNEL(k_perm, ALL(PERM))
KERNEL(k_1dpp, ROW(DPP, ADD))
KERNEL(k_1sdwa, ROW(SDWA, ADD))
KERNEL(k_1max3, ROW(MAX3, ADD))
KERNEL(k_1add64, ROW(ADD64, ADD))
KERNEL(k_2dpp, ROW(DPP, DPP))
KERNEL(k_dpp_max3, ROW(DPP, MAX3))
KERNEL(k_2max3, ROW(MAX3, MAX3))
#define MOV(r) "v_mov_b32_e32 " r ", %8\n"
#define CND(r) "v_cndmask_b32_e32 " r ", %8, " r ", vcc\n"
KERNEL(k_mov, ALL(MOV))
KERNEL(k_cnd, ALL(CND))
KERNEL(k_sub, OP2("sub_u32_e32"))
KERNEL(k_maxu, OP2("max_u32_e32"))
KERNEL(k_min, OP2("min_i32_e32"))
KERNEL(k_and, OP2("and_b32_e32"))
KERNEL(k_lsh, OP2("lshlrev_b32_e32"))
KERNEL(k_maxf, OP2("max_f32_e32"))
KERNEL(k_addf, OP2("add_f32_e32"))
KERNEL(k_max16, OP2("max_i16_e32"))
KERNEL(k_pkmax, OP2("pk_max_i16"))
KERNEL(k_pkadd, OP2("pk_add_u16"))
KERNEL(k_maxxy, OPXY("max_i32_e32"))
KERNEL(k_addxy, OPXY("add_u32_e32"))
KERNEL(k_max3f, OP3("max3_f32"))
KERNEL(k_fma, OP3("fma_f32"))
KERNEL(k_add3, OP3("add3_u32"))
KERNEL(k_med3, OP3("med3_i32"))

typedef void (*Kern)(int, unsigned long long*, int*);

static double run(Kern k, int waves) {
    unsigned long long* d;
    int* s;
    (void)hipMalloc(&d, 8 * 16);
    (void)hipMalloc(&s, 4 * 1024);
    const int iters = 2000;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, iters, d, s);
    (void)hipDeviceSynchronize();
    unsigned long long h[16];
    (void)hipMemcpy(h, d, 8 * waves, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
    (void)hipFree(d);
    (void)hipFree(s);
    return (double)mx / (iters * 32.0);
}

static void row(const char* name, Kern k) {
    const double one = run(k, 4), two = run(k, 8);
    printf("%-34s 1 wave/SIMD %5.2f cyc/instr | 2 waves/SIMD %5.2f per wave = %5.2f per SIMD (gain %.2fx)\n", name,
           one, two, two / 2, one / (two / 2));
}

int main() {
    row("v_add_e32", k_add);
    row("v_add_e64", k_add64);
    row("v_max_e32", k_max);
    row("v_mov_dpp", k_dpp);
    row("v_add_dpp", k_dppadd);
    row("v_add_sdwa", k_sdwa);
    row("v_max3", k_max3);
    row("v_perm", k_perm);
    row("7 add + 1 dpp", k_1dpp);
    row("7 add + 1 sdwa", k_1sdwa);
    row("7 add + 1 max3", k_1max3);
    row("7 add + 1 add_e64", k_1add64);
    row("6 add + 2 dpp", k_2dpp);
    row("6 add + 1 dpp + 1 max3", k_dpp_max3);
    row("6 add + 2 max3", k_2max3);
    row("v_mov_e32", k_mov);
    row("v_cndmask_e32", k_cnd);
    row("v_sub_u32_e32", k_sub);
    row("v_max_u32_e32", k_maxu);
    row("v_min_i32_e32", k_min);
    row("v_and_b32_e32", k_and);
    row("v_lshlrev_b32_e32", k_lsh);
    row("v_max_f32_e32", k_maxf);
    row("v_add_f32_e32", k_addf);
    row("v_max_i16_e32", k_max16);
    row("v_pk_max_i16", k_pkmax);
    row("v_pk_add_u16", k_pkadd);
    row("v_max_i32 r, x, y (no dep)", k_maxxy);
    row("v_add_u32 r, x, y (no dep)", k_addxy);
    row("v_max3_f32", k_max3f);
    row("v_fma_f32", k_fma);
    row("v_add3_u32", k_add3);
    row("v_med3_i32", k_med3);
    return 0;
}
