// Cost of the fill step's 5-instruction pattern and variants (one wave, cycles per step).
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
// C D E A B: cmp, cndmask, add, dpp (reads c written by previous B), max3
#define STEP_DPP "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
                 "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
                 "v_add_u32_e32 %[a], %[t], %[w]\n"                                \
                 "v_mov_b32_dpp %[t], %[c] wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %[c], %[a], %[c], %[t]\n"
// same, DPP replaced by a plain move
#define STEP_MOV "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
                 "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
                 "v_add_u32_e32 %[a], %[t], %[w]\n"                                \
                 "v_mov_b32 %[t], %[c]\n"                                          \
                 "v_max3_i32 %[c], %[a], %[c], %[t]\n"
// DPP on an operand not written recently (x), result feeds max3
#define STEP_DPPX "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
                  "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
                  "v_add_u32_e32 %[a], %[t], %[w]\n"                                \
                  "v_mov_b32_dpp %[t], %[x] wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                  "v_max3_i32 %[c], %[a], %[c], %[t]\n"
// DPP result NOT consumed by the next instruction (max3 uses x)
#define STEP_DPPN "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
                  "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
                  "v_add_u32_e32 %[a], %[x], %[w]\n"                                \
                  "v_mov_b32_dpp %[t], %[c] wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                  "v_max3_i32 %[c], %[a], %[c], %[x]\n"
// dpp with row_shr instead of wave_shr
#define STEP_ROW "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
                 "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
                 "v_add_u32_e32 %[a], %[t], %[w]\n"                                \
                 "v_mov_b32_dpp %[t], %[c] row_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %[c], %[a], %[c], %[t]\n"
// two interleaved independent chains (c,t) and (c2,t2)
#define STEP_2 "v_cmp_eq_u32_sdwa vcc, %[q], %[s] src0_sel:DWORD src1_sel:BYTE_1\n" \
               "v_cndmask_b32_e32 %[w], %[wx], %[wm], vcc\n"                     \
               "v_add_u32_e32 %[a], %[t], %[w]\n"                                \
               "v_add_u32_e32 %[a2], %[t2], %[w]\n"                              \
               "v_mov_b32_dpp %[t], %[c] wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
               "v_mov_b32_dpp %[t2], %[c2] wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
               "v_max3_i32 %[c], %[a], %[c], %[t]\n"                             \
               "v_max3_i32 %[c2], %[a2], %[c2], %[t2]\n"

template <int T>
__global__ void k(int iters, unsigned long long* out, int* sink) {
    int c = threadIdx.x, t = 3, a = 0, w = 0, c2 = 7, t2 = 1, a2 = 0, x = threadIdx.x * 5;
    int q = threadIdx.x & 3, s = 0x01020304 * (threadIdx.x & 1), wm = 4, wx = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define OPS : [c] "+v"(c), [t] "+v"(t), [a] "+v"(a), [w] "+v"(w), [c2] "+v"(c2), [t2] "+v"(t2), [a2] "+v"(a2) \
            : [q] "v"(q), [s] "v"(s), [wm] "v"(wm), [wx] "v"(wx), [x] "v"(x) : "vcc"
        if (T == 0) asm volatile(R8(STEP_DPP) OPS);
        if (T == 1) asm volatile(R8(STEP_MOV) OPS);
        if (T == 2) asm volatile(R8(STEP_DPPX) OPS);
        if (T == 3) asm volatile(R8(STEP_DPPN) OPS);
        if (T == 4) asm volatile(R8(STEP_ROW) OPS);
        if (T == 5) asm volatile(R8(STEP_2) OPS);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = c + t + a + w + c2 + t2 + a2;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

const char* names[] = {"step C D E A(dpp c) B", "step with plain mov", "dpp of stale x", "dpp result unused next",
                       "row_shr dpp", "two chains interleaved (per step of both)"};

template <int T>
void run(int waves) {
    unsigned long long* d; int* s;
    hipMalloc(&d, 8); hipMalloc(&s, 4 * 64 * 8);
    const int iters = 2000;
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves), 0, 0, iters, d, s);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves), 0, 0, iters, d, s);
    unsigned long long h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-45s waves/WG=%d: %.2f cycles per step\n", names[T], waves, (double)h / (8.0 * iters));
    hipFree(d); hipFree(s);
}

int main() {
    run<0>(1); run<1>(1); run<2>(1); run<3>(1); run<4>(1); run<5>(1);
    run<0>(8); run<5>(8);
    return 0;
}
