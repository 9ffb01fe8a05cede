// Micro-benchmark of candidate affine steady-state steps (tools/micro/gen_aff_micro.py):
// cycles per step for one wave alone, one wave per SIMD (4 per CU) and two per SIMD
// (8 per CU), on one CU and on every CU.  Diagnostic tool, not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/aff_micro.hip -o tools/micro/bin/aff_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "aff_micro.inc"

#define RFL(x) __builtin_amdgcn_readfirstlane(x)

template <int V>
__global__ __launch_bounds__(512) void micro(int nblocks, unsigned long long* out, int* sink) {
    __shared__ uint32_t sbuf[64 * 8];
    __shared__ __attribute__((aligned(16))) uint32_t dsink[8 * 64 * 64];   // per-wave ds_write target (128 KiB)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 64 * 8; i += blockDim.x) sbuf[i] = 0x03020100u + 0x01010101u * (i & 3);
    __syncthreads();
    int cur = lane, fd = -5, dg = lane - 1, tfg = 0, tff = -5, e = -100, hg = -2, best = 0;
    const int q = 0x41 + (lane & 3), wm = 4, wx = 1, go = -2, ge = -1, zl = lane + 3;
    const int lh = 0x01010101, ll = 0x04010401;
    uint32_t z = RFL((uint32_t)(lane * 0 + 3)), zb = RFL((uint32_t)3), nge = RFL((uint32_t)1);
    const uint32_t sa = (uint32_t)(size_t)(sbuf + lane * 8);
    const uint32_t pa = (uint32_t)(size_t)(dsink + wave * 4096 + lane * 64);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nblocks; ++b) {
#define AFFM_RUN(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(cur), [fd] "+v"(fd), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(best), [z] "+s"(z), [zb] "+s"(zb)                                  \
                 : [q] "v"(q), [wm] "v"(wm), [wx] "v"(wx), [go] "v"(go), [ge] "v"(ge), [zl] "v"(zl), [lh] "v"(lh), \
                   [ll] "v"(ll), [nge] "s"(nge), [sa] "v"(sa), [pa] "v"(pa)                                      \
                 : AFFM_CLOBBERS, "memory")
        if constexpr (V == 0) AFFM_RUN(AFFM_L_cur);
        if constexpr (V == 1) AFFM_RUN(AFFM_L_x);
        if constexpr (V == 2) AFFM_RUN(AFFM_L_xl);
        if constexpr (V == 3) AFFM_RUN(AFFM_L_xl_np);
        if constexpr (V == 4) AFFM_RUN(AFFM_L_xl_ds);
        if constexpr (V == 5) AFFM_RUN(AFFM_G_cur);
        if constexpr (V == 6) AFFM_RUN(AFFM_G_l);
        if constexpr (V == 7) AFFM_RUN(AFFM_L_es_np);
        if constexpr (V == 8) AFFM_RUN(AFFM_L_ro);
        if constexpr (V == 9) AFFM_RUN(AFFM_L_ro_np);
        if constexpr (V == 10) AFFM_RUN(AFFM_G_ro);
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = cur + fd + dg + e + hg + best + (int)z + (int)zb;
    if (lane == 0) out[blockIdx.x * 8 + wave] = c1 - c0;
}

static const char* kNames[] = {"L_cur", "L_x", "L_xl", "L_xl_np", "L_xl_ds", "G_cur", "G_l", "L_es_np", "L_ro", "L_ro_np", "G_ro"};

template <int V>
void run(int waves, int wgs) {
    const int nblocks = 1024;
    unsigned long long* d_out;
    int* d_sink;
    hipMalloc(&d_out, 8 * 8 * wgs);
    hipMalloc(&d_sink, 4 * 512 * wgs);
    hipLaunchKernelGGL((micro<V>), dim3(wgs), dim3(64 * waves), 0, 0, nblocks, d_out, d_sink);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((micro<V>), dim3(wgs), dim3(64 * waves), 0, 0, nblocks, d_out, d_sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(8 * wgs);
    hipMemcpy(h.data(), d_out, 8 * 8 * wgs, hipMemcpyDeviceToHost);
    std::vector<double> c;
    for (int g = 0; g < wgs; ++g)
        for (int w = 0; w < waves; ++w) c.push_back((double)h[g * 8 + w] / (nblocks * 32.0));
    std::sort(c.begin(), c.end());
    const double steps = nblocks * 32.0;
    printf("%-8s waves/WG %d WGs %3d: cyc/step median %.2f (min %.2f max %.2f); ns/step from wall %.2f\n", kNames[V],
           waves, wgs, c[c.size() / 2], c.front(), c.back(), ms * 1e6 / steps);
    hipFree(d_out);
    hipFree(d_sink);
}

template <int V>
void all() {
    run<V>(1, 1);
    run<V>(4, 1);
    run<V>(8, 1);
    run<V>(4, 256);
    run<V>(8, 256);
}

int main() {
    all<0>();
    all<1>();
    all<2>();
    all<3>();
    all<4>();
    all<5>();
    all<6>();
    all<7>();
    all<8>();
    all<9>();
    all<10>();
    return 0;
}
