// Cycles per step of the PRODUCTION affine steady-state loop (tools/gen_block_asm.py
// gen_aff2, the same code object strings as fill_affine_kernel) with every hand-off
// counter already satisfied: the loop's own instruction and stall cost, without the
// band chain's waiting.  One to eight waves per workgroup, each with its own rings.
// Diagnostic tool, not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/aff_loop_micro.hip -o tools/micro/bin/aff_loop_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#ifdef ANYSEQ_ASM_INC
#include ANYSEQ_ASM_INC
#else
#include "../../anyseq_amd/csrc/anyseq_block_asm.inc"
#endif

#define RFL(x) __builtin_amdgcn_readfirstlane(x)
constexpr int kMaxW = 8;

struct alignas(16) Sh {
    int2 ring[kMaxW][16 * 32];    // each wave's in-ring (4 KiB)
    int2 next[kMaxW][16 * 32];    // each wave's out-ring
    uint32_t skew[32][8][64];     // pre-skewed subject codes (64 KiB)
    uint32_t ctr[kMaxW][8];       // prod, cons, next prod, next cons, s_filled, tail
    uint32_t dummy[kMaxW][320];   // "st" publishing: the non-publishing lanes' store targets
};

// IOV > 0: the last wave of the workgroup (wave 4 of 5: on SIMD 0 beside compute wave 0)
// stands in for the fill's I/O wave: passes of IOV independent VALU adds, each pass
// followed by s_sleep IOS (0: none), until every compute wave is done.
template <int V, int IOV = 0, int IOS = 1>
__global__ __launch_bounds__(512) void micro(int nblocks, unsigned long long* out, int* sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Sh& sh = *reinterpret_cast<Sh*>(smem);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 32 * 8 * 64; i += blockDim.x) (&sh.skew[0][0][0])[i] = 0x03020100u + 0x01010101u * (i & 3);
    for (int i = threadIdx.x; i < kMaxW * 16 * 32; i += blockDim.x) {
        (&sh.ring[0][0])[i] = make_int2(i & 63, (i & 31) - 7);
        (&sh.next[0][0])[i] = make_int2(0, 0);
    }
    if (lane < 8) sh.ctr[wave][lane] = 0x7fffffffu;
    __shared__ uint32_t ndone;
    if (threadIdx.x == 0) ndone = 0;
    __syncthreads();
    if (IOV > 0 && wave == (int)(blockDim.x >> 6) - 1) {
        const uint32_t nc = (blockDim.x >> 6) - 1;
        int a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3;
        unsigned long long passes = 0;
        while (__hip_atomic_load(&ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < nc) {
#pragma unroll
            for (int i = 0; i < IOV / 4; ++i)
                asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
            if (IOS > 0) __builtin_amdgcn_s_sleep(IOS);
            ++passes;
        }
        sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
        if (lane == 0) out[blockIdx.x * kMaxW + wave] = passes;
        return;
    }
    auto la = [](void* p) { return (uint32_t)(size_t)(__attribute__((address_space(3))) char*)p; };
    int g = lane, fdn = -5, dg = lane - 1, tfg = 0, tff = -5, e = -100, hg = -2, bx = 0;
    const int q = lane & 3, wm = 3, wx = 0, go = -2, zlp = lane + 3;
    uint32_t ll = 0, lh = 0;
    for (int c = 0; c < 4; ++c) {
        ll |= (uint32_t)((q == c ? wm : wx) & 0xff) << (8 * c);
        lh |= (uint32_t)((q == c + 4 ? wm : wx) & 0xff) << (8 * c);
    }
    const uint32_t rb = RFL(la(sh.ring[wave])), nb = RFL(la(sh.next[wave]));
    const uint32_t apr = la(&sh.ctr[wave][0]), acn = la(&sh.ctr[wave][1]), anp = la(&sh.ctr[wave][2]),
                   anc = la(&sh.ctr[wave][3]), asf = la(&sh.ctr[wave][4]), atl = la(&sh.ctr[wave][5]);
    const uint32_t skb = la(&sh.skew[0][0][0]) + 4u * lane, lo = 8u * (lane - 48), lid8 = 8u * lane;
    const uint32_t bvb = 0, bvs = RFL(1u);
    const uint32_t pm63 = lane == 63 ? 0xffffffffu : 0u, pdb = lane == 63 ? 0u : la(&sh.dummy[wave][0]) + 16u * lane;
    const int ge = RFL(-1);
    const uint64_t hm = 0xffff000000000000ull, gp = 0;
    uint32_t b = 0, sp = 0, sf = 0, sc = 0, pf = 0, st, x0, x1, x2, x3, x4, be = RFL((uint32_t)nblocks);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#define LOOP(NAME)                                                                                              \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4)                                                                              \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(wm), [wx] "v"(wx), [ll] "v"(ll), [lh] "v"(lh), [go] "v"(go), \
                   [ge] "s"(ge), [zlp] "v"(zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(apr), [acn] "v"(acn),     \
                   [anp] "v"(anp), [anc] "v"(anc), [asf] "v"(asf), [atl] "v"(atl), [skb] "v"(skb), [lo] "v"(lo),  \
                   [lid8] "v"(lid8), [bvb] "v"(bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [pm63] "v"(pm63),   \
                   [pdb] "v"(pdb)                                                                            \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
    if constexpr (V == 0) LOOP(ANYSEQ_AF2_L_B0_LDS_U1);
    if constexpr (V == 1) LOOP(ANYSEQ_AF2_L_B0_NONE_U1);
    if constexpr (V == 2) LOOP(ANYSEQ_AF2_G_B0_LDS_U1);
    if constexpr (V == 3) LOOP(ANYSEQ_AF2_G_B0_NONE_U1);
    if constexpr (V == 4) LOOP(ANYSEQ_AF2_L_B0_LDS_U0);

    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (IOV > 0 && lane == 0) __hip_atomic_fetch_add(&ndone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    sink[blockIdx.x * blockDim.x + threadIdx.x] = g + fdn + dg + e + hg + bx + tfg + tff + (int)st;
    if (lane == 0) out[blockIdx.x * kMaxW + wave] = c1 - c0;
}

// Which SIMD each wave of a 5-wave workgroup runs on (HW_ID bits 5:4): the fill's I/O wave
// is wave 4 of 5.
__global__ void simd_ids(unsigned* out) {
    const unsigned id = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id;
}

static const char* kNames[] = {"L lds-pub lut", "L no-pub lut", "G lds-pub lut", "G no-pub lut", "L lds-pub cmp"};

template <int V>
void run(int waves, int wgs) {
    const int nblocks = 2048;
    unsigned long long* d_out;
    int* d_sink;
    (void)hipMalloc(&d_out, 8 * kMaxW * wgs);
    (void)hipMalloc(&d_sink, 4 * 64 * kMaxW * wgs);
    (void)hipFuncSetAttribute((const void*)micro<V>, hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(Sh));
    hipLaunchKernelGGL((micro<V>), dim3(wgs), dim3(64 * waves), sizeof(Sh), 0, nblocks, d_out, d_sink);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((micro<V>), dim3(wgs), dim3(64 * waves), sizeof(Sh), 0, nblocks, d_out, d_sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(kMaxW * wgs);
    (void)hipMemcpy(h.data(), d_out, 8 * kMaxW * wgs, hipMemcpyDeviceToHost);
    std::vector<double> c;
    for (int g = 0; g < wgs; ++g)
        for (int w = 0; w < waves; ++w) c.push_back((double)h[g * kMaxW + w] / (nblocks * 32.0));
    std::sort(c.begin(), c.end());
    const double steps = nblocks * 32.0;
    printf("%-14s waves/WG %d WGs %3d: cyc/step median %.2f (min %.2f max %.2f); ns/step from wall %.2f; "
           "GCUPS %.0f\n", kNames[V], waves, wgs, c[c.size() / 2], c.front(), c.back(), ms * 1e6 / steps,
           64.0 * steps * waves * wgs / (ms * 1e-3) / 1e9);
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
}

// compute waves 0..3 + the stand-in I/O wave: cycles per step of wave 0 (shares SIMD 0)
// and of waves 1..3, and the I/O wave's VALU issue rate
template <int IOV, int IOS>
void run_io() {
    const int nblocks = 2048, wgs = 256, waves = 5;
    unsigned long long* d_out;
    int* d_sink;
    (void)hipMalloc(&d_out, 8 * kMaxW * wgs);
    (void)hipMalloc(&d_sink, 4 * 64 * kMaxW * wgs);
    (void)hipFuncSetAttribute((const void*)micro<0, IOV, IOS>, hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(Sh));
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((micro<0, IOV, IOS>), dim3(wgs), dim3(64 * waves), sizeof(Sh), 0, nblocks, d_out, d_sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(kMaxW * wgs);
    (void)hipMemcpy(h.data(), d_out, 8 * kMaxW * wgs, hipMemcpyDeviceToHost);
    std::vector<double> w0, w13, io;
    for (int g = 0; g < wgs; ++g) {
        w0.push_back((double)h[g * kMaxW] / (nblocks * 32.0));
        for (int w = 1; w < 4; ++w) w13.push_back((double)h[g * kMaxW + w] / (nblocks * 32.0));
        io.push_back((double)h[g * kMaxW + 4] * IOV / (nblocks * 32.0) / (h[g * kMaxW] / (nblocks * 32.0)));
    }
    std::sort(w0.begin(), w0.end());
    std::sort(w13.begin(), w13.end());
    std::sort(io.begin(), io.end());
    printf("io VALU/pass %3d sleep %d: wave0 cyc/step %.2f, waves1-3 %.2f; io wave VALU per cycle %.3f "
           "(%.2f per wave0 step)\n", IOV, IOS, w0[w0.size() / 2], w13[w13.size() / 2], io[io.size() / 2],
           io[io.size() / 2] * w0[w0.size() / 2]);
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
}

template <int V>
void all() {
    run<V>(1, 1);
    run<V>(4, 1);
    run<V>(4, 256);
    run<V>(8, 256);
}

int main() {
    {
        unsigned* d;
        (void)hipMalloc(&d, 8 * 4 * 256);
        hipLaunchKernelGGL(simd_ids, dim3(256), dim3(320), 0, 0, d);
        std::vector<unsigned> h(8 * 256);
        (void)hipMemcpy(h.data(), d, 8 * 4 * 256, hipMemcpyDeviceToHost);
        for (int g = 0; g < 4; ++g) {
            printf("WG %d (5 waves): SIMD of waves 0..4:", g);
            for (int w = 0; w < 5; ++w) printf(" %u", (h[g * 8 + w] >> 4) & 3);
            printf("\n");
        }
        (void)hipFree(d);
    }
    all<0>();
    all<1>();
    all<2>();
    all<3>();
    all<4>();
    run_io<4, 1>();
    run_io<16, 1>();
    run_io<64, 1>();
    run_io<16, 0>();
    run_io<64, 0>();
    return 0;
}
