// The production affine steady-state loop by instruction subset, at one and two compute
// waves per SIMD (verdict round 4, item 4: why does a second wave per SIMD add so little?).
// The subsets come from tools/micro/gen_mix_micro.py (every hand-off counter satisfied,
// poll loops and loop branches cut out; two blocks per asm statement).  Prints cycles per
// step per wave (s_memtime, median over waves) and the pair's cycles per step per SIMD.
// Diagnostic tool, not part of the product.
// build: python3 tools/micro/gen_mix_micro.py ANYSEQ_AF2_G_B0_LDS_U1 build/mix_lds.inc &&
//        hipcc --offload-arch=gfx950 -O3 -DMIX_INC='"../../build/mix_lds.inc"' tools/micro/mix_micro.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include MIX_INC
#include "../../anyseq_amd/csrc/anyseq_block_asm.inc"   // (ANYSEQ_AF2_ASM_CLOBBERS)

#define RFL(x) __builtin_amdgcn_readfirstlane(x)
constexpr int kMaxW = 8;

struct alignas(16) Sh {
    int2 ring[kMaxW][16 * 32];
    int2 next[kMaxW][16 * 32];
    uint32_t ctr[kMaxW][8];
    int2 dum[kMaxW][96];   // (DSFULL: the per-step publish of lanes 0..62)
};

template <int V>
__global__ __launch_bounds__(512) void mix(int nblocks, const uint8_t* codes, unsigned long long* out, int* sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Sh& sh = *reinterpret_cast<Sh*>(smem);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kMaxW * 16 * 32; i += blockDim.x) {
        (&sh.ring[0][0])[i] = make_int2(i & 63, (i & 31) - 7);
        (&sh.next[0][0])[i] = make_int2(0, 0);
    }
    if (lane < 8) sh.ctr[wave][lane] = 0x7fffffffu;
    __syncthreads();
    auto la = [](void* p) { return (uint32_t)(size_t)(__attribute__((address_space(3))) char*)p; };
    int g = lane, fdn = -5, dg = lane - 1, tfg = 0, tff = -5, e = -100, hg = -2, bx = 0;
    int eb = -90, hgb = -3, ec = -80, hgc = -4;   // (R2 / R3 variants: cells B / C's E chains)
    const uint32_t llb = 0x00000300u, lhb = 0x00000003u, llc = 0x00030000u, lhc = 0x00000300u;
    const int q = lane & 3, wm = 3, wx = 0, go = -2, zlp = lane + 3;
    uint32_t ll = 0x00030000u, lh = 0x03000000u;
    const uint32_t rb = RFL(la(sh.ring[wave])), nb = RFL(la(sh.next[wave]));
    const uint32_t apr = la(&sh.ctr[wave][0]), acn = la(&sh.ctr[wave][1]), anp = la(&sh.ctr[wave][2]),
                   anc = la(&sh.ctr[wave][3]), asf = la(&sh.ctr[wave][4]), atl = la(&sh.ctr[wave][5]);
    const uint32_t skb = (uint32_t)(63 - lane), lo = 8u * (lane - 48), lid8 = 8u * lane;
    const uint32_t bvb = 0, bvs = RFL(1u);
    const uint32_t pm63 = lane == 63 ? 0xffffffffu : 0u, pdb = 0;
    const uint32_t pds = lane == 63 ? 0u : la(&sh.dum[wave][lane]);
    const int ge = RFL(-1);
    const uint64_t hm = 0xffff000000000000ull, gp = 0;
    const uint8_t* sg = codes;
    uint32_t b = 0, sp = 0x7fffffffu, sf = 0x7fffffffu, sc = 0x7fffffffu, pf = 0, st = 0, x0 = 0, x1 = 0, x2 = 0,
             x3 = 0, x4 = 0, be = RFL((uint32_t)nblocks);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#define MIXLOOP(NAME)                                                                                            \
    for (int it = 0; it < nblocks / 2; ++it)                                                                    \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "+s"(st), [x0] "+s"(x0), [x1] "+s"(x1), [x2] "+s"(x2), [x3] "+s"(x3),     \
                   [x4] "+s"(x4)                                                                               \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(wm), [wx] "v"(wx), [ll] "v"(ll), [lh] "v"(lh), [go] "v"(go), \
                   [ge] "s"(ge), [zlp] "v"(zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(apr), [acn] "v"(acn),     \
                   [anp] "v"(anp), [anc] "v"(anc), [asf] "v"(asf), [atl] "v"(atl), [skb] "v"(skb), [lo] "v"(lo),  \
                   [lid8] "v"(lid8), [bvb] "v"(bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [pm63] "v"(pm63),   \
                   [pdb] "v"(pdb), [sg] "s"(sg), [pds] "v"(pds)                                              \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
#define MIXLOOP2(NAME)                                                                                           \
    for (int it = 0; it < nblocks / 2; ++it)                                                                    \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "+s"(st), [x0] "+s"(x0), [x1] "+s"(x1), [x2] "+s"(x2), [x3] "+s"(x3),     \
                   [x4] "+s"(x4), [eb] "+v"(eb), [hgb] "+v"(hgb)                                               \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(wm), [wx] "v"(wx), [ll] "v"(ll), [lh] "v"(lh), [go] "v"(go), \
                   [ge] "s"(ge), [zlp] "v"(zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(apr), [acn] "v"(acn),     \
                   [anp] "v"(anp), [anc] "v"(anc), [asf] "v"(asf), [atl] "v"(atl), [skb] "v"(skb), [lo] "v"(lo),  \
                   [lid8] "v"(lid8), [bvb] "v"(bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [pm63] "v"(pm63),   \
                   [pdb] "v"(pdb), [sg] "s"(sg), [llb] "v"(llb), [lhb] "v"(lhb)                              \
                 : ANYSEQ_AF2_ASM_CLOBBERS, MIX_R2_CLOBBERS, "memory")
#define MIXLOOP3(NAME)                                                                                           \
    for (int it = 0; it < nblocks / 2; ++it)                                                                    \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "+s"(st), [x0] "+s"(x0), [x1] "+s"(x1), [x2] "+s"(x2), [x3] "+s"(x3),     \
                   [x4] "+s"(x4), [eb] "+v"(eb), [hgb] "+v"(hgb), [ec] "+v"(ec), [hgc] "+v"(hgc)               \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(wm), [wx] "v"(wx), [ll] "v"(ll), [lh] "v"(lh), [go] "v"(go), \
                   [ge] "s"(ge), [zlp] "v"(zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(apr), [acn] "v"(acn),     \
                   [anp] "v"(anp), [anc] "v"(anc), [asf] "v"(asf), [atl] "v"(atl), [skb] "v"(skb), [lo] "v"(lo),  \
                   [lid8] "v"(lid8), [bvb] "v"(bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [pm63] "v"(pm63),   \
                   [pdb] "v"(pdb), [sg] "s"(sg), [llb] "v"(llb), [lhb] "v"(lhb), [llc] "v"(llc), [lhc] "v"(lhc) \
                 : ANYSEQ_AF2_ASM_CLOBBERS, MIX_R3_CLOBBERS, "memory")
    if constexpr (V == 0) MIXLOOP(MIX_FULL);
    if constexpr (V == 1) MIXLOOP(MIX_VALU);
    if constexpr (V == 2) MIXLOOP(MIX_VALU_LDS);
    if constexpr (V == 3) MIXLOOP(MIX_VALU_SALU);
    if constexpr (V == 4) MIXLOOP(MIX_VALU_WAIT);
    if constexpr (V == 5) MIXLOOP(MIX_VALU_GLOB);
    if constexpr (V == 6) MIXLOOP(MIX_NODPP);
    if constexpr (V == 7) MIXLOOP(MIX_NOSDWA);
    if constexpr (V == 8) MIXLOOP(MIX_NOMAX3);
    if constexpr (V == 9) MIXLOOP(MIX_PLAIN);
    if constexpr (V == 10) MIXLOOP(MIX_PLAIN64);
    if constexpr (V == 11) MIXLOOP2(MIX_R2FULL);
    if constexpr (V == 12) MIXLOOP2(MIX_R2VALU);
    if constexpr (V == 13) MIXLOOP3(MIX_R3FULL);
    if constexpr (V == 14) MIXLOOP3(MIX_R3VALU);
    if constexpr (V == 15) MIXLOOP(MIX_SPFULL);
    if constexpr (V == 16) MIXLOOP(MIX_DSFULL);
    if constexpr (V == 17) MIXLOOP(MIX_DS1FULL);
    if constexpr (V == 18) MIXLOOP(MIX_PK2);
    if constexpr (V == 19) MIXLOOP(MIX_PK3);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * blockDim.x + threadIdx.x] = g + fdn + dg + e + hg + bx + tfg + tff + (int)st + eb + hgb + ec + hgc;
    if (lane == 0) out[blockIdx.x * kMaxW + wave] = c1 - c0;
}

static const char* kNames[] = {"FULL", "VALU", "VALU+LDS", "VALU+SALU", "VALU+WAIT", "VALU+GLOB",
                               "NODPP", "NOSDWA", "NOMAX3", "PLAIN", "PLAIN64", "R2FULL", "R2VALU",
                               "R3FULL", "R3VALU", "SPFULL", "DSFULL", "DS1FULL", "PK2", "PK3"};
static const int kN[] = {MIX_FULL_N, MIX_VALU_N, MIX_VALU_LDS_N, MIX_VALU_SALU_N, MIX_VALU_WAIT_N, MIX_VALU_GLOB_N,
                         MIX_NODPP_N, MIX_NOSDWA_N, MIX_NOMAX3_N, MIX_PLAIN_N, MIX_PLAIN64_N, MIX_R2FULL_N,
                         MIX_R2VALU_N, MIX_R3FULL_N, MIX_R3VALU_N, MIX_SPFULL_N, MIX_DSFULL_N, MIX_DS1FULL_N, MIX_PK2_N,
                         MIX_PK3_N};

template <int V>
double run(int waves, int wgs, const uint8_t* codes, int nblocks) {
    unsigned long long* d_out;
    int* d_sink;
    (void)hipMalloc(&d_out, 8 * kMaxW * wgs);
    (void)hipMalloc(&d_sink, 4 * 64 * kMaxW * wgs);
    (void)hipFuncSetAttribute((const void*)mix<V>, hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(Sh));
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((mix<V>), dim3(wgs), dim3(64 * waves), sizeof(Sh), 0, nblocks, codes, d_out, d_sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(kMaxW * wgs);
    (void)hipMemcpy(h.data(), d_out, 8 * kMaxW * wgs, hipMemcpyDeviceToHost);
    std::vector<double> c;
    for (int g = 0; g < wgs; ++g)
        for (int w = 0; w < waves; ++w) c.push_back((double)h[g * kMaxW + w] / (nblocks * 32.0));
    std::sort(c.begin(), c.end());
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
    return c[c.size() / 2];
}

template <int V>
void all(const uint8_t* codes, int nblocks, int wgs = 256) {
    const double one = run<V>(4, wgs, codes, nblocks), two = run<V>(8, wgs, codes, nblocks);
    const double ipb = kN[V] / 64.0;   // instructions per step (two blocks of 32 steps)
    printf("%-10s WGs %3d %5.2f instr/step | 1 wave/SIMD: %6.2f cyc/step (%.2f per instr) | 2 waves/SIMD: %6.2f per "
           "wave, %6.2f per SIMD-step (%.2f per instr), pair gain %.2fx\n",
           kNames[V], wgs, ipb, one, one / ipb, two, two / 2, two / 2 / ipb, one / (two / 2));
}

int main() {
    const int nblocks = 4096;
    uint8_t* codes;
    (void)hipMalloc(&codes, (size_t)nblocks * 32 + 8192);
    (void)hipMemset(codes, 1, (size_t)nblocks * 32 + 8192);
    printf("%s\n", MIX_INC);
    // the steady-state path, and publishing by a per-step ds_write instead of the shift register
    all<15>(codes, nblocks);
    all<16>(codes, nblocks);
    all<17>(codes, nblocks);
    all<15>(codes, nblocks, 128);
    all<16>(codes, nblocks, 128);
    if (getenv("MIX_ONLY_DS")) return 0;
    // the packed 16-bit projection (two problems per register, 2 / 3 rows per lane: 256 /
    // 384 cells per wave step) against the product's three-row loop and its VALU subset
    all<18>(codes, nblocks);
    all<19>(codes, nblocks);
    all<13>(codes, nblocks);
    all<14>(codes, nblocks);
    if (getenv("MIX_ONLY_PK")) return 0;
    all<1>(codes, nblocks);
    all<2>(codes, nblocks);
    all<3>(codes, nblocks);
    all<4>(codes, nblocks);
    all<5>(codes, nblocks);
    all<0>(codes, nblocks);
    all<6>(codes, nblocks);
    all<7>(codes, nblocks);
    all<8>(codes, nblocks);
    all<9>(codes, nblocks);
    all<10>(codes, nblocks);
    // two rows per lane (128 cells per wave step: compare cycles per step / 2 with FULL)
    all<11>(codes, nblocks);
    all<12>(codes, nblocks);
    // three rows per lane (192 cells per wave step)
    all<13>(codes, nblocks);
    all<14>(codes, nblocks);
    // the instruction fetch: one busy CU against all of them
    for (int wgs : {1, 8, 64, 128}) {
        all<1>(codes, nblocks, wgs);
        all<9>(codes, nblocks, wgs);
        all<10>(codes, nblocks, wgs);
    }
    (void)hipFree(codes);
    return 0;
}
