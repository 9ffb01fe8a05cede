// One-way hand-off latency between two workgroups (a flag ping-pong): same XCD (blocks b
// and b + 8) vs different XCDs, producer store flavour (plain / sc1) x consumer poll
// (sc1 / sc0 sc1).  Diagnostic tool for the fill's HBM hop, not part of
// the product.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/pingpong_micro.hip -o tools/micro/bin/pingpong_micro
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int ST, int LD>
__device__ __forceinline__ void st(uint32_t* p, uint32_t v) {
    if constexpr (ST == 0) asm volatile("global_store_dword %0, %1, off\n s_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
    if constexpr (ST == 1) asm volatile("global_store_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
    if constexpr (ST == 2) asm volatile("global_store_dword %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" ::"v"(p), "v"(v) : "memory");
}
template <int LD>
__device__ __forceinline__ uint32_t ld(const uint32_t* p) {
    uint32_t v;
    if constexpr (LD == 0) asm volatile("global_load_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    if constexpr (LD == 1) asm volatile("global_load_dword %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    if constexpr (LD == 2) asm volatile("global_load_dword %0, %1, off nt\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// pairs: (a, b) ping-pong `iters` times on flags f[2*pair], f[2*pair+1] (128 B apart)
template <int ST, int LD>
__global__ void pp(uint32_t* flags, const int* partner, int iters, unsigned long long* out, uint32_t* xcc) {
    if (threadIdx.x != 0) return;
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    xcc[blockIdx.x] = id & 0xf;
    const int me = blockIdx.x, other = partner[me];
    if (other < 0) return;
    const bool first = me < other;
    const int pair = first ? me : other;
    uint32_t* mine = flags + 64 * (2 * pair + (first ? 0 : 1));
    uint32_t* theirs = flags + 64 * (2 * pair + (first ? 1 : 0));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // every poll bounded: a form whose store never becomes visible ends after ~0.2 s (out = 0)
    const uint64_t limit = t0 + 20000000ull;
    bool ok = true;
    for (int i = 1; i <= iters && ok; ++i) {
        if (first) {
            st<ST, LD>(mine, (uint32_t)i);
            while (ld<LD>(theirs) != (uint32_t)i)
                if (__builtin_amdgcn_s_memrealtime() > limit) { ok = false; break; }
        } else {
            while (ld<LD>(theirs) != (uint32_t)i)
                if (__builtin_amdgcn_s_memrealtime() > limit) { ok = false; break; }
            st<ST, LD>(mine, (uint32_t)i);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[me] = ok ? t1 - t0 : 0;
}

template <int ST, int LD>
void run(const char* name, bool same) {
    const int nb = 16, iters = 2000;
    int hp[nb];
    for (int b = 0; b < nb; ++b) hp[b] = -1;
    if (same) { hp[0] = 8; hp[8] = 0; hp[3] = 11; hp[11] = 3; }
    else { hp[0] = 1; hp[1] = 0; hp[3] = 6; hp[6] = 3; }
    uint32_t* flags; int* partner; unsigned long long* out; uint32_t* xcc;
    (void)hipMalloc(&flags, 64 * 4 * 2 * nb);
    (void)hipMemset(flags, 0, 64 * 4 * 2 * nb);
    (void)hipMalloc(&partner, sizeof hp);
    (void)hipMemcpy(partner, hp, sizeof hp, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 8 * nb);
    (void)hipMalloc(&xcc, 4 * nb);
    hipLaunchKernelGGL((pp<ST, LD>), dim3(nb), dim3(64), 0, 0, flags, partner, iters, out, xcc);
    (void)hipDeviceSynchronize();
    unsigned long long h[nb]; uint32_t x[nb];
    (void)hipMemcpy(h, out, 8 * nb, hipMemcpyDeviceToHost);
    (void)hipMemcpy(x, xcc, 4 * nb, hipMemcpyDeviceToHost);
    const int a = same ? 0 : 0, b = same ? 8 : 1;
    printf("%-22s %-10s xcc %u/%u: one-way hop %.3f us (pair 2: %.3f us)\n", name, same ? "same-XCD" : "cross-XCD", x[a],
           x[b], h[a] / 100.0 / (2.0 * iters), h[3] / 100.0 / (2.0 * iters));
    (void)hipFree(flags); (void)hipFree(partner); (void)hipFree(out); (void)hipFree(xcc);
}

int main() {
    for (int s = 0; s < 2; ++s) {
        run<0, 0>("plain st / sc1 ld", s);
        run<1, 0>("sc1 st / sc1 ld", s);
        run<2, 0>("sc0sc1 st / sc1 ld", s);
        run<1, 1>("sc1 st / sc0sc1 ld", s);
        run<0, 2>("plain st / nt ld", s);
    }
    return 0;
}
