// Microbenchmark of the fill kernel's inner step (band_block) in isolation:
// cycles per step for one wave, with / without DPP and LDS operands.
#include "../../anyseq_amd/csrc/anyseq_kernels.hip"
#include <cstdio>
#include <vector>

using namespace anyseq;

template <int R, int MODE>
__global__ void micro(int nblocks, unsigned long long* out, int* sink) {
    constexpr int CH = 32;
    __shared__ int32_t ring[16 * CH];
    __shared__ uint8_t sr[kSRing + 64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 16 * CH; i += blockDim.x) ring[i] = i & 7;
    for (int i = threadIdx.x; i < kSRing + 64; i += blockDim.x) sr[i] = "ACGT"[(i * 7) & 3];
    __syncthreads();
    int qv[R]; bool dead[R]; int cur[R], prev[R];
    for (int k = 0; k < R; ++k) { qv[k] = "ACGT"[(lane + k) & 3]; dead[k] = false; cur[k] = 0; prev[k] = 0; }
    int dg = 0, upc = 0, best = 0, outv[CH];
    CellK ck{4, 1, 1};
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nblocks; ++b) {
        const int t0 = b * CH + 64;
        const int32_t* ring_blk = ring + (t0 & (16 * CH - 1));
        const uint8_t* s_blk[R];
        for (int k = 0; k < R; ++k) s_blk[k] = sr + ((t0 - 2 - (R + 1) * lane - k) & (kSRing - 1));
        if (MODE == 0) {
            band_block<KIND_GLOBAL, R, CH, false, false>(t0, lane, 1 << 30, ring[(t0 - 1) & 511], ring_blk, s_blk, qv,
                                                         dead, cur, prev, upc, dg, outv, best, ck);
        } else {
            // MODE 1: same arithmetic, no DPP and no LDS operands
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                int up = cur[R - 1] + 1, diag = dg; dg = up;
                const int sc = (t0 + u) & 3;
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int wgt = (qv[k] == sc) ? 4 : 1;
                    int v = max(max(diag + wgt, cur[k]), up);
                    diag = cur[k]; cur[k] = v; up = v;
                }
                outv[u] = cur[R - 1];
            }
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    int acc = best + dg;
    for (int k = 0; k < R; ++k) acc += cur[k];
    for (int u = 0; u < 32; ++u) acc += outv[u];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) { out[blockIdx.x * 2] = c1 - c0; out[blockIdx.x * 2 + 1] = r1 - r0; }
}

template <int R, int MODE>
void run(int waves, int blocks_per_grid) {
    const int nblocks = 2048;   // 65536 steps
    unsigned long long* d_out; int* d_sink;
    hipMalloc(&d_out, 16 * blocks_per_grid); hipMalloc(&d_sink, 4 * 64 * waves * blocks_per_grid);
    hipLaunchKernelGGL((micro<R, MODE>), dim3(blocks_per_grid), dim3(64 * waves), 0, 0, nblocks, d_out, d_sink);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((micro<R, MODE>), dim3(blocks_per_grid), dim3(64 * waves), 0, 0, nblocks, d_out, d_sink);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * blocks_per_grid);
    hipMemcpy(h.data(), d_out, 16 * blocks_per_grid, hipMemcpyDeviceToHost);
    const double steps = nblocks * 32.0;
    printf("R=%d mode=%d waves/WG=%d WGs=%d: %.2f cyc/step (memtime), %.2f ns/step (realtime), kernel %.3f ms, clk %.2f GHz\n",
           R, MODE, waves, blocks_per_grid, h[0] / steps, h[1] * 10.0 / steps, ms, (double)h[0] / (h[1] * 10.0));
    hipFree(d_out); hipFree(d_sink);
}

int main() {
    run<1, 0>(1, 1); run<1, 1>(1, 1);
    run<2, 0>(1, 1); run<2, 1>(1, 1);
    run<4, 0>(1, 1); run<4, 1>(1, 1);
    run<1, 0>(4, 1); run<1, 0>(8, 1);
    run<1, 0>(4, 256); run<2, 0>(4, 256); run<4, 0>(4, 256); run<1, 0>(8, 256);
    return 0;
}
