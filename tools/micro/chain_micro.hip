// Microbenchmark of the fill kernel's band chain without HBM hand-offs: NW compute
// waves of one workgroup run run_band() on NW consecutive bands, chained through
// the LDS rings exactly as in fill_kernel; the subject ring is pre-filled, so no
// I/O wave is needed.  Prints ns per 32-step block for the first and last wave.
#define ANYSEQ_MICRO
#include "../../anyseq_amd/csrc/anyseq_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace anyseq;

template <int NW>
__global__ __launch_bounds__(64 * NW) void chain(const uint8_t* q, int w, uint32_t* err, unsigned long long* out, int32_t* col, unsigned long long* dbg) {
    constexpr int CH = 32;
    __shared__ __attribute__((aligned(16))) FillShared<NW, CH> sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < kSRing + 64; i += blockDim.x) sh.s_ring[i] = "ACGT"[(i * 7 + (i >> 5)) & 3];
    if (threadIdx.x <= NW) { sh.prod[threadIdx.x] = 0; sh.cons[threadIdx.x] = 0; }
    if (threadIdx.x == 0) { sh.s_filled = 0x7fffffff; sh.tail = 0; }
    __syncthreads();
    DPProblem P;
    memset(&P, 0, sizeof P);
    P.q = q; P.s = nullptr; P.q_off = 0; P.q_step = 1; P.h = 64 * NW; P.w = w; P.nbands = NW; P.ngroups = 1;
    P.out_col = col + blockIdx.x * 64 * NW;   // keeps the DP live
    CellK ck;
    ck.ng = 1; ck.wm = 4; ck.wx = 1;
    WaveIO io;
    io.in_border = wave == 0;
    io.trailing = wave == NW - 1;
    io.my_ring = sh.in_ring[wave];
    io.my_prod = &sh.prod[wave];
    io.my_cons = &sh.cons[wave];
    io.s_ring = sh.s_ring;
    io.s_filled = &sh.s_filled;
    io.tail = &sh.tail;
    io.dummy = sh.dummy[wave];
    io.skew = &sh.skew[0][0][0];
    io.gout = nullptr;
    io.out_lds = wave < NW - 1;
    io.next_ring = sh.in_ring[wave + 1];
    io.next_prod = &sh.prod[wave + 1];
    io.next_cons = &sh.cons[wave + 1];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    run_band<KIND_GLOBAL, 1, 0, CH, false>(P, wave, lane, io, err, ck, dbg);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) { out[2 * (blockIdx.x * NW + wave)] = t0; out[2 * (blockIdx.x * NW + wave) + 1] = t1; }
}

template <int NW>
void run(int grid, int w) {
    uint8_t* q; uint32_t* err; unsigned long long* out;
    hipMalloc(&q, 64 * NW); hipMemset(q, 'A', 64 * NW);
    hipMalloc(&err, 4); hipMemset(err, 0, 4);
    hipMalloc(&out, 16 * grid * NW);
    int32_t* col; hipMalloc(&col, 4 * 64 * NW * grid);
    unsigned long long* dbg; hipMalloc(&dbg, 8 * 64); hipMemset(dbg, 0, 8 * 64);
    hipLaunchKernelGGL(chain<NW>, dim3(grid), dim3(64 * NW), 0, 0, q, w, err, out, col, nullptr);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain<NW>, dim3(grid), dim3(64 * NW), 0, 0, q, w, err, out, col, dbg);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * grid * NW);
    hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
    uint32_t e; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    const double nb = (w + 31) / 32 + 2;
    printf("NW=%d grid=%d w=%d: kernel %.3f ms | wave0 %.1f ns/block | last wave %.1f ns/block, start lag %.2f us/band | err %u\n",
           NW, grid, w, ms, (h[1] - h[0]) * 10.0 / nb, (h[2 * NW - 1] - h[2 * NW - 2]) * 10.0 / nb,
           (h[2 * NW - 2] - h[0]) / 100.0 / (NW > 1 ? NW - 1 : 1), e);
#ifdef ANYSEQ_STAMPS
    unsigned long long hd[16];
    hipMemcpy(hd, dbg, 128, hipMemcpyDeviceToHost);
    const double bands = hd[ST_BANDS] ? (double)hd[ST_BANDS] : 1.0, blocks = hd[ST_BLOCKS] ? (double)hd[ST_BLOCKS] : 1.0;
    printf("    stamps per block (cycles): total %.0f | acquire %.0f (wait_in %.0f wait_s %.0f) | compute %.0f | "
           "publish %.0f (wait_out %.0f)\n",
           hd[ST_TOTAL] / blocks, hd[ST_ACQ] / blocks, hd[ST_WAIT_IN] / blocks, hd[ST_WAIT_S] / blocks,
           hd[ST_COMPUTE] / blocks, hd[ST_PUB] / blocks, hd[ST_WAIT_OUT] / blocks);
    (void)bands;
#endif
    hipFree(q); hipFree(err); hipFree(out); hipFree(col); hipFree(dbg);
}

int main(int argc, char** argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 65536;
    run<1>(1, w); run<2>(1, w); run<4>(1, w); run<8>(1, w);
    run<4>(256, w); run<8>(256, w);
    return 0;
}
