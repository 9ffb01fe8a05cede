// Final-level (aff_predwalk_kernel) phase timing on synthetic diagonal blocks: the
// kernel with its sweep, walk or symbol output run twice, so each phase's cost is the
// difference to the plain launch.  Diagnostic tool, not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 -DANYSEQ_MICRO -DANYSEQ_PW_PHASES -I anyseq_amd/csrc tools/micro/pw_micro.hip -o tools/micro/bin/pw_micro
#include "../../anyseq_amd/csrc/anyseq_kernels.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace anyseq;

int main(int argc, char** argv) {
    const int nb = 512;
    std::mt19937 rng(7);
    const char A[4] = {'A', 'C', 'G', 'T'};
    for (int h : {64, 128, 192}) {
        const int n = nb * h, m = nb * 128;
        std::vector<uint8_t> q(n), s(m);
        for (auto& c : q) c = A[rng() & 3];
        for (int j = 0; j < m; ++j) s[j] = (rng() % 10 == 0) ? A[rng() & 3] : q[(int64_t)j * h / 128];
        std::vector<BlockInfo> bl(nb);
        for (int b = 0; b < nb; ++b) {
            BlockInfo bi{};
            bi.oi = b * h;
            bi.h = h;
            bi.oj = b * 128;
            bi.w = 128;
            bi.smode = BM_NORMAL;
            bi.e_end = 0;
            bi.flags = 0;
            bl[b] = bi;
        }
        uint8_t *dq, *ds, *dal, *das, *dpred;
        BlockInfo* dbl;
        (void)hipMalloc(&dq, n);
        (void)hipMalloc(&ds, m);
        (void)hipMalloc(&dal, n + m);
        (void)hipMalloc(&das, n + m);
        (void)hipMalloc(&dpred, 16);
        (void)hipMalloc(&dbl, nb * sizeof(BlockInfo));
        (void)hipMemcpy(dq, q.data(), n, hipMemcpyHostToDevice);
        (void)hipMemcpy(ds, s.data(), m, hipMemcpyHostToDevice);
        const int rows = 480;
        const int bytes = pred_lds_bytes(rows);
        (void)hipFuncSetAttribute((const void*)aff_predwalk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        float base = 0;
        for (int rep : {0, 1, 2, 4, 0}) {
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pw_rep), &rep, sizeof rep);
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                (void)hipMemcpy(dbl, bl.data(), nb * sizeof(BlockInfo), hipMemcpyHostToDevice);
                hipEvent_t e0, e1;
                (void)hipEventCreate(&e0);
                (void)hipEventCreate(&e1);
                (void)hipEventRecord(e0);
                hipLaunchKernelGGL(aff_predwalk_kernel, dim3(nb), dim3(128), bytes, 0, dbl, nb, dq, ds, dpred, 2, -1,
                                   -2, -1, dal, das, rows, nullptr, 0);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                best = std::min(best, ms);
            }
            if (rep == 0) base = best;
            printf("h %3d reps %d (sweep x%d walk x%d out x%d): %.1f us  (+%.1f)\n", h, rep, 1 + (rep & 1),
                   1 + ((rep >> 1) & 1), 1 + ((rep >> 2) & 1), best * 1e3, (best - base) * 1e3);
        }
        (void)hipFree(dq);
        (void)hipFree(ds);
        (void)hipFree(dal);
        (void)hipFree(das);
        (void)hipFree(dpred);
        (void)hipFree(dbl);
    }
    return 0;
}
