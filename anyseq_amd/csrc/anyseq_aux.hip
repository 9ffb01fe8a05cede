// anyseq_aux.hip — small device helpers of the affine construct's host-built levels.
//
// Inherited Hirschberg halves: a level's column vectors are moved
// between the capture arrays and the level's LH / LE / RH / RE, and a split half's
// second block has its outputs moved back from its own frame, by one launch of
// `i32_jobs_kernel` over a job table: dst[i] = src[i] + delta for i < n.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "anyseq_internal.h"

namespace anyseq {

__global__ __launch_bounds__(256) void i32_jobs_kernel(const I32Job* __restrict__ jobs, int njobs) {
    for (int j = blockIdx.y; j < njobs; j += gridDim.y) {
        const I32Job J = jobs[j];
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < J.n; i += blockDim.x * gridDim.x)
            J.dst[i] = J.src[i] + J.delta;
    }
}

}  // namespace anyseq

extern "C" hipError_t anyseq_launch_i32_jobs(const void* jobs, int njobs, int maxn, hipStream_t st) {
    if (njobs <= 0 || maxn <= 0) return hipSuccess;
    const dim3 grid(std::max(1, std::min(64, (maxn + 255) / 256)), std::min(njobs, 4096));
    hipLaunchKernelGGL(anyseq::i32_jobs_kernel, grid, dim3(256), 0, st, (const anyseq::I32Job*)jobs, njobs);
    return hipGetLastError();
}
