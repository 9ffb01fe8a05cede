// anyseq_kernels.hip — hand-written CDNA4 (gfx950) kernels for the AnySeq hot path.
//
//  fill_kernel   the anti-diagonal DP fill (replaces iteration_acc.impala:16-172 +
//                scoring_acc.impala:1-145).  Lane-owns-rows wavefront: lane l of a
//                wave owns R consecutive rows of a 64*R-row band and processes column
//                c = t - l at step t; the up/diag dependency crosses lanes with one DPP
//                wave_shr:1 per step, the left dependency stays in VGPRs.  NW waves of
//                a workgroup run NW consecutive bands, chained through LDS rings; the
//                last band of a workgroup hands its bottom row to the next workgroup
//                through HBM (write-through sc1 stores + a progress flag).  Persistent
//                grid, work units dequeued in dependency order.
//  hb_sum_kernel column-split selection of traceback_lintime.impala:44-135 (CPU
//                BLOCK_WIDTH = 1024 candidate order).
//  pred_kernel   blockwise predecessor fill of the final 128-column blocks
//                (iteration_acc.impala:174-224, scoring_acc.impala:147-180,
//                mapping_acc.impala:133-153); anti-diagonal-major byte layout.
//  walk_kernel   per-block traceback walk (traceback.impala:47-80), i+j+1 layout.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "anyseq_internal.h"

namespace anyseq {

#define DPP_WAVE_SHL1 0x130
#define DPP_WAVE_SHR1 0x138

__device__ __forceinline__ int wave_shr1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, DPP_WAVE_SHR1, 0xf, 0xf, false);
}
__device__ __forceinline__ int wave_shl1(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, DPP_WAVE_SHL1, 0xf, 0xf, false);
}

// Spin limit: 10 s of s_memrealtime (100 MHz) — a bug never hangs the GPU.
#define SPIN_TICKS 1000000000ull

__device__ __forceinline__ bool err_set(uint32_t* err) {
    return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

__device__ __forceinline__ bool spin_lds_ge(uint32_t* p, uint32_t target, uint32_t* err) {
    if (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err)) {
            atomicOr(err, ERR_SPIN_TIMEOUT);
            return false;
        }
    }
    return true;
}

__device__ __forceinline__ bool spin_glb_ge(uint32_t* p, uint32_t target, uint32_t* err) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err)) {
            atomicOr(err, ERR_SPIN_TIMEOUT);
            return false;
        }
    }
    return true;
}

// ------------------------------------------------------------------ fill --
// Border values and value-space conversion per kind (ng = -gap > 0).
template <int KIND>
__device__ __forceinline__ int border_top(int c, int ng) {      // row -1, column c >= -1
    return KIND == KIND_SEMIGLOBAL ? (c + 1) * ng : 0;
}
template <int KIND>
__device__ __forceinline__ int border_left(int r, int ng) {     // column -1, row r >= -1
    return KIND == KIND_SEMIGLOBAL ? (r + 1) * ng : 0;
}
template <int KIND>
__device__ __forceinline__ int to_h(int v, int r, int c, int ng) {
    return KIND == KIND_LOCAL ? v : v - (r + c + 2) * ng;
}

constexpr int kSlots = 16;    // in-ring depth in chunks
constexpr int kSRing = 256;   // subject ring bytes per wave (+64 mirrored)

// LDS of one workgroup: NW compute waves + 1 I/O wave.  in_ring[w] feeds compute
// wave w (written by wave w-1, or by the I/O wave for w = 0); in_ring[NW] is the
// out-ring from the group's last compute wave to the I/O wave.
template <int NW, int CH>
struct FillShared {
    int32_t in_ring[NW + 1][kSlots * CH];
    uint8_t s_ring[NW][kSRing + 64];
    uint32_t prod[NW + 1];
    uint32_t cons[NW + 1];
    int32_t group;
};

// Cell constants: G kinds wm = match - 2 gap, wx = mismatch - 2 gap;
// local wm = match - gap, wx = mismatch - gap, and H = sat(x - ng).
struct CellK {
    int wm, wx, ng;
};

__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One step of the band wavefront: lane l processes column c = t - 1 - l.
// MASK: some lanes are outside [0, w) in this step.  PARTIAL: rows >= h (dead
// rows) pass the value from above through, so lane 63 always carries row h-1.
template <int KIND, int R, bool MASK, bool PARTIAL>
__device__ __forceinline__ void band_step(int t, int lane, int w, int topv, int sc, const int (&qv)[R],
                                          const bool (&dead)[R], int (&cur)[R], int& dg, int& outv, int& best,
                                          const CellK ck) {
    int up = wave_shr1(topv, cur[R - 1]);
    int diag = dg;
    dg = up;
    const bool act = MASK ? ((unsigned)(t - 1 - lane) < (unsigned)w) : true;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int wgt = (qv[k] == sc) ? ck.wm : ck.wx;
        int v = max(max(diag + wgt, cur[k]), up);
        if (KIND == KIND_LOCAL) v = (int)__builtin_elementwise_sub_sat((unsigned)v, (unsigned)ck.ng);
        if (PARTIAL && dead[k]) v = up;
        diag = cur[k];
        if (act) {
            cur[k] = v;
            if (KIND == KIND_LOCAL) best = max(best, v);
        }
        up = v;
    }
    outv = cur[R - 1];
}

struct WaveIO {
    bool in_border;            // band 0: inputs are the scheme's top border
    int32_t* my_ring;
    uint32_t* my_prod;
    uint32_t* my_cons;
    bool out_lds;              // publish the bottom row into next_ring
    int32_t* next_ring;
    uint32_t* next_prod;
    uint32_t* next_cons;
    uint8_t* s_ring;
};

template <int KIND, int R, int CH, bool MASK, bool PARTIAL>
__device__ __forceinline__ void band_block(int t0, int lane, int w, int top_first, const int32_t* ring_blk,
                                           const uint8_t* s_blk, const int (&qv)[R], const bool (&dead)[R],
                                           int (&cur)[R], int& dg, int (&outv)[CH], int& best, const CellK ck) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int topv = u == 0 ? top_first : ring_blk[u - 1];
        const int sc = s_blk[u];
        band_step<KIND, R, MASK, PARTIAL>(t0 + u, lane, w, topv, sc, qv, dead, cur, dg, outv[u], best, ck);
    }
}

template <int KIND, int R, int CH, bool PARTIAL>
__device__ void run_band(const DPProblem& P, int band, int lane, const WaveIO& io, uint32_t* err, const CellK ck) {
    constexpr int IRM = kSlots * CH - 1;
    constexpr int LAG = 64 / CH;      // blocks between computing and publishing a chunk
    const int h = P.h, w = P.w, ng = ck.ng;
    const int rb = band * 64 * R;
    const int row0 = rb + lane * R;

    int qv[R];
    bool dead[R];
    int cur[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int r = row0 + k;
        dead[k] = r >= h;
        qv[k] = dead[k] ? 0x100 : (int)P.q[P.q_off + P.q_step * r];
        cur[k] = border_left<KIND>(r, ng);
    }
    int dg = border_left<KIND>(row0 - 1, ng);
    int outv[CH];
    int best = 0;

    const int nchunks = (w + CH - 1) / CH;
    const int nblocks = nchunks + LAG;
    auto schar = [&](int c) -> uint8_t { return c < w ? P.s[P.s_off + P.s_step * c] : (uint8_t)0; };
    auto sput = [&](int c, uint8_t v) {
        const int p = c & (kSRing - 1);
        io.s_ring[p] = v;
        if (p < 64) io.s_ring[p + kSRing] = v;
    };
    // prologue: subject chars of block 0 into the ring, block 1 into registers
    if (lane < CH) sput(lane, schar(lane));
    uint8_t pf1 = lane < CH ? schar(CH + lane) : 0;

    for (int b = 0; b < nblocks; ++b) {
        const int t0 = b * CH;
        // ---- input chunk b (columns [t0, t0+CH))
        if (b < nchunks) {
            if (io.in_border) {
                if (lane < CH) io.my_ring[(t0 + lane) & IRM] = border_top<KIND>(t0 + lane, ng);
            } else {
                if (!spin_lds_ge(io.my_prod, (uint32_t)(b + 1), err)) return;
            }
        }
        const int top_first = b == 0 ? border_left<KIND>(rb - 1, ng) : io.my_ring[(t0 - 1) & IRM];
        // ---- prefetch subject chars of block b+2
        const uint8_t pf2 = lane < CH ? schar(t0 + 2 * CH + lane) : (uint8_t)0;

        const int32_t* ring_blk = io.my_ring + (t0 & IRM);
        const uint8_t* s_blk = io.s_ring + ((t0 - 1 - lane) & (kSRing - 1));
        const bool full = (t0 >= 64) && (t0 + CH <= w + 1);
        if (full)
            band_block<KIND, R, CH, false, PARTIAL>(t0, lane, w, top_first, ring_blk, s_blk, qv, dead, cur, dg, outv,
                                                    best, ck);
        else
            band_block<KIND, R, CH, true, PARTIAL>(t0, lane, w, top_first, ring_blk, s_blk, qv, dead, cur, dg, outv,
                                                   best, ck);

        // ---- release chunks < b (column t0+CH-1 of chunk b is still read by block b+1)
        if (!io.in_border) lds_st(io.my_cons, (uint32_t)b);
        // ---- subject chars of block b+1 into the ring
        if (lane < CH) sput(t0 + CH + lane, pf1);
        pf1 = pf2;

        // ---- publish bottom-row chunk j = b - LAG (lane 63 holds it in outv)
        const int j = b - LAG;
        if (io.out_lds && j >= 0) {
            if (!spin_lds_ge(io.next_cons, (uint32_t)max(0, j - kSlots + 1), err)) return;
            if (lane == 63) {
                int4* dst = reinterpret_cast<int4*>(io.next_ring + ((j * CH) & IRM));
#pragma unroll
                for (int q = 0; q < CH / 4; ++q)
                    dst[q] = make_int4(outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]);
            }
            lds_st(io.next_prod, (uint32_t)(j + 1));
        }
    }
    if (!io.in_border) lds_st(io.my_cons, (uint32_t)(nchunks + kSlots));

    // ---- last column (H space) and local maximum
    if (P.out_col) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int r = row0 + k;
            if (r < h) P.out_col[r] = to_h<KIND>(cur[k], r, w - 1, ng);
        }
    }
    if (KIND == KIND_LOCAL && P.best) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
        if (lane == 0) atomicMax(P.best, best);
    }
}

// The I/O wave: copies the previous group's bottom row (HBM, sc1 loads behind a
// relaxed progress flag) into compute wave 0's in-ring, and this group's bottom
// row from the out-ring to HBM (sc1 stores, vmcnt(0), then the flag) — the
// global hand-off latency never sits on a compute wave's critical path.
template <int CH>
__device__ void io_wave(int lane, int nchunks, const int32_t* g_in, uint32_t* g_in_flag, int32_t* ring0,
                        uint32_t* prod0, uint32_t* cons0, int32_t* g_out, uint32_t* g_out_flag, int32_t* oring,
                        uint32_t* oprod, uint32_t* ocons, uint32_t* err) {
    constexpr int IRM = kSlots * CH - 1;
    const bool need_in = g_in != nullptr, need_out = g_out != nullptr;
    int in_next = 0, out_next = 0;
    uint32_t avail = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    while ((need_in && in_next < nchunks) || (need_out && out_next < nchunks)) {
        bool progress = false;
        if (need_in && in_next < nchunks) {
            if ((int)avail <= in_next)
                avail = __hip_atomic_load(g_in_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int lim = min(min((int)avail, (int)lds_ld(cons0) + kSlots), nchunks);
            if (lim > in_next) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int col = in_next * CH + lane; col < lim * CH; col += 64)
                    ring0[col & IRM] = __hip_atomic_load(g_in + col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lds_st(prod0, (uint32_t)lim);
                in_next = lim;
                progress = true;
            }
        }
        if (need_out && out_next < nchunks) {
            const int p = min((int)lds_ld(oprod), nchunks);
            if (p > out_next) {
                for (int col = out_next * CH + lane; col < p * CH; col += 64)
                    __hip_atomic_store(g_out + col, oring[col & IRM], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lds_st(ocons, (uint32_t)p);
                if (g_out_flag) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0)
                        __hip_atomic_store(g_out_flag, (uint32_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                out_next = p;
                progress = true;
            }
        }
        if (!progress) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t_start > SPIN_TICKS || err_set(err)) {
                atomicOr(err, ERR_SPIN_TIMEOUT);
                lds_st(prod0, (uint32_t)nchunks);
                return;
            }
        }
    }
}

template <int KIND, int R, int NW, int CH>
__global__ __launch_bounds__(64 * (NW + 1)) void fill_kernel(const DPProblem* __restrict__ probs,
                                                              const GroupRef* __restrict__ groups, int ngroups_total,
                                                              uint32_t* dq, uint32_t* err, FillParams fp) {
    __shared__ __attribute__((aligned(16))) FillShared<NW, CH> sh;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    CellK ck;
    ck.ng = -fp.gap;
    if (KIND == KIND_LOCAL) {
        ck.wm = fp.match - fp.gap;
        ck.wx = fp.mismatch - fp.gap;
    } else {
        ck.wm = fp.match - 2 * fp.gap;
        ck.wx = fp.mismatch - 2 * fp.gap;
    }
    for (;;) {
        if (threadIdx.x == 0) sh.group = (int32_t)atomicAdd(dq, 1u);
        if (threadIdx.x <= NW) {
            sh.prod[threadIdx.x] = 0;
            sh.cons[threadIdx.x] = 0;
        }
        __syncthreads();
        const int gi = sh.group;
        if (gi >= ngroups_total || err_set(err)) break;
        const GroupRef g = groups[gi];
        const DPProblem P = probs[g.prob];
        const int first = g.group * NW;
        const int last = min(P.nbands, first + NW) - 1;   // last band of this group
        // where the group's bottom row goes: the next group, the problem's out_row, or nowhere
        int32_t* g_out = nullptr;
        uint32_t* g_out_flag = nullptr;
        if (last < P.nbands - 1) {
            g_out = P.rowbuf + (size_t)g.group * P.wpad;
            g_out_flag = P.flags + g.group;
        } else if (P.out_row) {
            g_out = P.out_row;
        }
        if (wave == NW) {
            const int nchunks = (P.w + CH - 1) / CH;
            const int32_t* g_in = g.group > 0 ? P.rowbuf + (size_t)(g.group - 1) * P.wpad : nullptr;
            uint32_t* g_in_flag = g.group > 0 ? P.flags + (g.group - 1) : nullptr;
            io_wave<CH>(lane, nchunks, g_in, g_in_flag, sh.in_ring[0], &sh.prod[0], &sh.cons[0], g_out, g_out_flag,
                        sh.in_ring[NW], &sh.prod[NW], &sh.cons[NW], err);
        } else {
            const int band = first + wave;
            if (band <= last) {
                WaveIO io;
                io.in_border = band == 0;
                io.my_ring = sh.in_ring[wave];
                io.my_prod = &sh.prod[wave];
                io.my_cons = &sh.cons[wave];
                io.s_ring = sh.s_ring[wave];
                if (band < last) {
                    io.out_lds = true;
                    io.next_ring = sh.in_ring[wave + 1];
                    io.next_prod = &sh.prod[wave + 1];
                    io.next_cons = &sh.cons[wave + 1];
                } else {
                    io.out_lds = g_out != nullptr;
                    io.next_ring = sh.in_ring[NW];
                    io.next_prod = &sh.prod[NW];
                    io.next_cons = &sh.cons[NW];
                }
                const bool partial = (band + 1) * 64 * R > P.h;
                if (partial)
                    run_band<KIND, R, CH, true>(P, band, lane, io, err, ck);
                else
                    run_band<KIND, R, CH, false>(P, band, lane, io, err, ck);
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ reductions --
// Semiglobal score (scoring.impala:39-77): max over the last row (raw G values,
// index -1 = border 0 first) and the last column (H values); writes the max.
__global__ void semiglobal_reduce_kernel(const int32_t* __restrict__ row_g, int m, const int32_t* __restrict__ col_h,
                                         int n, int ng, int32_t* out) {
    int best = 0;  // row[-1] / col[-1] border values are 0
    for (int j = threadIdx.x + blockIdx.x * blockDim.x; j < m; j += blockDim.x * gridDim.x)
        best = max(best, row_g[j] - (n - 1 + j + 2) * ng);
    for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < n; i += blockDim.x * gridDim.x)
        best = max(best, col_h[i]);
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
}

// ---------------------------------------------------------------- hb_sum --
// Stage 1: one thread per (part, stride class) — traceback_lintime.impala:56-96.
__global__ void hb_sum_stage1(const PartInfo* __restrict__ parts, int nparts, int bpp, int half,
                              const int32_t* __restrict__ L, const int32_t* __restrict__ Rc, int kind, int gap,
                              int32_t* bmax, int32_t* bind) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nparts * bpp) return;
    const int part = id / bpp, pb = id % bpp;
    const PartInfo pi = parts[part];
    const int po = pi.off, len = pi.len;
    auto init = [&](int i) { return kind == KIND_GLOBAL ? (i + 1) * gap : 0; };
    int mx = -2147483647, index = -1;
    if (pb == 0 && len > 0) {
        mx = init(half - 1) + Rc[po + len - 1];
        index = -1;
        const int last = L[po + len - 1] + init(pi.rhw - 1);
        if (last > mx) {
            mx = last;
            index = len - 1;
        }
    }
    for (int i = pb; i < len - 1; i += bpp) {
        const int val = L[po + i] + Rc[po + len - i - 2];
        if (val > mx) {
            mx = val;
            index = i;
        }
    }
    bmax[id] = mx;
    bind[id] = index;
}

// Stage 2: one thread per part — traceback_lintime.impala:101-126 (ascending class order).
// splits is the logical-(-1) vector: storage index = logical + 1.
__global__ void hb_sum_stage2(const PartInfo* __restrict__ parts, int nparts, int bpp,
                              const int32_t* __restrict__ bmax, const int32_t* __restrict__ bind, int32_t* splits) {
    const int part = blockIdx.x * blockDim.x + threadIdx.x;
    if (part >= nparts) return;
    const int bo = part * bpp;
    int mx = bmax[bo], index = bind[bo];
    for (int i = 1; i < bpp; ++i) {
        if (bmax[bo + i] > mx) {
            mx = bmax[bo + i];
            index = bind[bo + i];
        }
    }
    splits[parts[part].split_index + 1] = parts[part].off + index + 1;
}

// ------------------------------------------------------------------ preds --
// Final level: one wave per 128-column block; lane l owns columns 2l and 2l+1
// and sweeps anti-diagonals d (cell A = (d-2l, 2l), cell B = (d-2l-1, 2l+1)).
// Predecessors are stored anti-diagonal-major: pred[base + d*128 + j].
__device__ __forceinline__ int relax_pred(int kind, int ng_entry, int gq_entry, int gs_entry, int sub, int gap,
                                          int& pred) {
    int score = ng_entry + sub;
    int p = 3;  // PRED_NO_GAP
    const int qg = gq_entry + gap;
    if (qg > score) {
        score = qg;
        p = 1;  // PRED_GAP_Q
    }
    const int sg = gs_entry + gap;
    if (sg > score) {
        score = sg;
        p = 2;  // PRED_GAP_S
    }
    if (kind == KIND_LOCAL && 0 > score) {
        score = 0;
        p = 0;  // PRED_NONE
    }
    pred = p;
    return score;
}

__global__ __launch_bounds__(64) void pred_kernel(const BlockInfo* __restrict__ blocks, int nblocks,
                                                  const uint8_t* __restrict__ Q, const uint8_t* __restrict__ S,
                                                  uint8_t* __restrict__ pred, FillParams fp) {
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    const BlockInfo bi = blocks[b];
    if (bi.h <= 0) return;
    const int lane = threadIdx.x;
    const int kind = fp.kind, gap = fp.gap;
    auto init = [&](int i) { return kind == KIND_GLOBAL ? (i + 1) * gap : 0; };
    const int jA = 2 * lane, jB = 2 * lane + 1;
    const int sA = jA < bi.w ? (int)S[bi.oj + jA] : 0x100;
    const int sB = jB < bi.w ? (int)S[bi.oj + jB] : 0x100;
    int A = init(jA);            // H[iA-1][jA]: up for A (row -1 border before A starts)
    int Bv = init(jB);           // H[iB-1][jB]: up for B
    int leftA_prev = init(-1);   // diag for A (lane 0: border H[iA-1][-1])
    int A_old = init(jA);        // A one step earlier: diag for B
    uint16_t* out16 = reinterpret_cast<uint16_t*>(pred + bi.pred_base);
    const int nsteps = bi.h + 127;
    for (int d = 0; d < nsteps; ++d) {
        const int iA = d - jA, iB = d - jB;
        // lane 0 border for A: H[iA][-1] = init(iA); diag = init(iA-1)
        const int leftA = wave_shr1(init(iA), Bv);
        const int diagA = leftA_prev;
        leftA_prev = leftA;
        const bool actA = (iA >= 0) && (iA < bi.h) && (jA < bi.w);
        const bool actB = (iB >= 0) && (iB < bi.h) && (jB < bi.w);
        const int qA = (iA >= 0 && iA < bi.h) ? (int)Q[bi.oi + iA] : 0x200;
        const int qB = (iB >= 0 && iB < bi.h) ? (int)Q[bi.oi + iB] : 0x200;
        int pA = 0, pB = 0;
        const int subA = qA == sA ? fp.match : fp.mismatch;
        const int subB = qB == sB ? fp.match : fp.mismatch;
        // B uses A at (iB, jA) = current A (before update) as left, A_old as diag
        const int nB = relax_pred(kind, A_old, A, Bv, subB, gap, pB);
        const int nA = relax_pred(kind, diagA, leftA, A, subA, gap, pA);
        // A_old tracks A value at the row above the current row for B's diag next step
        if (actB) Bv = nB;
        A_old = A;
        if (actA) A = nA;
        const uint16_t pk = (uint16_t)((actA ? pA : 0) | ((actB ? pB : 0) << 8));
        out16[(size_t)d * 64 + lane] = pk;
    }
}

// ------------------------------------------------------------------- walk --
// One thread per block: traceback_offset (traceback.impala:47-80) from (h-1, w-1).
__global__ void walk_kernel(const BlockInfo* __restrict__ blocks, int nblocks, const uint8_t* __restrict__ Q,
                            const uint8_t* __restrict__ S, const uint8_t* __restrict__ pred, int kind,
                            uint8_t* alq, uint8_t* als) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    const BlockInfo bi = blocks[b];
    auto P = [&](int i, int j) -> int {
        if (i < 0 || j < 0) {
            if (kind != KIND_GLOBAL || (i < 0 && j < 0)) return 0;
            return i < 0 ? 1 : 2;  // row -1: GAP_Q; column -1: GAP_S
        }
        return pred[bi.pred_base + (int64_t)(i + j) * 128 + j];
    };
    int i = bi.h - 1, j = bi.w - 1;
    int p = P(i, j);
    const int64_t base = (int64_t)bi.oi + bi.oj;
    while (p != 0) {
        uint8_t sq = '_', ss = '_';
        const int pos = i + j + 1;
        if (p == 3 || p == 2) {
            sq = Q[bi.oi + i];
            --i;
        }
        if (p == 3 || p == 1) {
            ss = S[bi.oj + j];
            --j;
        }
        alq[base + pos] = sq;
        als[base + pos] = ss;
        p = P(i, j);
    }
}

// --------------------------------------------------------------- launchers --
template <int KIND, int R, int NW, int CH>
static hipError_t launch_fill_t(const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    hipLaunchKernelGGL((fill_kernel<KIND, R, NW, CH>), dim3(grid), dim3(64 * (NW + 1)), 0, st, probs, groups,
                       ngroups, dq, err, fp);
    return hipGetLastError();
}

template <int R, int NW, int CH>
static hipError_t launch_fill_r(const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    switch (fp.kind) {
        case KIND_GLOBAL:
            return launch_fill_t<KIND_GLOBAL, R, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        case KIND_SEMIGLOBAL:
            return launch_fill_t<KIND_SEMIGLOBAL, R, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        default:
            return launch_fill_t<KIND_LOCAL, R, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
    }
}

}  // namespace anyseq

extern "C" {

// Fill launcher: R rows per lane in {1,2,4}; NW compute waves per workgroup in {4,8}; CH = 32.
hipError_t anyseq_launch_fill(int R, int NW, const anyseq::DPProblem* probs, const anyseq::GroupRef* groups,
                              int ngroups, uint32_t* dq, uint32_t* err, const anyseq::FillParams* fp, int grid,
                              hipStream_t st) {
    using namespace anyseq;
    if (NW == 4) {
        switch (R) {
            case 1: return launch_fill_r<1, 4, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
            case 2: return launch_fill_r<2, 4, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
            default: return launch_fill_r<4, 4, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
        }
    }
    switch (R) {
        case 1: return launch_fill_r<1, 8, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
        case 2: return launch_fill_r<2, 8, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
        default: return launch_fill_r<4, 8, 32>(probs, groups, ngroups, dq, err, *fp, grid, st);
    }
}

hipError_t anyseq_launch_semiglobal_reduce(const int32_t* row_g, int m, const int32_t* col_h, int n, int ng,
                                           int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(anyseq::semiglobal_reduce_kernel, dim3(64), dim3(256), 0, st, row_g, m, col_h, n, ng, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_hb_sum(const void* parts, int nparts, int bpp, int half, const int32_t* L, const int32_t* R,
                                int kind, int gap, int32_t* bmax, int32_t* bind, int32_t* splits, hipStream_t st) {
    using namespace anyseq;
    const int n1 = nparts * bpp;
    if (n1 > 0) {
        hipLaunchKernelGGL(hb_sum_stage1, dim3((n1 + 255) / 256), dim3(256), 0, st, (const PartInfo*)parts, nparts,
                           bpp, half, L, R, kind, gap, bmax, bind);
        hipLaunchKernelGGL(hb_sum_stage2, dim3((nparts + 255) / 256), dim3(256), 0, st, (const PartInfo*)parts,
                           nparts, bpp, bmax, bind, splits);
    }
    return hipGetLastError();
}

hipError_t anyseq_launch_pred(const void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S, uint8_t* pred,
                              const anyseq::FillParams* fp, hipStream_t st) {
    if (nblocks > 0)
        hipLaunchKernelGGL(anyseq::pred_kernel, dim3(nblocks), dim3(64), 0, st, (const anyseq::BlockInfo*)blocks,
                           nblocks, Q, S, pred, *fp);
    return hipGetLastError();
}

hipError_t anyseq_launch_walk(const void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S,
                              const uint8_t* pred, int kind, uint8_t* alq, uint8_t* als, hipStream_t st) {
    if (nblocks > 0)
        hipLaunchKernelGGL(anyseq::walk_kernel, dim3((nblocks + 63) / 64), dim3(64), 0, st,
                           (const anyseq::BlockInfo*)blocks, nblocks, Q, S, pred, kind, alq, als);
    return hipGetLastError();
}

}  // extern "C"
