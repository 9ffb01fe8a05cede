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

#include <algorithm>
#include <type_traits>

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

// Waits until *p >= target; returns the observed value (wave-uniform), or 0 on timeout/error.
__device__ __forceinline__ uint32_t spin_lds_ge(uint32_t* p, uint32_t target, uint32_t* err) {
    uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v >= target) {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        return v;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t it = 0;
    while ((v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) < target) {
        __builtin_amdgcn_s_sleep(1);
        // the error word lives in HBM: look at it (and the clock) only every 256 polls
        if ((++it & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
            atomicOr(err, ERR_SPIN_TIMEOUT);
            return 0;
        }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}

__device__ __forceinline__ bool spin_glb_ge(uint32_t* p, uint32_t target, uint32_t* err) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t it = 0;
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
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


constexpr int kSlots = 16;     // in-ring depth in chunks
constexpr int kSRing = 4096;   // shared subject ring bytes per workgroup (+64 mirrored)
constexpr int kSkewBlocks = 32;   // pre-skewed subject blocks held per workgroup (R = 1, X = 0, CH = 32)
constexpr int kMaxBack = 5 * 64 + 32;   // deepest look-back of a reader: D = 64(R+1) for R <= 4, + 1 chunk

// LDS of one workgroup: NW compute waves + 1 I/O wave.  in_ring[w] feeds compute
// wave w (written by wave w-1, or by the I/O wave for w = 0); in_ring[NW] is the
// out-ring from the group's last compute wave to the I/O wave.  s_ring holds the
// subject bytes of the group's columns, staged by the I/O wave ahead of wave 0
// and recycled behind the trailing wave.
template <int NW, int CH>
struct FillShared {
    int32_t in_ring[NW + 1][kSlots * CH];
    uint8_t s_ring[kSRing + 64];
    uint32_t prod[NW + 1];
    uint32_t cons[NW + 1];
    int32_t dummy[NW][64];   // per-wave sink of the block asm's non-publishing lanes
    // Pre-skewed subject (R = 1, X = 0, CH = 32 only): skew[b % kSkewBlocks][i][l] =
    // the 4 subject bytes lane l needs at steps 32b + 4i .. 32b + 4i + 3, i.e.
    // s[32b + 4i - 1 - l ..] -- one conflict-free ds_read_b32 per dword, no realignment.
    uint32_t skew[kSkewBlocks][8][64];
    uint32_t s_filled;   // subject chunks staged
    uint32_t tail;       // blocks completed by the trailing compute wave
    int32_t group;
};

// Cell constants: G kinds wm = match - 2 gap, wx = mismatch - 2 gap;
// local wm = match - gap, wx = mismatch - gap, and H = sat(x - ng).
struct CellK {
    int wm, wx, ng;
    int thr;   // FillParams::throttle
};

// LDS progress counters between waves of one workgroup.  The LDS executes one
// wave's DS instructions in issue order, so a counter store issued after the
// data stores is observed after them, and a data load issued after the counter
// load returned reads the published data: relaxed DS accesses plus compiler
// fences suffice.
__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
    uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Global-memory views (address space 1): global_load/global_store count only
// vmcnt, never lgkmcnt.
#define GLOBAL_AS __attribute__((address_space(1)))
#define LDS_AS __attribute__((address_space(3)))
template <typename T>
__device__ __forceinline__ GLOBAL_AS T* gmem(T* p) {
    return (GLOBAL_AS T*)p;
}

// Diagnostic stamps (separate build with -DANYSEQ_STAMPS; never in the product build):
// per-launch sums of wave cycles spent in compute blocks and in each kind of wait.
#ifdef ANYSEQ_STAMPS
#define STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, v) acc[slot] += (v)
#else
#define STAMP(var)
#define STAMP_ADD(slot, v)
#endif
enum { ST_TOTAL = 0, ST_COMPUTE, ST_WAIT_IN, ST_WAIT_S, ST_WAIT_OUT, ST_BANDS, ST_BLOCKS, ST_IO_TOTAL, ST_ACQ, ST_PUB, ST_POLL_S, ST_POLL_IN, ST_POLL_OUT, ST_NSLOTS };

// Band geometry.  Lane l owns rows r_k = rb + R*l + k (k < R) and at step t
// row k processes column
//     c_k(t) = t - BASE - S*l - k,   S = R + X,  BASE = 1 + X.
// Consequences (derived in DESIGN.md §3.1):
//  * rows k >= 1 read up = cur[k-1] and diag = prev[k-1] of their own lane, so
//    the R cells of a step are independent (ILP = R);
//  * row 0 reads lane l-1's row R-1 at the same column, produced 1 + X steps
//    earlier and moved by one DPP wave_shr:1 (X = 1 issues it one step ahead,
//    off the critical path, at the price of a 2-step lane skew);
//  * lane 63's row R-1 produces column t - D, D = 64 (R + X), so bottom-row
//    chunks stay CH-aligned.
template <int R, int X>
struct BandGeom {
    static constexpr int S = R + X;             // lane skew (steps)
    static constexpr int BASE = 1 + X;          // lane 0 / row 0 processes column t - BASE
    static constexpr int D = 64 * R + 64 * X;   // lane 63 / row R-1 processes column t - D
};

// One step.  MASK: some rows are outside [0, w) in this step.  PARTIAL: rows
// >= h pass the value from above through (so lane 63 carries row h-1).
template <int KIND, int R, int X, bool MASK, bool PARTIAL, bool VIRT = false>
__device__ __forceinline__ void band_step(int t, int lane, int w, int topv, const int (&sc)[R], const int (&qv)[R],
                                          const bool (&dead)[R], int (&cur)[R], int (&prev)[R], int& upc, int& dg,
                                          int& outv, int& best, const CellK ck) {
    constexpr int S = BandGeom<R, X>::S;
    constexpr int BASE = BandGeom<R, X>::BASE;
    // X = 1: DPP for the NEXT step (lane l-1's row R-1 at its start-of-step value);
    // X = 0: DPP for this step.
    const int up_dpp = wave_shr1(topv, cur[R - 1]);
    if (X == 0) upc = up_dpp;
    int nv[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int up = k == 0 ? upc : cur[k - 1];
        const int diag = k == 0 ? dg : prev[k - 1];
        const int wgt = (qv[k] == sc[k]) ? ck.wm : ck.wx;
        int v = max(max(diag + wgt, cur[k]), up);
        if (KIND == KIND_LOCAL) v = (int)__builtin_elementwise_sub_sat((unsigned)v, (unsigned)ck.ng);
        if (PARTIAL && dead[k]) v = up;
        nv[k] = v;
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        prev[k] = cur[k];
        // VIRT: columns < 0 are virtual (see run_band) and computed like real ones
        const bool act = MASK ? (VIRT ? (t - BASE - S * lane - k < w) : ((unsigned)(t - BASE - S * lane - k) < (unsigned)w))
                              : true;
        if (act) {
            cur[k] = nv[k];
            if (KIND == KIND_LOCAL) best = max(best, nv[k]);
        }
    }
    dg = upc;
    if (X == 1) upc = up_dpp;
    outv = cur[R - 1];
}

struct WaveIO {
    bool in_border;            // band 0: inputs are the scheme's top border
    bool trailing;             // last compute wave of the group: reports `tail`
    int32_t* my_ring;
    uint32_t* my_prod;
    uint32_t* my_cons;
    bool out_lds;              // publish the bottom row into next_ring
    int32_t* next_ring;
    uint32_t* next_prod;
    uint32_t* next_cons;
    const uint8_t* s_ring;
    uint32_t* s_filled;
    uint32_t* tail;
    int32_t* dummy;            // 64 ints of this wave's scratch
    const uint32_t* skew;      // pre-skewed subject blocks (FillShared::skew)
    int32_t* gout;             // last band of a group: global destination of the bottom row (or null)
};

// CH steps t0 .. t0+CH-1 from registers: top_first = top row at column t0-1,
// rv[u] = top row at column t0+u (only u < CH-1 is used here; rv[CH-1] becomes
// the next block's top_first), sw[k][u/4] = subject bytes of row k, 4 per dword.
template <int KIND, int R, int X, int CH, bool MASK, bool PARTIAL, bool VIRT = false>
__device__ __forceinline__ void band_block(int t0, int lane, int w, int top_first, const int (&rv)[CH],
                                           const uint32_t (&sw)[R][CH / 4], const int (&qv)[R],
                                           const bool (&dead)[R], int (&cur)[R], int (&prev)[R], int& upc, int& dg,
                                           int (&outv)[CH], int& best, const CellK ck) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        const int topv = u == 0 ? top_first : rv[u - 1];
        int sc[R];
#pragma unroll
        for (int k = 0; k < R; ++k) sc[k] = (int)((sw[k][u >> 2] >> (8 * (u & 3))) & 0xffu);
        band_step<KIND, R, X, MASK, PARTIAL, VIRT>(t0 + u, lane, w, topv, sc, qv, dead, cur, prev, upc, dg, outv[u],
                                                   best, ck);
    }
}

#ifdef ANYSEQ_ASM_INC   // (experimental builds: another generated loop, Makefile `lean`)
#include ANYSEQ_ASM_INC
#else
#include "anyseq_block_asm.inc"
#endif

// A full 32-step block (all 64 lanes inside [0, w) or on virtual columns, no dead
// rows) as ONE asm statement (tools/gen_block_asm.py): ra = LDS byte address of
// the block's 32 top-row values, tf = top row at column t0 - 1 (on return: the
// block's last top-row value, the next tf); lane 63 stores the block's 32 bottom
// cells through a DPP shift register: one ds_write_b32 at the per-lane LDS byte
// address pa (lanes 32..63: the 32 consecutive slots of the chunk; lanes 0..31 and
// non-publishing blocks: the wave's dummy area).
template <int KIND>
__device__ __forceinline__ void band_block_asm(int& tf, uint32_t ra, uint32_t pa, uint64_t pm,
                                               const uint32_t (&sw)[8], int q, int& cur, int& dg, int& best,
                                               const CellK& ck) {
    uint64_t sv;
    if constexpr (KIND == KIND_LOCAL) {
        asm volatile(ANYSEQ_BLOCK_ASM_L
                     : [cur] "+v"(cur), [dg] "+v"(dg), [tf] "+v"(tf), [best] "+v"(best), [sv] "=&s"(sv)
                     : [ra] "v"(ra), [pa] "v"(pa), [pm] "s"(pm), [s0] "v"(sw[0]), [s1] "v"(sw[1]), [s2] "v"(sw[2]),
                       [s3] "v"(sw[3]), [s4] "v"(sw[4]), [s5] "v"(sw[5]), [s6] "v"(sw[6]), [s7] "v"(sw[7]),
                       [q] "v"(q), [wm] "v"(ck.wm), [wx] "v"(ck.wx), [ng] "v"(ck.ng)
                     : ANYSEQ_BLOCK_ASM_CLOBBERS, "memory");
    } else {
        asm volatile(ANYSEQ_BLOCK_ASM_G
                     : [cur] "+v"(cur), [dg] "+v"(dg), [tf] "+v"(tf), [sv] "=&s"(sv)
                     : [ra] "v"(ra), [pa] "v"(pa), [pm] "s"(pm), [s0] "v"(sw[0]), [s1] "v"(sw[1]), [s2] "v"(sw[2]),
                       [s3] "v"(sw[3]), [s4] "v"(sw[4]), [s5] "v"(sw[5]), [s6] "v"(sw[6]), [s7] "v"(sw[7]),
                       [q] "v"(q), [wm] "v"(ck.wm), [wx] "v"(ck.wx)
                     : ANYSEQ_BLOCK_ASM_CLOBBERS, "memory");
    }
}

// Addresses and flags of one band's steady-state loop (ANYSEQ_LOOP_ASM_*).
struct LoopArgs {
    uint32_t rb, nb;                        // LDS byte address of my in-ring / the next ring
    uint32_t apr, acn, anp, anc, asf, atl;  // LDS byte addresses: my prod/cons, next prod/cons, s_filled, tail
    uint32_t skb;                           // skew base + 4*lane
    uint32_t lo;                            // 4*(lane-32) (publishing lanes 32..63)
    uint32_t lid4;                          // 4*lane
    uint32_t bvb;                           // border value of column `lane` (band 0)
    uint32_t bvs;                           // border value step per column (band 0)
    uint32_t fl;                            // bit0 in_border, bit1 trailing, bit2 publishes (LDS), bit3 (global)
    uint64_t gp;                            // global bottom-row destination (bit 3)
};

// Blocks b .. be-1 of a band (all full) in one asm statement (tools/gen_block_asm.py,
// gen_loop2), specialised by the band's role: BORDER (band 0 writes the top border)
// and PUB (0: no bottom row, 1: LDS ring of the next band, 2: HBM row of the next
// group / out_row).  Returns 0, or 1 on a spin timeout; b is advanced to be.
#ifdef ANYSEQ_STAMPS   // diagnostic build: also block 0's ready time and poll counts
#define AQ_NAME(K, B, P) ANYSEQ_LOOP2_##K##_##B##_##P##_TS
#define AQ_TS_OUT , [ts] "+s"(tsv), [nsf] "+s"(npoll[0]), [npr] "+s"(npoll[1]), [nbp] "+s"(npoll[2])
#else
#define AQ_NAME(K, B, P) ANYSEQ_LOOP2_##K##_##B##_##P
#define AQ_TS_OUT
#endif
#define AQ_ASM_G(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(cur), [dg] "+v"(dg), [tf] "+v"(tf), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf),     \
                   [sc] "+s"(sc), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4) AQ_TS_OUT                                                                    \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(ck.wm), [wx] "v"(ck.wx), [rb] "s"(rb), [nb] "s"(nb),       \
                   [apr] "v"(la.apr), [acn] "v"(la.acn), [anp] "v"(la.anp), [anc] "v"(la.anc), [asf] "v"(la.asf), \
                   [atl] "v"(la.atl), [skb] "v"(la.skb), [lo] "v"(la.lo), [lid4] "v"(la.lid4), [bvb] "v"(la.bvb), \
                   [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [thr] "s"(thr)                                   \
                 : ANYSEQ_LOOP2_ASM_CLOBBERS, "memory")
#define AQ_ASM_L(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(cur), [dg] "+v"(dg), [tf] "+v"(tf), [best] "+v"(best), [b] "+s"(b), [sp] "+s"(sp), \
                   [sf] "+s"(sf), [sc] "+s"(sc), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), \
                   [x3] "=&s"(x3), [x4] "=&s"(x4) AQ_TS_OUT                                                    \
                 : [be] "s"(be), [q] "v"(q), [wm] "v"(ck.wm), [wx] "v"(ck.wx), [ng] "v"(ck.ng), [rb] "s"(rb),   \
                   [nb] "s"(nb), [apr] "v"(la.apr), [acn] "v"(la.acn), [anp] "v"(la.anp), [anc] "v"(la.anc),     \
                   [asf] "v"(la.asf), [atl] "v"(la.atl), [skb] "v"(la.skb), [lo] "v"(la.lo), [lid4] "v"(la.lid4), \
                   [bvb] "v"(la.bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [thr] "s"(thr)                \
                 : ANYSEQ_LOOP2_ASM_CLOBBERS, "memory")
template <int KIND, bool BORDER, int PUB>
__device__ __forceinline__ uint32_t band_loop_asm(uint32_t& b, uint32_t be, uint32_t& sp, uint32_t& sf, uint32_t& sc,
                                                  const LoopArgs& la, int q, int& cur, int& dg, int& tf, int& best,
                                                  const CellK& ck, uint64_t& tsv, uint32_t (&npoll)[3]) {
    uint32_t st, x0, x1, x2, x3, x4;
    const uint64_t hm = 0xffffffff00000000ull;
    // "s" operands must be provably uniform SGPR values
#define RFL(x) __builtin_amdgcn_readfirstlane(x)
    b = RFL(b);
    sp = RFL(sp);
    sf = RFL(sf);
    sc = RFL(sc);
    be = RFL(be);
    const uint32_t rb = RFL(la.rb), nb = RFL(la.nb), bvs = RFL(la.bvs), thr = RFL((uint32_t)ck.thr);
    // (readfirstlane returns int: widen through uint32_t, or bit 31 sign-extends into the high half)
    const uint64_t gp = ((uint64_t)(uint32_t)RFL((uint32_t)(la.gp >> 32)) << 32) | (uint32_t)RFL((uint32_t)la.gp);
#undef RFL
    if constexpr (KIND == KIND_LOCAL) {
        if constexpr (BORDER && PUB == 0) AQ_ASM_L(AQ_NAME(L, B1, NONE));
        if constexpr (BORDER && PUB == 1) AQ_ASM_L(AQ_NAME(L, B1, LDS));
        if constexpr (BORDER && PUB == 2) AQ_ASM_L(AQ_NAME(L, B1, GLOB));
        if constexpr (!BORDER && PUB == 0) AQ_ASM_L(AQ_NAME(L, B0, NONE));
        if constexpr (!BORDER && PUB == 1) AQ_ASM_L(AQ_NAME(L, B0, LDS));
        if constexpr (!BORDER && PUB == 2) AQ_ASM_L(AQ_NAME(L, B0, GLOB));
    } else {
        if constexpr (BORDER && PUB == 0) AQ_ASM_G(AQ_NAME(G, B1, NONE));
        if constexpr (BORDER && PUB == 1) AQ_ASM_G(AQ_NAME(G, B1, LDS));
        if constexpr (BORDER && PUB == 2) AQ_ASM_G(AQ_NAME(G, B1, GLOB));
        if constexpr (!BORDER && PUB == 0) AQ_ASM_G(AQ_NAME(G, B0, NONE));
        if constexpr (!BORDER && PUB == 1) AQ_ASM_G(AQ_NAME(G, B0, LDS));
        if constexpr (!BORDER && PUB == 2) AQ_ASM_G(AQ_NAME(G, B0, GLOB));
    }
    return st;
}

template <typename T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(size_t)(LDS_AS T*)p;
}

// 32 subject bytes starting at ring position p (any alignment) -> 8 dwords:
// 9 aligned ds_read_b32 + 8 v_alignbit (unaligned b64/b128 LDS reads replay).
template <int CH>
__device__ __forceinline__ void load_sbytes(const uint8_t* s_ring, int p, uint32_t (&out)[CH / 4]) {
    const int pa = p & ~3;
    const uint32_t sh = (uint32_t)(p & 3) * 8u;
    const uint32_t* base = reinterpret_cast<const uint32_t*>(s_ring + pa);
    uint32_t d[CH / 4 + 1];
#pragma unroll
    for (int i = 0; i <= CH / 4; ++i) d[i] = base[i];
#pragma unroll
    for (int i = 0; i < CH / 4; ++i) out[i] = __builtin_amdgcn_alignbit(d[i + 1], d[i], sh);
}

// Column-block sharding: wait until the transported left column holds every row
// this band reads (rows rb-1 .. min(rb+span-1, h-1), rb = lane 0's row): the chunk
// flag of the band's last row (flags are set in chunk order, DPProblem::left_flag).
// Without flags (local direct mode) the kernel-written words themselves are polled
// against the sentinel.  Returns false on timeout.
__device__ __forceinline__ bool wait_left(const DPProblem& P, int row, uint32_t* err, int span = 64) {
    if (!P.left_flag) return true;
    const int rb = __builtin_amdgcn_readfirstlane(row);
    const int last = min(rb + span - 1, P.h - 1);
    if (last < 0) return true;
    uint32_t* f = const_cast<uint32_t*>(P.left_flag) + last / P.left_chunk;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t it = 0;
    while (__hip_atomic_load(gmem(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        __builtin_amdgcn_s_sleep(4);
        if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
            atomicOr(err, ERR_SPIN_TIMEOUT | 2u);
            return false;
        }
    }
    return true;
}

// This lane's left-border values H[row][-1] and H[row-1][-1] from the problem's
// left_in buffer (row -1 is the corner, whose value is the scheme's border in
// every shard frame).  Returns false on timeout.
__device__ __forceinline__ bool poll_left(const DPProblem& P, int row, int32_t& v1, int32_t& v0, uint32_t* err,
                                          int span = 64) {
    if (!wait_left(P, row, err, span)) return false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t it = 0;
    for (;;) {
        const bool has1 = row < P.h, has0 = row >= 1 && row - 1 < P.h;
        v1 = has1 ? __hip_atomic_load(gmem(P.left_in) + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        v0 = has0 ? __hip_atomic_load(gmem(P.left_in) + row - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        if (P.left_flag || __ballot((has1 && v1 == kShardSentinel) || (has0 && v0 == kShardSentinel)) == 0) break;
        __builtin_amdgcn_s_sleep(4);
        if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
            atomicOr(err, ERR_SPIN_TIMEOUT | 2u);
            return false;
        }
    }
    v1 += P.left_shift;
    v0 += P.left_shift;
    return true;
}

// Affine shard: this lane's E[row][-1] from left_in_e (after poll_left: with flags
// the chunk has landed; without, the words are sentinel-polled like poll_left).
__device__ __forceinline__ bool poll_left_e(const DPProblem& P, int row, int32_t& e1, uint32_t* err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t it = 0;
    for (;;) {
        const bool has1 = row < P.h;
        e1 = has1 ? __hip_atomic_load(gmem(P.left_in_e) + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        if (P.left_flag || __ballot(has1 && e1 == kShardSentinel) == 0) break;
        __builtin_amdgcn_s_sleep(4);
        if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
            atomicOr(err, ERR_SPIN_TIMEOUT | 2u);
            return false;
        }
    }
    e1 += P.left_shift;
    return true;
}

// After a band has stored its out_col rows: publish "band + 1 bands complete" in
// band order (waits for the band above to publish first), system scope, so the
// transport stream's hipStreamWaitValue32 and the kernel that sends the rows see
// the data.  Returns false on timeout.
// (units: 64-row bands; a band of `units` x 64 rows publishes that many at once)
__device__ __forceinline__ bool publish_progress(const DPProblem& P, int band, int lane, uint32_t* err,
                                                 int units = 1) {
    __threadfence_system();
    bool ok = true;
    band *= units;
    if (lane == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t it = 0;
        while (__hip_atomic_load(P.progress, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != (uint32_t)band) {
            __builtin_amdgcn_s_sleep(2);
            if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
                atomicOr(err, ERR_SPIN_TIMEOUT | 4u);
                ok = false;
                break;
            }
        }
        if (ok) __hip_atomic_store(P.progress, (uint32_t)(band + units), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return __shfl(ok ? 1 : 0, 0) != 0;
}

template <int KIND, int R, int X, int CH, bool PARTIAL>
__device__ void run_band(const DPProblem& P, int band, int lane, const WaveIO& io, uint32_t* err, const CellK ck,
                         unsigned long long* dbg) {
#ifdef ANYSEQ_STAMPS
    uint64_t acc[ST_NSLOTS] = {0};
    STAMP(t_begin);
#endif
    constexpr int IRM = kSlots * CH - 1;
    constexpr int S = BandGeom<R, X>::S;
    constexpr int BASE = BandGeom<R, X>::BASE;
    constexpr int D = BandGeom<R, X>::D;
    constexpr int LAG = D / CH;      // blocks between computing and publishing a chunk
    static_assert(D % CH == 0, "bottom-row chunks must stay aligned");
    const int h = P.h, w = P.w, ng = ck.ng;
    const int rb = band * 64 * R;
    const int row0 = rb + lane * R;

    // VIRT: the prologue needs no masking.  Lanes left of column 0 compute virtual
    // cells: every cell of columns <= -2 starts at kVirtNeg (and stays far below any
    // real value), so column -1 computes max3(neg, neg, up) = the cell above = 0,
    // which is the left border of global (G space) and local (H space).  Semiglobal's
    // left border grows with the row in G space and keeps the masked prologue.
    constexpr bool VIRT = KIND != KIND_SEMIGLOBAL && R == 1 && X == 0 && !PARTIAL;
    constexpr int kVirtNeg = -(1 << 29);
    // a shard with a received left column (R = 1 only, enforced by the host) runs
    // the masked prologue on the received values instead of the virtual one
    const bool shard_left = P.left_in != nullptr;
    const bool virt = VIRT && !shard_left;
    int lv1 = 0, lv0 = 0;   // H[row0][-1], H[row0-1][-1] in kernel value space
    if (P.stage && lane == 0) P.stage[band] = 1 | ((uint32_t)(__builtin_amdgcn_s_memrealtime() >> 4) & ~7u);
    if (shard_left) {
        if (!poll_left(P, row0, lv1, lv0, err)) return;
        if (P.stage && lane == 0) P.stage[band] = 2;
        if (KIND != KIND_LOCAL) {
            lv1 += (row0 + 1) * ng;
            lv0 += row0 * ng;
        }
        if (row0 == 0) lv0 = border_left<KIND>(-1, ng);
    }
    auto left_val = [&](int r) { return shard_left ? (r == row0 ? lv1 : lv0) : border_left<KIND>(r, ng); };
    int qv[R];
    bool dead[R];
    int cur[R], prev[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int r = row0 + k;
        dead[k] = r >= h;
        qv[k] = dead[k] ? 0x100 : (int)gmem(P.q)[P.q_off + P.q_step * r];
        cur[k] = virt ? kVirtNeg : left_val(r);
        prev[k] = cur[k];
    }
    // settle the query loads here: no global load is in flight inside the block loop
#pragma unroll
    for (int k = 0; k < R; ++k) asm volatile("" : "+v"(qv[k]));
    int dg = virt ? kVirtNeg : left_val(row0 - 1);   // diag of row 0 at its first column
    int upc = 0;                                 // up of row 0 for the current step
    int outv[CH];
    int best = 0;

    const int nchunks = (w + CH - 1) / CH;
    const int nblocks = nchunks + LAG;
    // last observed values of the LDS counters: most blocks need no LDS round trip
    uint32_t seen_prod = 0, seen_sfill = 0, seen_cons = 0;
    int rv[CH];
    uint32_t sw[R][CH / 4];

    // the hand-scheduled steady-state block reads its top-row values itself
    constexpr bool ASM = R == 1 && X == 0 && CH == 32 && !PARTIAL;

    // Acquire block bb's inputs: wait for the top-row chunk bb (in-ring) and the
    // subject bytes, load the subject bytes of every row and (unless the asm block
    // reads them itself) the top-row chunk.  Returns false on timeout.
    auto acquire = [&](int bb, bool asm_blk) -> bool {
        const int tb = bb * CH;
        STAMP(ta);
        if (bb < nchunks && seen_sfill < (uint32_t)(bb + 1)) {
            if (!(seen_sfill = spin_lds_ge(io.s_filled, (uint32_t)(bb + 1), err))) return false;
        }
        STAMP(tb2);
        STAMP_ADD(ST_WAIT_S, tb2 - ta);
        // subject words first: their latency overlaps the wait for the top row
        if constexpr (ASM) {
            if (asm_blk) {
                const uint32_t* src = io.skew + (bb % kSkewBlocks) * 8 * 64 + lane;
#pragma unroll
                for (int i = 0; i < 8; ++i) sw[0][i] = src[64 * i];
            }
        }
        if (!asm_blk) {
#pragma unroll
            for (int k = 0; k < R; ++k)
                load_sbytes<CH>(io.s_ring, (tb - BASE - S * lane - k) & (kSRing - 1), sw[k]);
        }
        if (bb < nchunks) {
            if (io.in_border) {
                if (lane < CH) io.my_ring[(tb + lane) & IRM] = border_top<KIND>(tb + lane, ng);
            } else if (seen_prod < (uint32_t)(bb + 1)) {
                if (!(seen_prod = spin_lds_ge(io.my_prod, (uint32_t)(bb + 1), err))) return false;
            }
            STAMP(tc);
            STAMP_ADD(ST_WAIT_IN, tc - tb2);
            if (!asm_blk) {
                const int4* src = reinterpret_cast<const int4*>(io.my_ring + (tb & IRM));
#pragma unroll
                for (int q = 0; q < CH / 4; ++q) {
                    const int4 v = src[q];
                    rv[4 * q] = v.x;
                    rv[4 * q + 1] = v.y;
                    rv[4 * q + 2] = v.z;
                    rv[4 * q + 3] = v.w;
                }
            }
        }
        return true;
    };

    // lane 0's top value at column -1: H[rb-1][-1] (lane 0 of a shard holds it in lv0)
    int top_first = shard_left ? __shfl(lv0, 0) : border_left<KIND>(rb - 1, ng);
    // full blocks end at fe (they start at 0 for VIRT, at D / CH otherwise)
    const int fe = w + BASE >= CH ? (w + BASE - CH) / CH + 1 : 0;
    LoopArgs la;
    if constexpr (ASM) {
        la.rb = lds_addr(io.my_ring);
        la.nb = io.out_lds ? lds_addr(io.next_ring) : 0u;
        la.apr = lds_addr(io.my_prod);
        la.acn = lds_addr(io.my_cons);
        la.anp = io.out_lds ? lds_addr(io.next_prod) : 0u;
        la.anc = io.out_lds ? lds_addr(io.next_cons) : 0u;
        la.asf = lds_addr(io.s_filled);
        la.atl = lds_addr(io.tail);
        la.skb = lds_addr(io.skew) + 4u * lane;
        la.lo = 4u * (lane - 32);
        la.lid4 = 4u * lane;
        la.bvb = (uint32_t)border_top<KIND>(lane, ng);
        la.bvs = (uint32_t)(border_top<KIND>(1, ng) - border_top<KIND>(0, ng));
        la.fl = (io.in_border ? 1u : 0u) | (io.trailing ? 2u : 0u) | (io.out_lds ? 4u : 0u) |
                (io.gout ? 8u : 0u);
        la.gp = (uint64_t)(size_t)io.gout;
    }
    for (int b = 0; b < nblocks; ++b) {
        const int t0 = b * CH;
        const bool full = (virt || t0 >= D) && (t0 + CH <= w + BASE);
        if constexpr (ASM) {
            if (full) {
#ifdef ANYSEQ_STAMPS
                if (b == 0 && dbg && lane == 0 && band < 2048) dbg[16 + 4 * (band + (P.q_step < 0 ? 2048 : 0))] = __builtin_amdgcn_s_memrealtime();
                STAMP(tl0);
#endif
                uint32_t bb = (uint32_t)b;
                uint64_t tsv = 0;
                uint32_t npoll[3] = {0, 0, 0};
                const int role = (io.in_border ? 3 : 0) + (io.out_lds ? 1 : (io.gout ? 2 : 0));
                uint32_t st = 0;
#define AQ_CALL(BD, PB)                                                                                          \
    st = band_loop_asm<KIND, BD, PB>(bb, (uint32_t)fe, seen_prod, seen_sfill, seen_cons, la, qv[0], cur[0], dg,   \
                                     top_first, best, ck, tsv, npoll)
                switch (role) {
                    case 0: AQ_CALL(false, 0); break;
                    case 1: AQ_CALL(false, 1); break;
                    case 2: AQ_CALL(false, 2); break;
                    case 3: AQ_CALL(true, 0); break;
                    case 4: AQ_CALL(true, 1); break;
                    default: AQ_CALL(true, 2); break;
                }
#undef AQ_CALL
                if (st) {
                    atomicOr(err, ERR_SPIN_TIMEOUT);
                    return;
                }
#ifdef ANYSEQ_STAMPS
                STAMP(tl1);
                STAMP_ADD(ST_COMPUTE, tl1 - tl0);
                if (b == 0 && dbg && lane == 0 && band < 2048) dbg[16 + 4 * (band + (P.q_step < 0 ? 2048 : 0))] = tsv;
                acc[ST_POLL_S] += npoll[0];
                acc[ST_POLL_IN] += npoll[1];
                acc[ST_POLL_OUT] += npoll[2];
#endif
                b = (int)bb - 1;   // ++b of the for
                continue;
            }
        }
        // inputs of this block (rv/sw live only inside one iteration)
        STAMP(t_acq0);
        if (!acquire(b, ASM && full)) return;
        STAMP(t_comp0);
        STAMP_ADD(ST_ACQ, t_comp0 - t_acq0);
#ifdef ANYSEQ_STAMPS
        if (b == 0 && dbg && lane == 0 && band < 2048) dbg[16 + 4 * (band + (P.q_step < 0 ? 2048 : 0))] = __builtin_amdgcn_s_memrealtime();
#endif
        // bottom-row chunk j = b - LAG is complete after this block: make room for it
        const int j = b - LAG;
        const bool pub = io.out_lds && j >= 0;
        if (pub) {
            const uint32_t need = (uint32_t)max(0, j - kSlots + 1);
            STAMP(to0);
            if (seen_cons < need) {
                if (!(seen_cons = spin_lds_ge(io.next_cons, need, err))) return;
            }
            STAMP(to1);
            STAMP_ADD(ST_WAIT_OUT, to1 - to0);
        }
        if (ASM && full) {
            if constexpr (ASM) {
                const bool st = pub;
                const uint32_t pa = st && lane >= 32 ? lds_addr(io.next_ring + ((j * CH) & IRM) + (lane - 32))
                                                     : lds_addr(io.dummy + lane);
                const uint64_t pm = 0;
                band_block_asm<KIND>(top_first, lds_addr(io.my_ring + (t0 & IRM)), pa, pm, sw[0], qv[0], cur[0], dg,
                                     best, ck);
            }
        } else {
            if (full)
                band_block<KIND, R, X, CH, false, PARTIAL>(t0, lane, w, top_first, rv, sw, qv, dead, cur, prev, upc,
                                                           dg, outv, best, ck);
            else if (virt)
                band_block<KIND, R, X, CH, true, PARTIAL, VIRT>(t0, lane, w, top_first, rv, sw, qv, dead, cur, prev,
                                                                upc, dg, outv, best, ck);
            else
                band_block<KIND, R, X, CH, true, PARTIAL, false>(t0, lane, w, top_first, rv, sw, qv, dead, cur, prev,
                                                                 upc, dg, outv, best, ck);
            top_first = rv[CH - 1];
            if (pub && lane == 63) {
                int4* dst = reinterpret_cast<int4*>(io.next_ring + ((j * CH) & IRM));
#pragma unroll
                for (int q = 0; q < CH / 4; ++q)
                    dst[q] = make_int4(outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]);
            }
            if (io.gout && j >= 0 && lane == 63) {
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    if (j * CH + u < w)
                        __hip_atomic_store(gmem(io.gout) + j * CH + u, outv[u], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        STAMP(t_comp1);
        STAMP_ADD(ST_COMPUTE, t_comp1 - t_comp0);
        // chunk b has been read: the producer may reuse its slot
        if (!io.in_border && b < nchunks) lds_st(io.my_cons, (uint32_t)(b + 1));
        if (io.trailing) lds_st(io.tail, (uint32_t)(b + 1));
        if (pub) {
            lds_st(io.next_prod, (uint32_t)(j + 1));
#ifdef ANYSEQ_STAMPS
            if (j == 0 && dbg && lane == 0 && band < 2048) dbg[16 + 4 * (band + (P.q_step < 0 ? 2048 : 0)) + 1] = __builtin_amdgcn_s_memrealtime();
#endif
        }
    }
    if (!io.in_border) lds_st(io.my_cons, (uint32_t)(nchunks + kSlots));
    if (io.trailing) lds_st(io.tail, 0x7fffffffu);

    // ---- last column (H space) and local maximum
    if (P.out_col) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int r = row0 + k;
            if (r < h) gmem(P.out_col)[r] = to_h<KIND>(cur[k], r, w - 1, ng);
        }
    }
    if (P.stage && lane == 0) P.stage[band] = 3;
    if (P.progress && !publish_progress(P, band, lane, err)) return;
    if (P.stage && lane == 0) P.stage[band] = 4 | ((uint32_t)(__builtin_amdgcn_s_memrealtime() >> 4) & ~7u);
    if (KIND == KIND_LOCAL && P.best) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
        if (lane == 0) atomicMax(P.best, best);
    }
#ifdef ANYSEQ_STAMPS
    if (dbg && lane == 0 && band < 2048) dbg[16 + 4 * (band + (P.q_step < 0 ? 2048 : 0)) + 2] = __builtin_amdgcn_s_memrealtime();
    STAMP(t_end);
    acc[ST_TOTAL] = t_end - t_begin;
    acc[ST_BANDS] = 1;
    acc[ST_BLOCKS] = nblocks;
    if (dbg && lane == 0)
        for (int i = 0; i < ST_NSLOTS; ++i) atomicAdd(dbg + i, (unsigned long long)acc[i]);
#endif
}

// The I/O wave of a workgroup:
//  * stages the subject bytes of the group's columns into the shared s_ring
//    (ahead of wave 0, never overwriting bytes the trailing wave still reads);
//  * copies the previous group's bottom row (HBM, sc1 loads behind a relaxed
//    progress flag) into compute wave 0's in-ring;
//  * copies this group's bottom row from the out-ring to HBM (sc1 stores,
//    vmcnt(0), then the flag).
// The HBM hand-off latency therefore never sits on a compute wave's critical path.
// Hand-off element: the linear fill passes one int per column (G or H), the affine
// fill an int2 (G, F-down).  Rows waiting for data hold a sentinel no kernel value
// takes: -1 for linear (G >= 0, local H >= 0), 0x80808080 in .x for affine.
template <typename T>
struct HandOff;
template <>
struct HandOff<int32_t> {
    __device__ static int32_t load(const int32_t* p) {
        return __hip_atomic_load(gmem(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static void store(int32_t* p, int32_t v) {
        __hip_atomic_store(gmem(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static bool pending(int32_t v) { return v == -1; }
    __device__ static int32_t zero() { return 0; }
    __device__ static int32_t sentinel() { return -1; }
    __device__ static int32_t neg() { return -(1 << 29); }
};
template <>
struct HandOff<int2> {
    __device__ static int2 load(const int2* p) {
        const uint64_t u = __hip_atomic_load(gmem(reinterpret_cast<const uint64_t*>(p)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return make_int2((int)(uint32_t)u, (int)(uint32_t)(u >> 32));
    }
    __device__ static void store(int2* p, int2 v) {
        const uint64_t u = (uint64_t)(uint32_t)v.x | ((uint64_t)(uint32_t)v.y << 32);
        __hip_atomic_store(gmem(reinterpret_cast<uint64_t*>(p)), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ static bool pending(int2 v) { return v.x == (int)0x80808080; }
    __device__ static int2 zero() { return make_int2(0, 0); }
    __device__ static int2 sentinel() { return make_int2((int)0x80808080, (int)0x80808080); }
    __device__ static int2 neg() { return make_int2(-(1 << 29), -(1 << 29)); }   // (kAffNeg, kAffNeg)
};

#ifndef ANYSEQ_IO_SKEW_POLLING
#define ANYSEQ_IO_SKEW_POLLING 8
#endif
constexpr int kIoSkewPolling = ANYSEQ_IO_SKEW_POLLING;   // skewed blocks per I/O pass while a hand-off poll is out
#ifndef ANYSEQ_IO_SLEEP
#define ANYSEQ_IO_SLEEP 1
#endif
constexpr int kIoSleep = ANYSEQ_IO_SLEEP;   // s_sleep units of an affine I/O pass without progress

// The affine I/O wave when the compute waves read their own subject codes (GS, round 5):
// it only forwards the previous group's bottom row from the HBM hand-off row into wave
// 0's LDS ring.  One poll of 128 columns (8 granules of 16, 2 loads per lane) is always
// in flight; after a poll is consumed the next one goes out BEFORE the consumed granules
// get their sentinel back, so the next poll's wait never covers those stores.  Same data
// protocol as io_wave: a granule is in when none of its columns < w holds the sentinel;
// ext: "minus infinity" past the last granule; pscale: ring counter units per chunk.
template <typename T>
__device__ void io_forward(int lane, int w, const T* g_in, T* ring0, uint32_t* prod0, uint32_t* cons0, uint32_t* err,
                           bool reset_in, int ext, int pscale, bool hprio, unsigned long long* evp) {
    constexpr int CH = 32, GR = 16, GPC = CH / GR, IRM = kSlots * CH - 1;
    const int nchunks = (w + CH - 1) / CH, ngran = (w + GR - 1) / GR;
    if (!g_in) return;
    int in_gran = 0, plim = 0;
    T pv[2];
    uint32_t idle = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#ifdef ANYSEQ_STAMPS
    uint64_t t_poll = 0;
#endif
    auto issue = [&]() {
        int lim = min(((int)lds_ld(cons0) + kSlots) * GPC, ngran);   // ring space
        plim = min(lim, in_gran + 8);
#ifdef ANYSEQ_STAMPS
        t_poll = evp ? __builtin_amdgcn_s_memrealtime() : 0;
#endif
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int col = in_gran * GR + i * 64 + lane;
            pv[i] = col < plim * GR && col < w ? HandOff<T>::load(g_in + col) : HandOff<T>::zero();
        }
    };
    issue();
    while (in_gran < ngran) {
        if (hprio) __builtin_amdgcn_s_setprio(3);
        int ready = 0;
        bool stop = false;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint64_t bad = __ballot(HandOff<T>::pending(pv[i]));
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int gi = in_gran + 4 * i + g;
                if (!stop && gi < plim && ((bad >> (16 * g)) & 0xffffu) == 0u) ++ready;
                else stop = true;
            }
        }
        if (ready > 0) {
#ifdef ANYSEQ_STAMPS
            if (evp && lane == 0 && in_gran <= 2000 && in_gran + ready > 2000) {
                evp[11] = __builtin_amdgcn_s_memrealtime();
                evp[12] = t_poll;
            }
#endif
            const int base = in_gran, c0 = in_gran * GR, c2 = (in_gran + ready) * GR;
            const T done0 = pv[0], done1 = pv[1];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int col = base * GR + i * 64 + lane;
                if (col >= c0 && col < c2) ring0[col & IRM] = i ? done1 : done0;
            }
            in_gran += ready;
            if (ext && in_gran >= ngran) {   // (as io_wave: the last chunk's unpolled columns)
                const int c = ngran * GR + lane;
                if (c < nchunks * CH) ring0[c & IRM] = HandOff<T>::neg();
            }
            lds_st(prod0, in_gran >= ngran ? (uint32_t)(nchunks * pscale) : (uint32_t)(in_gran * pscale / GPC));
            if (hprio) __builtin_amdgcn_s_setprio(0);
            if (in_gran < ngran) issue();
            if (reset_in) {   // whole granules, also past w (io_wave)
                T* gw = const_cast<T*>(g_in);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int col = base * GR + i * 64 + lane;
                    if (col >= c0 && col < c2) HandOff<T>::store(gw + col, HandOff<T>::sentinel());
                }
            }
            idle = 0;
        } else {
            if (hprio) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_s_sleep(kIoSleep);
            if ((++idle & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t_start > SPIN_TICKS || err_set(err))) {
                atomicOr(err, ERR_SPIN_TIMEOUT | 8u);
                lds_st(prod0, (uint32_t)(nchunks * pscale));
                return;
            }
            issue();
        }
    }
    if (reset_in) {   // (as io_wave: the producer's last chunk past w)
        T* gw = const_cast<T*>(g_in);
        for (int c = ngran * GR + lane; c < nchunks * CH; c += 64) HandOff<T>::store(gw + c, HandOff<T>::sentinel());
    }
}

template <int CH, bool SKEW, typename T = int32_t>
__device__ void io_wave(int lane, int w, const uint8_t* s, int s_off, int s_step, uint8_t* s_ring, uint32_t* skew,
                        uint32_t* s_filled, uint32_t* tail, const T* g_in, T* ring0, uint32_t* prod0,
                        uint32_t* cons0, uint32_t* err, bool reset_in = false, int ext = 0, int pscale = 1,
                        bool hprio = false, unsigned long long* evp = nullptr, int io_stage = 3,
                        int io_skew = kIoSkewPolling, bool io_poll2 = false, bool no_subject = false) {
    constexpr int IRM = kSlots * CH - 1;
    constexpr int SCH = kSRing / CH;   // chunks held by the subject ring
    constexpr int GR = 16;             // hand-off poll granule (columns)
    constexpr int GPC = CH / GR;       // granules per chunk
    const int nchunks = (w + CH - 1) / CH;
    const int ngran = (w + GR - 1) / GR;
    // ext: skewed blocks staged past the last chunk (the affine asm epilogue's), whose
    // columns >= w all hold code 0xFF; pscale: units of the ring counter per chunk (the
    // affine fill counts half chunks = granules)
    const int nskew = nchunks + ext;
    const bool need_in = g_in != nullptr;
    const GLOBAL_AS uint8_t* sg = gmem(s);
    int s_next = 0, sk_next = 0, in_gran = 0;
    int st_lim = 0;   // subject chunks whose loads are issued (s_next: stored in the ring)
    // no_subject: the compute waves read their codes from HBM (DPProblem::scode, round 5):
    // no subject staging and no skewed copy, only the hand-off rows.  (io_skew < 0 on the
    // LDS path: the same, as a DIAGNOSTIC that times the hand-off without the subject work
    // -- the compute waves then read stale LDS: wrong scores.)
    if (no_subject || io_skew < 0) {
        s_next = st_lim = nchunks;
        sk_next = SKEW ? nskew : 0;
        lds_st(s_filled, (uint32_t)nskew);
        io_skew = 8;
    }

    uint8_t sv[4];    // the loaded, not yet stored subject bytes (4 x 64 columns)
    T qv[2] = {HandOff<T>::zero(), HandOff<T>::zero()};   // io_poll2: the poll in flight
    int q_lim = 0, q_base = 0;
#ifdef ANYSEQ_STAMPS
    uint64_t q_t = 0;
#endif
    uint32_t idle = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    while (s_next < nchunks || (SKEW && sk_next < nskew) || (need_in && in_gran < ngran)) {
        bool progress = false;
        // The hand-off poll goes out first (the band chain waits on it): 128 columns from
        // the first granule not yet in, consumed after this iteration's skew work, so the
        // load's round trip overlaps it.  The previous group's last band stores its
        // bottom row straight into g_in (sc1), which the host filled with the sentinel
        // (never a kernel value): a granule is in when none of its columns < w holds it.
        // io_poll2: two polls in flight -- a pass issues one and consumes the one the
        // previous pass issued (half the cadence of a poll's round trip); the consumed
        // poll's granules start at pbase <= in_gran (those before in_gran came in through
        // the other poll)
        T pv[2];
        int plim = 0, pbase = in_gran;
#ifdef ANYSEQ_STAMPS
        uint64_t t_poll = evp ? __builtin_amdgcn_s_memrealtime() : 0;   // diagnostic build
#endif
        if (need_in && in_gran < ngran) {
            int lim = min(((int)lds_ld(cons0) + kSlots) * GPC, ngran);   // ring space
            lim = min(lim, in_gran + 8);
            T nv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int col = in_gran * GR + i * 64 + lane;
                nv[i] = col < lim * GR && col < w ? HandOff<T>::load(g_in + col) : HandOff<T>::zero();
            }
            if (io_poll2) {
                pv[0] = qv[0];
                pv[1] = qv[1];
                plim = q_lim;
                pbase = q_base;
                qv[0] = nv[0];
                qv[1] = nv[1];
                q_lim = lim;
                q_base = in_gran;
#ifdef ANYSEQ_STAMPS
                const uint64_t tq = q_t;
                q_t = t_poll;
                t_poll = tq;
#endif
            } else {
                pv[0] = nv[0];
                pv[1] = nv[1];
                plim = lim;
            }
        }
        // Subject staging (io_stage, FillParams::io_stage):
        //  0: whatever chunks the trailing wave has freed, loaded and stored in the same
        //     pass (a load round trip in nearly every pass, between the hand-off poll's
        //     issue and its consumption);
        //  1: the same in whole 1024-column batches (a round trip every 32 blocks);
        //  2: asynchronous -- a pass stores the bytes the previous pass loaded (up to 256
        //     columns) and issues the next loads, here, before the skew work;
        //  3: as 2, after the poll's consumption (the poll's wait never covers a younger
        //     staging load).
        // The first batch (up to 1024 columns) always waits for its loads.
        auto stage = [&]() {
            if (io_stage >= 2 && st_lim > s_next) {   // (loaded by the previous pass)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int c = s_next * CH + i * 64 + lane;
                    if (c < st_lim * CH) {
                        const int p = c & (kSRing - 1);
                        s_ring[p] = sv[i];
                        if (p < 64) s_ring[p + kSRing] = sv[i];
                    }
                }
                if (!SKEW) lds_st(s_filled, (uint32_t)st_lim);
                s_next = st_lim;
                progress = true;
            }
            if (st_lim >= nchunks) return;
            const uint32_t tl = lds_ld(tail);
            // the trailing wave in block `tl` still reads columns >= tl*CH - kMaxBack
            int lim = (int)min((uint32_t)nchunks, tl >= 0x7fffffffu ? (uint32_t)nchunks
                                                                     : tl + SCH - kMaxBack / CH - 1);
            if (st_lim == 0 || io_stage < 2) {
                lim = min(lim, st_lim + 1024 / CH);   // one batch: 16 loads in flight per lane
                const bool go_ = st_lim == 0 || io_stage == 0 || lim - st_lim >= 1024 / CH || lim >= nchunks ||
                                 st_lim < sk_next + 16;
                if (lim <= st_lim || !go_) return;
                const int c0 = st_lim * CH;
                uint8_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int c = c0 + i * 64 + lane;
                    v[i] = (c < w && c < lim * CH) ? sg[s_off + s_step * c] : (uint8_t)0;
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int c = c0 + i * 64 + lane;
                    if (c < lim * CH) {
                        const int p = c & (kSRing - 1);
                        s_ring[p] = v[i];
                        if (p < 64) s_ring[p + kSRing] = v[i];
                    }
                }
                if (!SKEW) lds_st(s_filled, (uint32_t)lim);
                s_next = st_lim = lim;
                progress = true;
            } else {
                lim = min(lim, st_lim + 256 / CH);
                if (lim >= st_lim + 2 || (lim >= nchunks && lim > st_lim)) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int c = st_lim * CH + i * 64 + lane;
                        sv[i] = (c < w && c < lim * CH) ? sg[s_off + s_step * c] : (uint8_t)0;
                    }
                    st_lim = lim;
                }
            }
        };
        if (io_stage < 3) stage();
        const int sk_avail = s_next >= nchunks ? nskew : s_next;
        if (SKEW && sk_next < sk_avail) {
            // skewed copy of block b needs raw columns 32b-64 .. 32b+31 (staged: b < s_next)
            // and a free slot: the trailing wave has finished block b - kSkewBlocks
            const uint32_t tl = lds_ld(tail);
            int lim = min(sk_avail, tl >= 0x7fffffffu ? nskew : (int)tl + kSkewBlocks);
            lim = min(lim, sk_next + (plim > in_gran ? io_skew : 8));
            for (int b = sk_next; b < lim; ++b) {
                uint32_t d[8];
                load_sbytes<32>(s_ring, (32 * b - 1 - lane) & (kSRing - 1), d);
                // columns left of 0 (virtual prologue lanes): code 0xFF, which matches no
                // query code (the LUT weight of 0xFF is -1); so are the
                // columns >= w of the epilogue's blocks
                const int cneg = 32 * b - 1 - lane;
                if (cneg < 0 || (ext && cneg + 31 >= w)) {
#pragma unroll
                    for (int i = 0; i < 8; ++i)
#pragma unroll
                        for (int kb = 0; kb < 4; ++kb) {
                            const int c = cneg + 4 * i + kb;
                            if (c < 0 || (ext && c >= w)) d[i] |= 0xffu << (8 * kb);
                        }
                }
                uint32_t* dst = skew + (b % kSkewBlocks) * 8 * 64 + lane;
#pragma unroll
                for (int i = 0; i < 8; ++i) dst[64 * i] = d[i];
            }
            if (lim > sk_next) {
                lds_st(s_filled, (uint32_t)lim);
                sk_next = lim;
                progress = true;
            }
        }
        if (plim > in_gran) {
            // hprio: the hand-off step runs at top issue priority (this wave shares a SIMD
            // with a compute wave, which otherwise wins every VALU slot); staging and skew
            // stay at the bottom, in the compute wave's bubbles
            if (hprio) __builtin_amdgcn_s_setprio(3);
            // leading run of complete granules (16 lanes each) from in_gran
            int ready = 0;
            bool stop = false;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint64_t bad = __ballot(HandOff<T>::pending(pv[i]));
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int gi = pbase + 4 * i + g;
                    if (gi < in_gran) continue;   // (came in through the other poll)
                    if (!stop && gi < plim && ((bad >> (16 * g)) & 0xffffu) == 0u) ++ready;
                    else stop = true;
                }
            }
            if (ready > 0) {
#ifdef ANYSEQ_STAMPS
                // diagnostic build: when the granule of column 32000 (chunk 1000) came in
                if (evp && lane == 0 && in_gran <= 2000 && in_gran + ready > 2000) {
                    evp[11] = __builtin_amdgcn_s_memrealtime();
                    evp[12] = t_poll;
                }
#endif
                const int c0 = in_gran * GR, c2 = (in_gran + ready) * GR;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int col = pbase * GR + i * 64 + lane;
                    if (col >= c0 && col < c2) ring0[col & IRM] = pv[i];
                }
                // ring of hand-off rows (DPProblem::nslots < ngroups - 1): put the sentinel
                // back, so the group that reuses this slot 2*grid+2 groups later is polled
                // against fresh data.  Whole granules, also their columns past w: the
                // producer stores whole 16-column halves, and a word it left past w would
                // sit inside the row of a later launch with another layout (device-planned
                // levels reuse the rows without a sentinel fill) and be read
                // there as data before that launch's producer wrote it
                if (reset_in) {
                    T* gw = const_cast<T*>(g_in);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int col = pbase * GR + i * 64 + lane;
                        if (col >= c0 && col < c2) HandOff<T>::store(gw + col, HandOff<T>::sentinel());
                    }
                }
                in_gran += ready;
                // ext: the consumer's blocks run past w to the end of the last chunk, whose
                // columns past the last granule (16 when ceil(w/16) is odd) no poll brings
                // in: "minus infinity" there, not whatever an earlier workgroup left in
                // this LDS (those cells' best counts in the capture-free band end, round 5)
                if (ext && in_gran >= ngran) {
                    const int c = ngran * GR + lane;
                    if (c < nchunks * CH) ring0[c & IRM] = HandOff<T>::neg();
                }
                // the counter: granules (pscale 2, CH 32), else whole chunks
                lds_st(prod0, in_gran >= ngran ? (uint32_t)(nchunks * pscale) : (uint32_t)(in_gran * pscale / GPC));
                progress = true;
            }
            if (hprio) __builtin_amdgcn_s_setprio(0);
        }
        if (io_stage == 3) stage();
        if (!progress) {
            __builtin_amdgcn_s_sleep(kIoSleep);
            if ((++idle & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t_start > SPIN_TICKS || err_set(err))) {
                atomicOr(err, ERR_SPIN_TIMEOUT | 8u);
                lds_st(prod0, (uint32_t)(nchunks * pscale));
                lds_st(s_filled, (uint32_t)nskew);
                return;
            }
        }
    }
    // the producer's last chunk may extend past w (whole-chunk stores of the asm
    // epilogue): those columns get the sentinel back too, so a ring that is reset
    // after every read is all sentinel again once the launch is over
    if (need_in && reset_in) {
        T* gw = const_cast<T*>(g_in);
        for (int c = ngran * GR + lane; c < nchunks * CH; c += 64) HandOff<T>::store(gw + c, HandOff<T>::sentinel());
    }
}

// The linear fill's I/O wave (round 2): whole-chunk hand-off polls.  The affine
// fill's io_wave above polls 16-column granules ahead of its staging work; on the
// linear kernel (configs[1], 65536^2) that variant measured 3.44 ms per launch against
// 3.11 ms with this one (profiles/r03e_c1_kernel_stats.csv, r03f_bench_c1_c3_c4.json),
// so the linear fill keeps it.
template <int CH, bool SKEW, typename T = int32_t>
__device__ void io_wave_lin(int lane, int w, const uint8_t* s, int s_off, int s_step, uint8_t* s_ring, uint32_t* skew,
                        uint32_t* s_filled, uint32_t* tail, const T* g_in, T* ring0, uint32_t* prod0,
                        uint32_t* cons0, uint32_t* err, bool reset_in = false) {
    constexpr int IRM = kSlots * CH - 1;
    constexpr int SCH = kSRing / CH;   // chunks held by the subject ring
    const int nchunks = (w + CH - 1) / CH;
    const bool need_in = g_in != nullptr;
    const GLOBAL_AS uint8_t* sg = gmem(s);
    int s_next = 0, sk_next = 0, in_next = 0;
    uint32_t idle = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    while (s_next < nchunks || (SKEW && sk_next < nchunks) || (need_in && in_next < nchunks)) {
        bool progress = false;
        if (s_next < nchunks) {
            const uint32_t tl = lds_ld(tail);
            // the trailing wave in block `tl` still reads columns >= tl*CH - kMaxBack
            int lim = (int)min((uint32_t)nchunks, tl >= 0x7fffffffu ? (uint32_t)nchunks
                                                                     : tl + SCH - kMaxBack / CH - 1);
            lim = min(lim, s_next + 1024 / CH);   // one batch: 16 loads in flight per lane
            if (lim > s_next) {
                const int c0 = s_next * CH;
                uint8_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int c = c0 + i * 64 + lane;
                    v[i] = (c < w && c < lim * CH) ? sg[s_off + s_step * c] : (uint8_t)0;
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int c = c0 + i * 64 + lane;
                    if (c < lim * CH) {
                        const int p = c & (kSRing - 1);
                        s_ring[p] = v[i];
                        if (p < 64) s_ring[p + kSRing] = v[i];
                    }
                }
                if (!SKEW) lds_st(s_filled, (uint32_t)lim);
                s_next = lim;
                progress = true;
            }
        }
        if (SKEW && sk_next < s_next) {
            // skewed copy of block b needs raw columns 32b-64 .. 32b+31 (staged: b < s_next)
            // and a free slot: the trailing wave has finished block b - kSkewBlocks
            const uint32_t tl = lds_ld(tail);
            int lim = min(s_next, tl >= 0x7fffffffu ? nchunks : (int)tl + kSkewBlocks);
            lim = min(lim, sk_next + 8);
            for (int b = sk_next; b < lim; ++b) {
                uint32_t d[8];
                load_sbytes<32>(s_ring, (32 * b - 1 - lane) & (kSRing - 1), d);
                uint32_t* dst = skew + (b % kSkewBlocks) * 8 * 64 + lane;
#pragma unroll
                for (int i = 0; i < 8; ++i) dst[64 * i] = d[i];
            }
            if (lim > sk_next) {
                lds_st(s_filled, (uint32_t)lim);
                sk_next = lim;
                progress = true;
            }
        }
        if (need_in && in_next < nchunks) {
            // The previous group's last band stores its bottom row straight into g_in
            // (sc1), which the host filled with the sentinel -1 (never a kernel value:
            // G >= 0 and local H >= 0).  Poll the data itself: a chunk is ready when
            // none of its columns < w still holds -1.
            const int lim = min((int)lds_ld(cons0) + kSlots, nchunks);
            if (lim > in_next) {
                constexpr int PER = kSlots * CH / 64;   // 2 chunks per load row
                T v[PER];
                const int c0 = in_next * CH, c1 = lim * CH;
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int col = c0 + i * 64 + lane;
                    v[i] = col < c1 && col < w ? HandOff<T>::load(g_in + col) : HandOff<T>::zero();
                }
                // leading run of complete chunks
                int ready = 0;
                bool stop = false;
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const uint64_t bad = __ballot(HandOff<T>::pending(v[i]));
                    if (!stop && in_next + 2 * i < lim && (uint32_t)bad == 0u) ++ready; else stop = true;
                    if (!stop && in_next + 2 * i + 1 < lim && (uint32_t)(bad >> 32) == 0u) ++ready; else stop = true;
                }
                if (ready > 0) {
                    const int c2 = (in_next + ready) * CH;
#pragma unroll
                    for (int i = 0; i < PER; ++i) {
                        const int col = c0 + i * 64 + lane;
                        if (col < c2) ring0[col & IRM] = v[i];
                    }
                    // ring of hand-off rows (DPProblem::nslots < ngroups - 1): put the sentinel
                    // back, so the group that reuses this slot 2*grid+2 groups later is polled
                    // against fresh data
                    if (reset_in) {
                        T* gw = const_cast<T*>(g_in);
#pragma unroll
                        for (int i = 0; i < PER; ++i) {
                            const int col = c0 + i * 64 + lane;
                            if (col < c2 && col < w) HandOff<T>::store(gw + col, HandOff<T>::sentinel());
                        }
                    }
                    lds_st(prod0, (uint32_t)(in_next + ready));
                    in_next += ready;
                    progress = true;
                }
            }
        }
        if (!progress) {
            __builtin_amdgcn_s_sleep(1);
            if ((++idle & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t_start > SPIN_TICKS || err_set(err))) {
                atomicOr(err, ERR_SPIN_TIMEOUT | 8u);
                lds_st(prod0, (uint32_t)nchunks);
                lds_st(s_filled, (uint32_t)nchunks);
                return;
            }
        }
    }
}

template <int KIND, int R, int X, int NW, int CH>
__global__ __launch_bounds__(64 * (NW + 1)) void fill_kernel(const DPProblem* __restrict__ probs,
                                                              const GroupRef* __restrict__ groups, int ngroups_total,
                                                              uint32_t* dq, uint32_t* err, FillParams fp) {
    __shared__ __attribute__((aligned(16))) FillShared<NW, CH> sh;
    // wave index via readfirstlane: everything derived from it is provably wave-uniform (SGPRs,
    // scalar branches instead of exec-mask flow)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    CellK ck;
    ck.ng = -fp.gap;
    ck.thr = fp.throttle;
    if (KIND == KIND_LOCAL) {
        ck.wm = fp.match - fp.gap;
        ck.wx = fp.mismatch - fp.gap;
    } else {
        ck.wm = fp.match - 2 * fp.gap;
        ck.wx = fp.mismatch - 2 * fp.gap;
    }
    // issue priority: 1 = compute waves before the I/O wave, 2 = the I/O wave first (it
    // sleeps when idle; its hand-off polls sit on the band chain)
    if (fp.prio == 1 && wave < NW) __builtin_amdgcn_s_setprio(3);
    if (fp.prio == 2 && wave == NW) __builtin_amdgcn_s_setprio(3);
    for (;;) {
        if (threadIdx.x == 0) {
            sh.group = (int32_t)atomicAdd(dq, 1u);
            sh.s_filled = 0;
            sh.tail = 0;
        }
        if (threadIdx.x <= NW) {
            sh.prod[threadIdx.x] = 0;
            sh.cons[threadIdx.x] = 0;
        }
        __syncthreads();
        const int gi = __builtin_amdgcn_readfirstlane(sh.group);
        if (gi >= ngroups_total || err_set(err)) break;
        const GroupRef g = groups[gi];
        const DPProblem P = probs[g.prob];
        if (g.epoch != fp.epoch || g.check != group_check(g.prob, g.group, g.epoch) ||
            P.magic != prob_magic(&probs[g.prob], g.prob, fp.epoch) || g.group >= P.ngroups) {
            if (threadIdx.x == 0) atomicOr(err, ERR_BAD_DESC);
            break;
        }
        const int first = g.group * NW;
        const int last = min(P.nbands, first + NW) - 1;   // last band of this group
        // where the group's bottom row goes: the next group's input row (rowbuf, pre-filled
        // with the sentinel -1), the problem's out_row, or nowhere.  The group's last band
        // stores it there itself.
        int32_t* g_out = nullptr;
        if (last < P.nbands - 1)
            g_out = P.rowbuf + (size_t)(g.group % P.nslots) * P.wpad;
        else if (P.out_row)
            g_out = P.out_row;
        if (wave == NW) {
            const int32_t* g_in = g.group > 0 ? P.rowbuf + (size_t)((g.group - 1) % P.nslots) * P.wpad : nullptr;
            io_wave_lin<CH, R == 1 && X == 0 && CH == 32>(lane, P.w, P.s, P.s_off, P.s_step, sh.s_ring, &sh.skew[0][0][0],
                                                      &sh.s_filled, &sh.tail, g_in, sh.in_ring[0], &sh.prod[0],
                                                      &sh.cons[0], err, P.nslots < P.ngroups - 1);
        } else {
            const int band = first + wave;
            if (band <= last) {
                WaveIO io;
                io.in_border = band == 0;
                io.trailing = band == last;
                io.my_ring = sh.in_ring[wave];
                io.my_prod = &sh.prod[wave];
                io.my_cons = &sh.cons[wave];
                io.s_ring = sh.s_ring;
                io.s_filled = &sh.s_filled;
                io.tail = &sh.tail;
                io.dummy = sh.dummy[wave];
                io.skew = &sh.skew[0][0][0];
                io.gout = nullptr;
                if (band < last) {
                    io.out_lds = true;
                    io.next_ring = sh.in_ring[wave + 1];
                    io.next_prod = &sh.prod[wave + 1];
                    io.next_cons = &sh.cons[wave + 1];
                } else {
                    io.out_lds = false;
                    io.gout = g_out;
                    io.next_ring = nullptr;
                    io.next_prod = nullptr;
                    io.next_cons = nullptr;
                }
                const bool partial = (band + 1) * 64 * R > P.h;
                if (partial)
                    run_band<KIND, R, X, CH, true>(P, band, lane, io, err, ck, fp.dbg);
                else
                    run_band<KIND, R, X, CH, false>(P, band, lane, io, err, ck, fp.dbg);
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------- affine fill --
// Gotoh (build-defined: affine_scoring_scheme, align.impala:153-166, is dead in the
// reference; semantics = oracle_affine_score / aff_fill in oracle/anyseq_oracle.c):
//   E[r][c] = max(E[r][c-1] + ge, H[r][c-1] + go + ge)   (horizontal, left)
//   F[r][c] = max(F[r-1][c] + ge, H[r-1][c] + go + ge)   (vertical, up)
//   H[r][c] = max(H[r-1][c-1] + sub, E, F)               (clamped: max(., 0))
// All problems run in G-space, X_G = X - (r+c+2)*ge for X in {H,E,F}: every gap
// extension is free there, so
//   E_G = max(E_G, G_left + go),  F_G = max(F_G, G_up + go),
//   G   = max3(G_diag + sub - 2 ge, E_G, F_G),
// and the local clamp H >= 0 becomes G >= Z_t = (r+c+2)(-ge), which is the SAME for
// every lane of a step (r + c = rb + t - 1 on the anti-diagonal): one v_max with a
// wave-uniform bound.  Same geometry as fill_kernel (R = 1, X = 0, CH = 32): lane l
// owns row rb + l of a 64-row band and processes column t - 1 - l at step t.  From
// the lane above it receives, by DPP wave_shr:1, G[r-1][c] (the next step's
// diagonal) and F[r][c] ("F-down" of the row above); lane 0 reads both from the
// band's input ring (int2 per column).  G + go is computed once per cell and
// serves both the F-down of this cell and the E of the next column.
//
// The kind of a problem is runtime data, so ONE launch can mix the sub-problems of
// a Hirschberg level whose ends are anchored or free:
//   DPProblem::bmode  borders (BM_*: the scheme corner / a continuing or paid gap /
//                     free local / free semiglobal borders),
//   DPProblem::amode  bit 0 the local clamp, bits 1-2 the best-cell output into
//                     *best (1: every cell, 2: the last row), H space.
// Problems with amode 0 run the plain steady-state loop (11 VALU per step), the
// others the clamp + best loop (14).
constexpr int kAffNeg = -(1 << 29);   // "minus infinity" of the E/F states (the oracle's AFF_NEG_INF)
// Round 5: the compute waves read their subject codes from the problem's code rows in
// HBM (DPProblem::scode, two 16-byte loads per lane and block) instead of the I/O wave's
// pre-skewed LDS copy, so the I/O wave only forwards the hand-off rows.
// 0: the round-4 LDS path (A/B builds, tools/gen_block_asm.py GS=0).
#ifndef ANYSEQ_AFF_GS
#define ANYSEQ_AFF_GS 1
#endif
constexpr bool kAffGS = ANYSEQ_AFF_GS != 0;

struct AffK {
    int wm, wx;   // diagonal weight sub - 2 ge
    int go;       // gap open (<= 0): added to a cell to open a gap (G space)
    int nge;      // -ge > 0
    int flags;    // bit 0: no asm steady state (diagnostics)
    int thr;      // FillParams::throttle
    bool codes;   // q / s hold alphabet codes (0xFF never a code): the virtual prologue may clamp
    bool lut;     // codes 0..7 and int8 weights: the v_perm weight table
    int slack;    // FillParams::slack
    int slack_io; // FillParams::slack_io
    bool lin;     // gap open 0 (a linear score through this kernel): the linear asm loop (gen_aff2 lin)
};

// Borders of a problem in G space (H border values by border mode, see
// bm_corner / bm_top / bm_left in oracle/anyseq_oracle.c):
//   corner G[-1][-1] = cg;  top G[-1][c] = tfree ? (c+1)(-ge) : tg;  left likewise.
struct AffBorder {
    int cg, tg, lg;
    bool tfree, lfree;
    __device__ AffBorder(int bm, int go) {
        // the transposed modes (FFREE, FPAID, FREE_SEMI_T) swap the top and left borders
        cg = (bm == BM_EFREE || bm == BM_EPAID || bm == BM_FFREE || bm == BM_FPAID) ? kAffNeg : 0;
        tfree = bm == BM_FREE_LOCAL || bm == BM_FREE_SEMI || bm == BM_FREE_SEMI_OPEN;
        lfree = bm == BM_FREE_LOCAL || bm == BM_FREE_SEMI_T || bm == BM_FREE_SEMI_OPEN;
        tg = bm == BM_EFREE ? 0 : (bm == BM_NORMAL || bm == BM_EPAID) ? go : kAffNeg;
        lg = bm == BM_FFREE ? 0 : (bm == BM_NORMAL || bm == BM_FPAID) ? go : kAffNeg;
    }
    __device__ int top(int c, int nge) const { return c < 0 ? cg : (tfree ? (c + 1) * nge : tg); }
    __device__ int left(int r, int nge) const { return r < 0 ? cg : (lfree ? (r + 1) * nge : lg); }
};
__device__ __forceinline__ int aff_to_h(int v, int r, int c, int nge) { return v - (r + c + 2) * nge; }

template <int NW>
struct AffShared {
    int2 in_ring[NW + 1][kSlots * 32];
    uint8_t s_ring[kSRing + 64];
    uint32_t prod[NW + 1];
    uint32_t cons[NW + 1];
    uint32_t skew[kSkewBlocks][8][64];   // pre-skewed subject, as FillShared::skew
    int2 neg[32];   // "minus infinity" top row: the capture-free epilogue's blocks past the last chunk
    uint32_t s_filled;
    uint32_t tail;
    int32_t group;
};

struct AffIO {
    bool in_border, trailing, out_lds;
    bool io_fed = false;   // the group's first band behind the HBM hand-off, fed by the I/O wave
    int2* my_ring;
    uint32_t* my_prod;
    uint32_t* my_cons;
    int2* next_ring;
    uint32_t* next_prod;
    uint32_t* next_cons;
    const uint8_t* s_ring;
    const uint32_t* skew;
    const int2* neg;
    uint32_t* s_filled;
    uint32_t* tail;
    int2* gout;   // last band of a group: HBM destination of the bottom row (G, F)
    // Self-forwarding (round 5, no I/O wave): the group's first band copies the previous
    // group's bottom row from this HBM hand-off row into its own ring, a segment ahead
    const int2* g_in;
    bool reset_in;   // put the sentinel back (the row is reused)
};

// Self-forwarding first band of a group (round 5): io_forward's protocol run by the band
// itself between its asm segments -- granules of 16 columns are in when none of their
// columns < w holds the sentinel; the ring gets them, the HBM row gets the sentinel back.
// Brings the ring (and *my_prod, in half chunks) up to chunk `cend` (exclusive), never
// more than kSlots - 1 chunks past the band's current block `b`.  false on timeout.
struct SelfFwd {
    int gran = 0;   // granules forwarded
    __device__ bool forward_to(const AffIO& io, int lane, int w, int b, int cend, uint32_t* err) {
        constexpr int CH = 32, GR = 16, IRM = kSlots * CH - 1;
        const int nchunks = (w + CH - 1) / CH, ngran = (w + GR - 1) / GR;
        const int tg = min(2 * min(cend, b + kSlots - 1), ngran);
        if (gran >= tg) return true;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t idle = 0;
        while (gran < tg) {
            const int lim = min(gran + 8, tg);
            int2 pv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int col = gran * GR + i * 64 + lane;
                pv[i] = col < lim * GR && col < w ? HandOff<int2>::load(io.g_in + col) : HandOff<int2>::zero();
            }
            int ready = 0;
            bool stop = false;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint64_t bad = __ballot(HandOff<int2>::pending(pv[i]));
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (!stop && gran + 4 * i + g < lim && ((bad >> (16 * g)) & 0xffffu) == 0u) ++ready;
                    else stop = true;
                }
            }
            if (ready == 0) {
                __builtin_amdgcn_s_sleep(1);
                if ((++idle & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
                    atomicOr(err, ERR_SPIN_TIMEOUT | 8u);
                    return false;
                }
                continue;
            }
            const int c0 = gran * GR, c2 = (gran + ready) * GR;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int col = c0 + i * 64 + lane;
                if (col < c2) io.my_ring[col & IRM] = pv[i];
                if (io.reset_in && col < c2) HandOff<int2>::store(const_cast<int2*>(io.g_in) + col, HandOff<int2>::sentinel());
            }
            gran += ready;
            if (gran >= ngran) {   // "minus infinity" past the last granule; the producer's last chunk past w
                const int c = ngran * GR + lane;
                if (c < nchunks * CH) {
                    io.my_ring[c & IRM] = HandOff<int2>::neg();
                    if (io.reset_in) HandOff<int2>::store(const_cast<int2*>(io.g_in) + c, HandOff<int2>::sentinel());
                }
            }
            idle = 0;
        }
        lds_st(io.my_prod, gran >= ngran ? (uint32_t)(2 * nchunks) : (uint32_t)gran);
        return true;
    }
};

// 32 steps in C++ (prologue / epilogue / partial bands; the steady state is the asm
// loop below).  c0 = this lane's column at the first step, tf = top row at column
// t0 - 1, rv[u] = top row at column t0 + u, zc / zb = clamp bound / true Z_t of the
// first step (zc is far below zb when the problem does not clamp).
// MASK: some lanes are outside [0, w).  PARTIAL: rows >= h pass the row above
// through (so lane 63 publishes the last row's G and F-down).  og/of: this lane's
// (G, F-down) after each step (lane 63's are the band's bottom row).
// lbrd: a zero-open left border (semiglobal) forced at column -1 (VIRT; kAffNeg: none)
template <bool MASK, bool PARTIAL, bool VIRT>
__device__ __forceinline__ void aff_block(int c0, int w, int2 tf, const int2 (&rv)[32], const uint32_t (&sw)[8], int q,
                                          bool dead, int zc, int zb, int& g, int& e, int& hg, int& fdn, int& dg,
                                          int& best, int (&og)[32], int (&of)[32], const AffK k, int lbrd = kAffNeg) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
        const int2 top = u == 0 ? tf : rv[u - 1];
        const int upg = wave_shr1(top.x, g);
        const int fin = wave_shr1(top.y, fdn);
        // virtual columns (< 0): no diagonal gain (the asm LUT gives their code 0xFF
        // -1 in X space; the mismatch could be positive, which under the clamp would
        // lift column -1 above the local border -- round 5); they only shape column -1
        const bool vcol = VIRT && c0 + u < 0;
        const int sb = (int)((sw[u >> 2] >> (8 * (u & 3))) & 0xffu);
        const int wgt = vcol ? kAffNeg : (q == sb ? k.wm : k.wx);
        const int en = max(e, hg);
        int v = max(max(dg + wgt, en), fin);
        v = max(v, zc + u * k.nge);
        if (VIRT && c0 + u == -1 && lbrd != kAffNeg) v = lbrd;
        const int hn = v + k.go;
        int fn = max(fin, hn);
        if (PARTIAL && dead) {
            v = upg;
            fn = fin;
        }
        // VIRT: columns < 0 are virtual and computed like real ones
        const bool act = MASK ? (VIRT ? (c0 + u < w) : ((unsigned)(c0 + u) < (unsigned)w)) : true;
        // branch-free masking: inactive lanes keep their state
        e = act ? en : e;
        g = act ? v : g;
        hg = act ? hn : hg;
        fdn = act ? fn : fdn;
        best = act ? max(best, v - (zb + u * k.nge)) : best;
        dg = upg;
        og[u] = g;
        of[u] = fdn;
    }
}


// Round-3 steady state (tools/gen_block_asm.py gen_aff2): blocks b .. be-1, kind
// L = X space (clamp / best) or G space, weights by LUT or compare.  pf: the first
// half of block b's top row is already in the TOP registers (never on entry from
// C++: 0).  Returns 0, or 1 on a spin timeout.
struct Aff2Args {
    uint32_t rb, nb, apr, acn, anp, anc, asf, atl, skb, lo, lid8, bvb, bvs, thr, neg;
    uint64_t gp;
    uint64_t sg;   // GS: the problem's subject-code rows (skb: the lane's byte offset at block 0)
    int q, wm, wx, ll, lh, zlp;
    int qb, llb, lhb, zlpb;   // rows per lane > 1: row 1's query code, LUT and clamp bound
    int qx, llx, lhx, zlpx;   // three rows per lane: row 2's
};
#ifdef ANYSEQ_STAMPS
#define AF2_NAME(NAME) NAME##_TS
#define AF2_TS_OUT , [ts] "+s"(ts_v), [te] "+s"(te_v), [tsf] "+s"(ts_f), [nmiss] "+s"(nmiss), [dbp] "+s"(dbp)
#else
#define AF2_NAME(NAME) NAME
#define AF2_TS_OUT
#endif
#define AF2_ASM(NAME)                                                                                           \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4) AF2_TS_OUT                                                                   \
                 : [be] "s"(be), [q] "v"(a.q), [wm] "v"(a.wm), [wx] "v"(a.wx), [ll] "v"(a.ll), [lh] "v"(a.lh),   \
                   [go] "v"(go), [ge] "s"(ge), [zlp] "v"(a.zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(a.apr),   \
                   [acn] "v"(a.acn), [anp] "v"(a.anp), [anc] "v"(a.anc), [asf] "v"(a.asf), [atl] "v"(a.atl),     \
                   [skb] "v"(a.skb), [lo] "v"(a.lo), [lid8] "v"(a.lid8), [bvb] "v"(a.bvb), [bvs] "s"(bvs),        \
                   [hm] "s"(hm), [gp] "s"(gp), [thr] "s"(thr), [sg] "s"(sg)                                    \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
// the band's last blocks (gen_aff2 epi): + the column-(w-1) capture and the poll clamp
#define AF2E_ASM(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4), [cnt] "+v"(cnt), [gc] "+v"(gc), [ec] "+v"(ec), [fc] "+v"(fc) AF2_TS_OUT     \
                 : [be] "s"(be), [q] "v"(a.q), [wm] "v"(a.wm), [wx] "v"(a.wx), [ll] "v"(a.ll), [lh] "v"(a.lh),   \
                   [go] "v"(go), [ge] "s"(ge), [zlp] "v"(a.zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(a.apr),   \
                   [acn] "v"(a.acn), [anp] "v"(a.anp), [anc] "v"(a.anc), [asf] "v"(a.asf), [atl] "v"(a.atl),     \
                   [skb] "v"(a.skb), [lo] "v"(a.lo), [lid8] "v"(a.lid8), [bvb] "v"(a.bvb), [bvs] "s"(bvs),        \
                   [hm] "s"(hm), [gp] "s"(gp), [nch] "s"(nch), [thr] "s"(thr), [sg] "s"(sg)                    \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
// the band's first blocks with the zero-open left border forced (gen_aff2 pro)
#define AF2P_ASM(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4), [pcnt] "+v"(pcnt) AF2_TS_OUT                                                \
                 : [be] "s"(be), [q] "v"(a.q), [wm] "v"(a.wm), [wx] "v"(a.wx), [ll] "v"(a.ll), [lh] "v"(a.lh),   \
                   [go] "v"(go), [ge] "s"(ge), [zlp] "v"(a.zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(a.apr),   \
                   [acn] "v"(a.acn), [anp] "v"(a.anp), [anc] "v"(a.anc), [asf] "v"(a.asf), [atl] "v"(a.atl),     \
                   [skb] "v"(a.skb), [lo] "v"(a.lo), [lid8] "v"(a.lid8), [bvb] "v"(a.bvb), [bvs] "s"(bvs),        \
                   [hm] "s"(hm), [gp] "s"(gp), [thr] "s"(thr), [sg] "s"(sg), [pbrd] "v"(pbrd)                  \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
// the band's last blocks without the column-(w-1) capture (gen_aff2 cap=False)
#define AF2F_ASM(NAME)                                                                                          \
    asm volatile(NAME                                                                                          \
                 : [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(e),  \
                   [hg] "+v"(hg), [best] "+v"(bx), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),     \
                   [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3), \
                   [x4] "=&s"(x4) AF2_TS_OUT                                                                   \
                 : [be] "s"(be), [q] "v"(a.q), [wm] "v"(a.wm), [wx] "v"(a.wx), [ll] "v"(a.ll), [lh] "v"(a.lh),   \
                   [go] "v"(go), [ge] "s"(ge), [zlp] "v"(a.zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(a.apr),   \
                   [acn] "v"(a.acn), [anp] "v"(a.anp), [anc] "v"(a.anc), [asf] "v"(a.asf), [atl] "v"(a.atl),     \
                   [skb] "v"(a.skb), [lo] "v"(a.lo), [lid8] "v"(a.lid8), [bvb] "v"(a.bvb), [bvs] "s"(bvs),        \
                   [hm] "s"(hm), [gp] "s"(gp), [nch] "s"(nch), [thr] "s"(thr), [neg] "s"(negp), [sg] "s"(sg)    \
                 : ANYSEQ_AF2_ASM_CLOBBERS, "memory")
// EPI: 0 the steady state, 1 the band's last blocks with the capture, 2 without it, 3 the
// band's first blocks with the zero-open left border forced (cap = {steps to column -1,
// the border in the loop's space}).  LIN: the linear loop (gen_aff2 lin: kinds N = G space,
// M = X space)
template <bool L, bool BORDER, int PUB, bool LUT, int EPI = 0, bool LIN = false>
__device__ __forceinline__ uint32_t aff2_loop_asm(uint32_t& b, uint32_t be, uint32_t& sp, uint32_t& sf, uint32_t& sc,
                                                  const Aff2Args& a, int go, int nge, int& g, int& fdn, int& dg,
                                                  int2& tf, int& e, int& hg, int& bx, uint64_t& ts_v, uint64_t& te_v,
                                                  uint32_t& ts_f, uint32_t& nmiss, uint32_t nch = 0, int* cap = nullptr,
                                                  uint64_t dbp = 0) {
    uint32_t st, x0, x1, x2, x3, x4, pf = 0;
    const uint64_t hm = 0xffff000000000000ull;   // lanes 48..63 (publishing)
#define RFL(x) __builtin_amdgcn_readfirstlane(x)
    b = RFL(b);
    sp = RFL(sp);
    sf = RFL(sf);
    sc = RFL(sc);
    be = RFL(be);
    const uint32_t rb = RFL(a.rb), nb = RFL(a.nb), bvs = RFL(a.bvs), thr = RFL(a.thr);
    const int ge = RFL(-nge);
    const uint64_t gp = ((uint64_t)(uint32_t)RFL((uint32_t)(a.gp >> 32)) << 32) | (uint32_t)RFL((uint32_t)a.gp);
    const uint64_t sg = ((uint64_t)(uint32_t)RFL((uint32_t)(a.sg >> 32)) << 32) | (uint32_t)RFL((uint32_t)a.sg);
#ifdef ANYSEQ_STAMPS
    ts_f = RFL(ts_f);
    nmiss = RFL(nmiss);
    dbp = ((uint64_t)(uint32_t)RFL((uint32_t)(dbp >> 32)) << 32) | (uint32_t)RFL((uint32_t)dbp);
    ts_v = ((uint64_t)(uint32_t)RFL((uint32_t)(ts_v >> 32)) << 32) | (uint32_t)RFL((uint32_t)ts_v);
    te_v = ((uint64_t)(uint32_t)RFL((uint32_t)(te_v >> 32)) << 32) | (uint32_t)RFL((uint32_t)te_v);
#else
    (void)ts_v, (void)te_v, (void)ts_f, (void)nmiss, (void)dbp;
#endif
#undef RFL
    int tfg = tf.x, tff = tf.y;
#define AF2_SEL(A, V, K, U)                                                                   \
    if constexpr (BORDER && PUB == 0) A(AF2_NAME(ANYSEQ_##V##_##K##_B1_NONE_U##U));          \
    if constexpr (BORDER && PUB == 1) A(AF2_NAME(ANYSEQ_##V##_##K##_B1_LDS_U##U));           \
    if constexpr (BORDER && PUB == 2) A(AF2_NAME(ANYSEQ_##V##_##K##_B1_GLOB_U##U));          \
    if constexpr (!BORDER && PUB == 0) A(AF2_NAME(ANYSEQ_##V##_##K##_B0_NONE_U##U));         \
    if constexpr (!BORDER && PUB == 1) A(AF2_NAME(ANYSEQ_##V##_##K##_B0_LDS_U##U));          \
    if constexpr (!BORDER && PUB == 2) A(AF2_NAME(ANYSEQ_##V##_##K##_B0_GLOB_U##U));
// (the linear loops have no diagnostic-stamp variants: their names stay plain)
#define AF2_SELN(A, V, K, U)                                                                  \
    if constexpr (BORDER && PUB == 0) A(ANYSEQ_##V##_##K##_B1_NONE_U##U);                    \
    if constexpr (BORDER && PUB == 1) A(ANYSEQ_##V##_##K##_B1_LDS_U##U);                     \
    if constexpr (BORDER && PUB == 2) A(ANYSEQ_##V##_##K##_B1_GLOB_U##U);                    \
    if constexpr (!BORDER && PUB == 0) A(ANYSEQ_##V##_##K##_B0_NONE_U##U);                   \
    if constexpr (!BORDER && PUB == 1) A(ANYSEQ_##V##_##K##_B0_LDS_U##U);                    \
    if constexpr (!BORDER && PUB == 2) A(ANYSEQ_##V##_##K##_B0_GLOB_U##U);
#define AF2_KINDS(A, V)                                          \
    if constexpr (!LIN && L && LUT) { AF2_SEL(A, V, L, 1) }       \
    if constexpr (!LIN && L && !LUT) { AF2_SEL(A, V, L, 0) }      \
    if constexpr (!LIN && !L && LUT) { AF2_SEL(A, V, G, 1) }      \
    if constexpr (!LIN && !L && !LUT) { AF2_SEL(A, V, G, 0) }     \
    if constexpr (LIN && L && LUT) { AF2_SELN(A, V, M, 1) }       \
    if constexpr (LIN && L && !LUT) { AF2_SELN(A, V, M, 0) }      \
    if constexpr (LIN && !L && LUT) { AF2_SELN(A, V, N, 1) }      \
    if constexpr (LIN && !L && !LUT) { AF2_SELN(A, V, N, 0) }
    if constexpr (EPI == 1) {
        nch = __builtin_amdgcn_readfirstlane(nch);
        int cnt = cap[0], gc = cap[1], ec = cap[2], fc = cap[3];
        AF2_KINDS(AF2E_ASM, AF2E)
        cap[0] = cnt, cap[1] = gc, cap[2] = ec, cap[3] = fc;
    } else if constexpr (EPI == 2) {
        nch = __builtin_amdgcn_readfirstlane(nch);
        const uint32_t negp = __builtin_amdgcn_readfirstlane(a.neg);
        (void)cap;
        AF2_KINDS(AF2F_ASM, AF2F)
    } else if constexpr (EPI == 3) {
        (void)nch;
        int pcnt = cap[0];
        const int pbrd = cap[1];
        if constexpr (!LIN && L && LUT) { AF2_SELN(AF2P_ASM, AF2P, L, 1) }
        if constexpr (!LIN && L && !LUT) { AF2_SELN(AF2P_ASM, AF2P, L, 0) }
        if constexpr (!LIN && !L && LUT) { AF2_SELN(AF2P_ASM, AF2P, G, 1) }
        if constexpr (!LIN && !L && !LUT) { AF2_SELN(AF2P_ASM, AF2P, G, 0) }
        if constexpr (LIN && L && LUT) { AF2_SELN(AF2P_ASM, AF2P, M, 1) }
        if constexpr (LIN && L && !LUT) { AF2_SELN(AF2P_ASM, AF2P, M, 0) }
        if constexpr (LIN && !L && LUT) { AF2_SELN(AF2P_ASM, AF2P, N, 1) }
        if constexpr (LIN && !L && !LUT) { AF2_SELN(AF2P_ASM, AF2P, N, 0) }
        cap[0] = pcnt;
    } else {
        (void)nch, (void)cap;
        AF2_KINDS(AF2_ASM, AF2)
    }
#undef AF2_KINDS
#undef AF2_SELN
#undef AF2_SEL
    tf = make_int2(tfg, tff);
    return st;
}
#undef AF2_ASM
#undef AF2E_ASM
#undef AF2F_ASM
#undef AF2P_ASM

// Two or three rows per lane (gen_aff2 nrows): the upper rows' state in gu / eu / hgu / bxu
// (row 0: %[ga] / %[e] / %[hg] / %[best], row 1 of three: %[gb] / %[eb] / %[hgb] / %[bestb]),
// the bottom row's in g / fdn (the lane-shifted cell, as one row's) and e / hg / bx (%[eb]..
// of two rows, %[ex].. of three).  No diagnostic-stamp variants.
#define AF2N_OUTS                                                                                              \
    [cur] "+v"(g), [fd] "+v"(fdn), [dg] "+v"(dg), [tfg] "+v"(tfg), [tff] "+v"(tff), [e] "+v"(eu[0]),           \
        [hg] "+v"(hgu[0]), [best] "+v"(bxu[0]), [b] "+s"(b), [sp] "+s"(sp), [sf] "+s"(sf), [sc] "+s"(sc),          \
        [pf] "+s"(pf), [st] "=&s"(st), [x0] "=&s"(x0), [x1] "=&s"(x1), [x2] "=&s"(x2), [x3] "=&s"(x3),            \
        [x4] "=&s"(x4), [ga] "+v"(gu[0])
#define AF2N_INS                                                                                               \
    [be] "s"(be), [q] "v"(a.q), [wm] "v"(a.wm), [wx] "v"(a.wx), [ll] "v"(a.ll), [lh] "v"(a.lh), [go] "v"(go),     \
        [ge] "s"(ge), [zlp] "v"(a.zlp), [rb] "s"(rb), [nb] "s"(nb), [apr] "v"(a.apr), [acn] "v"(a.acn),          \
        [anp] "v"(a.anp), [anc] "v"(a.anc), [asf] "v"(a.asf), [atl] "v"(a.atl), [skb] "v"(a.skb), [lo] "v"(a.lo),  \
        [lid8] "v"(a.lid8), [bvb] "v"(a.bvb), [bvs] "s"(bvs), [hm] "s"(hm), [gp] "s"(gp), [thr] "s"(thr),         \
        [sg] "s"(sg), [qb] "v"(a.qb), [llb] "v"(a.llb), [lhb] "v"(a.lhb), [zlpb] "v"(a.zlpb)
// two rows: row 1 is the bottom row
#define AF2R_OUTS AF2N_OUTS, [eb] "+v"(e), [hgb] "+v"(hg), [bestb] "+v"(bx)
#define AF2R_ASM(NAME) asm volatile(NAME : AF2R_OUTS : AF2N_INS : ANYSEQ_AF2R_ASM_CLOBBERS, "memory")
#define AF2RE_ASM(NAME)                                                                                   \
    asm volatile(NAME : AF2R_OUTS, [cnt] "+v"(cap[0]), [gc] "+v"(cap[1]), [ec] "+v"(cap[2]),               \
                 [gcb] "+v"(cap[3]), [ecb] "+v"(cap[4]), [fc] "+v"(cap[5]) : AF2N_INS, [nch] "s"(nch)      \
                 : ANYSEQ_AF2R_ASM_CLOBBERS, "memory")
#define AF2RF_ASM(NAME)                                                                                   \
    asm volatile(NAME : AF2R_OUTS : AF2N_INS, [nch] "s"(nch), [neg] "s"(negp) : ANYSEQ_AF2R_ASM_CLOBBERS, "memory")
// three rows: row 1 upper (gu[1] ..), row 2 the bottom row
#define AF2R3_OUTS                                                                                        \
    AF2N_OUTS, [gb] "+v"(gu[NU - 1]), [eb] "+v"(eu[NU - 1]), [hgb] "+v"(hgu[NU - 1]), [bestb] "+v"(bxu[NU - 1]), \
        [ex] "+v"(e), [hgx] "+v"(hg), [bestx] "+v"(bx)
#define AF2R3_INS AF2N_INS, [qx] "v"(a.qx), [llx] "v"(a.llx), [lhx] "v"(a.lhx), [zlpx] "v"(a.zlpx)
#define AF2R3_ASM(NAME) asm volatile(NAME : AF2R3_OUTS : AF2R3_INS : ANYSEQ_AF2R3_ASM_CLOBBERS, "memory")
#define AF2R3E_ASM(NAME)                                                                                  \
    asm volatile(NAME : AF2R3_OUTS, [cnt] "+v"(cap[0]), [gc] "+v"(cap[1]), [ec] "+v"(cap[2]),              \
                 [gcb] "+v"(cap[3]), [ecb] "+v"(cap[4]), [gcx] "+v"(cap[5]), [ecx] "+v"(cap[6]),           \
                 [fc] "+v"(cap[7]) : AF2R3_INS, [nch] "s"(nch) : ANYSEQ_AF2R3_ASM_CLOBBERS, "memory")
#define AF2R3F_ASM(NAME)                                                                                  \
    asm volatile(NAME : AF2R3_OUTS : AF2R3_INS, [nch] "s"(nch), [neg] "s"(negp) : ANYSEQ_AF2R3_ASM_CLOBBERS, "memory")
// EPI as aff2_loop_asm; cap = {cnt, then (g, e) of rows 0 .. RR-1, then the bottom row's F-down} (EPI 1)
template <int RR, bool L, bool BORDER, int PUB, bool LUT, int EPI = 0, int NU = RR - 1>
__device__ __forceinline__ uint32_t aff2n_loop_asm(uint32_t& b, uint32_t be, uint32_t& sp, uint32_t& sf, uint32_t& sc,
                                                   const Aff2Args& a, int go, int nge, int& g, int& fdn, int& dg,
                                                   int2& tf, int& e, int& hg, int& bx, int (&gu)[NU], int (&eu)[NU],
                                                   int (&hgu)[NU], int (&bxu)[NU], uint32_t nch = 0,
                                                   int* cap = nullptr) {
    static_assert(RR == 2 || RR == 3, "two or three rows per lane");
    uint32_t st, x0, x1, x2, x3, x4, pf = 0;
    const uint64_t hm = 0xffff000000000000ull;   // lanes 48..63 (publishing)
#define RFL(x) __builtin_amdgcn_readfirstlane(x)
    b = RFL(b);
    sp = RFL(sp);
    sf = RFL(sf);
    sc = RFL(sc);
    be = RFL(be);
    const uint32_t rb = RFL(a.rb), nb = RFL(a.nb), bvs = RFL(a.bvs), thr = RFL(a.thr);
    const int ge = RFL(-nge);
    const uint64_t gp = ((uint64_t)(uint32_t)RFL((uint32_t)(a.gp >> 32)) << 32) | (uint32_t)RFL((uint32_t)a.gp);
    const uint64_t sg = ((uint64_t)(uint32_t)RFL((uint32_t)(a.sg >> 32)) << 32) | (uint32_t)RFL((uint32_t)a.sg);
#undef RFL
    int tfg = tf.x, tff = tf.y;
#define AF2R_SEL(A, V, K, U)                                                          \
    if constexpr (BORDER && PUB == 0) A(ANYSEQ_##V##_##K##_B1_NONE_U##U);            \
    if constexpr (BORDER && PUB == 1) A(ANYSEQ_##V##_##K##_B1_LDS_U##U);             \
    if constexpr (BORDER && PUB == 2) A(ANYSEQ_##V##_##K##_B1_GLOB_U##U);            \
    if constexpr (!BORDER && PUB == 0) A(ANYSEQ_##V##_##K##_B0_NONE_U##U);           \
    if constexpr (!BORDER && PUB == 1) A(ANYSEQ_##V##_##K##_B0_LDS_U##U);            \
    if constexpr (!BORDER && PUB == 2) A(ANYSEQ_##V##_##K##_B0_GLOB_U##U);
#define AF2R_KINDS(A, V)                                  \
    if constexpr (L && LUT) { AF2R_SEL(A, V, L, 1) }      \
    if constexpr (L && !LUT) { AF2R_SEL(A, V, L, 0) }     \
    if constexpr (!L && LUT) { AF2R_SEL(A, V, G, 1) }     \
    if constexpr (!L && !LUT) { AF2R_SEL(A, V, G, 0) }
    if constexpr (EPI == 1) {
        nch = __builtin_amdgcn_readfirstlane(nch);
        if constexpr (RR == 2) { AF2R_KINDS(AF2RE_ASM, AF2RE) } else { AF2R_KINDS(AF2R3E_ASM, AF2R3E) }
    } else if constexpr (EPI == 2) {
        nch = __builtin_amdgcn_readfirstlane(nch);
        const uint32_t negp = __builtin_amdgcn_readfirstlane(a.neg);
        (void)cap;
        if constexpr (RR == 2) { AF2R_KINDS(AF2RF_ASM, AF2RF) } else { AF2R_KINDS(AF2R3F_ASM, AF2R3F) }
    } else {
        (void)nch, (void)cap;
        if constexpr (RR == 2) { AF2R_KINDS(AF2R_ASM, AF2R) } else { AF2R_KINDS(AF2R3_ASM, AF2R3) }
    }
#undef AF2R_KINDS
#undef AF2R_SEL
    tf = make_int2(tfg, tff);
    return st;
}
#undef AF2N_OUTS
#undef AF2N_INS
#undef AF2R_OUTS
#undef AF2R_ASM
#undef AF2RE_ASM
#undef AF2RF_ASM
#undef AF2R3_OUTS
#undef AF2R3_INS
#undef AF2R3_ASM
#undef AF2R3E_ASM
#undef AF2R3F_ASM

// RR rows per lane (2 or 3): aff_block for rows RR l .. RR l + RR-1 of a 64 RR-row band
// at the same column (the lane's column c0 + u at step u).  Row 0 takes its up / F-in
// from the bottom row of the lane above (DPP, lane 0: the top row); row i > 0 its diagonal
// from row i-1's previous cell, its up and F-in from row i-1's new cell.  The upper rows'
// state in gu / eu / hgu / bestu, the bottom row's in g / e / hg / fdn / best; og / of:
// the bottom row's (the band's bottom row at lane 63).  zc0 / zb0: row 0's clamp bound /
// true Z of the first step (row i's are i (-ge) further).  PARTIAL: a dead row passes the
// row above through.
template <int RR, bool MASK, bool PARTIAL, bool VIRT, int NU = RR - 1>
__device__ __forceinline__ void aff_blockn(int c0, int w, int2 tf, const int2 (&rv)[32], const uint32_t (&sw)[8],
                                           const int (&qu)[NU], int q, const bool (&deadu)[NU], bool dead, int zc0,
                                           int zb0, int (&gu)[NU], int (&eu)[NU], int (&hgu)[NU], int& dg, int& g,
                                           int& e, int& hg, int& fdn, int (&bestu)[NU], int& best, int (&og)[32],
                                           int (&of)[32], const AffK k) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
        const int2 top = u == 0 ? tf : rv[u - 1];
        const int upg = wave_shr1(top.x, g);
        const int fin = wave_shr1(top.y, fdn);
        const bool vcol = VIRT && c0 + u < 0;
        const int sb = (int)((sw[u >> 2] >> (8 * (u & 3))) & 0xffu);
        const int zu = zc0 + u * k.nge, zt = zb0 + u * k.nge;
        const bool act = MASK ? (VIRT ? (c0 + u < w) : ((unsigned)(c0 + u) < (unsigned)w)) : true;
        int dgi = dg, upi = upg, fi = fin;   // row i's diagonal, up, F-in
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int wi = vcol ? kAffNeg : (qu[i] == sb ? k.wm : k.wx);
            const int en = max(eu[i], hgu[i]);
            int v = max(max(max(dgi + wi, en), fi), zu + i * k.nge);
            const int hn = v + k.go;
            int fn = max(fi, hn);
            if (PARTIAL && deadu[i]) {
                v = upi;
                fn = fi;
            }
            dgi = gu[i];   // the next row's diagonal: this row's previous cell
            eu[i] = act ? en : eu[i];
            gu[i] = act ? v : gu[i];
            hgu[i] = act ? hn : hgu[i];
            bestu[i] = act ? max(bestu[i], v - (zt + i * k.nge)) : bestu[i];
            upi = v;
            fi = fn;
        }
        const int wb = vcol ? kAffNeg : (q == sb ? k.wm : k.wx);
        const int enb = max(e, hg);
        int vb = max(max(max(dgi + wb, enb), fi), zu + NU * k.nge);
        const int hnb = vb + k.go;
        int fnb = max(fi, hnb);
        if (PARTIAL && dead) {
            vb = upi;
            fnb = fi;
        }
        e = act ? enb : e;
        g = act ? vb : g;
        hg = act ? hnb : hg;
        fdn = act ? fnb : fdn;
        best = act ? max(best, vb - (zt + NU * k.nge)) : best;
        dg = upg;
        og[u] = g;
        of[u] = fdn;
    }
}

// RR: rows per lane.  RR 2 / 3 (round 5): lane l holds rows RR l .. RR l + RR-1 of a
// 64 RR-row band at the same column (aff_blockn, gen_aff2 nrows); `row`, g / e / hg / fdn
// are the lane's bottom row, gu / eu / hgu / bestu its upper rows (row rowt + i), dg row
// 0's diagonal.  The hand-off rows, rings and steps are the one-row band's.
template <bool PARTIAL, int RR>
__device__ __forceinline__ void run_band_aff(const DPProblem& P, int band, int lane, const AffIO& io, uint32_t* err, const AffK k,
                             unsigned long long* dbg) {
    static_assert(RR >= 1 && RR <= 3, "one to three rows per lane");
    constexpr int NU = RR > 1 ? RR - 1 : 1;   // upper rows (unused for RR 1)
    constexpr int CH = 32;
    constexpr int IRM = kSlots * CH - 1;
    constexpr int LAG = 2;   // lane 63 finishes column c at step c + 64: chunk j is complete after block j + 2
    const int h = P.h, w = P.w, go = k.go, nge = k.nge;
    const int bm = __builtin_amdgcn_readfirstlane(P.bmode);
    const int amode = __builtin_amdgcn_readfirstlane(P.amode);
    const bool clamp = amode & 1;
    const int bestmode = (amode >> 1) & 3;
    const AffBorder B(bm, go);
    // X space: a problem with the clamp or a best-cell output runs its
    // asm steady state in X = H + (r+2)|ge| (a per-row shift: the clamp bound is a
    // per-lane constant folded into E, the best cell is max X).  Its rings, hand-off
    // rows and out_row hold X values; the C++ blocks compute in G space (X + c|ge|) and
    // convert what they read and publish.
    const bool xs = amode != 0;
    auto to_g = [nge](int v, int c) { return v + c * nge; };
    auto to_x = [nge](int v, int c) { return v - c * nge; };
    // column-block shard: the left border column (H and E of column
    // -1, H space, sender's frame + left_shift) arrives from the neighbour shard;
    // such a band runs the masked C++ prologue on the received values
    const bool shard_left = P.left_in != nullptr;
    // Virtual prologue: lanes left of column 0 compute virtual cells from "minus
    // infinity" states (subject code 0xFF there matches nothing), and lane 0's top value
    // at column -1 is the left border of the row above, so column -1 reproduces the
    // border: NORMAL / FPAID a vertical gap paid from the corner, FFREE a continuing
    // one, FREE_LOCAL zeros by the clamp, the -inf borders -inf.  Not for a zero left
    // border without clamp (FREE_SEMI_OPEN / _T), nor where a finite border cell could
    // win a last-row best (the border is no candidate there).
    constexpr bool ASM_OK = !PARTIAL;
    const bool zero_open = bm == BM_FREE_SEMI_OPEN || bm == BM_FREE_SEMI_T;
    const bool finite_left = bm == BM_NORMAL || bm == BM_FFREE || bm == BM_FPAID;
    // A best of every cell without the clamp takes the virtual cells too: those left of
    // column -1 are "minus infinity", column -1 is the border.  It cannot win where the
    // left border is -inf, nor under NORMAL when min(match, mismatch) >= go + ge (flags
    // bit 4, set by the host): then cell (0,0) >= the largest border cell go + ge.
    const bool best_border_ok = !(bestmode == 1 && !clamp) || !finite_left || (bm == BM_NORMAL && (k.flags & 16));
    // Under the clamp the virtual cells are clamped to H = 0, so a diagonal step into
    // them must not gain: code 0xFF's weight is -1 (X space) in the LUT, but the compare
    // weights give it the mismatch -- a positive mismatch would lift column -1 above the
    // local left border (round 5: local scores too high with > 8 symbols and mismatch > 0)
    const bool ff_loses = k.lut || k.wx <= 2 * nge;
    // A zero-open left border (semiglobal) is forced at column -1 instead: the asm
    // prologue variant (gen_aff2 pro) and the C++ blocks' lbrd (one row per lane; round 5)
    // (not with a best of the last row or of every cell: the forced border cell, H = 0, would
    // become a candidate the C++ path never offers)
    const bool force_lb = zero_open && RR == 1 && !(k.flags & 512) && (bestmode == 0 || bestmode == 3);
    const bool virt = ASM_OK && !shard_left && (!zero_open || force_lb) && !(bestmode == 2 && finite_left) &&
                      best_border_ok && (!clamp || (k.codes && ff_loses)) && !(k.flags & 1);
    const int rb = band * 64 * RR;
    const int row = rb + RR * lane + (RR - 1);   // the lane's bottom row
    const int rowt = row - (RR - 1);             // its top row
    const bool dead = row >= h;
    const bool lastrow = row == h - 1;
    int q = dead ? 0x100 : (int)gmem(P.q)[P.q_off + P.q_step * row];
    int qu[NU];
    bool deadu[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        deadu[i] = RR == 1 || rowt + i >= h;
        qu[i] = deadu[i] ? 0x100 : (int)gmem(P.q)[P.q_off + P.q_step * (rowt + i)];
    }
    // settle the query loads here: a vmcnt wait inside the step loop would also wait
    // for lane 63's HBM row stores
    if constexpr (NU > 1)
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(q), "+v"(qu[0]), "+v"(qu[1])::"memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(q), "+v"(qu[0])::"memory");
    if (kAffGS && !P.scode) {   // (a planned level whose code rows did not fit: its bound check fails too)
        if (lane == 0) atomicOr(err, ERR_BAD_DESC);
        return;
    }
    int g, e = kAffNeg, hg, fdn = kAffNeg, dg;
    int gu[NU], eu[NU], hgu[NU];   // RR > 1: the upper rows
#pragma unroll
    for (int i = 0; i < NU; ++i) gu[i] = eu[i] = hgu[i] = kAffNeg;
    int2 tf;
    if (shard_left) {
        int32_t lh1 = 0, lh0 = 0, le1 = 0;
        if constexpr (RR > 1) {
            // row 0 first (waits for the band's 64 RR rows), then the rows below (landed)
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                int32_t a1 = 0, a0 = 0, ae = 0;
                if (!poll_left(P, rowt + i, a1, a0, err, 64 * RR - i)) return;
                if (!poll_left_e(P, rowt + i, ae, err)) return;
                gu[i] = a1 + (rowt + i + 1) * nge;
                eu[i] = ae + (rowt + i + 1) * nge;
                hgu[i] = gu[i] + go;
                if (i == 0) lh0 = a0;
            }
        }
        int32_t l0 = 0;
        if (!poll_left(P, row, lh1, l0, err, 64 * RR - (RR - 1))) return;
        if constexpr (RR == 1) lh0 = l0;
        if (!poll_left_e(P, row, le1, err)) return;
        // H space -> G space at column -1: G = H + (r + 1) (-ge); row -1 is the top
        // border of the shard frame (the scheme's: global go, free 0)
        g = lh1 + (row + 1) * nge;
        e = le1 + (row + 1) * nge;
        hg = g + go;
        dg = rowt == 0 ? (bm == BM_NORMAL ? go : 0) : lh0 + rowt * nge;
        tf = make_int2(__shfl(dg, 0), kAffNeg);
    } else if (virt) {
        g = kAffNeg;
        hg = kAffNeg;
        dg = kAffNeg;
        // (G, F-down) of the left border cell of row rb-1 (the corner for rb = 0)
        const int tg = B.left(rb - 1, nge);
        const int tff = (bm == BM_NORMAL || bm == BM_FPAID) ? (rb == 0 ? B.cg + go : go)
                        : bm == BM_FFREE ? 0 : bm == BM_FREE_LOCAL ? tg + go : kAffNeg;
        tf = make_int2(tg, bm == BM_FPAID && rb == 0 ? go : tff);
    } else {
        g = B.left(row, nge);
        hg = g + go;   // the next column's E candidate: G[r][-1] + go
        dg = B.left(rowt - 1, nge);
        tf = make_int2(B.left(rb - 1, nge), kAffNeg);
        if constexpr (RR > 1) {
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                gu[i] = B.left(rowt + i, nge);   // (also row i+1's diagonal at column 0)
                hgu[i] = gu[i] + go;
            }
        }
    }
    int best = kAffNeg, bestu[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) bestu[i] = kAffNeg;
    const int nchunks = (w + CH - 1) / CH;
    const int nblocks = nchunks + LAG;
    const int fe = w >= CH - 1 ? (w - (CH - 1)) / CH + 1 : 0;   // full blocks: 32b + 30 < w
    uint32_t seen_prod = 0, seen_sfill = 0, seen_cons = 0;
    // self-forwarding first band (no I/O wave): asm segments of kFwdSeg blocks, the ring
    // brought up to the segment's end before each
    const bool self_fwd = io.g_in != nullptr;
    constexpr int kFwdSeg = kSlots - 4;
    SelfFwd fw;
    uint64_t ts_v = 0, te_v = 0;   // diagnostic build: steady-state start / end (s_memrealtime)
    uint32_t ts_f = 0, nmiss = 0;  // diagnostic build: + hand-off waits
    // diagnostic build: hand-off event record of the band (tools/probes/_aff_timeline.py)
    const uint64_t dbp = dbg && band < 2048 ? (uint64_t)(size_t)(dbg + 16 + 4 * 4096 + 16 * (band + (P.q_step < 0 ? 2048 : 0))) : 0;
#ifdef ANYSEQ_STAMPS
    auto ev_store = [&](int slot, uint64_t v) {
        if (dbp && lane == 0) reinterpret_cast<unsigned long long*>(dbp)[slot] = v;
    };
#endif
#ifdef ANYSEQ_STAMPS
    uint64_t t_b0 = 0;             // diagnostic build: C++ block 0 start
    // diagnostic build: shader clock and 100 MHz time at the band's start and end (clock per band)
    const uint64_t ck_mt0 = __builtin_amdgcn_s_memtime(), ck_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // clamp bound far below any cell when the problem does not clamp
    const int zoff = clamp ? 0 : 2 * kAffNeg;
    // asm epilogue (the blocks past column w-1, whose cells feed no real cell): needs
    // codes (0xFF beyond w) and not a last-row best (the last row's cells are read per
    // column); the loop's best takes real cells only
    const bool epi = k.codes && !(k.flags & 3) && bestmode != 2 && !(k.flags & (bestmode == 1 ? 4 : 8));
    // gap open 0: the linear loop (one row per lane; its band end keeps no exact E for out_col_e)
    const bool lin = RR == 1 && k.lin && !P.out_col_e;
    Aff2Args la;
    if constexpr (ASM_OK) {
        la.rb = lds_addr(io.my_ring);
        la.nb = io.out_lds ? lds_addr(io.next_ring) : 0u;
        la.apr = lds_addr(io.my_prod);
        la.acn = lds_addr(io.my_cons);
        la.anp = io.out_lds ? lds_addr(io.next_prod) : 0u;
        la.anc = io.out_lds ? lds_addr(io.next_cons) : 0u;
        la.asf = lds_addr(io.s_filled);
        la.atl = lds_addr(io.tail);
        la.skb = lds_addr(io.skew) + 4u * lane;
        la.lo = 8u * (lane - 48);   // publishing lanes 48..63: 16 columns each half block
        la.lid8 = 8u * lane;
        la.thr = (uint32_t)max(k.thr, 0);   // band 0's pace (FillParams::throttle)
        la.neg = lds_addr(io.neg);
        if constexpr (kAffGS) {
            // the lane's 32 codes of block b: columns 32b-1-lane .. 32b+30-lane, i.e. row
            // bytes i .. i+31 with i = 32b + 63 - lane, from the copy shifted by i & 3
            const int i0 = 63 - lane, r = i0 & 3;
            la.skb = (uint32_t)(r * scode_len(w) + (i0 - r));
            la.sg = (uint64_t)(size_t)P.scode;
        } else {
            la.sg = 0;
        }
        // band 0's top border (value, value + go) in the loop's space
        la.bvb = (uint32_t)(xs ? to_x(B.top(lane, nge), lane) : B.top(lane, nge));
        la.bvs = (uint32_t)(B.top(1, nge) - B.top(0, nge) - (xs ? nge : 0));
        la.gp = (uint64_t)(size_t)io.gout;
        // diagonal weights in the loop's space: G adds sub - 2 ge, X adds sub - ge
        const int wm = xs ? k.wm - nge : k.wm, wx = xs ? k.wx - nge : k.wx;
        la.wm = wm;
        la.wx = wx;
        // per row: the query code, its LUT (weights against subject codes 0..7) and the
        // X-space clamp bound - ge (RR 2: %[q] / %[ll] / %[lh] / %[zlp] row A's)
        auto row_consts = [&](int qr, int r, int& qo, int& llo, int& lho, int& zo) {
            uint32_t ll = 0, lh = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                ll |= (uint32_t)((qr == c ? wm : wx) & 0xff) << (8 * c);
                lh |= (uint32_t)((qr == c + 4 ? wm : wx) & 0xff) << (8 * c);
            }
            qo = qr;
            llo = (int)ll;
            lho = (int)lh;
            zo = clamp ? (r + 3) * nge : 2 * kAffNeg;
        };
        row_consts(RR == 1 ? q : qu[0], rowt, la.q, la.ll, la.lh, la.zlp);
        if constexpr (RR == 2) row_consts(q, row, la.qb, la.llb, la.lhb, la.zlpb);
        if constexpr (RR == 3) {
            row_consts(qu[NU - 1], rowt + 1, la.qb, la.llb, la.lhb, la.zlpb);
            row_consts(q, row, la.qx, la.llx, la.lhx, la.zlpx);
        }
    }
    for (int b = 0; b < nblocks; ++b) {
        const int t0 = b * CH;
        if constexpr (ASM_OK) {
            // (a forced left border needs both prologue blocks in the forcing loop: with fewer
            // full blocks the band's first blocks stay in C++, where lbrd forces it)
            if ((virt || t0 >= 64) && b < fe && !(k.flags & 1) && !(force_lb && b < 2 && fe < 2)) {
                // self-forwarding: the fused end once the band's remaining chunks fit the ring,
                // else a main-loop segment of kFwdSeg blocks
                // (a zero-open left border: its first two blocks in the forcing prologue variant)
                const bool pro = force_lb && b < 2;
                const bool fwd_end = !pro && (!self_fwd || nblocks - b <= kFwdSeg + 1);
                const int seg_end = pro ? min(2, fe) : self_fwd ? min(fe, b + kFwdSeg) : fe;
                if (self_fwd && !fw.forward_to(io, lane, w, b, fwd_end ? nchunks : seg_end, err)) return;
                // one block of slack: block b starts once chunk b+1 is published, so in the
                // steady state the loop's poll (step 16) already sees the next chunk and
                // prefetches its top row -- no wait on the band chain's critical path
                // (without slack the loop's own block-start poll waits for the same half
                // 2b: entering it right away overlaps the conversions and the loop's
                // prologue with that wait -- round 4)
                const int slk = k.slack + (io.io_fed ? k.slack_io : 0);
                if (!io.in_border && (slk > 0 || (k.flags & 64))) {
                    const uint32_t need = (uint32_t)min(2 * b + 1 + slk, 2 * nchunks);
                    if (seen_prod < need && !(seen_prod = spin_lds_ge(io.my_prod, need, err))) return;
                }
                // state into the loop's space: the lane's cell of step t0-1 is column t0-2-lane
                const int cs = t0 - 2 - lane;
                int bx = kAffNeg;
                int bxu[NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) bxu[i] = kAffNeg;
                if (xs) {
                    g = to_x(g, cs);
                    hg = to_x(hg, cs);
                    e = to_x(e, cs);
                    fdn = to_x(fdn, cs);
                    dg = to_x(dg, cs);
                    tf = make_int2(to_x(tf.x, t0 - 1), to_x(tf.y, t0 - 1));
                    if constexpr (RR > 1) {
#pragma unroll
                        for (int i = 0; i < NU; ++i) {
                            gu[i] = to_x(gu[i], cs);
                            hgu[i] = to_x(hgu[i], cs);
                            eu[i] = to_x(eu[i], cs);
                        }
                    }
                }
                uint32_t bb = (uint32_t)b;
                const int role = (io.in_border ? 3 : 0) + (io.out_lds ? 1 : (io.gout ? 2 : 0));
                uint32_t st = 0;
#define AF2_ROLES(LV, LU)                          \
    switch (role) {                                \
        case 0: AF2_CALL(LV, false, 0, LU); break; \
        case 1: AF2_CALL(LV, false, 1, LU); break; \
        case 2: AF2_CALL(LV, false, 2, LU); break; \
        case 3: AF2_CALL(LV, true, 0, LU); break;  \
        case 4: AF2_CALL(LV, true, 1, LU); break;  \
        default: AF2_CALL(LV, true, 2, LU); break; \
    }
                // A band whose column-(w-1) state nobody reads (no out_col / out_col_e,
                // last-row F or last-column best: the transposed Hirschberg halves, the
                // score fronts) runs its last blocks in the same loop as the rest -- the
                // capture-free epilogue variant (gen_aff2 cap=False), whose polls stop at
                // the last half -- so there is no transition between two loops, and no
                // capture work, on the band chain at the band's end (round 4)
                // A best of every cell takes the cells past w too.
                // They never exceed the best real cell when (1) a diagonal step past w never
                // gains -- the LUT's weight of code 0xFF is -1 in X space (H - 1 - |ge|),
                // the compare's is the mismatch -- (2) the top row past w is cells of the
                // band above, or "minus infinity" (the I/O wave's pad past the last granule,
                // the masked top row past the last chunk), and (3) band 0's top border past
                // w cannot seed a winner: -inf, or the free border under the clamp (H = 0,
                // every real cell >= 0).  Else the capturing end (best over real cells).
                const bool top_safe = !io.in_border || (B.tfree ? clamp : B.tg == kAffNeg);
                const bool best_safe = bestmode == 0 || (bestmode == 1 && ff_loses && top_safe);
                const bool need_cap = P.out_col || P.out_col_e || P.out_f_last || !best_safe || (k.flags & 32);
                if (epi && !need_cap && fwd_end) {   // (never in the prologue: fwd_end is false there)
#define AF2_CALL(LV, BD, PB, LU)                                                                                  \
    if constexpr (RR > 1)                                                                                         \
        st = aff2n_loop_asm<RR, LV, BD, PB, LU, 2>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, \
                                                   nge, g, fdn, dg, tf, e, hg, bx, gu, eu, hgu, bxu,             \
                                                   (uint32_t)(2 * nchunks));                                     \
    else if (lin)                                                                                                 \
        st = aff2_loop_asm<LV, BD, PB, LU, 2, true>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, \
                                                    nge, g, fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss,        \
                                                    (uint32_t)(2 * nchunks), nullptr, dbp);                         \
    else                                                                                                          \
        st = aff2_loop_asm<LV, BD, PB, LU, 2>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, nge, g, \
                                              fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, (uint32_t)(2 * nchunks), \
                                              nullptr, dbp)
                    if (xs) {
                        if (k.lut) { AF2_ROLES(true, true) } else { AF2_ROLES(true, false) }
                    } else {
                        if (k.lut) { AF2_ROLES(false, true) } else { AF2_ROLES(false, false) }
                    }
#undef AF2_CALL
                    if (st) {
                        atomicOr(err, ERR_SPIN_TIMEOUT);
                        return;
                    }
                    if (xs) {
                        best = max(best, bx - (row + 2) * nge);
#pragma unroll
                        for (int i = 0; i < NU; ++i) bestu[i] = max(bestu[i], bxu[i] - (rowt + i + 2) * nge);
                    }
                    break;   // band done (g / e / fdn: nobody reads them)
                }
                // (the forcing prologue: steps until the lane's column -1, the border there)
                int pcap[2] = {lane - t0, xs ? to_x(B.left(row, nge), -1) : B.left(row, nge)};
#define AF2_CALL(LV, BD, PB, LU)                                                                               \
    if constexpr (RR > 1)                                                                                      \
        st = aff2n_loop_asm<RR, LV, BD, PB, LU>(bb, (uint32_t)seg_end, seen_prod, seen_sfill, seen_cons, la, go, \
                                                nge, g, fdn, dg, tf, e, hg, bx, gu, eu, hgu, bxu);               \
    else if (pro && lin)                                                                                       \
        st = aff2_loop_asm<LV, BD, PB, LU, 3, true>(bb, (uint32_t)seg_end, seen_prod, seen_sfill, seen_cons, la, go, \
                                                    nge, g, fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, 0u,     \
                                                    pcap, dbp);                                                      \
    else if (pro)                                                                                              \
        st = aff2_loop_asm<LV, BD, PB, LU, 3>(bb, (uint32_t)seg_end, seen_prod, seen_sfill, seen_cons, la, go, nge, \
                                              g, fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, 0u, pcap, dbp);  \
    else if (lin)                                                                                              \
        st = aff2_loop_asm<LV, BD, PB, LU, 0, true>(bb, (uint32_t)seg_end, seen_prod, seen_sfill, seen_cons, la, go, \
                                                    nge, g, fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, 0u,     \
                                                    nullptr, dbp);                                                   \
    else                                                                                                       \
        st = aff2_loop_asm<LV, BD, PB, LU>(bb, (uint32_t)seg_end, seen_prod, seen_sfill, seen_cons, la, go, nge, g, \
                                           fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, 0u, nullptr, dbp)
                if (xs) {
                    if (k.lut) { AF2_ROLES(true, true) } else { AF2_ROLES(true, false) }
                } else {
                    if (k.lut) { AF2_ROLES(false, true) } else { AF2_ROLES(false, false) }
                }
#undef AF2_CALL
                if (!st && epi && (int)bb >= fe) {
                    // the band's last blocks in the loop too: every lane runs on past column
                    // w-1 (subject code 0xFF there) and keeps its column-(w-1) state
                    if (self_fwd && !fw.forward_to(io, lane, w, (int)bb, nchunks, err)) return;
#ifdef ANYSEQ_STAMPS
                    ev_store(7, te_v);                               // main loop end
                    ev_store(8, __builtin_amdgcn_s_memrealtime());   // epilogue entry
#endif
                    // steps until column w-1, then the state kept there: (g, e) of rows 0 .. RR-1, the
                    // bottom row's F-down
                    int cap[2 * RR + 2];
                    cap[0] = w + lane - (int)bb * CH;
#pragma unroll
                    for (int i = 0; i < RR - 1; ++i) {
                        cap[1 + 2 * i] = gu[i];
                        cap[2 + 2 * i] = eu[i];
                    }
                    cap[2 * RR - 1] = g;
                    cap[2 * RR] = e;
                    cap[2 * RR + 1] = fdn;
#define AF2_CALL(LV, BD, PB, LU)                                                                               \
    if constexpr (RR > 1)                                                                                      \
        st = aff2n_loop_asm<RR, LV, BD, PB, LU, 1>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, \
                                                   nge, g, fdn, dg, tf, e, hg, bx, gu, eu, hgu, bxu,             \
                                                   (uint32_t)(2 * nchunks), cap);                                \
    else if (lin)                                                                                              \
        st = aff2_loop_asm<LV, BD, PB, LU, 1, true>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, \
                                                    nge, g, fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss,        \
                                                    (uint32_t)(2 * nchunks), cap, dbp);                             \
    else                                                                                                       \
        st = aff2_loop_asm<LV, BD, PB, LU, 1>(bb, (uint32_t)nblocks, seen_prod, seen_sfill, seen_cons, la, go, nge, g, \
                                              fdn, dg, tf, e, hg, bx, ts_v, te_v, ts_f, nmiss, (uint32_t)(2 * nchunks), \
                                              cap, dbp)
                    if (xs) {
                        if (k.lut) { AF2_ROLES(true, true) } else { AF2_ROLES(true, false) }
                    } else {
                        if (k.lut) { AF2_ROLES(false, true) } else { AF2_ROLES(false, false) }
                    }
#undef AF2_CALL
                    if (st) {
                        atomicOr(err, ERR_SPIN_TIMEOUT);
                        return;
                    }
#ifdef ANYSEQ_STAMPS
                    ev_store(9, te_v);   // epilogue end
#endif
#pragma unroll
                    for (int i = 0; i < RR - 1; ++i) {
                        gu[i] = cap[1 + 2 * i];
                        eu[i] = cap[2 + 2 * i];
                    }
                    g = cap[2 * RR - 1];
                    e = cap[2 * RR];
                    fdn = cap[2 * RR + 1];
                    if (xs) {
                        g = to_g(g, w - 1);
                        e = to_g(e, w - 1);
                        fdn = to_g(fdn, w - 1);
                        best = max(best, bx - (row + 2) * nge);
#pragma unroll
                        for (int i = 0; i < RR - 1; ++i) {
                            gu[i] = to_g(gu[i], w - 1);
                            eu[i] = to_g(eu[i], w - 1);
                            bestu[i] = max(bestu[i], bxu[i] - (rowt + i + 2) * nge);
                        }
                    }
                    break;   // band done
                }
#undef AF2_ROLES
                if (st) {
                    atomicOr(err, ERR_SPIN_TIMEOUT);
                    return;
                }
                // back to G space for the C++ epilogue; the loop's best (X) to H
                const int t1 = (int)bb * CH, ce = t1 - 2 - lane;
                if (xs) {
                    g = to_g(g, ce);
                    hg = to_g(hg, ce);
                    e = to_g(e, ce);
                    fdn = to_g(fdn, ce);
                    dg = to_g(dg, ce);
                    tf = make_int2(to_g(tf.x, t1 - 1), to_g(tf.y, t1 - 1));
                    best = max(best, bx - (row + 2) * nge);
#pragma unroll
                    for (int i = 0; i < RR - 1; ++i) {
                        gu[i] = to_g(gu[i], ce);
                        hgu[i] = to_g(hgu[i], ce);
                        eu[i] = to_g(eu[i], ce);
                        bestu[i] = max(bestu[i], bxu[i] - (rowt + i + 2) * nge);
                    }
                }
                b = (int)bb - 1;   // ++b of the for
                continue;
            }
        }
        uint32_t sw[8];
        if constexpr (kAffGS) {
            const int i0 = t0 + 63 - lane, r = i0 & 3;
            const GLOBAL_AS uint32_t* src =
                reinterpret_cast<const GLOBAL_AS uint32_t*>(gmem(P.scode) + r * scode_len(w) + (i0 - r));
#pragma unroll
            for (int i = 0; i < 8; ++i) sw[i] = src[i];
        } else {
            if (b < nchunks && seen_sfill < (uint32_t)(b + 1)) {
                if (!(seen_sfill = spin_lds_ge(io.s_filled, (uint32_t)(b + 1), err))) return;
            }
            load_sbytes<CH>(io.s_ring, (t0 - 1 - lane) & (kSRing - 1), sw);
        }
        int2 rv[CH];
        if (b < nchunks) {
            if (io.in_border) {
                const int bv = B.top(t0 + lane, nge);
                const int bvr = xs ? to_x(bv, t0 + lane) : bv;   // rings hold the loop's space
                io.my_ring[(t0 + lane) & IRM] = make_int2(bvr, bvr + go);
            } else if (seen_prod < (uint32_t)(2 * b + 2)) {
                if (self_fwd && !fw.forward_to(io, lane, w, b, b + 4, err)) return;
                if (!(seen_prod = spin_lds_ge(io.my_prod, (uint32_t)(2 * b + 2), err))) return;
            }
            const int4* src = reinterpret_cast<const int4*>(io.my_ring + (t0 & IRM));
#pragma unroll
            for (int i = 0; i < CH / 2; ++i) {
                const int4 v = src[i];
                rv[2 * i] = make_int2(v.x, v.y);
                rv[2 * i + 1] = make_int2(v.z, v.w);
            }
            if (xs) {
#pragma unroll
                for (int u = 0; u < CH; ++u) rv[u] = make_int2(to_g(rv[u].x, t0 + u), to_g(rv[u].y, t0 + u));
            }
        } else {
#pragma unroll
            for (int i = 0; i < CH; ++i) rv[i] = make_int2(kAffNeg, kAffNeg);
        }
        const int j = b - LAG;
        const bool pub = io.out_lds && j >= 0;
        if (pub) {
            const uint32_t need = (uint32_t)max(0, j - kSlots + 1);
            if (seen_cons < need) {
                if (!(seen_cons = spin_lds_ge(io.next_cons, need, err))) return;
            }
        }
        int og[CH], of[CH];
#ifdef ANYSEQ_STAMPS
        if (b == 0) t_b0 = __builtin_amdgcn_s_memrealtime();   // block 0's inputs are ready
#endif
        const int c0 = t0 - 1 - lane;
        // Z of the lane's first step (row 0): (r + c + 2)(-ge), r + c = rb + t0 - 1 + (RR-1) lane
        const int zb = (rb + t0 + 1 + (RR - 1) * lane) * nge;
        const int zc = zb + zoff;
        const bool full = (virt || t0 >= 64) && b < fe;
        if constexpr (RR > 1) {
            if (full) {
                if (virt)
                    aff_blockn<RR, false, PARTIAL, true>(c0, w, tf, rv, sw, qu, q, deadu, dead, zc, zb, gu, eu, hgu, dg,
                                                         g, e, hg, fdn, bestu, best, og, of, k);
                else
                    aff_blockn<RR, false, PARTIAL, false>(c0, w, tf, rv, sw, qu, q, deadu, dead, zc, zb, gu, eu, hgu,
                                                          dg, g, e, hg, fdn, bestu, best, og, of, k);
            } else if (virt) {
                aff_blockn<RR, true, PARTIAL, true>(c0, w, tf, rv, sw, qu, q, deadu, dead, zc, zb, gu, eu, hgu, dg, g,
                                                    e, hg, fdn, bestu, best, og, of, k);
            } else {
                aff_blockn<RR, true, PARTIAL, false>(c0, w, tf, rv, sw, qu, q, deadu, dead, zc, zb, gu, eu, hgu, dg, g,
                                                     e, hg, fdn, bestu, best, og, of, k);
            }
        } else if (full) {
            if (virt)
                aff_block<false, PARTIAL, true>(c0, w, tf, rv, sw, q, dead, zc, zb, g, e, hg, fdn,
                                                        dg, best, og, of, k, force_lb ? B.left(row, nge) : kAffNeg);
            else
                aff_block<false, PARTIAL, false>(c0, w, tf, rv, sw, q, dead, zc, zb, g, e, hg, fdn,
                                                         dg, best, og, of, k);
        } else if (virt) {
            aff_block<true, PARTIAL, true>(c0, w, tf, rv, sw, q, dead, zc, zb, g, e, hg, fdn, dg,
                                                   best, og, of, k, force_lb ? B.left(row, nge) : kAffNeg);
        } else {   // masked prologue / epilogue (also a shard's received border column)
            aff_block<true, PARTIAL, false>(c0, w, tf, rv, sw, q, dead, zc, zb, g, e, hg, fdn, dg,
                                                    best, og, of, k);
        }
        tf = rv[CH - 1];
        if (xs) {
            // lane 63's cell of step t0+u is column t0+u-64 (the published chunk j)
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                og[u] = to_x(og[u], t0 + u - 64);
                of[u] = to_x(of[u], t0 + u - 64);
            }
        }
        if (pub && lane == 63) {
            int4* dst = reinterpret_cast<int4*>(io.next_ring + ((j * CH) & IRM));
#pragma unroll
            for (int i = 0; i < CH / 2; ++i) dst[i] = make_int4(og[2 * i], of[2 * i], og[2 * i + 1], of[2 * i + 1]);
        }
        if (io.gout && j >= 0 && lane == 63) {
            // 16-byte write-through stores of two (G, F) columns; each column's 8 bytes
            // land together, so the consumer's 64-bit poll never sees half a column
            int2* dst = io.gout + j * CH;
            if (j * CH + CH <= w && !(k.flags & 2)) {
#pragma unroll
                for (int i = 0; i < CH / 2; ++i) {
                    typedef int v4i __attribute__((ext_vector_type(4)));
                    const v4i v = {og[2 * i], of[2 * i], og[2 * i + 1], of[2 * i + 1]};
                    // s_nop: a >64-bit store's data VGPRs must not be rewritten by the next
                    // VALU (VMEM store-data hazard; the compiler cannot pad inline asm)
                    asm volatile("global_store_dwordx4 %0, %1, off sc1\n s_nop 1" ::"v"(dst + 2 * i), "v"(v)
                                 : "memory");
                }
            } else {
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    if (j * CH + u < w) HandOff<int2>::store(io.gout + j * CH + u, make_int2(og[u], of[u]));
            }
        }
        if (!io.in_border && b < nchunks) lds_st(io.my_cons, (uint32_t)(b + 1));
        if (io.trailing) lds_st(io.tail, (uint32_t)(b + 1));
        if (pub) lds_st(io.next_prod, (uint32_t)(2 * j + 2));
    }
    if (!io.in_border) lds_st(io.my_cons, (uint32_t)(nchunks + kSlots));
    if (io.trailing) lds_st(io.tail, 0x7fffffffu);
#ifdef ANYSEQ_STAMPS
    // timeline: slot 0 = first steady-state block start, 1 = steady-state end, 2 = band end
    if (dbg && lane == 0 && band < 2048 && ts_f) {
        const int slot = 16 + 4 * (band + (P.q_step < 0 ? 2048 : 0));
        dbg[slot] = ts_v;
        dbg[slot + 1] = te_v;
        dbg[slot + 2] = __builtin_amdgcn_s_memrealtime();
        dbg[slot + 3] = t_b0 ? t_b0 : (uint64_t)nmiss;   // (asm path: prefetch misses)
    }
    ev_store(10, __builtin_amdgcn_s_memrealtime());   // band end
    if (dbg && lane == 0 && band < 2048) {
        unsigned long long* ck = dbg + 16 + 20 * 4096 + 4 * (band + (P.q_step < 0 ? 2048 : 0));
        ck[0] = ck_mt0;
        ck[1] = ck_rt0;
        ck[2] = __builtin_amdgcn_s_memtime();
        ck[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (!dead) {
        if (P.out_col) gmem(P.out_col)[row] = aff_to_h(g, row, w - 1, nge);
        if (P.out_col_e) gmem(P.out_col_e)[row] = aff_to_h(e, row, w - 1, nge);
        // shard: F-down of the last row at the last column (the combine pairs it across shards)
        if (lastrow && P.out_f_last) *gmem(P.out_f_last) = aff_to_h(fdn, row, w - 1, nge);
    }
    if constexpr (RR > 1) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int r = rowt + i;
            if (deadu[i]) continue;
            if (P.out_col) gmem(P.out_col)[r] = aff_to_h(gu[i], r, w - 1, nge);
            if (P.out_col_e) gmem(P.out_col_e)[r] = aff_to_h(eu[i], r, w - 1, nge);
            // (an upper row last: the rows below are dead and passed its F-down through, in fdn)
            if (r == h - 1 && P.out_f_last) *gmem(P.out_f_last) = aff_to_h(fdn, r, w - 1, nge);
        }
    }
    if (P.progress && !publish_progress(P, band, lane, err, RR)) return;
    if (bestmode && P.best) {
        // the lane's best covers its row; last-row mode keeps the problem's last row only,
        // last-column mode the lane's cell in the last column
        if (bestmode == 3) best = aff_to_h(g, row, w - 1, nge);
        if (dead || (bestmode == 2 && !lastrow)) best = kAffNeg;
        if constexpr (RR > 1) {
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                int bu = bestu[i];
                if (bestmode == 3) bu = aff_to_h(gu[i], rowt + i, w - 1, nge);
                if (deadu[i] || (bestmode == 2 && rowt + i != h - 1)) bu = kAffNeg;
                best = max(best, bu);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
        if (lane == 0) atomicMax(P.best, best);
    }
}

// NW 8 (round 5): eight compute waves and no I/O wave -- each group's first band forwards
// its own input row (SelfFwd), so every SIMD runs two compute waves
template <int NW, int RR>
__global__ __launch_bounds__(NW == 8 ? 512 : 64 * (NW + 1)) void fill_affine_kernel(const DPProblem* __restrict__ probs,
                                                                     const GroupRef* __restrict__ groups,
                                                                     int ngroups_total, uint32_t* dq, uint32_t* err,
                                                                     FillParams fp) {
    __shared__ __attribute__((aligned(16))) AffShared<NW> sh;
    // logical wave: compute waves 0 .. NW-1, the I/O wave NW.  FillParams::pad bit 8: the
    // I/O wave is the workgroup's first hardware wave, so it shares its SIMD with the
    // group's last band instead of its first (waves are dealt to the SIMDs in order)
    const int hw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int wave = (fp.pad & 256) && NW != 8 ? (hw == 0 ? NW : hw - 1) : hw;
    AffK k;
    k.go = fp.gap_open;
    k.nge = -fp.gap_extend;
    k.wm = fp.match + 2 * k.nge;
    k.wx = fp.mismatch + 2 * k.nge;
    k.flags = fp.pad;
    k.thr = fp.throttle;
    // alphabet codes: *fp.alpha is the number of distinct symbols of the
    // pair, which q / s hold as codes 0 .. n-1
    const int nsym = fp.alpha ? __builtin_amdgcn_readfirstlane(*fp.alpha) : 0;
    k.codes = nsym > 0 && nsym < 255;
    k.lut = nsym > 0 && nsym <= 8 && fp.lut_ok;
    k.slack = fp.slack;
    k.slack_io = fp.slack_io;
    k.lin = fp.gap_open == 0 && !(fp.pad & 128);
    // issue priority: 1 = compute waves before the I/O wave, 2 = the I/O wave first (it
    // sleeps when idle; its hand-off polls sit on the band chain)
    if (fp.prio == 1 && wave < NW) __builtin_amdgcn_s_setprio(3);
    if (fp.prio == 2 && wave == NW) __builtin_amdgcn_s_setprio(3);
    // XCD-local groups (FillParams::xq): this workgroup's XCD first, then the others
    uint32_t xcc = 0;
    if (fp.xq) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= kXcds - 1;
    for (;;) {
        if (threadIdx.x == 0) {
            if (fp.xq) {
                int32_t g = ngroups_total;
                for (uint32_t i = 0; i < (uint32_t)kXcds; ++i) {
                    const uint32_t y = (xcc + i) & (kXcds - 1), lo = fp.xq[y], hi = fp.xq[y + 1];
                    if (lo >= hi || __hip_atomic_load(dq + kXcdCtr + y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                                        hi - lo)
                        continue;
                    const uint32_t j = atomicAdd(dq + kXcdCtr + y, 1u);
                    if (j < hi - lo) {
                        g = (int32_t)(lo + j);
                        break;
                    }
                }
                sh.group = g;
            } else {
                sh.group = (int32_t)atomicAdd(dq, 1u);
            }
            sh.s_filled = 0;
            sh.tail = 0;
        }
        if (threadIdx.x <= NW) {
            sh.prod[threadIdx.x] = 0;
            sh.cons[threadIdx.x] = 0;
        }
        if (threadIdx.x < 32) sh.neg[threadIdx.x] = make_int2(kAffNeg, kAffNeg);
        __syncthreads();
        const int gi = __builtin_amdgcn_readfirstlane(sh.group);
        if (gi >= ngroups_total || err_set(err)) break;
        const GroupRef gr = groups[gi];
        const DPProblem P = probs[gr.prob];
        if (gr.epoch != fp.epoch || gr.check != group_check(gr.prob, gr.group, gr.epoch) ||
            P.magic != prob_magic(&probs[gr.prob], gr.prob, fp.epoch) ||
            (gr.group >= P.ngroups && P.pad_ != kPlannedDesc)) {
            if (threadIdx.x == 0) atomicOr(err, ERR_BAD_DESC);
            break;
        }
        if (gr.group >= P.ngroups) {   // a device-planned level's unused group slot
            __syncthreads();
            continue;
        }
        const int first = gr.group * NW;
        const int last = min(P.nbands, first + NW) - 1;
        int2* rows = reinterpret_cast<int2*>(P.rowbuf);
        int2* g_out = nullptr;
        if (last < P.nbands - 1)
            g_out = rows + (size_t)(gr.group % P.nslots) * P.wpad;
        else if (P.out_row)
            g_out = reinterpret_cast<int2*>(P.out_row);
        // (GS: always the forwarder -- the I/O wave has no subject work; io_wave, a called
        // function, would give the kernel a stack and every launch a scratch setup)
        constexpr bool kSelfFwd = NW == 8;
        static_assert(!kSelfFwd || kAffGS, "self-forwarding needs the code rows");
        if (kSelfFwd && wave == NW) {
        } else if (wave == NW && (kAffGS || fp.io_fwd)) {
            const int2* g_in = gr.group > 0 ? rows + (size_t)((gr.group - 1) % P.nslots) * P.wpad : nullptr;
            io_forward<int2>(lane, P.w, g_in, sh.in_ring[0], &sh.prod[0], &sh.cons[0], err,
                             P.nslots < P.ngroups - 1 || P.pad_ == kPlannedDesc, 2, 2, fp.prio == 3,
                             fp.dbg && first < 2048 ? fp.dbg + 16 + 4 * 4096 + 16 * (first + (P.q_step < 0 ? 2048 : 0))
                                                    : nullptr);
        } else if (wave == NW) {
          if constexpr (!kAffGS) {
            const int2* g_in = gr.group > 0 ? rows + (size_t)((gr.group - 1) % P.nslots) * P.wpad : nullptr;
            io_wave<32, true, int2>(lane, P.w, P.s, P.s_off, P.s_step, sh.s_ring, &sh.skew[0][0][0], &sh.s_filled,
                                    &sh.tail, g_in, sh.in_ring[0], &sh.prod[0], &sh.cons[0], err,
                                    P.nslots < P.ngroups - 1 || P.pad_ == kPlannedDesc, 2, 2, fp.prio == 3,
                                    fp.dbg && first < 2048 ? fp.dbg + 16 + 4 * 4096 + 16 * (first + (P.q_step < 0 ? 2048 : 0))
                                                           : nullptr,
                                    fp.io_stage, fp.io_skew != 0 ? fp.io_skew : kIoSkewPolling, fp.io_poll2 != 0,
                                    kAffGS);
          }
        } else {
            const int band = first + wave;
            if (band <= last) {
                AffIO io;
                io.in_border = band == 0;
                io.io_fed = !kSelfFwd && wave == 0 && gr.group > 0;
                io.trailing = band == last;
                io.my_ring = sh.in_ring[wave];
                io.my_prod = &sh.prod[wave];
                io.my_cons = &sh.cons[wave];
                io.s_ring = sh.s_ring;
                io.skew = &sh.skew[0][0][0];
                io.neg = sh.neg;
                io.s_filled = &sh.s_filled;
                io.tail = &sh.tail;
                io.out_lds = band < last;
                io.next_ring = band < last ? sh.in_ring[wave + 1] : nullptr;
                io.next_prod = band < last ? &sh.prod[wave + 1] : nullptr;
                io.next_cons = band < last ? &sh.cons[wave + 1] : nullptr;
                io.gout = band < last ? nullptr : g_out;
                io.g_in = kSelfFwd && wave == 0 && gr.group > 0 ? rows + (size_t)((gr.group - 1) % P.nslots) * P.wpad
                                                                : nullptr;
                io.reset_in = P.nslots < P.ngroups - 1 || P.pad_ == kPlannedDesc;
                if ((band + 1) * 64 * RR > P.h) run_band_aff<true, RR>(P, band, lane, io, err, k, fp.dbg);
                else run_band_aff<false, RR>(P, band, lane, io, err, k, fp.dbg);
            }
        }
        __syncthreads();
    }
}

// Affine score reductions (H space; rows are (G, F) pairs of the kernel value space).
// Single front: semiglobal max over the last row (index -1 = border 0), the last
// column and 0.  Two fronts (top rows [0,h1) forward, bottom rows [h1,n) reversed):
// for every split column j in [-1, m-1], with jb = m-2-j,
//     max(Ht[j] + Hb[jb], Ft[j] + Fb[jb] - go)
// (F = the last row's F-down, max(F, H + go): the maximum is that of the exact F
// join, whose extra terms never exceed Ht + Hb; a vertical gap across the split is
// opened once), plus the semiglobal end columns / the local best cells.
__global__ void aff_reduce_kernel(int kind, int two, const int2* __restrict__ rowF, int h1,
                                  const int2* __restrict__ rowB, int h2, int m, int go, int ge,
                                  const int32_t* __restrict__ colF, const int32_t* __restrict__ colB, int32_t* out) {
    // global / semiglobal fronts run in G space, local ones (clamp + best) in X space
    auto toh = [&](int v, int r, int c) { return v + (r + (kind == KIND_LOCAL ? 0 : c) + 2) * ge; };
    const int NEG2 = 2 * kAffNeg;
    int best = kind == KIND_SEMIGLOBAL ? 0 : -2147483647;
    const int tid = threadIdx.x + blockIdx.x * blockDim.x, nth = blockDim.x * gridDim.x;
    if (two) {
        const int bt = kind == KIND_GLOBAL ? go + h1 * ge : 0;   // H[h1-1][-1]
        const int bb = kind == KIND_GLOBAL ? go + h2 * ge : 0;
        const int ft = kind == KIND_GLOBAL ? bt : kAffNeg;       // global borders are vertical gaps
        const int fb = kind == KIND_GLOBAL ? bb : kAffNeg;
        for (int j = tid - 1; j < m; j += nth) {
            int Ht = bt, Ft = ft, Hb = bb, Fb = fb;
            if (j >= 0) {
                const int2 t = rowF[j];
                Ht = toh(t.x, h1 - 1, j);
                Ft = toh(t.y, h1 - 1, j);
            }
            const int jb = m - 2 - j;
            if (jb >= 0) {
                const int2 t = rowB[jb];
                Hb = toh(t.x, h2 - 1, jb);
                Fb = toh(t.y, h2 - 1, jb);
            }
            best = max(best, max(Ht + Hb, max(Ft + Fb - go, NEG2)));
        }
        if (kind == KIND_SEMIGLOBAL) {
            for (int i = tid; i < h1; i += nth) best = max(best, colF[i]);
            for (int i = tid; i < h2; i += nth) best = max(best, colB[i]);
        }
    } else if (kind == KIND_SEMIGLOBAL) {
        for (int j = tid; j < m; j += nth) best = max(best, toh(rowF[j].x, h1 - 1, j));
        for (int i = tid; i < h1; i += nth) best = max(best, colF[i]);
    }
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
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

// Two-front score combine (Hirschberg row split at h1): the top front is the
// forward DP of rows [0,h1), the bottom front the DP of rows [h1,n) with query
// and subject reversed.  For every split column j in [-1, m-1]:
//     F[j] + B[m-2-j]    (F = top bottom-row H, B = bottom-front bottom-row H,
//                         index -1 = the scheme's border)
// is the best path crossing rows h1-1 -> h1 after consuming s[0..j].  Semiglobal
// adds paths ending on the right column in the top half (top out_col) and paths
// starting on the left column in the bottom half (bottom out_col); local adds
// the best cell of either front (already in *out via atomicMax).
__global__ void front_combine_kernel(int kind, const int32_t* __restrict__ rowF, int h1, const int32_t* __restrict__ rowB,
                                     int h2, int m, int gap, const int32_t* __restrict__ colF,
                                     const int32_t* __restrict__ colB, int32_t* out) {
    const int ng = -gap;
    auto init = [&](int i) { return kind == KIND_GLOBAL ? (i + 1) * gap : 0; };
    auto toh = [&](int v, int r, int c) { return kind == KIND_LOCAL ? v : v - (r + c + 2) * ng; };
    // semiglobal: row[-1] = col[-1] = 0 borders are part of the reference's max (scoring.impala:51-63)
    int best = kind == KIND_SEMIGLOBAL ? 0 : -2147483647;
    for (int j = (int)(threadIdx.x + blockIdx.x * blockDim.x) - 1; j < m; j += blockDim.x * gridDim.x) {
        const int F = j < 0 ? init(h1 - 1) : toh(rowF[j], h1 - 1, j);
        const int jb = m - 2 - j;
        const int B = jb < 0 ? init(h2 - 1) : toh(rowB[jb], h2 - 1, jb);
        best = max(best, F + B);
    }
    if (kind == KIND_SEMIGLOBAL) {
        for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < h1; i += blockDim.x * gridDim.x) best = max(best, colF[i]);
        for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < h2; i += blockDim.x * gridDim.x) best = max(best, colB[i]);
    }
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
}

// Column-block shard combine: the two-front split of
// front_combine_kernel restricted to one shard's columns [c0, c0+w).  Split
// columns j in [-1, w-1) (+ j = w-1 on the last shard): F = top front's last row
// at local column j (j = -1: the received left column lT[h1-1] + sT, or the
// scheme border on shard 0), B = bottom front's last row at reversed local column
// w-2-j (-1: the bottom front's received column lB[h2-1] + sB, or the border on
// the last shard).  adj moves the sum from the two shard frames to the true
// score.  Semiglobal adds the end columns colT (last shard) / colB (shard 0).
__global__ void shard_combine_kernel(int kind, const int32_t* __restrict__ rowT, int h1,
                                     const int32_t* __restrict__ rowB, int h2, int w, int gap,
                                     const int32_t* __restrict__ lT, int sT, const int32_t* __restrict__ lB, int sB,
                                     int last, const int32_t* __restrict__ colT, const int32_t* __restrict__ colB,
                                     int adj, int32_t* out) {
    const int ng = -gap;
    auto init = [&](int i) { return kind == KIND_GLOBAL ? (i + 1) * gap : 0; };
    auto toh = [&](int v, int r, int c) { return kind == KIND_LOCAL ? v : v - (r + c + 2) * ng; };
    int best = kind == KIND_SEMIGLOBAL ? 0 : -2147483647;
    const int jend = last ? w : w - 1;
    for (int j = (int)(threadIdx.x + blockIdx.x * blockDim.x) - 1; j < jend; j += blockDim.x * gridDim.x) {
        const int F = j >= 0 ? toh(rowT[j], h1 - 1, j) : (lT ? lT[h1 - 1] + sT : init(h1 - 1));
        const int jb = w - 2 - j;
        const int B = jb >= 0 ? toh(rowB[jb], h2 - 1, jb) : (lB ? lB[h2 - 1] + sB : init(h2 - 1));
        best = max(best, F + B + adj);
    }
    if (kind == KIND_SEMIGLOBAL) {
        if (colT)
            for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < h1; i += blockDim.x * gridDim.x)
                best = max(best, colT[i]);
        if (colB)
            for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < h2; i += blockDim.x * gridDim.x)
                best = max(best, colB[i]);
    }
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
}

// Affine shard combine: aff_reduce_kernel's two-front split-row join over this
// shard's columns (true-score units via adj), with the split column left of the
// block paired through the received left column (H[h1-1], F of the last row at
// lTf) and the one right of it through the bottom front's received column.
__global__ void shard_aff_combine_kernel(int kind, const int2* __restrict__ rowT, int h1, const int2* __restrict__ rowB,
                                         int h2, int w, int go, int ge, const int32_t* __restrict__ lT,
                                         const int32_t* __restrict__ lTf, int sT, const int32_t* __restrict__ lB,
                                         const int32_t* __restrict__ lBf, int sB, int last,
                                         const int32_t* __restrict__ colT, const int32_t* __restrict__ colB, int adj,
                                         int32_t* out) {
    // global / semiglobal fronts run in G space, local ones (clamp + best) in X space
    auto toh = [&](int v, int r, int c) { return v + (r + (kind == KIND_LOCAL ? 0 : c) + 2) * ge; };
    const int NEG2 = 2 * kAffNeg;
    int best = kind == KIND_SEMIGLOBAL ? 0 : -2147483647;
    const int bt = kind == KIND_GLOBAL ? go + h1 * ge : 0;   // H[h1-1][-1] of the whole matrix
    const int bb = kind == KIND_GLOBAL ? go + h2 * ge : 0;
    const int jend = last ? w : w - 1;
    const int tid = threadIdx.x + blockIdx.x * blockDim.x, nth = blockDim.x * gridDim.x;
    for (int j = tid - 1; j < jend; j += nth) {
        int Ht, Ft, Hb, Fb;
        if (j >= 0) {
            const int2 t = rowT[j];
            Ht = toh(t.x, h1 - 1, j);
            Ft = toh(t.y, h1 - 1, j);
        } else if (lT) {
            Ht = lT[h1 - 1] + sT;
            Ft = *lTf + sT;
        } else {
            Ht = bt;
            Ft = kind == KIND_GLOBAL ? bt : kAffNeg;
        }
        const int jb = w - 2 - j;
        if (jb >= 0) {
            const int2 t = rowB[jb];
            Hb = toh(t.x, h2 - 1, jb);
            Fb = toh(t.y, h2 - 1, jb);
        } else if (lB) {
            Hb = lB[h2 - 1] + sB;
            Fb = *lBf + sB;
        } else {
            Hb = bb;
            Fb = kind == KIND_GLOBAL ? bb : kAffNeg;
        }
        best = max(best, max(Ht + Hb, max(Ft + Fb - go, NEG2)) + adj);
    }
    if (kind == KIND_SEMIGLOBAL) {
        if (colT)
            for (int i = tid; i < h1; i += nth) best = max(best, colT[i]);
        if (colB)
            for (int i = tid; i < h2; i += nth) best = max(best, colB[i]);
    }
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

// ----------------------------------------------------------------- fulltb --
// construct_*_alignment_fulltb (export.impala:37-53,93-109,150-166; all three use
// global_scheme, export.impala:52,108,165): traceback_full (align.impala:190-216)
// = one fill of the whole matrix writing every predecessor, then traceback_offset
// from (n-1, m-1).  The matrix is cut into 128-column strips; one wave per strip,
// lane l owns strip columns 2l and 2l+1 and sweeps anti-diagonals exactly like
// pred_kernel, with the GLOBAL top border and the left column H[r][oj-1] polled
// from the strip on the left (which stores its last column as it goes, sentinel
// 0x80808080, 64 rows per poll).  Strips are taken by ticket, so a strip only
// waits on a strip that is already running.  Predecessors are anti-diagonal-major
// per strip: pred[k*(n+127)*128 + (i+jl)*128 + jl].
__global__ __launch_bounds__(64) void fulltb_strip_kernel(const uint8_t* __restrict__ Q, int n,
                                                          const uint8_t* __restrict__ S, int m, uint8_t* pred,
                                                          int32_t* cols, uint32_t* ticket, uint32_t* err, int match,
                                                          int mismatch, int gap) {
    const int lane = threadIdx.x;
    int k = 0;
    if (lane == 0) k = (int)atomicAdd(ticket, 1u);
    k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
    const int nstrips = (m + 127) / 128;
    if (k >= nstrips) return;
    const int oj = k * 128, w = min(128, m - oj);
    const int32_t* left_in = k > 0 ? cols + (size_t)(k - 1) * n : nullptr;
    int32_t* right_out = (k < nstrips - 1) ? cols + (size_t)k * n : nullptr;
    auto init = [&](int i) { return (i + 1) * gap; };   // init_scores_global, align.impala:85
    const int jA = 2 * lane, jB = 2 * lane + 1;
    const int sA = jA < w ? (int)S[oj + jA] : 0x100;
    const int sB = jB < w ? (int)S[oj + jB] : 0x100;
    int A = init(oj + jA), Bv = init(oj + jB), A_old = A;
    int leftA_prev = init(oj - 1);   // H[-1][oj-1]: the corner of this strip
    uint16_t* out16 = reinterpret_cast<uint16_t*>(pred + (size_t)k * (size_t)(n + 127) * 128);
    int lchunk = 0;                  // left-column values of rows d & ~63 .. +63 (lane r holds row base + r)
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const int nsteps = n + 127;
    for (int d = 0; d < nsteps; ++d) {
        if (left_in && (d & 63) == 0 && d < n) {
            const int r = d + lane;
            uint32_t it = 0;
            for (;;) {
                lchunk = r < n ? __hip_atomic_load(gmem(left_in) + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0;
                if (__ballot(r < n && lchunk == kShardSentinel) == 0) break;
                __builtin_amdgcn_s_sleep(2);
                if ((++it & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || err_set(err))) {
                    atomicOr(err, ERR_SPIN_TIMEOUT | 16u);
                    return;
                }
            }
        }
        const int lv = left_in ? __shfl(lchunk, d & 63) : init(d);   // H[d][oj-1] for lane 0 (row iA = d)
        const int iA = d - jA, iB = d - jB;
        const int leftA = wave_shr1(lv, Bv);
        const int diagA = leftA_prev;
        leftA_prev = leftA;
        const bool actA = (iA >= 0) && (iA < n) && (jA < w);
        const bool actB = (iB >= 0) && (iB < n) && (jB < w);
        const int qA = (iA >= 0 && iA < n) ? (int)Q[iA] : 0x200;
        const int qB = (iB >= 0 && iB < n) ? (int)Q[iB] : 0x200;
        int pA = 0, pB = 0;
        const int nB = relax_pred(KIND_GLOBAL, A_old, A, Bv, qB == sB ? match : mismatch, gap, pB);
        const int nA = relax_pred(KIND_GLOBAL, diagA, leftA, A, qA == sA ? match : mismatch, gap, pA);
        if (actB) Bv = nB;
        A_old = A;
        if (actA) A = nA;
        if (right_out && actB && jB == 127)
            __hip_atomic_store(gmem(right_out) + iB, nB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out16[(size_t)d * 64 + lane] = (uint16_t)((actA ? pA : 0) | ((actB ? pB : 0) << 8));
    }
}

// One thread: traceback_offset (traceback.impala:47-80) from (n-1, m-1) over the
// strips, global border predecessors (predecessors.impala:17-18, align.impala:88-90).
__global__ void fulltb_walk_kernel(const uint8_t* __restrict__ Q, int n, const uint8_t* __restrict__ S, int m,
                                   const uint8_t* __restrict__ pred, uint8_t* alq, uint8_t* als) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const size_t strip = (size_t)(n + 127) * 128;
    auto P = [&](int i, int j) -> int {
        if (i < 0 && j < 0) return 0;
        if (i < 0) return 1;   // row -1: GAP_Q
        if (j < 0) return 2;   // column -1: GAP_S
        const int jl = j & 127;
        return pred[(size_t)(j >> 7) * strip + (size_t)(i + jl) * 128 + jl];
    };
    int i = n - 1, j = m - 1;
    int p = P(i, j);
    while (p != 0) {
        uint8_t sq = '_', ss = '_';
        const int pos = i + j + 1;
        if (p == 3 || p == 2) sq = Q[i--];
        if (p == 3 || p == 1) ss = S[j--];
        alq[pos] = sq;
        als[pos] = ss;
        p = P(i, j);
    }
}

// ======================================================= affine construct --
// Build-defined linear-space affine alignment (semantics =
// oracle_affine_construct in oracle/anyseq_oracle.c): one column-split Hirschberg
// over the whole matrix whose parts may have free starts / ends.

// H-space top border of a half at column c (oracle bm_top).
__device__ __forceinline__ int aff_top_h(int bm, int c, int go, int ge) {
    if (bm == BM_NORMAL || bm == BM_EPAID) return go + (c + 1) * ge;
    if (bm == BM_EFREE) return (c + 1) * ge;
    return 0;
}

// Hirschberg join of one part per workgroup, the first maximum (strict >) in the
// candidate order
//     BEFORE (free end: best end cell of the left half, pbest[2p]),
//     AFTER (free start: best start cell of the right half, pbest[2p+1]),
//     rows i = -1 .. len-1: HL(i) + HR(len-i-2), then EL(i) + ER(len-i-2) - go
// (L = forward left half's last column, R = reversed right half's; index -1 =
// the half's top border: a gap when anchored, no gap when free).  Writes the split
// row and its type (T_*) at the part's split index; an empty part passes its type
// on.  score: the value of part 0 (level 1: the optimal score).
__global__ __launch_bounds__(256) void aff_hb_join_kernel(const PartInfo* __restrict__ parts, int half,
                                                          const int32_t* __restrict__ LH, const int32_t* __restrict__ LE,
                                                          const int32_t* __restrict__ RH,
                                                          const int32_t* __restrict__ RE,
                                                          const int32_t* __restrict__ pbest, int go, int ge,
                                                          int32_t* splits, int32_t* types, int32_t* score) {
    __shared__ int sv[256], sk[256];
    const PartInfo pi = parts[blockIdx.x];
    const int off = pi.off, len = pi.len;
    if (pi.flags & 8) return;   // a one-block part (aff_part_geo): nothing to split
    if (pi.flags & 4) {
        if (threadIdx.x == 0) {
            splits[pi.split_index + 1] = off;
            types[pi.split_index + 1] = pi.empty_type;
        }
        return;
    }
    const bool sfree = pi.flags & 1, efree = pi.flags & 2;
    const int bLH = aff_top_h(pi.smode, pi.lhw - 1, go, ge), bLE = sfree ? kAffNeg : bLH;
    const int bRH = aff_top_h(pi.emode, pi.rhw - 1, go, ge), bRE = efree ? kAffNeg : bRH;
    int best = -2147483647, key = 0x7fffffff;   // key: 0 BEFORE, 1 AFTER, 2 + 2 (i + 1) + type
    if (threadIdx.x == 0) {
        if (efree && pbest[2 * blockIdx.x] > best) {
            best = pbest[2 * blockIdx.x];
            key = 0;
        }
        if (sfree && pbest[2 * blockIdx.x + 1] > best) {
            best = pbest[2 * blockIdx.x + 1];
            key = 1;
        }
    }
    for (int i = (int)threadIdx.x - 1; i < len; i += blockDim.x) {
        const int k = len - i - 2;
        const int hl = i < 0 ? bLH : LH[off + i], el = i < 0 ? bLE : LE[off + i];
        const int hr = k < 0 ? bRH : RH[off + k], er = k < 0 ? bRE : RE[off + k];
        const int vh = hl + hr, ve = el + er - go;
        if (vh > best) {
            best = vh;
            key = 2 + 2 * (i + 1);
        }
        if (ve > best) {
            best = ve;
            key = 3 + 2 * (i + 1);
        }
    }
    sv[threadIdx.x] = best;
    sk[threadIdx.x] = key;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const int v2 = sv[threadIdx.x + o], k2 = sk[threadIdx.x + o];
            if (v2 > sv[threadIdx.x] || (v2 == sv[threadIdx.x] && k2 < sk[threadIdx.x])) {
                sv[threadIdx.x] = v2;
                sk[threadIdx.x] = k2;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int kk = sk[0];
        int type, spl;
        if (kk == 0) {
            type = T_BEFORE;
            spl = off + len;
        } else if (kk == 1) {
            type = T_AFTER;
            spl = off;
        } else {
            type = (kk & 1) ? T_E : T_H;
            spl = off + (kk - 2) / 2;   // off + idx + 1
        }
        splits[pi.split_index + 1] = spl;
        types[pi.split_index + 1] = type;
        if (score && blockIdx.x == 0) *score = sv[0];
    }
}

// The same join in two stages for long parts: stage 1 takes the first maximum of one
// slice of a part's candidates per workgroup (slice 0 also tries BEFORE / AFTER),
// stage 2 combines a part's slices in order (larger value, then the earlier key).
constexpr int kJoinSlice = 4096;
__global__ __launch_bounds__(256) void aff_hb_join_slice_kernel(const PartInfo* __restrict__ parts, int half,
                                                                const int32_t* __restrict__ LH,
                                                                const int32_t* __restrict__ LE,
                                                                const int32_t* __restrict__ RH,
                                                                const int32_t* __restrict__ RE,
                                                                const int32_t* __restrict__ pbest, int go, int ge,
                                                                int nslices, int2* __restrict__ partial) {
    __shared__ int sv[256], sk[256];
    const int part = blockIdx.y, slice = blockIdx.x;
    const PartInfo pi = parts[part];
    const int off = pi.off, len = pi.len;
    int best = -2147483647, key = 0x7fffffff;
    if (!(pi.flags & 12)) {
        const bool sfree = pi.flags & 1, efree = pi.flags & 2;
        const int bLH = aff_top_h(pi.smode, pi.lhw - 1, go, ge), bLE = sfree ? kAffNeg : bLH;
        const int bRH = aff_top_h(pi.emode, pi.rhw - 1, go, ge), bRE = efree ? kAffNeg : bRH;
        if (slice == 0 && threadIdx.x == 0) {
            if (efree && pbest[2 * part] > best) {
                best = pbest[2 * part];
                key = 0;
            }
            if (sfree && pbest[2 * part + 1] > best) {
                best = pbest[2 * part + 1];
                key = 1;
            }
        }
        const int i0 = slice * kJoinSlice - 1, i1 = min(len, i0 + kJoinSlice);
        for (int i = i0 + (int)threadIdx.x; i < i1; i += blockDim.x) {
            const int k = len - i - 2;
            const int hl = i < 0 ? bLH : LH[off + i], el = i < 0 ? bLE : LE[off + i];
            const int hr = k < 0 ? bRH : RH[off + k], er = k < 0 ? bRE : RE[off + k];
            const int vh = hl + hr, ve = el + er - go;
            if (vh > best) {
                best = vh;
                key = 2 + 2 * (i + 1);
            }
            if (ve > best) {
                best = ve;
                key = 3 + 2 * (i + 1);
            }
        }
    }
    sv[threadIdx.x] = best;
    sk[threadIdx.x] = key;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const int v2 = sv[threadIdx.x + o], k2 = sk[threadIdx.x + o];
            if (v2 > sv[threadIdx.x] || (v2 == sv[threadIdx.x] && k2 < sk[threadIdx.x])) {
                sv[threadIdx.x] = v2;
                sk[threadIdx.x] = k2;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[(size_t)part * nslices + slice] = make_int2(sv[0], sk[0]);
}

__global__ void aff_hb_join_final_kernel(const PartInfo* __restrict__ parts, int nparts, int nslices,
                                         const int2* __restrict__ partial, int32_t* splits, int32_t* types,
                                         int32_t* score) {
    const int part = blockIdx.x * blockDim.x + threadIdx.x;
    if (part >= nparts) return;
    const PartInfo pi = parts[part];
    if (pi.flags & 8) return;
    if (pi.flags & 4) {
        splits[pi.split_index + 1] = pi.off;
        types[pi.split_index + 1] = pi.empty_type;
        return;
    }
    int best = -2147483647, kk = 0x7fffffff;
    for (int sl = 0; sl < nslices; ++sl) {
        const int2 v = partial[(size_t)part * nslices + sl];
        if (v.x > best || (v.x == best && v.y < kk)) {
            best = v.x;
            kk = v.y;
        }
    }
    int type, spl;
    if (kk == 0) {
        type = T_BEFORE;
        spl = pi.off + pi.len;
    } else if (kk == 1) {
        type = T_AFTER;
        spl = pi.off;
    } else {
        type = (kk & 1) ? T_E : T_H;
        spl = pi.off + (kk - 2) / 2;
    }
    splits[pi.split_index + 1] = spl;
    types[pi.split_index + 1] = type;
    if (score && part == 0) *score = best;
}

// Transposed Hirschberg halves: the bottom row (G, F-down) of
// the transposed problem is the original's last column (H, E-right) -> H space.
// E-right = max(E, H + go) instead of E changes no join decision: an E candidate
// that only its H + go term lifts never exceeds the H candidate of its row, which
// is tried first.
__global__ void aff_row_to_col_kernel(const RowToCol* __restrict__ jobs, int nge) {
    const RowToCol J = jobs[blockIdx.y];
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < J.n; c += blockDim.x * gridDim.x) {
        const int2 v = reinterpret_cast<const int2*>(J.row)[c];
        const int z = (J.hlast + (J.xs ? 0 : c + J.c0) + 2) * nge;
        J.H[c] = v.x - z;
        J.E[c] = v.y - z;
    }
}

// ---------------------------------------------------------------------------
// Device-planned Hirschberg level (AffLevelPlan): the host-side
// level builder of the affine construct (anyseq_engine.cpp add_half / fill_prepare)
// restated on the device, one workgroup: part table, the two half descriptors of
// every part (transposed when taller than wide), their hand-off ring and flag slots,
// the k-major group table and the row-to-column jobs.  Hand-off rows and transposed
// bottom rows are packed by block-wide exclusive scans over the parts in order.
struct AffHalfGeo {
    int32_t h, w;          // the problem as run (transposed: subject columns as rows)
    int32_t tr, ngroups, nslots, wpad;
    int64_t rowbuf;        // hand-off ring ints
    int64_t rowpool;       // transposed bottom row ints
    int64_t scode;         // subject-code row bytes (DPProblem::scode)
};
__device__ AffHalfGeo aff_half_geo(const AffLevelPlan& a, int len, int width) {
    AffHalfGeo g{};
    if (len <= 0) return g;
    g.tr = a.afft && len > width;
    g.h = g.tr ? width : len;
    g.w = g.tr ? len : width;
    const int nbands = (g.h + 63) / 64;
    g.ngroups = (nbands + a.NW - 1) / a.NW;
    g.wpad = (g.w + 63) & ~63;
    g.nslots = max(1, min(g.ngroups - 1, a.want_slots));
    g.rowbuf = g.ngroups > 1 ? (int64_t)g.nslots * g.wpad * 2 : 0;
    g.rowpool = g.tr ? (int64_t)((len + 63) & ~63) * 2 : 0;
    g.scode = 4 * scode_len(g.w);
    return g;
}

// block-wide exclusive scan (64 .. 1024 threads) of one 64-bit value; returns the prefix,
// *total the tile's sum
__device__ int64_t block_scan_excl(int64_t v, int64_t* sh, int64_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    if (tid == 0) {
        int64_t acc = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            const int64_t t = sh[i];
            sh[i] = acc;
            acc += t;
        }
        sh[16] = acc;
    }
    __syncthreads();
    const int64_t r = sh[wv] + x - v;
    *total = sh[16];
    __syncthreads();
    return r;
}

// Four block-wide exclusive scans at once (the plan's ring, bottom-row, code-row and
// half-ordinal packing): one pass of shuffles, the wave totals scanned by wave 0's lanes
// (no serial loop), three barriers for all four (round 5: four separate scans were
// 3.5 us of every level's tail).
struct Scan4 {
    int64_t v[4];
};
__device__ Scan4 block_scan_excl4(const Scan4& in, int64_t (*sh)[4], Scan4* total) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = (int)(blockDim.x >> 6);
    Scan4 x = in;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t y = __shfl_up(x.v[k], o);
            if (lane >= o) x.v[k] += y;
        }
    }
    if (lane == 63)
        for (int k = 0; k < 4; ++k) sh[wv][k] = x.v[k];
    __syncthreads();
    if (wv == 0) {   // exclusive scan of the (at most 16) wave totals
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t t = lane < nw ? sh[lane][k] : 0;
            int64_t c = t;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const int64_t y = __shfl_up(c, o);
                if (lane >= o) c += y;
            }
            if (lane < nw) sh[lane][k] = c - t;
            if (lane == nw - 1) sh[16][k] = c;
        }
    }
    __syncthreads();
    Scan4 r;
    for (int k = 0; k < 4; ++k) {
        r.v[k] = sh[wv][k] + x.v[k] - in.v[k];
        total->v[k] = sh[16][k];
    }
    __syncthreads();
    return r;
}

// The same within each wave alone (no LDS, no barrier): a level of at most 64 parts has
// all of them in wave 0 (the other waves scan zeros).
__device__ Scan4 wave_scan_excl4(const Scan4& in, Scan4* total) {
    const int lane = threadIdx.x & 63;
    Scan4 x = in, r;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t y = __shfl_up(x.v[k], o);
            if (lane >= o) x.v[k] += y;
        }
    }
    for (int k = 0; k < 4; ++k) {
        total->v[k] = __shfl(x.v[k], 63);
        r.v[k] = x.v[k] - in.v[k];
    }
    return r;
}

__device__ void aff_level_plan_body(const AffLevelPlan& a) {
    __shared__ int64_t sh[17];
    __shared__ int64_t sh4[17][4];
    __shared__ unsigned long long cells;
    __shared__ int32_t bad;
    auto stamp = [&](int k) {   // diagnostics: the plan's phases (a.stamps[k], ANYSEQ_TAIL_STAMPS)
        if (a.stamps && threadIdx.x == 0) a.stamps[k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    if (threadIdx.x == 0) {
        cells = 0;
        bad = 0;
    }
    __syncthreads();
    // kind != global with a level-1 value <= 0: the empty alignment, no halves
    const bool stop = a.score && a.kind != KIND_GLOBAL && *a.score <= 0;
    RowToCol* jobs = a.jobs;
    int64_t rb_base = 0, rp_base = 0, sc_base = 0, hb_base = 0;
    unsigned long long my_cells = 0;   // this thread's halves' cells (summed per wave below)
    for (int t0 = 0; t0 < a.parts; t0 += blockDim.x) {
        const int p = t0 + (int)threadIdx.x;
        PartInfo pi{};
        AffHalfGeo gl{}, gr{};
        int off = 0, len = 0, hoj_l = 0, hoj_r = 0, hw = 0;
        bool sfree = false, efree = false;
        if (p < a.parts) {
            const AffPartGeo pg = aff_part_geo(a.nb, a.m, a.parts, p);
            const int sb = pg.sb, eb = pg.eb;
            const int ts = a.typ[sb + 1], te = a.typ[eb + 1];
            pi.split_index = pg.mid;
            pi.lhw = pg.lw;
            off = a.spl[sb + 1];
            if (pg.lw <= 0 || pg.hw <= 0) {   // a one-block part: no split, no halves
                pi.flags = 8;
            } else if (stop || ts == T_BEFORE || te == T_AFTER) {   // empty part: so are both halves
                pi.flags = 4;
                pi.empty_type = ts == T_BEFORE ? T_BEFORE : T_AFTER;
                pi.off = off;
            } else {
                len = a.spl[eb + 1] - off;
                hoj_l = pg.hoj_l;
                hoj_r = pg.hoj_r;
                hw = pg.hw;
                sfree = ts == T_AFTER;
                efree = te == T_BEFORE;
                pi.off = off;
                pi.len = len;
                pi.rhw = hw;
                pi.smode = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : aff_free_bm(a.kind, hoj_l == 0);
                pi.emode = te == T_H ? BM_NORMAL : te == T_E ? BM_EPAID : aff_free_bm(a.kind, hoj_r + hw == a.m);
                pi.flags = (sfree ? 1 : 0) | (efree ? 2 : 0);
                gl = aff_half_geo(a, len, pg.lw);
                gr = aff_half_geo(a, len, hw);
            }
            a.parts_out[p] = pi;
            if (gl.ngroups > a.bound || gr.ngroups > a.bound) atomicOr(&bad, 1);
        }
        stamp(1);
        // ring, bottom-row and code-row offsets; sharded: the part's ordinal among the parts
        // with halves (the host's half_index / 2)
        Scan4 in4, tot4;
        in4.v[0] = gl.rowbuf + gr.rowbuf;
        in4.v[1] = gl.rowpool + gr.rowpool;
        in4.v[2] = gl.scode + gr.scode;
        in4.v[3] = p < a.parts && len > 0 ? 1 : 0;
        const Scan4 ex4 = a.parts <= 64 ? wave_scan_excl4(in4, &tot4) : block_scan_excl4(in4, sh4, &tot4);
        const int64_t rb = rb_base + ex4.v[0], rp = rp_base + ex4.v[1], sco = sc_base + ex4.v[2];
        const int64_t hord = hb_base + ex4.v[3];
        rb_base += tot4.v[0];
        rp_base += tot4.v[1];
        sc_base += tot4.v[2];
        hb_base += tot4.v[3];
        stamp(2);
        if (p < a.parts) {
            for (int side = 0; side < 2; ++side) {
                const AffHalfGeo& g = side ? gr : gl;
                const int idx = 2 * p + side;
                // sharded: the half's owner; view: where its columns / best cell go
                const int own = a.world > 1 ? (int)((2 * hord + side) % a.world) : 0;
                const bool mine = a.world <= 1 || a.rank < 0 || own == a.rank;
                const int64_t view = a.world > 1 && a.rank < 0 ? own : 0;
                DPProblem P{};
                RowToCol J{};
                if (g.h > 0) {
                    // the half as add_half builds it (original orientation first)
                    const int qoff = side ? off + len - 1 : off, qstep = side ? -1 : 1;
                    const int soff = side ? hoj_r + hw - 1 : hoj_l, sstep = side ? -1 : 1;
                    const int bm = side ? pi.emode : pi.smode;
                    const bool fr = side ? sfree : efree;
                    const int amode = (bm == BM_FREE_LOCAL ? AM_CLAMP : 0) | (fr ? a.best_bits : 0);
                    int32_t* H = (side ? a.RH : a.LH) + view * a.vstride + off;
                    int32_t* E = (side ? a.RE : a.LE) + view * a.vstride + off;
                    P.best = fr ? a.pbest + view * a.pstride + 2 * p + side : nullptr;
                    if (g.tr) {
                        P.q = a.s;
                        P.q_off = soff;
                        P.q_step = sstep;
                        P.s = a.q;
                        P.s_off = qoff;
                        P.s_step = qstep;
                        P.bmode = aff_transposed_bm(bm);
                        P.amode = (amode & AM_CLAMP) |
                                  ((amode & AM_BEST_LASTCOL) == AM_BEST_LAST ? AM_BEST_LASTCOL : (amode & AM_BEST_LASTCOL));
                        const int64_t ro = rp + (side ? gl.rowpool : 0);
                        P.out_row = a.rowpool + ro;
                        J.row = P.out_row;
                        J.H = H;
                        J.E = E;
                        J.n = len;
                        J.hlast = g.h - 1;
                        J.xs = P.amode != 0 ? 1 : 0;
                    } else {
                        P.q = a.q;
                        P.q_off = qoff;
                        P.q_step = qstep;
                        P.s = a.s;
                        P.s_off = soff;
                        P.s_step = sstep;
                        P.bmode = bm;
                        P.amode = amode;
                        P.out_col = H;
                        P.out_col_e = E;
                    }
                    P.h = g.h;
                    P.w = g.w;
                    P.nbands = (g.h + 63) / 64;
                    P.ngroups = mine ? g.ngroups : 0;   // (another rank's half: every group slot skipped)
                    P.wpad = g.wpad;
                    P.nslots = g.nslots;
                    P.rowbuf = a.rowbuf + rb + (side ? gl.rowbuf : 0);
                    const int64_t so = sco + (side ? gl.scode : 0);
                    P.scode = a.scode && so + g.scode <= a.scode_cap ? a.scode + so : nullptr;
                    if (mine) my_cells += (unsigned long long)((int64_t)g.h * g.w);
                } else {
                    P.nslots = 1;
                }
                P.flags = a.flags + (size_t)idx * a.bound;
                P.magic = prob_magic(&P, idx, a.epoch);
                P.pad_ = kPlannedDesc;
                a.probs[idx] = P;
                jobs[idx] = J;
            }
        }
    }
    {   // the level's cells: a wave sum, one LDS add per wave (not one per half)
        unsigned long long c = my_cells;
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(&cells, c);
    }
    stamp(3);
    // the group table, k-major over the half slots (a half's groups in increasing k);
    // XCD-local groups (a.xrun > 0, FillParams::xq): stably partitioned by XCD
    const int nh = 2 * a.parts;
    const int T = nh * a.bound;
    if (a.xrun <= 0) {
        for (int i = (int)threadIdx.x; i < T; i += blockDim.x) {
            const int k = i / nh, pr = i % nh;
            a.groups[i] = GroupRef{pr, k, a.epoch, group_check(pr, k, a.epoch)};
        }
    } else {
        __shared__ int32_t xcnt[kXcds], xoff[kXcds + 1];
        if (threadIdx.x < kXcds) xcnt[threadIdx.x] = 0;
        __syncthreads();
        for (int i = (int)threadIdx.x; i < T; i += blockDim.x)
            atomicAdd(&xcnt[xcd_of_group((int64_t)(i % nh) * a.bound + i / nh, a.xrun)], 1);
        __syncthreads();
        if (threadIdx.x == 0) {
            xoff[0] = 0;
            for (int x = 0; x < kXcds; ++x) xoff[x + 1] = xoff[x] + xcnt[x];
        }
        __syncthreads();
        if (threadIdx.x <= kXcds) a.xq[threadIdx.x] = (uint32_t)xoff[threadIdx.x];
        // rank within the XCD in k-major order: two block scans of four 16-bit counters
        int32_t base[kXcds] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int t0 = 0; t0 < T; t0 += blockDim.x) {
            const int i = t0 + (int)threadIdx.x;
            const int k = i / nh, pr = i % nh;
            const int x = i < T ? xcd_of_group((int64_t)pr * a.bound + k, a.xrun) : -1;
            const int64_t lo = x >= 0 && x < 4 ? (int64_t)1 << (16 * x) : 0;
            const int64_t hi = x >= 4 ? (int64_t)1 << (16 * (x - 4)) : 0;
            int64_t tlo, thi;
            const int64_t elo = block_scan_excl(lo, sh, &tlo);
            const int64_t ehi = block_scan_excl(hi, sh, &thi);
            if (x >= 0) {
                const int rank = (int)(((x < 4 ? elo >> (16 * x) : ehi >> (16 * (x - 4)))) & 0xffff) + base[x];
                a.groups[xoff[x] + rank] = GroupRef{pr, k, a.epoch, group_check(pr, k, a.epoch)};
            }
            for (int y = 0; y < kXcds; ++y) base[y] += (int)(((y < 4 ? tlo >> (16 * y) : thi >> (16 * (y - 4)))) & 0xffff);
        }
    }
    __syncthreads();
    stamp(4);
    if (threadIdx.x == 0) {
        a.hdr[0] = (uint32_t)(rb_base / 4);   // sentinel uint4s (every ring is a multiple of 128 ints)
        a.hdr[1] = (uint32_t)(bad || sc_base > a.scode_cap);
        reinterpret_cast<unsigned long long*>(a.hdr)[1] = cells;
    }
}

__global__ __launch_bounds__(1024) void aff_level_plan_kernel(const AffLevelPlan a) {
    // (level 1: what a memset, an upload and the fill prep did before -- three launches fewer)
    if (a.nzero_init > 0 || a.init_ends || a.nzero2 > 0 || a.ninit2 > 0) {
        for (int i = threadIdx.x; i < a.nzero_init; i += blockDim.x) a.zero_init[i] = 0u;
        for (int i = threadIdx.x; i < a.nzero2; i += blockDim.x) a.zero2[i] = 0u;
        for (int i = threadIdx.x; i < a.ninit2; i += blockDim.x) a.init2[i] = a.init2_value;
        if (a.init_ends && threadIdx.x == 0) {
            int32_t* spl = const_cast<int32_t*>(a.spl);
            int32_t* typ = const_cast<int32_t*>(a.typ);
            spl[0] = 0;
            spl[a.nb] = a.n;
            typ[0] = a.kind != KIND_GLOBAL ? T_AFTER : T_H;
            typ[a.nb] = a.kind != KIND_GLOBAL ? T_BEFORE : T_H;
        }
        __threadfence();
        __syncthreads();
    }
    aff_level_plan_body(a);
}

// Dwords [d0, d1) of problem P's subject-code rows (DPProblem::scode): column c at byte
// c + 64 of copy 0, copy r shifted left by r bytes, code 0xFF outside [0, w)
// (aff_scode_kernel).
__device__ __forceinline__ void aff_scode_dwords(const DPProblem& P, int64_t d0, int64_t d1, int64_t stride) {
    const int64_t nd = scode_len(P.w) / 4;   // dwords per copy (scode_len is a multiple of 16)
    const GLOBAL_AS uint8_t* s = gmem(P.s);
    uint32_t* out = reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(P.scode));
    for (int64_t d = d0; d < d1; d += stride) {
        const int r = (int)(d / nd);
        const int64_t c0 = (d % nd) * 4 - 64 + r;   // column of the dword's first byte
        uint32_t v = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t c = c0 + t;
            const uint32_t b = (c >= 0 && c < P.w) ? s[P.s_off + (int64_t)P.s_step * c] : 0xffu;
            v |= b << (8 * t);
        }
        out[d] = v;
    }
}

constexpr int kTailStage = 8192;   // partials staged in LDS per chunk of parts (64 KiB)
constexpr int kTailThreads = 1024;   // (16 waves: a join thread loads at most 4 rows of a 4096-row slice)
__global__ __launch_bounds__(kTailThreads) void aff_level_tail_kernel(const AffLevelTail t) {
    __shared__ int sv[kTailThreads / 64], sk[kTailThreads / 64];
    __shared__ int last;
    const int nj = t.nslices * t.nparts;
    const int b = blockIdx.x;
    // diagnostics: [0] first workgroup start, [1] last join done, [2] the last workgroup's
    // final pass done, [3] its counters / best cells, [4] the plan done (s_memrealtime)
    auto stamp = [&](int k, bool first) {
        if (t.stamps && threadIdx.x == 0) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (first) atomicMin(t.stamps + k, now);
            else atomicMax(t.stamps + k, now);
        }
    };
    stamp(0, true);
    if (t.has_next) {
        const uint4 v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
        for (size_t i = (size_t)b * blockDim.x + threadIdx.x; i < t.nsent16; i += (size_t)gridDim.x * blockDim.x)
            reinterpret_cast<uint4*>(t.sent)[i] = v;
    }
    const int part = b / max(t.nslices, 1), slice = b % max(t.nslices, 1);
    const PartInfo pi = b < nj ? t.parts[part] : PartInfo{};
    // slices past the part's candidates (the slice count covers the longest possible part)
    const bool idle = b < nj && (pi.flags & 12 || (slice > 0 && slice * t.slice_len - 1 >= pi.len));
    // partials: write-through (sc1) stores, drained before the counter, read back with sc1
    // loads -- no L2 write-back fence, which would also flush the sentinel rows
    int2* partial = reinterpret_cast<int2*>(t.partial);
    if (idle && threadIdx.x == 0)
        HandOff<int2>::store(partial + (size_t)part * t.nslices + slice, make_int2(-2147483647, 0x7fffffff));
    if (b < nj && !idle) {
        const int off = pi.off, len = pi.len, nge = -t.ge;
        int best = -2147483647, key = 0x7fffffff;
        if (!(pi.flags & 4)) {
            const bool sfree = pi.flags & 1, efree = pi.flags & 2;
            const int bLH = aff_top_h(pi.smode, pi.lhw - 1, t.go, t.ge), bLE = sfree ? kAffNeg : bLH;
            const int bRH = aff_top_h(pi.emode, pi.rhw - 1, t.go, t.ge), bRE = efree ? kAffNeg : bRH;
            const RowToCol JL = t.jobs[2 * part], JR = t.jobs[2 * part + 1];
            if (slice == 0 && threadIdx.x == 0) {
                if (efree && t.pbest[2 * part] > best) {
                    best = t.pbest[2 * part];
                    key = 0;
                }
                if (sfree && t.pbest[2 * part + 1] > best) {
                    best = t.pbest[2 * part + 1];
                    key = 1;
                }
            }
            const int i0 = slice * t.slice_len - 1, i1 = min(len, i0 + t.slice_len);
            for (int i = i0 + (int)threadIdx.x; i < i1; i += blockDim.x) {
                const int k = len - i - 2;
                int hl, el, hr, er;
                if (i < 0) {
                    hl = bLH;
                    el = bLE;
                } else if (JL.n > 0) {   // transposed left half: its bottom row, H space
                    const int2 v = reinterpret_cast<const int2*>(JL.row)[i];
                    const int z = (JL.hlast + (JL.xs ? 0 : i + JL.c0) + 2) * nge;
                    hl = v.x - z;
                    el = v.y - z;
                } else {
                    hl = t.LH[off + i];
                    el = t.LE[off + i];
                }
                if (k < 0) {
                    hr = bRH;
                    er = bRE;
                } else if (JR.n > 0) {
                    const int2 v = reinterpret_cast<const int2*>(JR.row)[k];
                    const int z = (JR.hlast + (JR.xs ? 0 : k + JR.c0) + 2) * nge;
                    hr = v.x - z;
                    er = v.y - z;
                } else {
                    hr = t.RH[off + k];
                    er = t.RE[off + k];
                }
                const int vh = hl + hr, ve = el + er - t.go;
                if (vh > best) {
                    best = vh;
                    key = 2 + 2 * (i + 1);
                }
                if (ve > best) {
                    best = ve;
                    key = 3 + 2 * (i + 1);
                }
            }
        }
        // the first maximum (larger value, then smaller key): lanes, then the waves
        for (int o = 32; o >= 1; o >>= 1) {
            const int v2 = __shfl_xor(best, o), k2 = __shfl_xor(key, o);
            if (v2 > best || (v2 == best && k2 < key)) {
                best = v2;
                key = k2;
            }
        }
        if ((threadIdx.x & 63) == 0) {
            sv[threadIdx.x >> 6] = best;
            sk[threadIdx.x >> 6] = key;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int wv = 1; wv < (int)(blockDim.x >> 6); ++wv)
                if (sv[wv] > best || (sv[wv] == best && sk[wv] < key)) {
                    best = sv[wv];
                    key = sk[wv];
                }
            HandOff<int2>::store(partial + (size_t)part * t.nslices + slice, make_int2(best, key));
        }
    }
    // the last workgroup to finish
    __syncthreads();
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(t.done, 1u) == gridDim.x - 1;
    }
    stamp(1, false);
    __syncthreads();
    if (!last) return;
    // the final pass over chunks of parts: every partial of the chunk is loaded at once
    // (independent write-through loads, one round trip) into LDS, then reduced per part
    __shared__ int2 stage[kTailStage];
    const int pc = min((int)blockDim.x, max(1, kTailStage / max(t.nslices, 1)));   // (host: nslices <= kTailStage)
    for (int p0 = 0; p0 < t.nparts; p0 += pc) {
        const int np = min(pc, t.nparts - p0);
        __syncthreads();
        for (int i = threadIdx.x; i < np * t.nslices; i += blockDim.x)
            stage[i] = HandOff<int2>::load(partial + (size_t)p0 * t.nslices + i);
        __syncthreads();
        const int part = p0 + (int)threadIdx.x;
        if ((int)threadIdx.x >= np) continue;
        const PartInfo pi = t.parts[part];
        if (pi.flags & 8) continue;   // a one-block part: nothing to split
        if (pi.flags & 4) {
            t.splits[pi.split_index + 1] = pi.off;
            t.types[pi.split_index + 1] = pi.empty_type;
            continue;
        }
        int best = -2147483647, kk = 0x7fffffff;
        for (int sl = 0; sl < t.nslices; ++sl) {
            const int2 v = stage[threadIdx.x * t.nslices + sl];
            if (v.x > best || (v.x == best && v.y < kk)) {
                best = v.x;
                kk = v.y;
            }
        }
        int type, spl;
        if (kk == 0) {
            type = T_BEFORE;
            spl = pi.off + pi.len;
        } else if (kk == 1) {
            type = T_AFTER;
            spl = pi.off;
        } else {
            type = (kk & 1) ? T_E : T_H;
            spl = pi.off + (kk - 2) / 2;
        }
        t.splits[pi.split_index + 1] = spl;
        t.types[pi.split_index + 1] = type;
        if (t.score && part == 0) *t.score = best;
    }
    __syncthreads();
    stamp(2, false);
    if (!t.has_next) return;
    __threadfence_block();
    for (int i = threadIdx.x; i < t.nzero; i += blockDim.x) t.zero[i] = 0u;
    for (int i = threadIdx.x; i < t.ninit; i += blockDim.x) t.init[i] = kAffNeg;
    __syncthreads();
    stamp(3, false);
    if (t.stamps) {
        AffLevelPlan nx = t.next;
        nx.stamps = t.stamps + 8;
        aff_level_plan_body(nx);
    } else {
        aff_level_plan_body(t.next);
    }
    __syncthreads();
    stamp(4, false);
}

// Final level: Gotoh with predecessor bytes for one 128-column block per wave,
// the geometry of pred_kernel (lane l owns columns 2l, 2l+1, anti-diagonal
// sweep, byte pred[base + (i+j)*128 + j]).  Byte: bits 0-1 H source (0 diag,
// 1 E, 2 F, 3 clamped), bit 2 E extends, bit 3 F extends.  Borders by the start
// mode (the local clamp for BM_FREE_LOCAL).  A free end (e_end 2) also finds the
// exit cell: local, the first maximum of all cells in row-major order;
// semiglobal, the first maximum of the last row, then of the last column (when
// the block holds it) if strictly greater -> blocks[b].xi / xj.
// PB: the predecessor slab (LDS or HBM), QB: the block's query rows (LDS:
// staged, HBM: Q + oi).  Returns the exit cell (xi, xj) of a free end in every lane.
// XFREE / XLOCAL: the block holds a free end (e_end 2), local (first maximum of
// all cells) or semiglobal (last row, then the last column).  The sweep is
// branch-free (selects), and a lane's query byte for the next step is read one
// step ahead (B's row is A's row of the previous step).
template <bool XFREE, bool XLOCAL, typename PB, typename QB>
__device__ __forceinline__ int2 aff_pred_sweep(const BlockInfo& bi, QB qrow, const uint8_t* __restrict__ S, PB pred,
                                               int match, int mismatch, int go, int ge) {
    const int lane = threadIdx.x;
    const int NEG = kAffNeg;
    const int bm = bi.smode;
    const bool clamp = bm == BM_FREE_LOCAL;
    const int C = (bm == BM_EFREE || bm == BM_EPAID) ? NEG : 0;
    const bool lnormal = bm == BM_NORMAL, lzero = bm == BM_FREE_LOCAL || bm == BM_FREE_SEMI_OPEN;
    auto top = [&](int j) { return j < 0 ? C : aff_top_h(bm, j, go, ge); };
    const bool xlastcol = bi.flags & 2;
    const int h = bi.h, w = bi.w;
    const int jA = 2 * lane, jB = 2 * lane + 1;
    const bool colA = jA < w, colB = jB < w;
    const int sA = colA ? (int)S[bi.oj + jA] : 0x100;
    const int sB = colB ? (int)S[bi.oj + jB] : 0x100;
    int HA = top(jA), FA = NEG, EA = NEG;   // A's current row state (row -1: the top border)
    int HB = top(jB), FB = NEG, EB = NEG;
    int HAo = top(jA);                       // A one step earlier: B's diagonal
    int dA = C;                              // A's diagonal (lane 0: the left border, row -1)
    int xvA = -2147483647, xrA = 0, xvB = -2147483647, xrB = 0, cv = -2147483647, cr = 0;
    const int nsteps = h + 127;
    int qA_next = (-jA >= 0 && -jA < h) ? (int)qrow[-jA] : 0x200;
    int qA_prev = 0x200;
    for (int d = 0; d < nsteps; ++d) {
        const int iA = d - jA, iB = iA - 1;
        const int qA = qA_next, qB = qA_prev;   // rows iA and iB (= iA of the previous step)
        qA_prev = qA;
        qA_next = (iA + 1 >= 0 && iA + 1 < h) ? (int)qrow[iA + 1] : 0x200;
        // A's left neighbour = lane l-1's B at row iA (lane 0: the left border)
        const int lb = iA < 0 ? C : (lnormal ? go + (iA + 1) * ge : (lzero ? 0 : NEG));
        const int lH = wave_shr1(lb, HB);
        const int lE = wave_shr1(NEG, EB);
        const bool actA = colA && iA >= 0 && iA < h;
        const bool actB = colB && iB >= 0 && iB < h;
        // B (uses A's state before A's update: A at row iB)
        const int e1B = EA + ge, e2B = HA + go + ge;
        const int eB = e1B > e2B ? e1B : e2B;
        const int f1B = FB + ge, f2B = HB + go + ge;
        const int fB = f1B > f2B ? f1B : f2B;
        int hB = HAo + (qB == sB ? match : mismatch), sB3 = 0;
        if (eB > hB) { hB = eB; sB3 = 1; }
        if (fB > hB) { hB = fB; sB3 = 2; }
        if (clamp && 0 > hB) { hB = 0; sB3 = 3; }
        const int pB = sB3 | (e1B > e2B ? 4 : 0) | (f1B > f2B ? 8 : 0);
        // A
        const int e1A = lE + ge, e2A = lH + go + ge;
        const int eA = e1A > e2A ? e1A : e2A;
        const int f1A = FA + ge, f2A = HA + go + ge;
        const int fA = f1A > f2A ? f1A : f2A;
        int hA = dA + (qA == sA ? match : mismatch), sA3 = 0;
        if (eA > hA) { hA = eA; sA3 = 1; }
        if (fA > hA) { hA = fA; sA3 = 2; }
        if (clamp && 0 > hA) { hA = 0; sA3 = 3; }
        const int pA = sA3 | (e1A > e2A ? 4 : 0) | (f1A > f2A ? 8 : 0);
        dA = lH;   // next step's diagonal of A: lane l-1's B at row iA
        HB = actB ? hB : HB;
        FB = actB ? fB : FB;
        EB = actB ? eB : EB;
        if constexpr (XFREE) {
            if constexpr (XLOCAL) {
                const bool u = actB && hB > xvB;
                xvB = u ? hB : xvB;
                xrB = u ? iB : xrB;
            } else {
                xvB = (actB && iB == h - 1) ? hB : xvB;
                const bool u = xlastcol && actB && jB == w - 1 && hB > cv;
                cv = u ? hB : cv;
                cr = u ? iB : cr;
            }
        }
        HAo = HA;
        HA = actA ? hA : HA;
        FA = actA ? fA : FA;
        EA = actA ? eA : EA;
        if constexpr (XFREE) {
            if constexpr (XLOCAL) {
                const bool u = actA && hA > xvA;
                xvA = u ? hA : xvA;
                xrA = u ? iA : xrA;
            } else {
                xvA = (actA && iA == h - 1) ? hA : xvA;
                const bool u = xlastcol && actA && jA == w - 1 && hA > cv;
                cv = u ? hA : cv;
                cr = u ? iA : cr;
            }
        }
        const uint16_t pk = (uint16_t)((actA ? pA : 0) | ((actB ? pB : 0) << 8));
        reinterpret_cast<uint16_t*>(pred)[d * 64 + lane] = pk;
    }
    if constexpr (XFREE) {
        // best (value, row, column) of the lane: A before B (same row: smaller column)
        int v = xvA, r = XLOCAL ? xrA : h - 1, c = jA;
        if (xvB > v || (xvB == v && XLOCAL && xrB < r)) {
            v = xvB;
            r = XLOCAL ? xrB : h - 1;
            c = jB;
        }
        if (!colA) v = -2147483647;
        // first maximum over lanes: larger value, then smaller row, then smaller column
        for (int o = 32; o >= 1; o >>= 1) {
            const int v2 = __shfl_xor(v, o), r2 = __shfl_xor(r, o), c2 = __shfl_xor(c, o);
            if (v2 > v || (v2 == v && (r2 < r || (r2 == r && c2 < c)))) {
                v = v2;
                r = r2;
                c = c2;
            }
        }
        if (!XLOCAL && xlastcol) {   // the last column's first maximum, if strictly greater
            const int owner = (w - 1) >> 1;
            const int cv0 = __shfl(cv, owner), cr0 = __shfl(cr, owner);
            if (cv0 > v) {
                v = cv0;
                r = cr0;
                c = w - 1;
            }
        }
        return make_int2(r, c);
    }
    return make_int2(0, 0);
}

template <typename PB, typename QB>
__device__ __forceinline__ int2 aff_pred_block(const BlockInfo& bi, QB qrow, const uint8_t* __restrict__ S, PB pred,
                                               int match, int mismatch, int go, int ge) {
    if (bi.e_end != 2) return aff_pred_sweep<false, false>(bi, qrow, S, pred, match, mismatch, go, ge);
    if (bi.flags & 1) return aff_pred_sweep<true, true>(bi, qrow, S, pred, match, mismatch, go, ge);
    return aff_pred_sweep<true, false>(bi, qrow, S, pred, match, mismatch, go, ge);
}

// The same predecessors by TWO waves per block, one column per lane (wave w owns
// columns 64w .. 64w+63): lane l of wave w computes row i = d - l at its step d, so
// a wave sweeps h + 63 anti-diagonals of one cell per lane (the single-wave sweep
// above: h + 127 of two cells).  Wave 1's lane 0 takes its left neighbour (H, E)
// of row i from wave 0's lane 63 through a 128-entry LDS ring; wave 1 runs kSw2Lag
// steps behind, and both waves meet at a barrier every kSw2Chunk steps, so a row is
// in the ring (written at wave 0's step i + 63) a chunk before wave 1 reads it and
// is overwritten (row i + 128) only after.  Same bytes, same exit cell.
constexpr int kSw2Chunk = 16, kSw2Lag = 80;   // kSw2Lag >= 63 + kSw2Chunk, a multiple of it
template <bool XFREE, bool XLOCAL>
__device__ __forceinline__ int2 aff_pred_sweep2(const BlockInfo& bi, const uint8_t* qrow, const uint8_t* __restrict__ S,
                                                uint8_t* pred, int2* ring, int match, int mismatch, int go, int ge) {
    // (readfirstlane: the wave index is uniform, and the compiler must know it -- else
    // every branch on it, and on the chunk's step range, juggles exec masks)
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int NEG = kAffNeg;
    const int bm = bi.smode;
    const bool clamp = bm == BM_FREE_LOCAL;
    const int C = (bm == BM_EFREE || bm == BM_EPAID) ? NEG : 0;
    const bool lnormal = bm == BM_NORMAL, lzero = bm == BM_FREE_LOCAL || bm == BM_FREE_SEMI_OPEN;
    const bool xlastcol = bi.flags & 2;
    const int h = bi.h, w = bi.w, goe = go + ge;
    const int j = 64 * wv + lane;
    const bool col = j < w;
    const int sj = col ? (int)S[bi.oj + j] : 0x100;
    // row -1: H(-1, j) = the top border, E = F = -inf; the diagonal of row 0: H(-1, j-1)
    int Hc = aff_top_h(bm, j, go, ge), Ec = NEG, F = NEG;
    int dH = j == 0 ? C : aff_top_h(bm, j - 1, go, ge);
    int xv = -2147483647, xr = 0, cv = -2147483647, cr = 0;
    const int nsteps = h + 63;
    const int nchunks = (nsteps + kSw2Lag + kSw2Chunk - 1) / kSw2Chunk;
    uint8_t* pw = pred + 64 * wv * 128 + j;   // + d * 128: anti-diagonal d + 64 wv
    // one chunk of a wave's steps, specialised per wave and per clamp (no per-step branch
    // on either)
    auto chunk = [&](auto wv_c, auto clamp_c, int d0) {
        constexpr int WV = decltype(wv_c)::value;
        constexpr bool CL = decltype(clamp_c)::value;
        // the chunk's LDS reads up front, one wait: the query bytes of the lane's 16 rows,
        // wave 1's 16 left neighbours from the ring (a step that waits for an LDS read
        // every step ran at ~550 cycles)
        int qk[kSw2Chunk];
        int2 rk[kSw2Chunk];
#pragma unroll
        for (int k = 0; k < kSw2Chunk; ++k) {   // (unconditional reads: one wait)
            const int i = d0 + k - lane;
            qk[k] = qrow[min(max(i, 0), h - 1)];
        }
#pragma unroll
        for (int k = 0; k < kSw2Chunk; ++k) {
            const int i = d0 + k - lane;
            qk[k] = (i >= 0 && i < h) ? qk[k] : 0x200;
        }
        if constexpr (WV == 1) {
#pragma unroll
            for (int k = 0; k < kSw2Chunk; ++k) rk[k] = ring[(d0 + k) & 127];   // (H, E) of (d, 63)
        }
#pragma unroll
        for (int k = 0; k < kSw2Chunk; ++k) {
            const int d = d0 + k;
            if (d >= nsteps) continue;   // (uniform; not a break: the loop stays unrolled)
            const int i = d - lane;
            int lH, lE;
            if constexpr (WV == 0) {
                // lane 0: the block's left border at row d (>= 0)
                const int lb = lnormal ? go + (d + 1) * ge : (lzero ? 0 : NEG);
                lH = wave_shr1(lb, Hc);
                lE = wave_shr1(NEG, Ec);
            } else {
                lH = wave_shr1(rk[k].x, Hc);
                lE = wave_shr1(rk[k].y, Ec);
            }
            const bool act = col && (unsigned)i < (unsigned)h;
            const int e1 = lE + ge, e2 = lH + goe;
            const int e = e1 > e2 ? e1 : e2;
            const int f1 = F + ge, f2 = Hc + goe;
            const int f = f1 > f2 ? f1 : f2;
            const int hd = dH + (qk[k] == sj ? match : mismatch);
            int hh = hd, src = 0;
            if (e > hh) { hh = e; src = 1; }
            if (f > hh) { hh = f; src = 2; }
            if (CL && 0 > hh) { hh = 0; src = 3; }
            pw[d * 128] = (uint8_t)(src | (e1 > e2 ? 4 : 0) | (f1 > f2 ? 8 : 0));
            dH = lH;
            Hc = act ? hh : Hc;
            Ec = act ? e : Ec;
            F = act ? f : F;
            if constexpr (WV == 0)
                if (lane == 63 && i >= 0) ring[i & 127] = make_int2(hh, e);
            if constexpr (XFREE) {
                if constexpr (XLOCAL) {
                    const bool u = act && hh > xv;
                    xv = u ? hh : xv;
                    xr = u ? i : xr;
                } else {
                    xv = (act && i == h - 1) ? hh : xv;
                    const bool u = xlastcol && act && j == w - 1 && hh > cv;
                    cv = u ? hh : cv;
                    cr = u ? i : cr;
                }
            }
        }
    };
    using W0 = std::integral_constant<int, 0>;
    using W1 = std::integral_constant<int, 1>;
    using CT = std::integral_constant<bool, true>;
    using CF = std::integral_constant<bool, false>;
    for (int c = 0; c < nchunks; ++c) {
        const int d0 = c * kSw2Chunk - (wv ? kSw2Lag : 0);
        if (d0 >= 0 && d0 < nsteps) {   // (d0 is a multiple of the chunk)
            if (wv == 0) {
                if (clamp) chunk(W0{}, CT{}, d0);
                else chunk(W0{}, CF{}, d0);
            } else {
                if (clamp) chunk(W1{}, CT{}, d0);
                else chunk(W1{}, CF{}, d0);
            }
        }
        __syncthreads();
    }
    if constexpr (XFREE) {
        // first maximum over the block: larger value, then smaller row, then smaller column
        int v = col ? xv : -2147483647, r = XLOCAL ? xr : h - 1, cc = j;
        for (int o = 32; o >= 1; o >>= 1) {
            const int v2 = __shfl_xor(v, o), r2 = __shfl_xor(r, o), c2 = __shfl_xor(cc, o);
            if (v2 > v || (v2 == v && (r2 < r || (r2 == r && c2 < cc)))) {
                v = v2;
                r = r2;
                cc = c2;
            }
        }
        // across the two waves (the ring is free now), then the last column's first
        // maximum if strictly greater (semiglobal)
        int* red = reinterpret_cast<int*>(ring);
        if (lane == 0) {
            red[3 * wv] = v;
            red[3 * wv + 1] = r;
            red[3 * wv + 2] = cc;
        }
        if (!XLOCAL && xlastcol && j == w - 1) {
            red[6] = cv;
            red[7] = cr;
        }
        __syncthreads();
        v = red[0];
        r = red[1];
        cc = red[2];
        const int v2 = red[3], r2 = red[4], c2 = red[5];
        if (v2 > v || (v2 == v && (r2 < r || (r2 == r && c2 < cc)))) {
            v = v2;
            r = r2;
            cc = c2;
        }
        if (!XLOCAL && xlastcol && red[6] > v) {
            r = red[7];
            cc = w - 1;
        }
        __syncthreads();
        return make_int2(r, cc);
    }
    return make_int2(0, 0);
}

__device__ __forceinline__ int2 aff_pred_block2(const BlockInfo& bi, const uint8_t* qrow, const uint8_t* __restrict__ S,
                                                uint8_t* pred, int2* ring, int match, int mismatch, int go, int ge) {
    if (bi.e_end != 2) return aff_pred_sweep2<false, false>(bi, qrow, S, pred, ring, match, mismatch, go, ge);
    if (bi.flags & 1) return aff_pred_sweep2<true, true>(bi, qrow, S, pred, ring, match, mismatch, go, ge);
    return aff_pred_sweep2<true, false>(bi, qrow, S, pred, ring, match, mismatch, go, ge);
}

// One thread: walk from the block's end (bottom-right in state H or E, or the
// free exit cell x) back to its start (anchored: the corner through the border's
// gap runs; free: a clamped cell or the border); sparse i+j+1 output.
// qrow / scol: the block's query rows and subject columns (LDS or HBM).
template <typename PB>
__device__ __forceinline__ void aff_walk_block(const BlockInfo& bi, int2 x, const uint8_t* qrow,
                                               const uint8_t* scol, PB pred, uint8_t* alq, uint8_t* als) {
    const bool free_start = bi.smode >= BM_FREE_LOCAL;
    const int64_t base = (int64_t)bi.oi + bi.oj;
    int i = bi.e_end == 2 ? x.x : bi.h - 1, j = bi.e_end == 2 ? x.y : bi.w - 1;
    int st = bi.e_end == 1 ? 1 : 0;
    while (i >= 0 || j >= 0) {
        const int64_t pos = base + i + j + 1;
        if (i < 0 || j < 0) {
            if (free_start) break;   // the path starts on the border
            if (i < 0) {
                alq[pos] = '_';
                als[pos] = scol[j];
                --j;
            } else {
                alq[pos] = qrow[i];
                als[pos] = '_';
                --i;
            }
            continue;
        }
        const int pb = pred[(i + j) * 128 + j];
        if (st == 0) {
            const int hs = pb & 3;
            if (hs == 3) break;   // clamped: the path starts after this cell
            if (hs == 0) {
                alq[pos] = qrow[i];
                als[pos] = scol[j];
                --i;
                --j;
            } else {
                st = hs;
            }
        } else if (st == 1) {
            alq[pos] = '_';
            als[pos] = scol[j];
            st = (pb & 4) ? 1 : 0;
            --j;
        } else {
            alq[pos] = qrow[i];
            als[pos] = '_';
            st = (pb & 8) ? 2 : 0;
            --i;
        }
    }
}

// The same walk over an LDS slab, by the whole wave in lock step (every value is
// wave-uniform: scalar registers and branches, no exec-mask juggling), recording
// only the path: position p = i + j + 1 gets (i + 1) << 2 | op (1 both symbols,
// 2 a gap in the query, 3 a gap in the subject; 0 the position a diagonal move
// skips) in bytes 126-127 of slab row p, which the walk has left behind (it reads
// anti-diagonals i + j < p from then on; row h + 127 is the slab's spare row).  The
// symbols are fetched afterwards by all lanes (aff_trace_out).  Returns the recorded
// range [lo, hi] of positions.
__device__ __forceinline__ int2 aff_walk_trace(const BlockInfo& bi, int2 x, uint8_t* slab) {
    // (readfirstlane: the values are uniform, and the compiler must know it)
    const bool free_start = __builtin_amdgcn_readfirstlane(bi.smode) >= BM_FREE_LOCAL;
    const int e_end = __builtin_amdgcn_readfirstlane(bi.e_end);
    int i = __builtin_amdgcn_readfirstlane(e_end == 2 ? x.x : bi.h - 1);
    int j = __builtin_amdgcn_readfirstlane(e_end == 2 ? x.y : bi.w - 1);
    int st = e_end == 1 ? 1 : 0;
    const int hi = i + j + 1;
    int lo = hi + 1;
    auto rec = [&](int p, int ii, int op) {
        *reinterpret_cast<uint16_t*>(slab + p * 128 + 126) = (uint16_t)(((ii + 1) << 2) | op);
    };
    // inside the block: one move per iteration, branch-free on scalars.  The cell's
    // source `eff` (0 diagonal, 1 E, 2 F, 3 clamped) is its H source in state H, else
    // the state; a gap move takes the next state from the same byte (bit 2 E extends,
    // bit 3 F extends: (pb >> (eff + 1)) & 1), as two iterations of the reference walk
    // do (the state switch, then the move)
    bool stop = false;
    while (i >= 0 && j >= 0) {
        const int p = i + j + 1;
        const int pb = __builtin_amdgcn_readfirstlane((int)slab[(i + j) * 128 + j]);
        const int eff = st ? st : (pb & 3);
        if (eff == 3) {   // clamped: the path starts after this cell
            stop = true;
            break;
        }
        rec(p, i, eff + 1);
        if (eff == 0) rec(p - 1, 0, 0);
        lo = eff == 0 ? p - 1 : p;
        st = ((pb >> (eff + 1)) & 1) * eff;
        i -= eff != 1;
        j -= eff != 2;
    }
    // on the border (anchored starts): the rest of the row above, or of the column left
    if (!stop && !free_start) {
        for (; i < 0 && j >= 0; --j) {
            rec(j, -1, 2);
            lo = j;
        }
        for (; j < 0 && i >= 0; --i) {
            rec(i, i, 3);
            lo = i;
        }
    }
    return make_int2(lo, hi);
}

// The recorded path's symbols, one position per lane: sparse i+j+1 output at oi+oj+p.
__device__ __forceinline__ void aff_trace_out(const BlockInfo& bi, int2 r, const uint8_t* slab,
                                              const uint8_t* __restrict__ Q, const uint8_t* __restrict__ S,
                                              uint8_t* alq, uint8_t* als) {
    const int64_t base = (int64_t)bi.oi + bi.oj;
    for (int p = r.x + (int)threadIdx.x; p <= r.y; p += blockDim.x) {
        const int t = *reinterpret_cast<const uint16_t*>(slab + p * 128 + 126);
        const int op = t & 3;
        if (op == 0) continue;
        const int i = (t >> 2) - 1, j = p - 1 - i;
        alq[base + p] = op == 2 ? (uint8_t)'_' : Q[bi.oi + i];
        als[base + p] = op == 3 ? (uint8_t)'_' : S[bi.oj + j];
    }
}

// Final level, one workgroup (two waves) per 128-column block: predecessors, then the
// walk in the same launch.  A block of h <= lds_rows rows (the launch's tallest
// block, capped at kPredLdsMaxRows) keeps its query rows and its (h + 127) x 128
// predecessor bytes in LDS, so neither the sweep's query reads nor the walk's
// dependent reads go to HBM: both waves sweep it (aff_pred_sweep2), wave 0 walks it
// in lock step (aff_walk_trace), both write the symbols.  Taller blocks (long
// vertical gaps) use the HBM slab at pred_base, wave 0's sweep (aff_pred_sweep) and
// lane 0's walk (aff_walk_block).
//
// Launch modes: list == nullptr walks block blockIdx.x (defer: skips blocks taller than
// lds_rows and those the path does not touch, flags bit 2 -- aff_final_blocks_kernel's
// table); else the workgroups walk the blocks list[1 .. list[0]] in turn (the tall
// blocks deferred by the first launch).
__device__ __forceinline__ void aff_predwalk_one(BlockInfo* __restrict__ blocks, int b, const uint8_t* __restrict__ Q,
                                                 const uint8_t* __restrict__ S, uint8_t* __restrict__ pred, int match,
                                                 int mismatch, int go, int ge, uint8_t* alq, uint8_t* als, int lds_rows,
                                                 uint8_t* pw_lds);

__global__ __launch_bounds__(128) void aff_predwalk_kernel(BlockInfo* __restrict__ blocks, int nblocks,
                                                          const uint8_t* __restrict__ Q, const uint8_t* __restrict__ S,
                                                          uint8_t* __restrict__ pred, int match, int mismatch, int go,
                                                          int ge, uint8_t* alq, uint8_t* als, int lds_rows,
                                                          const int32_t* __restrict__ list, int defer) {
    extern __shared__ __attribute__((aligned(16))) uint8_t pw_lds[];
    if (list) {
        const int cnt = min(list[0], nblocks);
        for (int k = blockIdx.x; k < cnt; k += gridDim.x) {
            aff_predwalk_one(blocks, list[1 + k], Q, S, pred, match, mismatch, go, ge, alq, als, lds_rows, pw_lds);
            __syncthreads();   // (the next block reuses the LDS slab)
        }
        return;
    }
    const int b = blockIdx.x;
    if (b >= nblocks) return;
    if (defer) {
        const BlockInfo bi = blocks[b];
        if ((bi.flags & 4) || bi.h > lds_rows) return;
    }
    aff_predwalk_one(blocks, b, Q, S, pred, match, mismatch, go, ge, alq, als, lds_rows, pw_lds);
}

#ifdef ANYSEQ_PW_PHASES   // tools/micro/pw_micro.hip: each phase repeated to time it
__device__ int g_pw_rep = 0;
#define PW_REPS(bit) (1 + ((g_pw_rep >> (bit)) & 1))
#else
#define PW_REPS(bit) 1
#endif
__device__ __forceinline__ void aff_predwalk_one(BlockInfo* __restrict__ blocks, int b, const uint8_t* __restrict__ Q,
                                                 const uint8_t* __restrict__ S, uint8_t* __restrict__ pred, int match,
                                                 int mismatch, int go, int ge, uint8_t* alq, uint8_t* als, int lds_rows,
                                                 uint8_t* pw_lds) {
    const BlockInfo bi = blocks[b];
    if (bi.flags & 4) return;                 // the path does not touch the block
    if (bi.e_end == 2 && bi.h <= 0) return;   // the path ended at the block's corner
    int2 x = make_int2(0, 0);
    if (bi.h <= lds_rows) {
        // LDS: the slab (+ the spare row), the h query rows, the two waves' ring
        uint8_t* qs = pw_lds + (lds_rows + 128) * 128;
        int2* ring = reinterpret_cast<int2*>(qs + ((lds_rows + 15) & ~15));
        if (bi.h > 0) {
            for (int i = threadIdx.x; i < bi.h; i += blockDim.x) qs[i] = Q[bi.oi + i];
            __syncthreads();
            for (int rep = 0; rep < PW_REPS(0); ++rep)
                x = aff_pred_block2(bi, (const uint8_t*)qs, S, pw_lds, ring, match, mismatch, go, ge);
        }
        // wave 0 walks (the walk's dependent reads are all LDS: an HBM read per step
        // would cost ~1 us), both waves write the symbols
        for (int rep = 0; rep < PW_REPS(1); ++rep) {
            if (threadIdx.x < 64) {
                const int2 r = aff_walk_trace(bi, x, pw_lds);
                if (threadIdx.x == 0) ring[0] = r;
            }
            __syncthreads();
        }
        for (int rep = 0; rep < PW_REPS(2); ++rep) aff_trace_out(bi, ring[0], pw_lds, Q, S, alq, als);
    } else {
        uint8_t* slab = pred + bi.pred_base;
        if (threadIdx.x < 64) {   // (one wave: the single-wave sweep, lane 0's walk)
            x = aff_pred_block(bi, Q + bi.oi, S, slab, match, mismatch, go, ge);
            __threadfence_block();
        }
        __syncthreads();
        if (threadIdx.x == 0) aff_walk_block(bi, x, Q + bi.oi, S + bi.oj, (const uint8_t*)slab, alq, als);
    }
    if (threadIdx.x == 0 && bi.e_end == 2) {
        blocks[b].xi = x.x;
        blocks[b].xj = x.y;
    }
}

// The final level's block table from the last level's splits (device-planned
// constructs), so the final level is enqueued behind the levels with
// no host round trip: block b spans rows [spl[b], spl[b+1]) and columns [128b,
// 128b + 128), its start / end types typ[b] / typ[b+1] (the host builder's rules,
// aff_construct_hb).  Blocks the path does not touch -- and every block when the
// level-1 value says the empty alignment (kind != global, <= 0) -- get flags bit 2.
// Blocks taller than small_rows go to `tall` (count, then indices) for the second
// predwalk launch; those taller than kPredLdsMaxRows use the HBM slab at (oi + 127 b)
// x 128 (no scan: the slabs of consecutive blocks abut).  Any split out of order or
// range, or type out of range, sets *err and leaves every block skipped.
__global__ __launch_bounds__(1024) void aff_final_blocks_kernel(const AffFinalPlan a) {
    __shared__ int bad, ntall;
    if (threadIdx.x == 0) {
        bad = 0;
        ntall = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= a.nb; i += blockDim.x) {
        const int v = a.spl[i], t = a.typ[i];
        const bool ok = v >= 0 && v <= a.n && (i == 0 || a.spl[i - 1] <= v) && t >= T_H && t <= T_AFTER;
        if (!ok) atomicOr(&bad, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) *a.err = bad ? 1u : 0u;
    // (score null: no Hirschberg level ran, the host has already checked the score)
    const bool stop = bad || (a.score && a.kind != KIND_GLOBAL && *a.score <= 0);
    for (int b = threadIdx.x; b < a.nb; b += blockDim.x) {
        BlockInfo bi{};
        const int ts = a.typ[b], te = a.typ[b + 1];
        bi.oi = a.spl[b];
        bi.h = a.spl[b + 1] - bi.oi;
        bi.oj = b * 128;   // (the final blocks' width, align.impala:18)
        bi.w = min(128, a.m - bi.oj);
        bi.pred_base = ((int64_t)bi.oi + 127 * (int64_t)b) * 128;
        bi.smode = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : aff_free_bm(a.kind, bi.oj == 0);
        bi.e_end = te == T_H ? 0 : te == T_E ? 1 : 2;
        bi.flags = (a.kind == KIND_LOCAL ? 1 : 0) | (bi.oj + bi.w == a.m ? 2 : 0);
        if (stop || ts == T_BEFORE || te == T_AFTER) bi.flags |= 4;
        if (a.world > 1 && b % a.world != a.rank) bi.flags |= 4;   // sharded: another rank walks it
        a.blocks[b] = bi;
        if (!(bi.flags & 4) && bi.h > a.small_rows) a.tall[1 + atomicAdd(&ntall, 1)] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) a.tall[0] = ntall;
}

// --------------------------------------------------------------- launchers --
#ifndef ANYSEQ_MICRO   // tools/micro includes the kernels without the launchers
template <int KIND, int R, int X, int NW, int CH>
static hipError_t launch_fill_t(const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    hipLaunchKernelGGL((fill_kernel<KIND, R, X, NW, CH>), dim3(grid), dim3(64 * (NW + 1)), 0, st, probs, groups,
                       ngroups, dq, err, fp);
    return hipGetLastError();
}

template <int R, int X, int NW, int CH>
static hipError_t launch_fill_r(const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    switch (fp.kind) {
        case KIND_GLOBAL:
            return launch_fill_t<KIND_GLOBAL, R, X, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        case KIND_SEMIGLOBAL:
            return launch_fill_t<KIND_SEMIGLOBAL, R, X, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        default:
            return launch_fill_t<KIND_LOCAL, R, X, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
    }
}

template <int NW, int CH>
static hipError_t launch_fill_n(int R, const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    switch (R) {
        case 1: return launch_fill_r<1, 0, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        case 2: return launch_fill_r<2, 0, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
        default: return launch_fill_r<4, 0, NW, CH>(probs, groups, ngroups, dq, err, fp, grid, st);
    }
}

template <int CH>
static hipError_t launch_fill_c(int R, int NW, const DPProblem* probs, const GroupRef* groups, int ngroups,
                                uint32_t* dq, uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    switch (NW) {
        case 3: return launch_fill_n<3, CH>(R, probs, groups, ngroups, dq, err, fp, grid, st);
        case 4: return launch_fill_n<4, CH>(R, probs, groups, ngroups, dq, err, fp, grid, st);
        case 7: return launch_fill_n<7, CH>(R, probs, groups, ngroups, dq, err, fp, grid, st);
        default: return launch_fill_n<8, CH>(R, probs, groups, ngroups, dq, err, fp, grid, st);
    }
}

template <int NW, int RR>
static hipError_t launch_fill_aff_n(const DPProblem* probs, const GroupRef* groups, int ngroups, uint32_t* dq,
                                    uint32_t* err, const FillParams& fp, int grid, hipStream_t st) {
    hipLaunchKernelGGL((fill_affine_kernel<NW, RR>), dim3(grid), dim3(NW == 8 ? 512 : 64 * (NW + 1)), 0, st, probs,
                       groups, ngroups, dq, err, fp);
    return hipGetLastError();
}
#endif  // ANYSEQ_MICRO
}  // namespace anyseq

#ifndef ANYSEQ_MICRO
extern "C" {

// Fill launcher: R rows per lane in {1,2,4}; NW compute waves per workgroup in
// {3,4,7,8} (+1 I/O wave); CH (steps per block = hand-off chunk) in {16,32}.
hipError_t anyseq_launch_fill(int R, int CH, int NW, const anyseq::DPProblem* probs, const anyseq::GroupRef* groups,
                              int ngroups, uint32_t* dq, uint32_t* err, const anyseq::FillParams* fp, int grid,
                              hipStream_t st) {
    using namespace anyseq;
    if (CH == 16) return launch_fill_c<16>(R, NW, probs, groups, ngroups, dq, err, *fp, grid, st);
    return launch_fill_c<32>(R, NW, probs, groups, ngroups, dq, err, *fp, grid, st);
}

// One launch instead of three memsets ahead of a fill (each host API call costs
// several microseconds on the level's critical path): zero the launch block's
// counters and flags, set the caller's best cells to "minus infinity", and fill the
// hand-off rows with the sentinel.
namespace anyseq {
__global__ __launch_bounds__(256) void fill_prep_kernel(uint32_t* zero, int nzero, int32_t* init, int ninit,
                                                        int32_t init_value, uint4* sent, size_t nsent, uint32_t sv,
                                                        const uint4* up_src, uint4* up_dst, int nup,
                                                        const uint32_t* nsent_dev) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    // a device-planned level: the plan kernel sized the hand-off rows (at most nsent)
    if (nsent_dev) nsent = min(nsent, (size_t)*nsent_dev);
    // the launch's descriptors, read straight from the host's pinned staging area (no
    // separate copy operation in front of this kernel)
    for (size_t i = tid; i < (size_t)nup; i += nth) up_dst[i] = up_src[i];
    for (size_t i = tid; i < (size_t)nzero; i += nth) zero[i] = 0u;
    for (size_t i = tid; i < (size_t)ninit; i += nth) init[i] = init_value;
    const uint4 v = make_uint4(sv, sv, sv, sv);
    for (size_t i = tid; i < nsent; i += nth) sent[i] = v;
}
}  // namespace anyseq

// Alphabet codes of a sequence pair.  The affine fill compares codes,
// which are equal iff the bytes are (raw byte equality, align.impala:130-133); with at
// most 8 distinct symbols its steady state reads the diagonal weights of 4 steps from a
// per-lane table with one v_perm_b32.  Code 0xFF is never a code of a pair with fewer
// than 255 symbols: the virtual prologue's columns left of 0 use it.
namespace anyseq {
// (+ optionally the ' ' prefill of a construct's two output strings, fill_len bytes each:
// one launch fewer in front of the construct's first fill)
__global__ __launch_bounds__(256) void seq_presence_kernel(const uint8_t* __restrict__ q, int n,
                                                           const uint8_t* __restrict__ s, int m, uint32_t* mask,
                                                           uint8_t* fill0, uint8_t* fill1, size_t fill_len) {
    __shared__ uint32_t sm[8];
    if (threadIdx.x < 8) sm[threadIdx.x] = 0;
    __syncthreads();
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < fill_len; i += nth) {
        fill0[i] = ' ';
        fill1[i] = ' ';
    }
    const size_t total = (size_t)n + (size_t)m;
    for (size_t i = tid; i < total; i += nth) {
        const uint32_t b = i < (size_t)n ? q[i] : s[i - n];
        const uint32_t bit = 1u << (b & 31);
        // (a repeated symbol only reads: the first lanes of a symbol set its bit)
        if (!(__hip_atomic_load(&sm[b >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & bit))
            atomicOr(&sm[b >> 5], bit);
    }
    __syncthreads();
    if (threadIdx.x < 8 && sm[threadIdx.x]) atomicOr(&mask[threadIdx.x], sm[threadIdx.x]);
}
// q ++ s -> their codes (one buffer of n + m bytes): every block builds the code table
// from the presence mask (code(byte) = rank of the byte among the present bytes, 0xfe
// for an absent one; block 0 also writes it out and alpha[0] = the number of symbols),
// then recodes its share; the last block to finish clears the mask for the next pair.
__global__ __launch_bounds__(256) void seq_recode_kernel(const uint8_t* __restrict__ q, int n,
                                                         const uint8_t* __restrict__ s, int m, uint8_t* table,
                                                         int32_t* alpha, uint8_t* out, uint32_t* mask,
                                                         uint32_t* done) {
    __shared__ uint8_t tb[256];
    __shared__ uint32_t sm[8];
    __shared__ int last;
    const int t = threadIdx.x;
    if (t < 8) sm[t] = mask[t];
    __syncthreads();
    {
        const uint32_t w = sm[t >> 5];
        int rank = __popc(w & ((1u << (t & 31)) - 1u));
        for (int k = 0; k < (t >> 5); ++k) rank += __popc(sm[k]);
        tb[t] = ((w >> (t & 31)) & 1u) ? (uint8_t)rank : (uint8_t)0xfe;
        if (blockIdx.x == 0) {
            table[t] = tb[t];
            if (t == 0) {
                int tot = 0;
                for (int k = 0; k < 8; ++k) tot += __popc(sm[k]);
                *alpha = tot;
            }
        }
    }
    __syncthreads();
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    const size_t total = (size_t)n + (size_t)m;
    for (size_t i = tid; i < total; i += nth) out[i] = tb[i < (size_t)n ? q[i] : s[i - n]];
    // (every block has read the mask: the last one clears it, and the counter)
    __syncthreads();
    if (t == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last && t < 8) mask[t] = 0u;
    if (last && t == 0) *done = 0u;
}
}  // namespace anyseq


hipError_t anyseq_launch_seq_codes(const uint8_t* q, int n, const uint8_t* s, int m, uint32_t* mask, uint8_t* table,
                                   int32_t* alpha, uint8_t* out, uint8_t* fill0, uint8_t* fill1, size_t fill_len,
                                   hipStream_t st) {
    const size_t total = (size_t)n + (size_t)m;
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>(1024, (std::max(total, fill_len) + 4095) / 4096));
    hipLaunchKernelGGL(anyseq::seq_presence_kernel, dim3(blocks), dim3(256), 0, st, q, n, s, m, mask, fill0, fill1,
                       fill0 ? fill_len : 0);
    hipLaunchKernelGGL(anyseq::seq_recode_kernel, dim3(blocks), dim3(256), 0, st, q, n, s, m, table, alpha, out, mask,
                       mask + 8);
    return hipGetLastError();
}

// Emulated ranks of the sharded construct (local mode): the views'
// level columns / best cells reduced over the views in place (op 0 SUM, 1 MAX), as the
// RCCL all-reduce does across processes; strings merged by a byte-wise MAX.
namespace anyseq {
__global__ void view_reduce_i32_kernel(int32_t* base, size_t stride, int nviews, size_t n, int op) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        int32_t a = base[i];
        for (int v = 1; v < nviews; ++v) {
            const int32_t x = base[(size_t)v * stride + i];
            a = op ? max(a, x) : a + x;
        }
        for (int v = 0; v < nviews; ++v) base[(size_t)v * stride + i] = a;
    }
}
__global__ void view_max_u8_kernel(uint8_t* dst, const uint8_t* others, size_t stride, int nothers, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint8_t a = dst[i];
        for (int v = 0; v < nothers; ++v) a = max(a, others[(size_t)v * stride + i]);
        dst[i] = a;
    }
}
}  // namespace anyseq

hipError_t anyseq_launch_view_reduce_i32(int32_t* base, size_t stride, int nviews, size_t n, int op, hipStream_t st) {
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>(1024, (n + 255) / 256));
    hipLaunchKernelGGL(anyseq::view_reduce_i32_kernel, dim3(blocks), dim3(256), 0, st, base, stride, nviews, n, op);
    return hipGetLastError();
}
hipError_t anyseq_launch_view_max_u8(uint8_t* dst, const uint8_t* others, size_t stride, int nothers, size_t n,
                                     hipStream_t st) {
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>(1024, (n + 255) / 256));
    hipLaunchKernelGGL(anyseq::view_max_u8_kernel, dim3(blocks), dim3(256), 0, st, dst, others, stride, nothers, n);
    return hipGetLastError();
}

// In-process sharded transport: one kernel per chunk copies the chunk's H rows (and
// affine E rows) into the neighbour's left column, then sets the chunk's ready
// flag with a release store after the data (one launch instead of two copies and
// a memset through the runtime's copy paths).
namespace anyseq {
__global__ __launch_bounds__(256) void shard_chunk_copy_kernel(int32_t* __restrict__ dst, const int32_t* __restrict__ src,
                                                               int n, int32_t* __restrict__ dst_e,
                                                               const int32_t* __restrict__ src_e, int ne,
                                                               uint32_t* flag) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    if (dst_e)
        for (int i = threadIdx.x; i < ne; i += blockDim.x) dst_e[i] = src_e[i];
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace anyseq

hipError_t anyseq_launch_shard_chunk_copy(int32_t* dst, const int32_t* src, int n, int32_t* dst_e,
                                          const int32_t* src_e, int ne, uint32_t* flag, hipStream_t st) {
    hipLaunchKernelGGL(anyseq::shard_chunk_copy_kernel, dim3(1), dim3(256), 0, st, dst, src, n, dst_e, src_e, ne, flag);
    return hipGetLastError();
}

hipError_t anyseq_launch_fill_prep(uint32_t* zero, int nzero, int32_t* init, int ninit, int32_t init_value,
                                   void* sent, size_t sent_bytes, uint32_t sent_value, const void* up_src, void* up_dst,
                                   size_t up_bytes, hipStream_t st) {
    const size_t n16 = sent_bytes / 16;   // (hand-off rows: whole 16-byte units)
    const int nup = (int)((up_bytes + 15) / 16);
    const size_t work = std::max<size_t>(std::max<size_t>((size_t)nzero, (size_t)ninit), std::max<size_t>(n16, nup));
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>(2048, (work + 255) / 256));
    hipLaunchKernelGGL(anyseq::fill_prep_kernel, dim3(blocks), dim3(256), 0, st, zero, nzero, init, ninit, init_value,
                       (uint4*)sent, n16, sent_value, (const uint4*)up_src, (uint4*)up_dst, nup, (const uint32_t*)nullptr);
    return hipGetLastError();
}

// The subject-code rows of an affine launch's problems (DPProblem::scode): problem
// blockIdx.y, grid-stride over its 4 shifted copies in dwords.  Column c sits at byte
// c + 64 of copy 0; copy r holds the row shifted left by r bytes.  Codes 0xFF outside
// [0, w): the virtual prologue's columns and the asm band end's columns past w.
namespace anyseq {
__global__ __launch_bounds__(256) void aff_scode_kernel(const DPProblem* __restrict__ probs, int nprobs) {
    if ((int)blockIdx.y >= nprobs) return;
    const DPProblem& P = probs[blockIdx.y];
    if (P.h <= 0 || P.w <= 0 || !P.scode) return;
    aff_scode_dwords(P, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, scode_len(P.w),
                     (int64_t)gridDim.x * blockDim.x);
}
}  // namespace anyseq

hipError_t anyseq_launch_aff_scode(const void* probs, int nprobs, int64_t max_w, hipStream_t st) {
    if (nprobs <= 0) return hipSuccess;
    const int64_t per = (4 * anyseq::scode_len((int)std::min<int64_t>(max_w, INT32_MAX - 256)) / 4 + 255) / 256;
    const int bx = (int)std::max<int64_t>(1, std::min<int64_t>(per, std::max(1, 2048 / nprobs)));
    hipLaunchKernelGGL(anyseq::aff_scode_kernel, dim3(bx, nprobs), dim3(256), 0, st,
                       (const anyseq::DPProblem*)probs, nprobs);
    return hipGetLastError();
}

// Affine fill launcher: NW compute waves per workgroup in {3, 4} (+1 I/O wave).
hipError_t anyseq_launch_fill_affine(int NW, const anyseq::DPProblem* probs, const anyseq::GroupRef* groups,
                                     int ngroups, uint32_t* dq, uint32_t* err, const anyseq::FillParams* fp, int grid,
                                     hipStream_t st) {
    using namespace anyseq;
    // (the asm steady state holds ~150 fixed VGPRs: at most 2 waves per SIMD -- NW <= 7 beside
    // the I/O wave, or NW 8 without it)
    // fp->arows 2 / 3: rows per lane (NW 4 or 7; the descriptors' nbands count 64 arows-row bands)
    // NW 8: eight compute waves, the groups' first bands forwarding their own input rows
    if (fp->arows == 2 || fp->arows == 3) {
        if (NW == 7 && fp->arows == 2) return launch_fill_aff_n<7, 2>(probs, groups, ngroups, dq, err, *fp, grid, st);
        if (NW == 4 && fp->arows == 2) return launch_fill_aff_n<4, 2>(probs, groups, ngroups, dq, err, *fp, grid, st);
        if (NW == 8 && fp->arows == 2) return launch_fill_aff_n<8, 2>(probs, groups, ngroups, dq, err, *fp, grid, st);
        if (NW == 7) return launch_fill_aff_n<7, 3>(probs, groups, ngroups, dq, err, *fp, grid, st);
        if (NW == 4) return launch_fill_aff_n<4, 3>(probs, groups, ngroups, dq, err, *fp, grid, st);
        if (NW == 8) return launch_fill_aff_n<8, 3>(probs, groups, ngroups, dq, err, *fp, grid, st);
        return hipErrorInvalidValue;
    }
    if (NW == 8) return launch_fill_aff_n<8, 1>(probs, groups, ngroups, dq, err, *fp, grid, st);
    if (NW == 3) return launch_fill_aff_n<3, 1>(probs, groups, ngroups, dq, err, *fp, grid, st);
    if (NW == 7) return launch_fill_aff_n<7, 1>(probs, groups, ngroups, dq, err, *fp, grid, st);
    return launch_fill_aff_n<4, 1>(probs, groups, ngroups, dq, err, *fp, grid, st);
}

hipError_t anyseq_launch_aff_reduce(int kind, int two, const void* rowF, int h1, const void* rowB, int h2, int m,
                                    int go, int ge, const int32_t* colF, const int32_t* colB, int32_t* out,
                                    hipStream_t st) {
    hipLaunchKernelGGL(anyseq::aff_reduce_kernel, dim3(64), dim3(256), 0, st, kind, two, (const int2*)rowF, h1,
                       (const int2*)rowB, h2, m, go, ge, colF, colB, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_semiglobal_reduce(const int32_t* row_g, int m, const int32_t* col_h, int n, int ng,
                                           int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(anyseq::semiglobal_reduce_kernel, dim3(64), dim3(256), 0, st, row_g, m, col_h, n, ng, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_front_combine(int kind, const int32_t* rowF, int h1, const int32_t* rowB, int h2, int m,
                                       int gap, const int32_t* colF, const int32_t* colB, int32_t* out,
                                       hipStream_t st) {
    hipLaunchKernelGGL(anyseq::front_combine_kernel, dim3(64), dim3(256), 0, st, kind, rowF, h1, rowB, h2, m, gap,
                       colF, colB, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_shard_combine(int kind, const int32_t* rowT, int h1, const int32_t* rowB, int h2, int w,
                                       int gap, const int32_t* lT, int sT, const int32_t* lB, int sB, int last,
                                       const int32_t* colT, const int32_t* colB, int adj, int32_t* out,
                                       hipStream_t st) {
    hipLaunchKernelGGL(anyseq::shard_combine_kernel, dim3(64), dim3(256), 0, st, kind, rowT, h1, rowB, h2, w, gap, lT,
                       sT, lB, sB, last, colT, colB, adj, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_hb_join(const void* parts, int nparts, int half, const int32_t* LH, const int32_t* LE,
                                     const int32_t* RH, const int32_t* RE, const int32_t* pbest, int go, int ge,
                                     int32_t* splits, int32_t* types, int32_t* score, hipStream_t st) {
    if (nparts > 0)
        hipLaunchKernelGGL(anyseq::aff_hb_join_kernel, dim3(nparts), dim3(256), 0, st,
                           (const anyseq::PartInfo*)parts, half, LH, LE, RH, RE, pbest, go, ge, splits, types, score);
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_hb_join2(const void* parts, int nparts, int maxlen, int half, const int32_t* LH,
                                      const int32_t* LE, const int32_t* RH, const int32_t* RE, const int32_t* pbest,
                                      int go, int ge, void* partial, int32_t* splits, int32_t* types, int32_t* score,
                                      hipStream_t st) {
    using namespace anyseq;
    const int nslices = std::max(1, (maxlen + 1 + kJoinSlice - 1) / kJoinSlice);
    if (nparts > 0) {
        hipLaunchKernelGGL(aff_hb_join_slice_kernel, dim3(nslices, nparts), dim3(256), 0, st,
                           (const PartInfo*)parts, half, LH, LE, RH, RE, pbest, go, ge, nslices, (int2*)partial);
        hipLaunchKernelGGL(aff_hb_join_final_kernel, dim3((nparts + 63) / 64), dim3(64), 0, st,
                           (const PartInfo*)parts, nparts, nslices, (const int2*)partial, splits, types, score);
    }
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_level_plan(const anyseq::AffLevelPlan* plan, hipStream_t st) {
    hipLaunchKernelGGL(anyseq::aff_level_plan_kernel, dim3(1), dim3(1024), 0, st, *plan);
    return hipGetLastError();
}

// One launch per level boundary of the device-planned construct (aff_level_tail_kernel):
// `fill_groups` workgroups at least, so the next level's sentinel fill spreads over the chip.
// Hand-off row invariant of the device-planned levels: between
// planned launches every word of the reused hand-off row buffer holds the sentinel
// (each consumer puts it back after a read; the I/O wave also on the columns past w).
// Debug check (ANYSEQ_CHECK_ROWS=1), run after each planned fill before the level's
// tail launch: out[0] counts non-sentinel words, out[1] the first (lowest) one's index,
// and the map kernel names its half, ring slot and column from the level's
// descriptors (out[2..5]: half, slot, column, half width; -1 when the word lies in no
// half's ring).  inject: first store a stale word past w of the first half with a ring
// (the check's own regression test), and put it back once found.
namespace anyseq {
__global__ __launch_bounds__(256) void rows_check_kernel(const uint32_t* __restrict__ rows, size_t nwords,
                                                         uint32_t sentinel, uint32_t* out) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    const size_t n4 = nwords / 4;
    const uint4* r4 = reinterpret_cast<const uint4*>(rows);
    for (size_t i = tid; i < n4; i += nth) {
        const uint4 v = r4[i];
        if (v.x != sentinel || v.y != sentinel || v.z != sentinel || v.w != sentinel) {
            const uint32_t k = v.x != sentinel ? 0 : v.y != sentinel ? 1 : v.z != sentinel ? 2 : 3;
            atomicAdd(&out[0], 1u);
            atomicMin(&out[1], (uint32_t)(4 * i + k));
        }
    }
    for (size_t i = 4 * n4 + tid; i < nwords; i += nth)
        if (rows[i] != sentinel) {
            atomicAdd(&out[0], 1u);
            atomicMin(&out[1], (uint32_t)i);
        }
}
__global__ void rows_check_map_kernel(const DPProblem* __restrict__ probs, int nprobs, int32_t* rows, uint32_t* out,
                                      int repair) {
    if (threadIdx.x != 0 || out[0] == 0) return;
    int32_t* w = rows + out[1];
    // (the check's own test: the injected word is put back, so later levels run on clean rows)
    if (repair) *w = (int32_t)0x80808080u;
    out[2] = out[3] = out[4] = 0xffffffffu;
    for (int p = 0; p < nprobs; ++p) {
        const DPProblem& P = probs[p];
        if (P.ngroups <= 1 || !P.rowbuf) continue;
        const size_t span = (size_t)P.nslots * P.wpad * 2;   // (G, F) int pairs
        if (w >= P.rowbuf && w < P.rowbuf + span) {
            const size_t off = (size_t)(w - P.rowbuf);
            out[2] = (uint32_t)p;
            out[3] = (uint32_t)(off / ((size_t)P.wpad * 2));
            out[4] = (uint32_t)((off % ((size_t)P.wpad * 2)) / 2);
            out[5] = (uint32_t)P.w;
            return;
        }
    }
}
// the first half with a hand-off ring: a stale G word at column w of its first slot
// (past the half's last column; column wpad-1 when w is a multiple of 64)
__global__ void rows_inject_kernel(const DPProblem* __restrict__ probs, int nprobs) {
    if (threadIdx.x != 0) return;
    for (int p = 0; p < nprobs; ++p) {
        const DPProblem& P = probs[p];
        if (P.ngroups <= 1 || !P.rowbuf) continue;
        P.rowbuf[2 * (size_t)min(P.w, P.wpad - 1)] = 0x12345678;
        return;
    }
}
}  // namespace anyseq

hipError_t anyseq_launch_rows_check(const void* rows, size_t nwords, uint32_t sentinel, const void* probs, int nprobs,
                                    uint32_t* out, int inject, hipStream_t st) {
    if (inject)
        hipLaunchKernelGGL(anyseq::rows_inject_kernel, dim3(1), dim3(64), 0, st, (const anyseq::DPProblem*)probs,
                           nprobs);
    const int grid = (int)std::max<size_t>(1, std::min<size_t>(2048, (nwords / 4 + 255) / 256));
    hipLaunchKernelGGL(anyseq::rows_check_kernel, dim3(grid), dim3(256), 0, st, (const uint32_t*)rows, nwords,
                       sentinel, out);
    hipLaunchKernelGGL(anyseq::rows_check_map_kernel, dim3(1), dim3(64), 0, st, (const anyseq::DPProblem*)probs,
                       nprobs, (int32_t*)rows, out, inject);
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_level_tail(const void* tail, int fill_groups, hipStream_t st) {
    const anyseq::AffLevelTail& t = *(const anyseq::AffLevelTail*)tail;
    const int grid = std::max(std::max(1, t.nslices * t.nparts), t.has_next ? fill_groups : 1);
    hipLaunchKernelGGL(anyseq::aff_level_tail_kernel, dim3(grid), dim3(anyseq::kTailThreads), 0, st, t);
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_row_to_col(const void* jobs, int njobs, int maxn, int nge, hipStream_t st) {
    if (njobs > 0)
        hipLaunchKernelGGL(anyseq::aff_row_to_col_kernel, dim3(std::max(1, std::min(64, (maxn + 255) / 256)), njobs),
                           dim3(256), 0, st, (const anyseq::RowToCol*)jobs, nge);
    return hipGetLastError();
}

hipError_t anyseq_launch_aff_predwalk(void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S, uint8_t* pred,
                                      int match, int mismatch, int go, int ge, uint8_t* alq, uint8_t* als, int lds_rows,
                                      hipStream_t st) {
    if (nblocks <= 0) return hipSuccess;
    const int bytes = anyseq::pred_lds_bytes(lds_rows);
    static int attr_set = 0;   // the kernel's dynamic-LDS limit, raised once to 160 KiB
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void*)anyseq::aff_predwalk_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 anyseq::pred_lds_bytes(anyseq::kPredLdsMaxRows));
        if (e != hipSuccess) return e;
        attr_set = 1;
    }
    hipLaunchKernelGGL(anyseq::aff_predwalk_kernel, dim3(nblocks), dim3(128), bytes, st, (anyseq::BlockInfo*)blocks,
                       nblocks, Q, S, pred, match, mismatch, go, ge, alq, als, lds_rows, nullptr, 0);
    return hipGetLastError();
}

// Device-planned final level: the block table (aff_final_blocks_kernel), the blocks of
// at most small_rows rows (one workgroup each, LDS slabs of small_rows rows), then the
// taller ones from the list (32 workgroups in turn -- tall blocks are rare, and an
// empty list costs little more than the launch -- the largest LDS slab or HBM).
hipError_t anyseq_launch_aff_final(const anyseq::AffFinalPlan* plan, const uint8_t* Q, const uint8_t* S,
                                   uint8_t* pred, int match, int mismatch, int go, int ge, uint8_t* alq, uint8_t* als,
                                   hipStream_t st) {
    const anyseq::AffFinalPlan& a = *plan;
    if (a.nb <= 0) return hipSuccess;
    static int attr_set = 0;
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void*)anyseq::aff_predwalk_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 anyseq::pred_lds_bytes(anyseq::kPredLdsMaxRows));
        if (e != hipSuccess) return e;
        attr_set = 1;
    }
    hipLaunchKernelGGL(anyseq::aff_final_blocks_kernel, dim3(1), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(anyseq::aff_predwalk_kernel, dim3(a.nb), dim3(128), anyseq::pred_lds_bytes(a.small_rows), st,
                       a.blocks, a.nb, Q, S, pred, match, mismatch, go, ge, alq, als, a.small_rows, nullptr, 1);
    hipLaunchKernelGGL(anyseq::aff_predwalk_kernel, dim3(std::min(a.nb, 32)), dim3(128),
                       anyseq::pred_lds_bytes(anyseq::kPredLdsMaxRows), st, a.blocks, a.nb, Q, S, pred, match,
                       mismatch, go, ge, alq, als, anyseq::kPredLdsMaxRows, a.tall, 0);
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

hipError_t anyseq_launch_shard_aff_combine(int kind, const void* rowT, int h1, const void* rowB, int h2, int w, int go,
                                           int ge, const int32_t* lT, const int32_t* lTf, int sT, const int32_t* lB,
                                           const int32_t* lBf, int sB, int last, const int32_t* colT,
                                           const int32_t* colB, int adj, int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(anyseq::shard_aff_combine_kernel, dim3(64), dim3(256), 0, st, kind, (const int2*)rowT, h1,
                       (const int2*)rowB, h2, w, go, ge, lT, lTf, sT, lB, lBf, sB, last, colT, colB, adj, out);
    return hipGetLastError();
}

hipError_t anyseq_launch_fulltb(const uint8_t* Q, int n, const uint8_t* S, int m, uint8_t* pred, int32_t* cols,
                                uint32_t* ticket, uint32_t* err, int match, int mismatch, int gap, uint8_t* alq,
                                uint8_t* als, hipStream_t st) {
    const int nstrips = (m + 127) / 128;
    if (n > 0 && m > 0)
        hipLaunchKernelGGL(anyseq::fulltb_strip_kernel, dim3(nstrips), dim3(64), 0, st, Q, n, S, m, pred, cols,
                           ticket, err, match, mismatch, gap);
    hipLaunchKernelGGL(anyseq::fulltb_walk_kernel, dim3(1), dim3(64), 0, st, Q, n, S, m, pred, alq, als);
    return hipGetLastError();
}

}  // extern "C"
#endif  // ANYSEQ_MICRO
