// anyseq_internal.h — shared types between the HIP kernels and the host engine.
//
// Value spaces used by the fill kernels:
//   * linear global / semiglobal run in "G-space": G[r][c] = H[r][c] - (r+c+2)*gap,
//     so the recurrence of align.impala:46-67 becomes G = max3(G_diag + w, G_left, G_up)
//     with w = sub - 2*gap (4 for a match, 1 for a mismatch under (2,-1,-1));
//   * linear local runs in "H-space": H = sat(max3(H_diag + sub - gap, H_left, H_up) + gap)
//     (align.impala:69-79, the clamp at 0 folded into one saturating subtract).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace anyseq {

enum Kind : int32_t { KIND_GLOBAL = 0, KIND_SEMIGLOBAL = 1, KIND_LOCAL = 2 };

// One rectangular DP sub-problem (a whole matrix, one Hirschberg half, ...).
// Row r of the sub-problem reads query byte q[q_off + q_step*r]; column c reads
// subject byte s[s_off + s_step*c] (q_step/s_step = +1 forward, -1 reversed:
// get_sequence_acc_half, traceback_lintime.impala:137-148).  Borders are the
// scheme's init relative to the sub-problem (scoring.impala:261-299).
struct DPProblem {
    const uint8_t* q;
    const uint8_t* s;
    int32_t q_off, q_step;
    int32_t s_off, s_step;
    int32_t h, w;
    int32_t nbands;        // ceil(h / (64*R))
    int32_t ngroups;       // ceil(nbands / NW)
    int32_t wpad;          // row-buffer pitch (multiple of 64, >= w)
    int32_t nslots;        // hand-off rows in the ring: group k writes slot k % nslots
    int32_t* out_col;      // optional: H[r][w-1] for r in [0,h)
    int32_t* out_row;      // optional: raw (kernel value space) bottom row, >= wpad ints (affine: G, F-down)
    int32_t* rowbuf;       // nslots * wpad ints: ring of group -> group hand-off rows
    uint32_t* flags;       // ngroups entries, chunk progress of each group's last band
    int32_t* best;         // optional (local): atomicMax of every cell
    int32_t* out_col_e;    // optional (affine): E[r][w-1] (H space) for r in [0,h)
    // Column-block sharding.  left_in: the left border column
    // H[r][-1] for r in [0,h), written progressively by the neighbour shard's
    // transport into a buffer pre-filled with kShardSentinel; the band polls it.
    // Values are in the sender's frame and move into this problem's frame by
    // + left_shift.  progress: bands whose out_col rows are complete, bumped in
    // band order with a system-scope release (the transport stream waits on it).
    const int32_t* left_in;
    const int32_t* left_in_e;   // affine: E[r][-1] (H space), polled like left_in
    int32_t* out_f_last;        // affine shard: F of the last row at the last column (H space)
    int32_t left_shift;
    // Chunk-ready flags of left_in / left_in_e (transported columns): the transport
    // writes flag k (0 -> 1) in stream order after chunk k's rows [k*left_chunk,
    // (k+1)*left_chunk) have landed.  A copy engine may write a chunk's bytes in any
    // order, so the data words themselves are never polled (a sentinel word can be
    // seen half overwritten).  Null: left_in is written by kernel dword stores (local
    // direct mode) and polled against kShardSentinel.
    const uint32_t* left_flag;
    int32_t left_chunk;
    // Affine fill: border mode (BM_*) and kind bits
    // (bit 0 the local clamp; bits 1-2 the best cell into *best, 1: every cell,
    // 2: the last row; H space).
    int32_t bmode;
    int32_t amode;
    uint32_t* progress;
    uint32_t* stage;       // diagnostics (ANYSEQ_SHARD_DEBUG): per-band stage reached
    // Affine fill (round 5): the problem's subject codes as the compute waves read them
    // from HBM -- column c at byte c + 64 of a padded row (code 0xFF left of column 0 and
    // from column w on), in four copies shifted by 0..3 bytes (scode_len(w) bytes each), so
    // a lane's 32 codes of a block are two dword-aligned 16-byte loads (aff_scode_kernel).
    const uint8_t* scode;
    // kProbMagic ^ (index in the launch's problem table) ^ (epoch << 12), set by
    // fill_prepare: a fill group checks it before it uses any pointer of the descriptor
    int32_t magic;
    int32_t pad_;
};
constexpr int32_t kProbMagic = 0x5eb1a700;
// bytes of one shifted copy of DPProblem::scode (columns -64 .. 32 ceil(w/32) + 95)
__host__ __device__ inline int64_t scode_len(int w) { return 32 * (int64_t)((w + 31) / 32) + 160; }

// Digest of a descriptor's words before `magic` (FNV-1a over 32-bit words).  magic =
// kProbMagic ^ index ^ (epoch << 12) ^ digest: a fill group recomputes it from the
// descriptor it read, so a descriptor that is stale or torn in ANY word (not only in
// its magic) raises ERR_BAD_DESC instead of running on its pointers.
// (round 5: four interleaved FNV-1a streams over words i = k mod 4, folded at the end --
// a quarter of the dependent multiply chain, which every group start and every planned
// half's descriptor pays)
__host__ __device__ inline uint32_t desc_digest(const uint32_t* w, int nwords) {
    uint32_t h[4] = {0x811c9dc5u, 0x811c9dc5u ^ 1u, 0x811c9dc5u ^ 2u, 0x811c9dc5u ^ 3u};
    for (int i = 0; i < nwords; ++i) h[i & 3] = (h[i & 3] ^ w[i]) * 16777619u;
    uint32_t r = 0x811c9dc5u;
    for (int k = 0; k < 4; ++k) r = (r ^ h[k]) * 16777619u;
    return r;
}
constexpr int kDescWords = (int)(offsetof(DPProblem, magic) / 4);
__host__ __device__ inline int32_t prob_magic(const DPProblem* P, int index, int epoch) {
    return (int32_t)((uint32_t)kProbMagic ^ (uint32_t)index ^ ((uint32_t)epoch << 12) ^
                     desc_digest(reinterpret_cast<const uint32_t*>(P), kDescWords));
}

// Affine border modes (H space; oracle bm_corner / bm_top / bm_left):
//   NORMAL     the scheme's global borders (corner 0, gaps paid from it);
//   EFREE      the path continues a horizontal gap (corner and left -inf, top
//              row without the open);
//   EPAID      the path starts with a horizontal gap that pays its open (corner
//              and left -inf, top row with the open);
//   FREE_LOCAL local: every border 0 (with the clamp, amode bit 0);
//   FREE_SEMI  semiglobal inside the matrix: top 0, left -inf;
//   FREE_SEMI_OPEN semiglobal at the matrix's left edge: top and left 0;
//   FFREE, FPAID, FREE_SEMI_T: EFREE, EPAID, FREE_SEMI of a TRANSPOSED problem
//              (query and subject swapped: the top and left borders trade places).
enum : int32_t {
    BM_NORMAL = 0, BM_EFREE = 1, BM_EPAID = 2, BM_FREE_LOCAL = 3, BM_FREE_SEMI = 4, BM_FREE_SEMI_OPEN = 5,
    BM_FFREE = 6, BM_FPAID = 7, BM_FREE_SEMI_T = 8
};
// amode: clamp; best of every cell / of the last row / of the last column
enum : int32_t { AM_CLAMP = 1, AM_BEST_ALL = 2, AM_BEST_LAST = 4, AM_BEST_LASTCOL = 6 };
// Split boundary types of the affine construct (oracle T_*).
enum : int32_t { T_H = 0, T_E = 1, T_BEFORE = 2, T_AFTER = 3 };

// Sentinel of a not-yet-received left-border value (memset byte 0x80): no H value
// of a supported problem reaches it.
constexpr int32_t kShardSentinel = (int32_t)0x80808080;

struct GroupRef {
    int32_t prob;
    int32_t group;
    int32_t epoch;   // FillParams::epoch of the launch that uploaded it
    int32_t check;   // group_check(prob, group, epoch): a torn entry is detected
};
__host__ __device__ inline int32_t group_check(int32_t prob, int32_t group, int32_t epoch) {
    return (int32_t)(((uint32_t)prob * 0x9e3779b1u) ^ ((uint32_t)group * 0x85ebca6bu) ^ ((uint32_t)epoch * 0xc2b2ae35u) ^
                     0x27d4eb2fu);
}

struct FillParams {
    int32_t kind;
    int32_t match, mismatch, gap;     // linear (gap < 0)
    int32_t gap_open, gap_extend;     // affine (gap_open <= 0, gap_extend < 0)
    int32_t affine;
    int32_t pad;                      // affine: bit 0 = C++ steady state only (diagnostics)
    unsigned long long* dbg;          // diagnostic build only (ANYSEQ_STAMPS): per-launch stamp sums
    int32_t epoch;                    // launch counter: descriptors carry it (stale uploads are detected)
    int32_t prio;                     // compute waves raise their issue priority (s_setprio 3) when set
    int32_t throttle;                 // s_sleep 1 units per block in a problem's band 0 (chain pace)
    // Affine fill: alpha -> number of distinct symbols of the pair when q / s
    // hold alphabet codes 0 .. n-1 (seq_code_kernel), else null; lut_ok: the diagonal weights
    // of both value spaces fit int8 (the v_perm weight table).
    const int32_t* alpha;
    int32_t lut_ok;
    int32_t slack;                    // affine: blocks a band starts behind the structural minimum (>= 0)
    int32_t io_stage;                 // affine I/O wave: subject staging mode (io_wave)
    int32_t io_skew;                  // affine I/O wave: skewed blocks per pass while a poll is out (0: 8)
    int32_t io_poll2;                 // affine I/O wave: two hand-off polls in flight
    int32_t io_fwd;                   // affine I/O wave with code rows (GS): 1 the forwarder io_forward, 0 io_wave
    int32_t arows;                    // affine: rows per lane, 1 or 2 (0 = 1); nbands counts 64 * arows rows
    // XCD-local groups (round 5): null = one global queue in group-table
    // order; else the table is partitioned by XCD (xcd_of_group), xq[x] .. xq[x+1] the
    // groups of XCD x in k-major order, dequeued by that XCD's workgroups through the
    // counter dq[kXcdCtr + x] (a workgroup whose queue is empty takes from the others)
    const uint32_t* xq;
    // affine (round 6): half chunks of extra start slack for the band fed through the
    // I/O wave (a group's first band after the HBM hand-off)
    int32_t slack_io;
};

// XCD-local group placement: the workgroups of a launch of `grid` >= 8 are dealt to the 8
// XCDs round-robin, grid / 8 each; a problem's groups go to the XCDs in runs of that many
// consecutive groups (v = the problem's first group index in problem-major order + k), so
// a hand-off between consecutive groups stays in one XCD's L2 but at run boundaries, and
// any grid-wide window of consecutive groups spreads evenly over the XCDs.
constexpr int kXcds = 8;
constexpr int kXcdCtr = 16;   // dq[16 .. 23]: the per-XCD dequeue counters (zeroed with the launch's counters)
__host__ __device__ inline int xcd_of_group(int64_t v, int run) { return (int)((v / (run > 0 ? run : 1)) % kXcds); }

// Part table entry of one Hirschberg level (traceback_lintime.impala:44-135).
struct PartInfo {
    int32_t off;          // first row of the part
    int32_t len;          // rows of the part
    int32_t rhw;          // right-half width
    int32_t split_index;  // logical index into splits set by set_split_position
    int32_t smode;        // affine construct: border mode of the left half (the part's start)
    int32_t emode;        // affine construct: border mode of the reversed right half (the part's end)
    int32_t flags;        // affine construct: bit 0 free start, bit 1 free end, bit 2 empty part
    int32_t empty_type;   // affine construct, empty part: the type its split inherits
    int32_t lhw;          // affine construct: left-half width (the parts' widths vary, aff_part_geo)
};

// Part p of a Hirschberg level of the build-defined affine construct (DESIGN.md §3.4,
// oracle aff_part): the level has P = 2^(k-1) parts; part p holds the 128-column blocks
// [floor(p nb / P), floor((p+1) nb / P)) and splits at block floor((2p+1) nb / 2P), its
// middle, so every level fills ~nm / 2^(k-1) cells for any m (nb a power of two: the
// reference construct's next_pow_2 parts).  sb / mid / eb: logical split indices of the
// part's start, split and end; lw / hw: the halves' widths (a one-block part has a zero
// one and no split).
struct AffPartGeo {
    int32_t sb, mid, eb, hoj_l, hoj_r, lw, hw;
};
__host__ __device__ inline AffPartGeo aff_part_geo(int nb, int m, int P, int p) {
    const int64_t b0 = (int64_t)p * nb / P, b1 = (int64_t)(p + 1) * nb / P, bm = (int64_t)(2 * p + 1) * nb / (2 * P);
    AffPartGeo a;
    a.sb = (int32_t)b0 - 1;
    a.eb = (int32_t)b1 - 1;
    a.mid = (int32_t)bm - 1;
    a.hoj_l = (int32_t)(b0 * 128);
    a.hoj_r = (int32_t)(bm * 128);
    a.lw = a.hoj_r - a.hoj_l;
    a.hw = (int32_t)(b1 * 128 < m ? b1 * 128 : m) - a.hoj_r;
    return a;
}

// One final-level 128-column block (iteration_*:121-173).
struct BlockInfo {
    int32_t oi, h;        // rows [oi, oi+h)
    int32_t oj, w;        // cols [oj, oj+w)
    int64_t pred_base;    // byte offset of the block's anti-diagonal-major predecessor slab
    int32_t smode;        // affine construct: start border mode (BM_*)
    int32_t e_end;        // affine construct: end at the bottom-right in H (0) or E (1), or free (2)
    int32_t flags;        // affine construct: bit 0 local (free end = any cell), bit 1 holds the last column
    int32_t xi, xj;       // affine construct, free end: the exit cell (written by aff_pred_kernel)
};

// Border mode of a free start / end (oracle free_bm): local clamps everywhere.
__host__ __device__ inline int32_t aff_free_bm(int kind, bool at_edge) {
    return kind == KIND_LOCAL ? BM_FREE_LOCAL : (at_edge ? BM_FREE_SEMI_OPEN : BM_FREE_SEMI);
}
// The same borders with query and subject swapped (a transposed half).
__host__ __device__ inline int32_t aff_transposed_bm(int bm) {
    return bm == BM_EFREE ? BM_FFREE : bm == BM_EPAID ? BM_FPAID : bm == BM_FREE_SEMI ? BM_FREE_SEMI_T : bm;
}

// Transposed Hirschberg half: its bottom row (G, F-down pairs) is the
// original's last column (H, E-right) -> H space (aff_row_to_col_kernel).
struct RowToCol {
    const void* row;
    int32_t* H;
    int32_t* E;
    int32_t n;      // columns of the transposed problem (rows of the original)
    int32_t hlast;  // last row of the transposed problem
    int32_t xs;     // the row holds X-space values (DPProblem::amode != 0)
    int32_t c0;     // G space: the row's first column in the half (a column block of a sharded level, §6.2)
};

// Inherited Hirschberg halves (anyseq_aux.hip): dst[i] = src[i] + delta, i < n.
struct I32Job {
    const int32_t* src;
    int32_t* dst;
    int32_t n;
    int32_t delta;
};

// Device-planned Hirschberg level of the affine construct (DESIGN.md §3.7,
// aff_level_plan_kernel): the level's part table, half descriptors, group table and
// row-to-column jobs are built on the device from the previous level's splits, so the
// host enqueues every level without reading anything back.  Slots are fixed by the
// level's geometry: half 2p / 2p+1 of part p (h = 0 when the part has no halves) and
// `bound` groups per half (a half spans at most `half` columns, so a transposed or
// square half has at most ceil(half / 64) bands); a group past its half's ngroups is
// skipped by the fill (DPProblem::pad_ = kPlannedDesc).
constexpr int32_t kPlannedDesc = 1;
struct AffLevelPlan {
    int32_t parts, bpp, nb, half, pw, m, n, kind;
    int32_t best_bits;     // AM_BEST_ALL (local) or AM_BEST_LAST (semiglobal / global)
    int32_t afft;          // halves taller than wide run transposed
    int32_t NW, want_slots, bound, epoch;
    const uint8_t* q;      // alphabet codes of the pair
    const uint8_t* s;
    int32_t *LH, *LE, *RH, *RE;   // the level's columns
    int32_t* pbest;               // 2 per part
    int32_t* rowpool;             // transposed halves' bottom rows
    int32_t* rowbuf;              // group -> group hand-off rows (sentinel-filled by the prep)
    uint32_t* flags;              // group flags: `bound` per half
    const int32_t* spl;           // the splits / types so far (storage index = logical + 1)
    const int32_t* typ;
    const int32_t* score;         // level-1 join value (levels >= 2; null at level 1)
    PartInfo* parts_out;
    DPProblem* probs;             // 2 * parts
    GroupRef* groups;             // 2 * parts * bound, k-major
    RowToCol* jobs;               // per half (n = 0: not transposed)
    uint32_t* hdr;                // [0] sentinel uint4s of rowbuf, [2..3] cells (u64)
    // level 1's own launch (aff_level_plan_kernel) only: words to zero first (every
    // level's header and error word), and the split table's two ends to set
    uint32_t* zero_init;
    int32_t nzero_init, init_ends;
    // (and what the level's fill prep did: the launch block's counters zeroed, the best
    // cells set to init2_value -- one launch fewer in front of level 1's fill)
    uint32_t* zero2;
    int32_t nzero2;
    int32_t* init2;
    int32_t ninit2, init2_value;
    // XCD-local groups (FillParams::xq): run > 0 -> the group table in XCD order and its
    // 9 offsets at xq (run: consecutive groups per XCD, the grid / 8)
    int32_t xrun;
    uint32_t* xq;
    uint8_t* scode;   // the level's subject-code rows (DPProblem::scode), packed by the plan
    int64_t scode_cap;   // their bytes (a plan that needs more fails the level's bound check)
    // sharded construct: world > 1 deals the level's halves
    // round-robin in part order (the host's half_owner: ordinal % world, counting only
    // parts with halves).  rank >= 0 (one rank per GPU): the other ranks' halves get no
    // groups; rank < 0 (emulated ranks): every half runs and writes the columns / best
    // cells of its owner's view (+ owner * vstride / + owner * pstride)
    int32_t world, rank;
    int64_t vstride, pstride;
    unsigned long long* stamps;   // diagnostics (ANYSEQ_TAIL_STAMPS): the plan's phases, or null
};

// The tail of a device-planned level, one launch: the join of level L
// (one workgroup per slice of kJoinSlice candidates per part; a transposed half's
// last column is read straight from its bottom row, which replaces the
// row-to-column pass), the sentinel fill of level L+1's hand-off rows (every
// workgroup, grid-stride over the host's bound), and -- in the last workgroup to
// finish -- the join's final pass (splits, types), then level L+1's counters, best
// cells and plan.
struct AffLevelTail {
    const PartInfo* parts;
    const RowToCol* jobs;
    const int32_t *LH, *LE, *RH, *RE;
    const int32_t* pbest;
    int32_t nparts, half, nslices, go, ge;
    int32_t slice_len;    // candidates per slice (nslices * slice_len > the longest possible part)
    void* partial;        // int2 per (part, slice)
    int32_t* splits;
    int32_t* types;
    int32_t* score;        // level 1: the join value
    uint32_t* done;        // zeroed before the launch
    void* sent;            // next level's hand-off rows (uint4 units)
    size_t nsent16;
    int32_t has_next;
    unsigned long long* stamps;   // diagnostics (ANYSEQ_TAIL_STAMPS): 16 s_memrealtime words, or null
    uint32_t* zero;        // next level's counters + group flags
    int32_t nzero;
    int32_t* init;         // next level's best cells
    int32_t ninit;
    AffLevelPlan next;
};

// Affine final level (aff_predwalk_kernel): blocks of at most `lds_rows` rows (the
// launch's tallest block, at most kPredLdsMaxRows) keep their predecessor bytes (plus
// a spare row for the walk's path record), query rows and the two sweeping waves'
// ring in LDS ((rows + 128) x 128 + rows + 1 KiB, <= 160 KiB); taller ones use an HBM
// slab.
constexpr int kPredLdsMaxRows = 1130;
// the device final level's first launch: LDS slabs of up to this many rows (78 KB:
// two workgroups per CU); taller blocks go to its second launch
constexpr int kPredSmallRows = 480;
// Device-planned final level (aff_final_blocks_kernel): the block table from the splits.
struct AffFinalPlan {
    const int32_t* spl;    // nb + 1 splits (rows), spl[0] = 0, spl[nb] = n
    const int32_t* typ;    // nb + 1 types (T_*)
    const int32_t* score;  // the level-1 value
    BlockInfo* blocks;     // nb entries
    int32_t* tall;         // 1 + nb: count, then the blocks taller than small_rows
    uint32_t* err;         // set to 1 on a bad split table
    int nb, n, m, kind, small_rows;
    int world, rank;       // sharded: only the blocks b with b % world == rank (world <= 1: all)
};
inline int pred_lds_bytes(int rows) { return (rows + 128) * 128 + ((rows + 15) & ~15) + 1024; }

// Device-side error codes written to the error word.
enum : uint32_t { ERR_NONE = 0, ERR_SPIN_TIMEOUT = 1, ERR_BAD_DESC = 0x100 };

}  // namespace anyseq
