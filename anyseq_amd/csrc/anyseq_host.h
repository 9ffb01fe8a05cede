// anyseq_host.h — host-side core shared by the engine (anyseq_engine.cpp) and the
// column-block sharded driver (anyseq_shard.cpp): per-device state, device
// buffers, error handling, and the asynchronous fill launch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/anyseq.h"
#include "anyseq_internal.h"

namespace anyseq {
namespace host {

constexpr int32_t SCORE_MIN_VALUE = -2147483647;  // align.impala:16
constexpr int32_t kAffNegH = -(1 << 29);          // affine "minus infinity" (the kernels' kAffNeg)

struct Failure {
    std::string msg;
};

[[noreturn]] void fail(const char* fmt, ...);

#define HIPCHECK(x)                                                                                         \
    do {                                                                                                    \
        hipError_t e_ = (x);                                                                                \
        if (e_ != hipSuccess)                                                                               \
            ::anyseq::host::fail("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

// Grow-only device buffer.  uncached: MTYPE UC (hipDeviceMallocUncached), for
// words that a running kernel polls while another kernel or engine writes them:
// per-XCD L2s are not coherent, an uncached line is never served stale.
// Growth never frees the old allocation on the spot: work queued on another stream
// (a shard's transport, a caller's stream) may still reference it.  The old block is
// retired and released by release_retired() once the device is idle.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool uncached = false;
    void* get(size_t bytes);
};

// Grow-only pinned host buffer: the source / destination of truly asynchronous copies
// (a pageable hipMemcpyAsync stages through the runtime and may block).  Callers must
// not rewrite it before the stream has passed the copy.  Allocated COHERENT
// (fine-grained, never cached in a GPU L2): kernels read the staged descriptors
// straight from it (fill_prep_kernel), and the host rewrites the same bytes for the
// next launch, so a non-coherent line cached by an earlier launch would be read
// stale.  Retired like DevBuf on growth.
struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    void* get(size_t bytes);
};

// Frees the allocations retired by DevBuf / PinBuf growth after a device-wide
// synchronisation.  Called at API entry, when no work of this library is in flight.
void release_retired();

// Debug pointer audit (ANYSEQ_CHECK_PTRS=1): every pointer a fill descriptor carries
// must lie, with its extent, inside a live library allocation or a caller buffer
// registered for the current call.  A violation fails the call before any launch.
bool check_ptrs_enabled();
void register_extern_range(const void* p, size_t bytes);   // caller buffers of this call
void register_static_range(const void* p, size_t bytes);   // allocations outside DevBuf / PinBuf
void clear_extern_ranges();
void check_range(const void* p, size_t bytes, const char* what);

int env_int(const char* name, int dflt);
// Diagnostics (ANYSEQ_FAULT_INFO): name a buffer for the GPU memory-fault report.
void register_fault_buf(const char* name, const DevBuf* b);

struct Tuning {
    int R = 1;
    int CH = 32;
    int NW = 4;
    int grid = 0;
    int fronts = 2;
    int NWa = 0;     // affine fill: compute waves per workgroup (3, 4 or 7; 0 = chosen per launch)
    int arows = 0;   // affine fill: rows per lane (1, 2, 3; 0 = chosen per launch, aff_rows_for)
    int selffwd = 1; // affine fill: throughput-bound launches with 8 compute waves, no I/O wave
    int linaff = 1;  // linear scores through the affine fill with gap open 0 (every kind; 0: fill_kernel)
    int linloop = 1; // ... with its linear asm loop (0: the affine loop with open 0)
    int iofirst = 0; // affine fill: the I/O wave on the workgroup's first hardware wave
    int forcelb = 1; // affine fill: a zero-open left border forced at column -1 (virtual prologue)
    int grida = 0;   // affine fill: persistent grid (0 = one workgroup per CU)
    int affasm = 1;  // affine fill: bit 0 asm steady state; bit 1 no asm epilogue; bits 2/3 none for best-all / other;
                     // bit 5 the round-3 band end (capturing epilogue), bit 6 its start (C++ spin) (A/B; round 5:
                     // 1 = the fused band end, every-cell bests included, and the spin-free start: configs[2] +2 %)
    int ring_slots = 0;  // hand-off rows per problem (0 = 4*grid+4; never below 2*grid+2)
    int afft = 1;        // affine construct: run Hirschberg halves taller than wide transposed
    int prio = -1;       // 1: compute waves at s_setprio 3; 2: the I/O wave at 3; 3: its hand-off step at 3;
                         // -1: per kind (affine 1, r04p A/B: +1.5-2 %; linear 0)
    int thr = 0;         // band 0 of every problem sleeps thr s_sleep-1 units per block (chain pace)
    int afflut = 1;      // affine fill: v_perm weight table when the pair has <= 8 symbols
    int slack = 0;       // affine fill: half chunks a band starts behind the structural minimum
    int slack_io = 0;    // ... the extra for the band fed through the I/O wave (HBM hop)
    int io_stage = 3;    // affine fill: the I/O wave's subject staging mode (io_wave; 0..3, r04o A/B)
    int io_skew = 0;     // affine fill: the I/O wave's skewed blocks per pass while a poll is out (0: 8)
    int io_poll2 = 0;    // affine fill: the I/O wave keeps two hand-off polls in flight
    int io_fwd = 1;      // affine fill with code rows: the I/O wave as the plain forwarder (io_forward)
    // HIP events around every fill launch (its duration for last_fill_stats); each record
    // costs a ~5 us gap in the queue before and after the launch (tools/micro/gap_micro.hip),
    // so bench.py times its steps with them off and the kernels in a separate pass
    int fill_events = 1;
    int devplan = 1;     // affine construct: Hirschberg levels planned on the device (one download)
    int devfinal = 1;    // affine construct, device-planned: the final level's blocks built on the device too
    int virtbest = 1;    // affine fill: virtual prologue for NORMAL-border best-of-every-cell problems when safe
    int plan_queues = 0; // sharded construct plan: hardware queues to plan for (0 = the process's, below)
    // affine fill: XCD-local groups on whole-chip launches (FillParams::xq).  Diagnostic
    // only, never a default: a worker takes from another XCD's queue only when its own is
    // empty, so an XCD with no resident workgroup (CUs held by another stream's kernels)
    // leaves its queue's groups undequeued and their successors spin to the timeout.
    int xcdq = 0;
    // extended API (anyseq_construct / anyseq_construct_device) with gap open 0: 0 = the
    // reference's compat construct (align.impala:292-311, per-block walk to the first
    // PRED_NONE), 1 = the true optimal alignment from the affine construct with open 0,
    // which is the linear recurrence.  The six import.h symbols
    // always keep the compat semantics.
    int ctrue = 0;
    // affine construct, host-built levels: inherited halves -- a filled
    // half of a throughput-bound level also records its child's split column, and the
    // child's half is then a lookup instead of a fill.  0 off, 1 throughput-bound levels
    // (default), 2 every level (tests).
    int inherit = 1;
    int inherit_depth = 2;   // descendant columns a split half records (1..4)
};
extern Tuning g_tuning;

// GPU_MAX_HW_QUEUES as HIP read it: snapshot once, at the first engine use (before the
// first HIP call of this library), so a later change of the variable cannot make the
// plan disagree with the real queue count.
int process_hw_queues();

// Buffers and events of one in-flight fill launch (one per concurrently running
// fill: the engine has one, each local shard of the sharded driver its own).
struct FillCtx {
    DevBuf probs;                           // launch block: counters | flags | descriptors | groups | extra
    DevBuf groups, rowbuf, flags, ctr;      // (groups, flags: unused since the launch block; ctr: result words)
    DevBuf scode;                           // affine: the problems' subject-code rows (DPProblem::scode)
    DevBuf rcheck;                          // ANYSEQ_CHECK_ROWS: the hand-off row check's result words
    bool rows_checked = false;
    bool timed = true;                      // ev0 / ev1 recorded around the launch (Tuning::fill_events)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int R = 1, NW = 4;
    unsigned long long* stamps = nullptr;   // diagnostic build only
    // the prepared launch (fill_prepare -> fill_launch)
    bool pending = false, aff = false;
    DPProblem* d_probs = nullptr;
    GroupRef* d_groups = nullptr;
    void* d_extra = nullptr;                // the caller's extra payload in the launch block (fill_prepare)
    int ngroups = 0, grid = 0;
    int64_t cells = 0;                      // DP cells of the prepared launch (sum of h*w)
    FillParams fp{};
    hipStream_t st = nullptr;
    // host sources of the launch's uploads: hipMemcpyAsync may read pageable host
    // memory after it returns, so they live as long as the context, not the call
    std::vector<DPProblem> h_probs;
    std::vector<GroupRef> h_groups;
    PinBuf pin;                  // staged descriptors + group table of the launch, and the error word
    hipEvent_t ev2 = nullptr;    // after the error word's copy to `pin`
    uint32_t* err_host = nullptr;
    void init();
};

struct Engine {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev_order = nullptr;   // orders a caller's stream behind the engine's stream
    std::mutex mu;
    FillCtx fc;
    DevBuf q, s, outcol, outrow, L, R, spl, parts, bmax, bind, blocks, pred, alq, als;
    DevBuf LE, RE, typ, pos;   // affine construct
    DevBuf status;             // affine construct: splits | types | score of a level (one download)
    DevBuf tall;               // affine construct, device final level: the tall blocks' list
    DevBuf joinbuf;            // affine construct: per-slice partial maxima of the level's joins
    PinBuf pin_up, pin_down;   // construct: staged uploads / downloads of a level
    PinBuf pin_blocks;         // construct: the final level's block table
    std::vector<int32_t> host_i32;
    std::vector<BlockInfo> host_blocks;
    std::vector<PartInfo> host_parts;
    std::vector<uint8_t> host_jobs;
    DevBuf jobs;
    DevBuf codes, codemeta;    // alphabet codes of the current pair (prepare_codes)
    DevBuf vstr;               // sharded construct, emulated ranks: their ' '-filled strings
    // affine construct, device-planned levels: launch block, hand-off rows, part table,
    // row-to-column jobs (their per-level header and error words sit in `status`)
    DevBuf pl_meta, pl_rowbuf, pl_parts, pl_jobs;
    DevBuf pl_scode;           // the planned levels' subject-code rows (DPProblem::scode)
    DevBuf tst;                // diagnostics: tail-launch stamps (ANYSEQ_TAIL_STAMPS)
    // host-built levels, inherited halves: the recorded child columns
    // (H, E by query row, left and right halves) and the level's copy / frame jobs
    DevBuf capL, capR, auxjobs;
    PinBuf pin_aux;
    std::vector<hipEvent_t> pl_ev;
    bool pl_dirty = true;      // pl_rowbuf may hold non-sentinel words (fresh, or a failed call)
    explicit Engine(int dev);
};

// A pair recoded to alphabet codes.
struct SeqCodes {
    const uint8_t* q;
    const uint8_t* s;
    const int32_t* alpha;   // device: number of distinct symbols
};
// (fill0 / fill1: optionally fill_len bytes of ' ' each, in the same launches)
SeqCodes prepare_codes(Engine& E, const uint8_t* dq, int n, const uint8_t* ds, int m, hipStream_t st,
                       uint8_t* fill0 = nullptr, uint8_t* fill1 = nullptr, size_t fill_len = 0);

Engine& engine();
int rows_per_lane();
int waves_per_group();
int aff_waves_per_group();
// the issue-priority mode of a fill launch (g_tuning.prio, per kind when -1)
inline int fill_prio(bool affine) { return g_tuning.prio >= 0 ? g_tuning.prio : (affine ? 1 : 0); }
int aff_waves_for(int64_t chain_steps, int64_t wave_steps, int grid);
// Column-block pipelines (round 5): stages ahead of the last one for the fills prepared
// while it is set (a rank starts one band sweep of its block after its left neighbour;
// aff_rows_for weighs that start against the throughput of more rows per lane)
extern thread_local int g_fill_stages;
struct FillStages {
    explicit FillStages(int s) { g_fill_stages = s > 0 ? s : 0; }
    ~FillStages() { g_fill_stages = 0; }
};

FillParams make_params(int kind, const anyseq_scoring& sc);
// An affine problem of kind `kind` over the whole matrix (or a shard of it): its
// border mode and clamp / best bits (DPProblem::bmode / amode).
void set_aff_kind(DPProblem& P, int kind);
void check_scoring(int kind, const anyseq_scoring& sc);
void check_value_range(const anyseq_scoring& sc, int64_t n, int64_t m);

// Enqueues one batched fill over `probs` on `st` (the problems' nbands/ngroups/
// wpad/rowbuf/flags are filled in here).  grid <= 0: the tuning's grid.
// fill_prepare does every allocation and upload (allocation and hipFree can
// synchronise the device, which must not happen while another shard's persistent
// fill waits for this one) and fill_launch only enqueues the kernel.
void fill_prepare(Engine& E, FillCtx& C, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st,
                  int grid_req = 0, const void* extra = nullptr, size_t extra_bytes = 0, int32_t* init = nullptr,
                  int init_words = 0, int32_t init_value = 0);
void fill_launch(FillCtx& C);
void fill_async(Engine& E, FillCtx& C, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st,
                int grid_req = 0, const void* extra = nullptr, size_t extra_bytes = 0, int32_t* init = nullptr,
                int init_words = 0, int32_t init_value = 0);
// Waits for the launch of fill_async, accounts its time, checks the error word.
void fill_finish(FillCtx& C);
// The same without waiting: for a caller that has already synchronised the stream
// past the launch (one synchronisation per Hirschberg level).
void fill_collect(FillCtx& C);
// fill_async + fill_finish on the engine's context.
void run_fill(Engine& E, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st);

void set_last_error(const std::string& m);

// Sharded affine construct: the half fills of every Hirschberg level
// and the final blocks are dealt round-robin to `world` ranks; after each level's fills
// the ranks' columns are summed (rows a rank did not fill are zero) and the free-end
// best cells max-reduced, so every rank joins every part and holds the same splits;
// the ranks' output strings merge by a byte-wise max.  local: `world` virtual ranks in
// this process, one fill launch each, sharing the buffers (no reduction needed).
//
// Column-blocked levels: a part's two halves, both transposed
// (subject columns as rows, query rows as columns), are the two fronts of ONE problem
// split at row `half` (the left half's width) -- so a part runs on a subgroup of ranks
// with the score sharding's boundary-column transport (anyseq_shard.cpp): rank g of
// the subgroup fills the part's query rows [off + g*len/G, off + (g+1)*len/G) of both
// halves and writes its segment of the level's columns (the halves' bottom rows).
// Level k with P parts is column-blocked when world >= 2P (P = 1: level 1 over all
// ranks; P = 2: each part over half of them; ...); part p takes ranks
// [p*world/P, (p+1)*world/P).
struct ShardPart {
    const uint8_t* cq = nullptr;   // query codes: the transposed halves' columns start at cq + off
    const uint8_t* cs = nullptr;   // subject codes: their rows start at cs + soff
    int off = 0, len = 0;          // the part's query rows
    int soff = 0, mw = 0, half = 0;   // its subject columns; forward half rows [0, half), reversed [half, mw)
    int bm_l = 0, am_l = 0;        // border mode / kind bits of the transposed forward half
    int bm_r = 0, am_r = 0;        // ... of the transposed reversed half
    int32_t* pbest = nullptr;      // view 0's two best cells of the part; view v at + v * pstride
    int r0 = 0, G = 1;             // its rank subgroup
};
struct ShardLevel {
    int kind = 0;
    anyseq_scoring sc{};
    FillParams fp{};
    std::vector<ShardPart> parts;
    int32_t *LH = nullptr, *LE = nullptr, *RH = nullptr, *RE = nullptr;   // view 0; view v at + v * nn
    size_t nn = 0;
    size_t pstride = 0;
    hipStream_t st = nullptr;      // the construct's stream (the level is ordered on it)
    Engine* E = nullptr;           // the construct's engine (held under E->mu by the caller)
};

struct ConstructShards {
    int rank = 0, world = 1;
    bool local = false;
    std::function<void(int32_t*, size_t, hipStream_t)> sum_i32, max_i32;
    std::function<void(uint8_t*, size_t, hipStream_t)> max_u8;
    std::function<void(const ShardLevel&)> blocked;   // column-blocked levels (null: round-robin)
};
int64_t construct_affine_dev(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n,
                             const uint8_t* ds, int m, uint8_t* d_alq, uint8_t* d_als, hipStream_t st,
                             const ConstructShards* shards = nullptr);

}  // namespace host
}  // namespace anyseq
