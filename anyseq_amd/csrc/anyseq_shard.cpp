// anyseq_shard.cpp — column-block sharded score fill.
//
// The matrix is split into contiguous subject column blocks, one per shard:
// shard g owns columns [c0_g, c0_g + w_g), query replicated.  Each shard runs the
// two-front fill of score_dev on its block:
//   * the top front (rows [0, h1), forward) needs H[r][c0_g - 1] from shard g-1
//     and sends its own last column to shard g+1;
//   * the bottom front (rows [h1, n), query and subject reversed) flows the other
//     way: it needs the column c0_g + w_g from shard g+1 and sends its first
//     column to shard g-1.
// A front's band publishes its last-column rows (out_col) and then bumps a
// progress counter in signal memory in band order (publish_progress); the
// transport stream of that front waits on the counter (hipStreamWaitValue32) and
// ships each chunk of rows to the neighbour, whose band polls the sentinel-filled
// left_in buffer (poll_left).  No host thread sits in the loop.
//
// Two transports:
//   * RCCL (one process per GPU, anyseq_shard_init): ncclSend / ncclRecv over
//     xGMI, four communicators so that every communicator is used by exactly one
//     stream of a rank (top/bottom direction x link parity);
//   * local (anyseq_shard_score_local): several shards in one process on one
//     device, hipMemcpyAsync between them -- the same kernels, counters and
//     chunk protocol, runnable on a single GPU (parity tests).
// The per-shard combine (shard_combine_kernel) gives every shard's best split
// candidate in true-score units; RCCL reduces them with a MAX all-reduce.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "anyseq_host.h"

extern "C" hipError_t anyseq_launch_shard_chunk_copy(int32_t* dst, const int32_t* src, int n, int32_t* dst_e,
                                                     const int32_t* src_e, int ne, uint32_t* flag, hipStream_t st);
extern "C" hipError_t anyseq_launch_shard_aff_combine(int kind, const void* rowT, int h1, const void* rowB, int h2,
                                                      int w, int go, int ge, const int32_t* lT, const int32_t* lTf,
                                                      int sT, const int32_t* lB, const int32_t* lBf, int sB, int last,
                                                      const int32_t* colT, const int32_t* colB, int adj, int32_t* out,
                                                      hipStream_t st);
extern "C" hipError_t anyseq_launch_aff_row_to_col(const void* jobs, int njobs, int maxn, int nge, hipStream_t st);
extern "C" hipError_t anyseq_launch_shard_combine(int kind, const int32_t* rowT, int h1, const int32_t* rowB, int h2,
                                                  int w, int gap, const int32_t* lT, int sT, const int32_t* lB,
                                                  int sB, int last, const int32_t* colT, const int32_t* colB, int adj,
                                                  int32_t* out, hipStream_t st);

namespace anyseq {
namespace host {
namespace {

#define NCCLCHECK(x)                                                                                   \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) fail("%s failed: %s (%s:%d)", #x, ncclGetErrorString(r_), __FILE__, __LINE__); \
    } while (0)

constexpr int kComms = 4;   // top even/odd links, bottom even/odd links

// Transport trigger: a host thread per direction polls the sender's progress
// counter in pinned host memory and issues each chunk's transfer.  With
// ANYSEQ_SHARD_WAITVALUE=1 every chunk transfer is instead enqueued up front on the
// direction's transport stream behind hipStreamWaitValue32 on the counter (signal
// memory).  ANYSEQ_SHARD_DIRECT=1 (local shards only): the receiver polls the
// sender's out_col itself.  Host-polled transport is the default (round 2, measured on MI355X with 2 and 4
// in-process shards at 16384^2 semiglobal affine: host polling 0 failures in 80
// runs at ~4 ms each; hipStreamWaitValue32 1 spin timeout in 80 runs and ~100 ms
// each).  ANYSEQ_SHARD_WAITVALUE=1 selects the stream-wait transport.
bool use_wait_value() { return env_int("ANYSEQ_SHARD_WAITVALUE", 0) != 0; }
bool use_direct() { return env_int("ANYSEQ_SHARD_DIRECT", 0) != 0; }


struct Front {
    // affine: out_col_e / left_in_e hold E of the last column, h rows, plus [h] = F of
    // the last row at the last column (the combine's vertical-gap join)
    DevBuf out_col, left_in, out_row, out_col_e, left_in_e;
    DevBuf left_flag;   // chunk-ready flags of left_in / left_in_e (DPProblem::left_flag)
    bool aff = false;
    uint32_t* progress = nullptr;     // device view of the counter (what the kernel bumps)
    uint32_t* progress_h = nullptr;   // host view (pinned, coherent) -- host-poll transport
    uint32_t* progress_sig = nullptr; // signal memory -- hipStreamWaitValue32 transport
    hipStream_t s_send = nullptr, s_recv = nullptr;
    int h = 0;
};

struct Shard {
    int g = 0, c0 = 0, w = 0;
    hipStream_t st = nullptr;
    hipEvent_t ready = nullptr;
    FillCtx fc;
    Front top, bot;
    DevBuf res;
    const int32_t* lT = nullptr;   // where the fronts read their received columns (combine reads them too)
    const int32_t* lB = nullptr;
    const int32_t* lTe = nullptr;  // affine: received E columns (+ [h] = F of the last row)
    const int32_t* lBe = nullptr;
    // column-blocked construct level: the two bottom rows -> the level's column segments
    DevBuf jobs;
    RowToCol h_jobs[2] = {};
    void init() {
        if (st) return;
        for (Front* f : {&top, &bot})
            for (DevBuf* b : {&f->out_col, &f->left_in, &f->out_row, &f->out_col_e, &f->left_in_e, &f->left_flag})
                register_fault_buf(f == &top ? "shard.top" : "shard.bot", b);
        for (DevBuf* b : {&fc.probs, &fc.groups, &fc.rowbuf, &fc.flags, &fc.ctr, &res}) register_fault_buf("shard.fc", b);
        // polled across kernels / XCDs: never L2-cached (see DevBuf::uncached)
        for (Front* f : {&top, &bot})
            f->out_col.uncached = f->left_in.uncached = f->out_col_e.uncached = f->left_in_e.uncached =
                f->left_flag.uncached = true;
        HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHECK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        for (Front* f : {&top, &bot}) {
            void* p = nullptr;
            HIPCHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
            f->progress_h = (uint32_t*)p;
            void* d = nullptr;
            HIPCHECK(hipHostGetDevicePointer(&d, p, 0));
            register_static_range(d, 64);
            HIPCHECK(hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory));
            f->progress_sig = (uint32_t*)p;
            register_static_range(p, 8);
            f->progress = use_wait_value() ? f->progress_sig : (uint32_t*)d;
        }
        fc.init();
    }
};

// Transport streams are created on first use: every stream of the process needs a
// hardware queue of its own.  HIP multiplexes streams over GPU_MAX_HW_QUEUES
// queues (default 4), and a queue is in-order: a transfer queued behind the
// persistent fill kernel (or behind another direction's stream wait) would never
// run while the fill waits for it.
hipStream_t lazy_stream(hipStream_t& s) {
    if (!s) HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

void check_hw_queues(int streams) {
    // this process's streams: the engine's, torch's null stream, the shards' fill and transport streams
    const int need = streams + 2;
    const int have = process_hw_queues();
    if (have < need)
        fail("the sharded fill runs %d concurrent streams: set GPU_MAX_HW_QUEUES >= %d (<= 32) in the environment "
             "before the first HIP call (it is %d); streams sharing a hardware queue would deadlock behind the "
             "persistent fill kernel", streams, need, have);
}

// Column block of shard g of N over m columns (balanced, contiguous).
inline int block_c0(int g, int N, int m) { return (int)((int64_t)g * m / N); }

struct RcclState {
    int rank = -1, world = 0;
    ncclComm_t comm[kComms] = {};
    Shard shard;
    // resident inputs of this rank (anyseq_shard_load)
    DevBuf q, s;
    int n = 0, m = 0, c0 = 0, w = 0;
};
std::unique_ptr<RcclState> g_rccl;

// Rows per transported chunk of a front of h rows: 1024 up to 256K rows, then h/256
// (a power of two, at most 16384), so a genome-length front (4.64M rows) ships ~280
// chunks per direction instead of ~4500 host-thread send calls, for a start lag of one
// chunk per rank (16384 rows ~ 0.6 ms of a ~1 s rank fill).  Both sides of a link
// derive it from the same front height.  ANYSEQ_SHARD_CHUNK forces it.
int chunk_rows(int h) {
    const int forced = env_int("ANYSEQ_SHARD_CHUNK", 0);
    if (forced > 0) return std::max(64, forced / 64 * 64);
    int c = 1024;
    while (c < 16384 && (int64_t)c * 256 < (int64_t)h) c *= 2;
    return c;
}

// Host-side wait with a deadline: a lost message must not hang the caller.
void wait_stream(hipStream_t s, double seconds, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) fail("%s: %s", what, hipGetErrorString(e));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds)
            fail("%s: timed out after %.0f s", what, seconds);
        std::this_thread::yield();
    }
}

// Per-step setup of one shard: problems, sentinel buffers, counters.
// h1_req >= 0: the top front's rows (a construct level splits at `half`, not n/2).
void setup_shard(Shard& S, int N, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n, const uint8_t* ds_block,
                 int m, std::vector<DPProblem>& probs, int& h1, int& h2, bool direct = false, int h1_req = -1) {
    h1 = h1_req >= 0 ? h1_req : n / 2;
    h2 = n - h1;
    const int g = S.g, w = S.w;
    const int wpad = (w + 63) & ~63;
    const bool has_left = g > 0, has_right = g < N - 1;
    const int ng = -sc.gap_extend;
    const bool aff = sc.gap_open != 0;
    S.top.h = h1;
    S.bot.h = h2;
    S.top.aff = S.bot.aff = aff;
    // rows: (G, F) pairs for affine
    int32_t* rowT = (int32_t*)S.top.out_row.get((size_t)wpad * (aff ? 8 : 4));
    int32_t* rowB = (int32_t*)S.bot.out_row.get((size_t)wpad * (aff ? 8 : 4));
    int32_t* colTe = aff ? (int32_t*)S.top.out_col_e.get((size_t)(h1 + 1) * 4) : nullptr;
    int32_t* colBe = aff ? (int32_t*)S.bot.out_col_e.get((size_t)(h2 + 1) * 4) : nullptr;
    int32_t* inTe = aff && has_left ? (int32_t*)S.top.left_in_e.get((size_t)(h1 + 1) * 4) : nullptr;
    int32_t* inBe = aff && has_right ? (int32_t*)S.bot.left_in_e.get((size_t)(h2 + 1) * 4) : nullptr;
    if (inTe) HIPCHECK(hipMemsetAsync(inTe, 0x80, (size_t)(h1 + 1) * 4, S.st));
    if (inBe) HIPCHECK(hipMemsetAsync(inBe, 0x80, (size_t)(h2 + 1) * 4, S.st));
    if (direct && aff) {
        HIPCHECK(hipMemsetAsync(colTe, 0x80, (size_t)(h1 + 1) * 4, S.st));
        HIPCHECK(hipMemsetAsync(colBe, 0x80, (size_t)(h2 + 1) * 4, S.st));
    }
    S.lTe = inTe;
    S.lBe = inBe;
    // out_col: sent downstream; also the semiglobal end column on the edge shards
    int32_t* colT = (int32_t*)S.top.out_col.get((size_t)h1 * 4);
    int32_t* colB = (int32_t*)S.bot.out_col.get((size_t)h2 * 4);
    int32_t* inT = has_left ? (int32_t*)S.top.left_in.get((size_t)h1 * 4) : nullptr;
    int32_t* inB = has_right ? (int32_t*)S.bot.left_in.get((size_t)h2 * 4) : nullptr;
    if (inT) HIPCHECK(hipMemsetAsync(inT, 0x80, (size_t)h1 * 4, S.st));
    if (inB) HIPCHECK(hipMemsetAsync(inB, 0x80, (size_t)h2 * 4, S.st));
    // chunk-ready flags of the received columns (the transport sets flag k after chunk k)
    const int CRT = chunk_rows(h1), CRB = chunk_rows(h2);
    uint32_t* flT = nullptr;
    uint32_t* flB = nullptr;
    if (inT && !direct) {
        flT = (uint32_t*)S.top.left_flag.get((size_t)((h1 + CRT - 1) / CRT) * 4);
        HIPCHECK(hipMemsetAsync(flT, 0, (size_t)((h1 + CRT - 1) / CRT) * 4, S.st));
    }
    if (inB && !direct) {
        flB = (uint32_t*)S.bot.left_flag.get((size_t)((h2 + CRB - 1) / CRB) * 4);
        HIPCHECK(hipMemsetAsync(flB, 0, (size_t)((h2 + CRB - 1) / CRB) * 4, S.st));
    }
    if (direct) {   // local direct mode: the neighbours poll these columns themselves
        HIPCHECK(hipMemsetAsync(colT, 0x80, (size_t)h1 * 4, S.st));
        HIPCHECK(hipMemsetAsync(colB, 0x80, (size_t)h2 * 4, S.st));
    }
    for (Front* f : {&S.top, &S.bot}) {
        if (use_wait_value()) HIPCHECK(hipMemsetAsync(f->progress, 0, 4, S.st));
        else __atomic_store_n(f->progress_h, 0u, __ATOMIC_RELEASE);   // before the launch below
    }
    HIPCHECK(hipEventRecord(S.ready, S.st));
    for (Front* f : {&S.top, &S.bot}) {
        if (f->s_send) HIPCHECK(hipStreamWaitEvent(f->s_send, S.ready, 0));
        if (f->s_recv) HIPCHECK(hipStreamWaitEvent(f->s_recv, S.ready, 0));
    }
    // frames: a shard's top border is the scheme's, so global values are shifted by
    // the shard's column offset; a received column moves by the sender's width
    const int shT = (kind == KIND_GLOBAL && has_left) ? block_c0(g, N, m) - block_c0(g - 1, N, m) : 0;
    const int shB = (kind == KIND_GLOBAL && has_right) ? block_c0(g + 2, N, m) - block_c0(g + 1, N, m) : 0;
    DPProblem P;
    memset(&P, 0, sizeof P);
    P.q = dq;
    P.s = ds_block;
    P.q_step = 1;
    P.s_step = 1;
    P.w = w;
    if (aff) set_aff_kind(P, kind);
    P.h = h1;
    P.out_row = rowT;
    P.out_col = colT;
    P.left_in = inT;
    P.left_in_e = inTe;
    P.left_flag = flT;
    P.left_chunk = CRT;
    P.out_col_e = colTe;
    P.out_f_last = colTe ? colTe + h1 : nullptr;
    S.lT = inT;
    S.lB = inB;
    P.left_shift = shT * ng;
    P.progress = S.top.progress;
    probs.push_back(P);
    P.q_off = n - 1;
    P.q_step = -1;
    P.s_off = w - 1;
    P.s_step = -1;
    P.h = h2;
    P.out_row = rowB;
    P.out_col = colB;
    P.left_in = inB;
    P.left_in_e = inBe;
    P.left_flag = flB;
    P.left_chunk = CRB;
    P.out_col_e = colBe;
    P.out_f_last = colBe ? colBe + h2 : nullptr;
    P.left_shift = shB * ng;
    P.progress = S.bot.progress;
    probs.push_back(P);
}

// Bands of rows [0, r1) of a front: chunk k of rows is shipped once they are done.
inline uint32_t bands_for_rows(int r1) { return (uint32_t)((r1 + 63) / 64); }

// One direction of one front: wait for the sender's progress, ship each chunk.
// Runs on its own host thread (hipStreamWaitValue32 may block the calling
// thread on some runtimes; a thread per direction never orders one direction's
// wait before another direction's enqueue).
struct Xfer {
    int device = 0;
    Front* src = nullptr;
    int32_t* dst = nullptr;         // local transport: the neighbour's left_in
    int32_t* dst_e = nullptr;       // affine: the neighbour's left_in_e (RCCL: receive E into it)
    uint32_t* flag = nullptr;       // the receiver's chunk-ready flags (set after each chunk's data)
    ncclComm_t comm = nullptr;      // RCCL transport
    int peer = -1;
    bool recv = false;              // RCCL: receive into dst instead of sending
    int h = 0;
    std::string error;
};

void run_xfer(Xfer* x) {
    try {
        HIPCHECK(hipSetDevice(x->device));
        const int CR = chunk_rows(x->h);
        for (int r0 = 0; r0 < x->h; r0 += CR) {
            const int r1 = std::min(x->h, r0 + CR);
            // affine: E rows follow the H rows; the last chunk's E carries one more
            // element, [h] = F of the last row at the last column
            const size_t ne = (size_t)(r1 - r0) + (r1 == x->h ? 1 : 0);
            if (x->recv) {
                NCCLCHECK(ncclRecv(x->dst + r0, (size_t)(r1 - r0), ncclInt32, x->peer, x->comm, x->src->s_recv));
                if (x->src->aff)
                    NCCLCHECK(ncclRecv(x->dst_e + r0, ne, ncclInt32, x->peer, x->comm, x->src->s_recv));
                // in stream order after the chunk's data: the only word the fill polls
                HIPCHECK(hipMemsetD32Async(x->flag + r0 / CR, 1u, 1, x->src->s_recv));
                continue;
            }
            const uint32_t need = bands_for_rows(r1);
            if (use_wait_value()) {
                HIPCHECK(hipStreamWaitValue32(x->src->s_send, x->src->progress, need, hipStreamWaitValueGte,
                                              0xffffffffu));
            } else {
                const auto t0 = std::chrono::steady_clock::now();
                while (__atomic_load_n(x->src->progress_h, __ATOMIC_ACQUIRE) < need) {
                    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 120.0)
                        fail("shard transport: no progress from the fill (chunk rows %d..%d)", r0, r1);
                    std::this_thread::yield();
                }
            }
            const int32_t* src = (const int32_t*)x->src->out_col.p + r0;
            const int32_t* src_e = x->src->aff ? (const int32_t*)x->src->out_col_e.p + r0 : nullptr;
            if (x->comm) {
                NCCLCHECK(ncclSend(src, (size_t)(r1 - r0), ncclInt32, x->peer, x->comm, x->src->s_send));
                if (src_e) NCCLCHECK(ncclSend(src_e, ne, ncclInt32, x->peer, x->comm, x->src->s_send));
            } else {
                HIPCHECK(anyseq_launch_shard_chunk_copy(x->dst + r0, src, r1 - r0, src_e ? x->dst_e + r0 : nullptr,
                                                        src_e, (int)ne, x->flag + r0 / CR, x->src->s_send));
            }
        }
    } catch (const Failure& f) {
        x->error = f.msg;
    }
}

// Starts every transfer on its own thread; returns the threads to join.
std::vector<std::thread> start_xfers(std::vector<Xfer>& xs) {
    std::vector<std::thread> th;
    for (Xfer& x : xs) th.emplace_back(run_xfer, &x);
    return th;
}

// After the fills ended: a failed fill never reaches its progress targets, so
// release every counter (waiting transfers then drain), join, report.
void finish_xfers(std::vector<std::thread>& th, std::vector<Xfer>& xs, std::vector<Shard*> shards, bool fill_ok) {
    if (!fill_ok)
        for (Shard* S : shards)
            for (Front* f : {&S->top, &S->bot}) {
                const uint32_t big = 0x7fffffffu;
                if (use_wait_value()) (void)hipMemcpy(f->progress, &big, 4, hipMemcpyHostToDevice);
                else __atomic_store_n(f->progress_h, big, __ATOMIC_RELEASE);
            }
    for (auto& t : th) t.join();
    for (auto& x : xs)
        if (!x.error.empty()) fail("shard transport: %s", x.error.c_str());
}

std::vector<Xfer> local_xfers(std::vector<Shard>& shards, int N, int device) {
    std::vector<Xfer> xs;
    for (int g = 0; g < N; ++g) {
        Shard& S = shards[g];
        if (g + 1 < N) {   // top: g -> g+1
            Xfer x;
            x.device = device;
            x.src = &S.top;
            x.dst = (int32_t*)shards[g + 1].top.left_in.p;
            x.dst_e = (int32_t*)shards[g + 1].top.left_in_e.p;
            x.flag = (uint32_t*)shards[g + 1].top.left_flag.p;
            x.h = S.top.h;
            xs.push_back(x);
        }
        if (g > 0) {       // bottom: g -> g-1
            Xfer x;
            x.device = device;
            x.src = &S.bot;
            x.dst = (int32_t*)shards[g - 1].bot.left_in.p;
            x.dst_e = (int32_t*)shards[g - 1].bot.left_in_e.p;
            x.flag = (uint32_t*)shards[g - 1].bot.left_flag.p;
            x.h = S.bot.h;
            xs.push_back(x);
        }
    }
    return xs;
}

std::vector<Xfer> rccl_xfers(RcclState& R, int device) {
    Shard& S = R.shard;
    const int g = R.rank, N = R.world;
    std::vector<Xfer> xs;
    // link a joins ranks a and a+1: top data a -> a+1 on comm[a % 2], bottom data
    // a+1 -> a on comm[2 + a % 2]; every communicator is used by one stream per rank
    auto add = [&](Front* f, bool recv, int peer, ncclComm_t c) {
        Xfer x;
        x.device = device;
        x.src = f;
        x.recv = recv;
        x.peer = peer;
        x.comm = c;
        x.dst = recv ? (int32_t*)f->left_in.p : nullptr;
        x.dst_e = recv ? (int32_t*)f->left_in_e.p : nullptr;
        x.flag = recv ? (uint32_t*)f->left_flag.p : nullptr;
        x.h = f->h;
        xs.push_back(x);
    };
    if (g > 0) {
        add(&S.top, true, g - 1, R.comm[(g - 1) % 2]);
        add(&S.bot, false, g - 1, R.comm[2 + (g - 1) % 2]);
    }
    if (g < N - 1) {
        add(&S.top, false, g + 1, R.comm[g % 2]);
        add(&S.bot, true, g + 1, R.comm[2 + g % 2]);
    }
    return xs;
}

// Combine of one shard into *res (true-score units).
void enqueue_combine(Shard& S, int N, int kind, const anyseq_scoring& sc, int m, int h1, int h2, int32_t* res) {
    const int g = S.g, w = S.w;
    const int gap = sc.gap_extend;
    const int shT = (kind == KIND_GLOBAL && g > 0) ? (block_c0(g, N, m) - block_c0(g - 1, N, m)) * -gap : 0;
    const int shB = (kind == KIND_GLOBAL && g < N - 1) ? (block_c0(g + 2, N, m) - block_c0(g + 1, N, m)) * -gap : 0;
    // top frame: H_true = H + c0 gap; bottom frame (reversed): H_true = H + (m - c0 - w) gap
    const int adj = kind == KIND_GLOBAL ? (m - w) * gap : 0;
    const int32_t* colT = (kind == KIND_SEMIGLOBAL && g == N - 1) ? (const int32_t*)S.top.out_col.p : nullptr;
    const int32_t* colB = (kind == KIND_SEMIGLOBAL && g == 0) ? (const int32_t*)S.bot.out_col.p : nullptr;
    if (sc.gap_open != 0) {
        HIPCHECK(anyseq_launch_shard_aff_combine(kind, S.top.out_row.p, h1, S.bot.out_row.p, h2, w, sc.gap_open, gap,
                                                 S.lT, S.lTe ? S.lTe + h1 : nullptr, shT, S.lB,
                                                 S.lBe ? S.lBe + h2 : nullptr, shB, g == N - 1 ? 1 : 0, colT, colB, adj,
                                                 res, S.st));
        return;
    }
    HIPCHECK(anyseq_launch_shard_combine(kind, (const int32_t*)S.top.out_row.p, h1, (const int32_t*)S.bot.out_row.p,
                                         h2, w, gap, S.lT, shT, S.lB, shB,
                                         g == N - 1 ? 1 : 0, colT, colB, adj, res, S.st));
}

// Diagnostics (ANYSEQ_SHARD_DUMP=<path>): every combine input of the last local
// sharded call, plus each shard's combine alone, written as text.
void dump_arr(FILE* f, const char* name, const void* d, size_t n) {
    std::vector<int32_t> h(n);
    if (d && n) (void)hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    fprintf(f, "%s:", name);
    if (!d) fprintf(f, " null");
    for (size_t i = 0; d && i < n; ++i) fprintf(f, " %d", h[i]);
    fprintf(f, "\n");
}

void dump_shards(const char* path, std::vector<Shard>& shards, int N, int kind, const anyseq_scoring& sc, int m, int h1,
                 int h2, int32_t v) {
    FILE* f = fopen(path, "w");
    if (!f) return;
    const bool aff = sc.gap_open != 0;
    fprintf(f, "kind %d N %d m %d h1 %d h2 %d result %d\n", kind, N, m, h1, h2, v);
    static DevBuf one;
    int32_t* r1 = (int32_t*)one.get(64);
    for (int g = 0; g < N; ++g) {
        Shard& S = shards[g];
        fprintf(f, "shard %d c0 %d w %d\n", g, S.c0, S.w);
        dump_arr(f, "rowT", S.top.out_row.p, (size_t)S.w * (aff ? 2 : 1));
        dump_arr(f, "rowB", S.bot.out_row.p, (size_t)S.w * (aff ? 2 : 1));
        dump_arr(f, "colT", S.top.out_col.p, (size_t)h1);
        dump_arr(f, "colB", S.bot.out_col.p, (size_t)h2);
        if (aff) dump_arr(f, "colTe", S.top.out_col_e.p, (size_t)h1 + 1);
        if (aff) dump_arr(f, "colBe", S.bot.out_col_e.p, (size_t)h2 + 1);
        dump_arr(f, "lT", S.lT, (size_t)h1);
        dump_arr(f, "lB", S.lB, (size_t)h2);
        if (aff) dump_arr(f, "lTe", S.lTe, (size_t)h1 + 1);
        if (aff) dump_arr(f, "lBe", S.lBe, (size_t)h2 + 1);
        HIPCHECK(hipMemset(r1, kind == KIND_LOCAL ? 0 : 0x80, 4));
        HIPCHECK(hipDeviceSynchronize());
        enqueue_combine(S, N, kind, sc, m, h1, h2, r1);
        HIPCHECK(hipStreamSynchronize(S.st));
        dump_arr(f, "combine", r1, 1);
    }
    fclose(f);
}

void check_shard_shape(int kind, const anyseq_scoring& sc, int n, int m, int N) {
    check_scoring(kind, sc);
    check_value_range(sc, n, m);
    if (N < 1) fail("sharded fill: need at least one shard");
    if (n < 2) fail("sharded fill: need at least 2 query rows (two fronts), got %d", n);
    if (m < N) fail("sharded fill: %d columns cannot be split over %d shards", m, N);
    if (g_tuning.R != 1) fail("sharded fill: rows_per_lane must be 1");
}

int grid_per_shard(const Engine& E, int nshards) {
    // One shard per GPU (the RCCL path): leave CUs for the transport (RCCL kernels)
    // next to the persistent fill.
    if (nshards <= 1) return std::max(8, E.num_cus - env_int("ANYSEQ_SHARD_RESERVE", 16));
    // Several persistent fills on one GPU that wait for each other (the in-process
    // transport): each fill workgroup needs a CU of its own (LDS), a launch spreads its
    // workgroups round-robin over the 8 XCDs, and a launch that cannot place all of its
    // workgroups holds back the dispatch of the launches behind it.  With (CUs-16)/N
    // workgroups per fill (60 at N = 4) the XCDs that get 8 of every launch's were full
    // (32 of 32 CUs) and about 1 % of 4-shard runs deadlocked until the 10 s spin limit
    // (DESIGN.md §8); at most (CUs/8 - 8)/N per XCD per fill leaves 8 CUs per XCD free:
    // 0 failures in 3200 runs.
    const int xcds = 8, per_xcd = E.num_cus / xcds;
    const int reserve = env_int("ANYSEQ_SHARD_RESERVE", 0);
    if (reserve > 0) return std::max(8, (E.num_cus - reserve) / nshards);
    return std::max(8, xcds * std::max(1, (per_xcd - 8) / nshards));
}

// The in-process shards (kept: streams, counters, buffers are reused; they never move,
// their buffers are registered by address).
std::vector<Shard>& local_shards() {
    static std::vector<Shard> shards;
    if (shards.capacity() < 64) shards.reserve(64);
    return shards;
}

int64_t shard_score_local(int kind, const anyseq_scoring& sc, const char* q, int n, const char* s, int m, int N) {
    check_shard_shape(kind, sc, n, m, N);
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    std::vector<Shard>& shards = local_shards();
    // every local shard's persistent fill must be co-resident with the others (they
    // wait for each other): grid_per_shard gives each at least one workgroup per XCD
    // and keeps 8 CUs per XCD free, so at most CUs/8 - 8 shards fit (24 on MI355X)
    const int max_local = std::max(1, E.num_cus / 8 - 8);
    if (N > max_local) fail("sharded fill: at most %d local shards on this device (got %d)", max_local, N);
    if (N > 64) fail("sharded fill: at most 64 local shards");
    if ((int)shards.size() < N) shards.resize(N);
    uint8_t* dq = (uint8_t*)E.q.get((size_t)n);
    uint8_t* ds = (uint8_t*)E.s.get((size_t)m);
    HIPCHECK(hipMemcpy(dq, q, (size_t)n, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(ds, s, (size_t)m, hipMemcpyHostToDevice));
    const bool direct = use_direct();
    check_hw_queues(direct || N == 1 ? N : 3 * N - 2);
    for (int g = 0; g < N; ++g) {
        shards[g].init();
        if (direct) continue;
        if (g + 1 < N) lazy_stream(shards[g].top.s_send);
        if (g > 0) lazy_stream(shards[g].bot.s_send);
    }
    int32_t* res = (int32_t*)E.fc.ctr.get(128) + 4;
    HIPCHECK(hipMemset(res, kind == KIND_LOCAL ? 0 : 0x80, 4));
    FillParams fp = make_params(kind, sc);
    // affine: the fills compare alphabet codes (the v_perm weight table);
    // the transported columns are values, so any consistent recoding is exact
    const uint8_t *fq = dq, *fs = ds;
    if (sc.gap_open != 0) {
        const SeqCodes cd = prepare_codes(E, dq, n, ds, m, E.stream);
        HIPCHECK(hipStreamSynchronize(E.stream));
        fq = cd.q;
        fs = cd.s;
        fp.alpha = cd.alpha;
    }
    std::vector<std::vector<DPProblem>> probs(N);
    int h1 = 0, h2 = 0;
    for (int g = 0; g < N; ++g) {
        Shard& S = shards[g];
        S.init();
        S.g = g;
        S.c0 = block_c0(g, N, m);
        S.w = block_c0(g + 1, N, m) - S.c0;
        setup_shard(S, N, kind, sc, fq, n, fs + S.c0, m, probs[g], h1, h2, direct);
        if (kind == KIND_LOCAL) {
            probs[g][0].best = res;
            probs[g][1].best = res;
        }
    }
    if (direct) {
        // each shard polls its neighbours' out_col: every sentinel fill precedes every fill
        for (int g = 0; g < N; ++g) {
            if (g > 0) shards[g].lT = probs[g][0].left_in = (const int32_t*)shards[g - 1].top.out_col.p;
            if (g + 1 < N) shards[g].lB = probs[g][1].left_in = (const int32_t*)shards[g + 1].bot.out_col.p;
            if (sc.gap_open != 0) {
                if (g > 0) shards[g].lTe = probs[g][0].left_in_e = (const int32_t*)shards[g - 1].top.out_col_e.p;
                if (g + 1 < N) shards[g].lBe = probs[g][1].left_in_e = (const int32_t*)shards[g + 1].bot.out_col_e.p;
            }
            for (int k = 0; k < N; ++k)
                if (k != g) HIPCHECK(hipStreamWaitEvent(shards[g].st, shards[k].ready, 0));
        }
    }
    // a copy lands in the neighbour's left_in: it must follow that shard's sentinel fill
    for (int g = 0; g < N; ++g)
        for (int k = 0; k < N; ++k)
            if (k != g) {
                if (shards[g].top.s_send) HIPCHECK(hipStreamWaitEvent(shards[g].top.s_send, shards[k].ready, 0));
                if (shards[g].bot.s_send) HIPCHECK(hipStreamWaitEvent(shards[g].bot.s_send, shards[k].ready, 0));
            }
    static DevBuf stage_buf;
    uint32_t* stage = nullptr;
    const int nbmax = std::max((n + 63) / 64 + 1, 128);
    if (env_int("ANYSEQ_SHARD_DEBUG", 0)) {
        stage = (uint32_t*)stage_buf.get((size_t)N * 2 * nbmax * 4);
        HIPCHECK(hipMemset(stage, 0, (size_t)N * 2 * nbmax * 4));
        for (int g = 0; g < N; ++g)
            for (int f = 0; f < 2; ++f) probs[g][f].stage = stage + (g * 2 + f) * nbmax;
    }
    const int grid = grid_per_shard(E, N);
    // every shard's allocations and uploads first: the fills wait for each other once launched
    {
        const FillStages stages(N - 1);
        for (int g = 0; g < N; ++g) fill_prepare(E, shards[g].fc, probs[g], fp, shards[g].st, grid);
    }
    for (int g = 0; g < N; ++g) fill_launch(shards[g].fc);
    std::vector<Xfer> xs = direct ? std::vector<Xfer>() : local_xfers(shards, N, E.device);
    std::vector<std::thread> th = start_xfers(xs);
    std::vector<Shard*> sp;
    for (int g = 0; g < N; ++g) sp.push_back(&shards[g]);
    bool ok = true;
    std::string err;
    for (int g = 0; g < N; ++g) {
        try {
            wait_stream(shards[g].st, 120.0, "sharded fill");
            fill_finish(shards[g].fc);
        } catch (const Failure& f) {
            ok = false;
            if (err.empty()) err = f.msg;
        }
    }
    if (!ok && stage) {
        std::vector<uint32_t> st((size_t)N * 2 * nbmax);
        (void)hipMemcpy(st.data(), stage, st.size() * 4, hipMemcpyDeviceToHost);
        for (int g = 0; g < N; ++g)
            for (int f = 0; f < 2; ++f) {
                fprintf(stderr, "shard %d front %d stages:", g, f);
                for (int b = 0; b < (f ? h2 : h1 + 63) / 64 + (f ? 1 : 0) && b < nbmax; ++b)
                    fprintf(stderr, " %u@%.1fus", st[(g * 2 + f) * nbmax + b] & 7u,
                            (double)((st[(g * 2 + f) * nbmax + b] & ~7u) - (st[0] & ~7u)) * 0.16);
                fprintf(stderr, "\n");
            }
    }
    if (!ok && env_int("ANYSEQ_SHARD_DEBUG", 0)) {
        for (int g = 0; g < N; ++g)
            for (Front* f : {&shards[g].top, &shards[g].bot}) {
                uint32_t pv = 0;
                pv = use_wait_value() ? 0u : __atomic_load_n(f->progress_h, __ATOMIC_ACQUIRE);
                if (use_wait_value()) (void)hipMemcpy(&pv, f->progress, 4, hipMemcpyDeviceToHost);
                int32_t lv[4] = {0, 0, 0, 0}, oc[4] = {0, 0, 0, 0};
                if (f->left_in.p) (void)hipMemcpy(lv, f->left_in.p, 4 * std::min(4, f->h), hipMemcpyDeviceToHost);
                (void)hipMemcpy(oc, f->out_col.p, 4 * std::min(4, f->h), hipMemcpyDeviceToHost);
                fprintf(stderr, "shard %d %s: progress %u left_in %d %d %d %d out_col %d %d %d %d flags", g,
                        f == &shards[g].top ? "top" : "bot", pv, lv[0], lv[1], lv[2], lv[3], oc[0], oc[1], oc[2],
                        oc[3]);
                if (f->left_flag.p) {
                    const int nfl = (f->h + chunk_rows(f->h) - 1) / chunk_rows(f->h);
                    std::vector<uint32_t> fl((size_t)nfl);
                    (void)hipMemcpy(fl.data(), f->left_flag.p, (size_t)nfl * 4, hipMemcpyDeviceToHost);
                    for (uint32_t x : fl) fprintf(stderr, " %u", x);
                }
                fprintf(stderr, "\n");
            }
    }
    finish_xfers(th, xs, sp, ok);
    // every transfer drains before returning, also after a failure: a copy still in
    // flight would land in the next call's freshly reset left columns and flags
    for (int g = 0; g < N; ++g)
        for (Front* f : {&shards[g].top, &shards[g].bot})
            if (f->s_send) wait_stream(f->s_send, 30.0, "shard transport");
    if (!ok) fail("%s", err.c_str());
    for (int g = 0; g < N; ++g) enqueue_combine(shards[g], N, kind, sc, m, h1, h2, res);
    int32_t v = 0;
    for (int g = 0; g < N; ++g) HIPCHECK(hipStreamSynchronize(shards[g].st));
    HIPCHECK(hipMemcpy(&v, res, 4, hipMemcpyDeviceToHost));
    if (const char* dump = getenv("ANYSEQ_SHARD_DUMP")) {
        dump_shards(dump, shards, N, kind, sc, m, h1, h2, v);
        if (stage) {
            FILE* f = fopen(dump, "a");
            for (int g = 0; f && g < N; ++g)
                for (int fr = 0; fr < 2; ++fr) {
                    char name[64];
                    snprintf(name, sizeof name, "probe shard %d front %d", g, fr);
                    dump_arr(f, name, stage + (g * 2 + fr) * nbmax + 64, 32);
                }
            if (f) fclose(f);
        }
    }
    return v;
}

int64_t shard_score_rccl(int kind, const anyseq_scoring& sc) {
    if (!g_rccl || g_rccl->rank < 0) fail("anyseq_shard_init has not been called");
    RcclState& R = *g_rccl;
    if (R.n <= 0) fail("anyseq_shard_load has not been called");
    check_shard_shape(kind, sc, R.n, R.m, R.world);
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    Shard& S = R.shard;
    S.init();
    check_hw_queues(1 + 2 * ((R.rank > 0) + (R.rank < R.world - 1)));
    if (R.rank > 0) {
        lazy_stream(S.top.s_recv);
        lazy_stream(S.bot.s_send);
    }
    if (R.rank < R.world - 1) {
        lazy_stream(S.top.s_send);
        lazy_stream(S.bot.s_recv);
    }
    S.g = R.rank;
    S.c0 = R.c0;
    S.w = R.w;
    int32_t* res = (int32_t*)S.res.get(64);
    HIPCHECK(hipMemsetAsync(res, kind == KIND_LOCAL ? 0 : 0x80, 4, S.st));
    FillParams fp = make_params(kind, sc);
    // affine: alphabet codes of this rank's query and subject block (each rank recodes
    // its own pair: only the equality of symbols enters the DP, and the ranks exchange
    // values, never symbols)
    const uint8_t* fq = (const uint8_t*)R.q.p;
    const uint8_t* fs = (const uint8_t*)R.s.p;
    if (sc.gap_open != 0) {
        const SeqCodes cd = prepare_codes(E, fq, R.n, fs, R.w, S.st);
        fq = cd.q;
        fs = cd.s;
        fp.alpha = cd.alpha;
    }
    std::vector<DPProblem> probs;
    int h1 = 0, h2 = 0;
    setup_shard(S, R.world, kind, sc, fq, R.n, fs, R.m, probs, h1, h2);
    if (kind == KIND_LOCAL) {
        probs[0].best = res;
        probs[1].best = res;
    }
    {
        const FillStages stages(R.world - 1);
        fill_async(E, S.fc, probs, fp, S.st, grid_per_shard(E, 1));
    }
    std::vector<Xfer> xs = rccl_xfers(R, E.device);
    std::vector<std::thread> th = start_xfers(xs);
    bool ok = true;
    std::string err;
    try {
        wait_stream(S.st, 300.0, "sharded fill");
        fill_finish(S.fc);
    } catch (const Failure& f) {
        ok = false;
        err = f.msg;
    }
    finish_xfers(th, xs, {&S}, ok);
    if (!ok) fail("%s", err.c_str());
    for (hipStream_t t : {S.top.s_send, S.top.s_recv, S.bot.s_send, S.bot.s_recv})
        if (t) wait_stream(t, 60.0, "shard transport");
    enqueue_combine(S, R.world, kind, sc, R.m, h1, h2, res);
    NCCLCHECK(ncclAllReduce(res, res, 1, ncclInt32, ncclMax, R.comm[0], S.st));
    int32_t v = 0;
    HIPCHECK(hipMemcpyAsync(&v, res, 4, hipMemcpyDeviceToHost, S.st));
    wait_stream(S.st, 60.0, "score all-reduce");
    return v;
}


// ---------------------------------------------------------------------------
// Column-blocked levels of the sharded affine construct (DESIGN.md §6.2,
// align.impala:254-259).  A part's halves, both transposed (subject codes as rows),
// are the two fronts of ONE problem split at row `half`: the forward half is the top
// front, the reversed one the bottom front.  Shard g of the part's rank subgroup fills
// query columns [c0, c0 + w) of both with the score sharding's boundary-column
// transport, and its two bottom rows become its segment of the level's columns (zero
// elsewhere, so the construct's SUM reduction assembles them).  The halves' border
// modes and kind bits replace the score's; a last-column best cell belongs to the
// shard that holds the half's last column (the reversed half's: the first).
void part_setup(Shard& S, const ShardLevel& J, const ShardPart& T, int view, std::vector<DPProblem>& probs) {
    const int N = T.G;
    int h1 = 0, h2 = 0;
    probs.clear();
    setup_shard(S, N, J.kind, J.sc, T.cs + T.soff, T.mw, T.cq + T.off + S.c0, T.len, probs, h1, h2, false, T.half);
    const bool holds_last[2] = {S.g == N - 1, S.g == 0};
    const int bm[2] = {T.bm_l, T.bm_r}, am[2] = {T.am_l, T.am_r};
    int32_t* pb = T.pbest + (size_t)view * J.pstride;
    for (int f = 0; f < 2; ++f) {
        DPProblem& P = probs[f];
        int a = am[f];
        if ((a & AM_BEST_LASTCOL) == AM_BEST_LASTCOL && !holds_last[f]) a &= ~AM_BEST_LASTCOL;
        P.bmode = bm[f];
        P.amode = a;
        P.best = (a & AM_BEST_LASTCOL) ? pb + f : nullptr;
    }
    // bottom row (kernel value space, G or X) -> H / E of the level's columns; a global
    // (G space) block's frame is shifted by its first column in the half (as the score
    // combine's), which the job's column offset takes out
    const size_t vo = (size_t)view * J.nn + (size_t)T.off;
    const int cr = T.len - S.c0 - S.w;   // the block's first column in the reversed half
    const bool glob = J.kind == KIND_GLOBAL;
    S.h_jobs[0] = RowToCol{S.top.out_row.p, J.LH + vo + S.c0, J.LE + vo + S.c0, S.w, h1 - 1,
                           probs[0].amode != 0 ? 1 : 0, glob ? S.c0 : 0};
    S.h_jobs[1] = RowToCol{S.bot.out_row.p, J.RH + vo + cr, J.RE + vo + cr, S.w, h2 - 1,
                           probs[1].amode != 0 ? 1 : 0, glob ? cr : 0};
    // (synchronous: every shard is set up before any fill is launched)
    HIPCHECK(hipMemcpy(S.jobs.get(sizeof S.h_jobs), S.h_jobs, sizeof S.h_jobs, hipMemcpyHostToDevice));
}

// After a shard's fill: its column segments, then the construct's stream waits for it.
void part_finish(Shard& S, const ShardLevel& J) {
    HIPCHECK(anyseq_launch_aff_row_to_col(S.jobs.p, 2, S.w, -J.sc.gap_extend, S.st));
    HIPCHECK(hipEventRecord(S.ready, S.st));
    HIPCHECK(hipStreamWaitEvent(J.st, S.ready, 0));
}

hipEvent_t level_event() {
    static hipEvent_t ev = nullptr;
    if (!ev) HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return ev;
}

void check_part(const ShardPart& T) {
    if (T.len < T.G) fail("sharded construct: %d query rows cannot be split over %d ranks", T.len, T.G);
    if (T.half < 1 || T.half >= T.mw) fail("internal: sharded part split %d of %d columns", T.half, T.mw);
    if (g_tuning.R != 1) fail("sharded construct: rows_per_lane must be 1");
}

// A shard's place: its part's subgroup, its column block of the part's query rows.
void place_shard(Shard& S, const ShardPart& T, int rank) {
    S.g = rank - T.r0;
    S.c0 = block_c0(S.g, T.G, T.len);
    S.w = block_c0(S.g + 1, T.G, T.len) - S.c0;
}

// The blocked levels run their shards' fills concurrently: emulated ranks need 3N-2
// streams (fill + transport) and N co-resident grids of >= 8 workgroups (one per XCD);
// one rank per GPU needs its fill and up to 4 transport streams.  When the process
// cannot give it that, the construct deals every level round-robin instead of failing
// (same result, bit for bit).
// (the process's queues as HIP read them, or the plan_hw_queues option's; less the
// engine's and torch's)
int hw_queues_available() {
    return (g_tuning.plan_queues > 0 ? std::min(g_tuning.plan_queues, process_hw_queues()) : process_hw_queues()) - 2;
}
int max_local_level1(int num_cus) { return std::max(1, num_cus / 8 - 8); }
bool level1_local_possible(int N, int num_cus) {
    return N >= 2 && N <= max_local_level1(num_cus) && 3 * N - 2 <= hw_queues_available();
}
// The same answer on every rank (the ranks must agree on the collectives a level runs):
// the worst case, an interior rank's fill + 2 transport streams per neighbour.
bool level1_rccl_possible(int world) {
    return world >= 2 && 1 + 2 * std::min(2, world - 1) <= hw_queues_available();
}

// Emulated ranks (anyseq_construct_local_sharded): N in-process shards, view g = rank g;
// every part's subgroup at once, transport links inside each subgroup only.
void blocked_local(const ShardLevel& J, int N) {
    for (const ShardPart& T : J.parts) check_part(T);
    Engine& E = *J.E;   // (the construct holds E.mu; no engine() here: it would release retired blocks mid-call)
    std::vector<Shard>& shards = local_shards();
    const int max_local = max_local_level1(E.num_cus);
    if (N > max_local) fail("sharded construct: at most %d emulated ranks on this device (got %d)", max_local, N);
    if ((int)shards.size() < N) shards.resize(N);
    check_hw_queues(3 * N - 2);
    std::vector<int> part_of(N, -1);
    for (size_t p = 0; p < J.parts.size(); ++p)
        for (int r = J.parts[p].r0; r < J.parts[p].r0 + J.parts[p].G; ++r) part_of[r] = (int)p;
    std::vector<int> act;   // the ranks with a part at this level
    for (int g = 0; g < N; ++g)
        if (part_of[g] >= 0) act.push_back(g);
    for (int g : act) {
        const ShardPart& T = J.parts[part_of[g]];
        shards[g].init();
        place_shard(shards[g], T, g);
        if (shards[g].g + 1 < T.G) lazy_stream(shards[g].top.s_send);
        if (shards[g].g > 0) lazy_stream(shards[g].bot.s_send);
    }
    // behind the construct's stream: the level's zeroed columns and reset best cells
    HIPCHECK(hipEventRecord(level_event(), J.st));
    std::vector<std::vector<DPProblem>> probs(N);
    for (int g : act) {
        HIPCHECK(hipStreamWaitEvent(shards[g].st, level_event(), 0));
        part_setup(shards[g], J, J.parts[part_of[g]], g, probs[g]);
    }
    for (int g : act)   // a copy lands in a neighbour's left_in after its sentinel fill
        for (int k : act)
            if (k != g) {
                if (shards[g].top.s_send) HIPCHECK(hipStreamWaitEvent(shards[g].top.s_send, shards[k].ready, 0));
                if (shards[g].bot.s_send) HIPCHECK(hipStreamWaitEvent(shards[g].bot.s_send, shards[k].ready, 0));
            }
    const int grid = grid_per_shard(E, (int)act.size());
    for (int g : act) fill_prepare(E, shards[g].fc, probs[g], J.fp, shards[g].st, grid);
    for (int g : act) fill_launch(shards[g].fc);
    std::vector<Xfer> xs;
    for (const ShardPart& T : J.parts) {   // links inside the subgroup
        for (int g = T.r0; g + 1 < T.r0 + T.G; ++g) {
            Shard &A = shards[g], &B = shards[g + 1];
            Xfer x;
            x.device = E.device;
            x.src = &A.top;   // top: g -> g+1
            x.dst = (int32_t*)B.top.left_in.p;
            x.dst_e = (int32_t*)B.top.left_in_e.p;
            x.flag = (uint32_t*)B.top.left_flag.p;
            x.h = A.top.h;
            xs.push_back(x);
            Xfer y;
            y.device = E.device;
            y.src = &B.bot;   // bottom: g+1 -> g
            y.dst = (int32_t*)A.bot.left_in.p;
            y.dst_e = (int32_t*)A.bot.left_in_e.p;
            y.flag = (uint32_t*)A.bot.left_flag.p;
            y.h = B.bot.h;
            xs.push_back(y);
        }
    }
    std::vector<std::thread> th = start_xfers(xs);
    std::vector<Shard*> sp;
    for (int g : act) sp.push_back(&shards[g]);
    bool ok = true;
    std::string err;
    for (int g : act) {
        try {
            wait_stream(shards[g].st, 120.0, "sharded construct level");
            fill_finish(shards[g].fc);
        } catch (const Failure& f) {
            ok = false;
            if (err.empty()) err = f.msg;
        }
    }
    finish_xfers(th, xs, sp, ok);
    for (int g : act)
        for (Front* f : {&shards[g].top, &shards[g].bot})
            if (f->s_send) wait_stream(f->s_send, 30.0, "shard transport");
    if (!ok) fail("%s", err.c_str());
    for (int g : act) part_finish(shards[g], J);
}

// One rank per GPU (anyseq_shard_construct): this rank's block of its part over RCCL.
void blocked_rccl(const ShardLevel& J) {
    if (!g_rccl || g_rccl->rank < 0) fail("anyseq_shard_init has not been called");
    RcclState& R = *g_rccl;
    for (const ShardPart& T : J.parts) check_part(T);
    const ShardPart* mine = nullptr;
    for (const ShardPart& T : J.parts)
        if (R.rank >= T.r0 && R.rank < T.r0 + T.G) mine = &T;
    if (!mine) return;   // no part for this rank at this level (its columns stay zero)
    const ShardPart& T = *mine;
    Engine& E = *J.E;   // (the construct holds E.mu)
    Shard& S = R.shard;
    S.init();
    place_shard(S, T, R.rank);
    const bool has_left = S.g > 0, has_right = S.g + 1 < T.G;
    check_hw_queues(1 + 2 * ((int)has_left + (int)has_right));
    if (has_left) {
        lazy_stream(S.top.s_recv);
        lazy_stream(S.bot.s_send);
    }
    if (has_right) {
        lazy_stream(S.top.s_send);
        lazy_stream(S.bot.s_recv);
    }
    HIPCHECK(hipEventRecord(level_event(), J.st));
    HIPCHECK(hipStreamWaitEvent(S.st, level_event(), 0));
    std::vector<DPProblem> probs;
    part_setup(S, J, T, 0, probs);
    fill_async(E, S.fc, probs, J.fp, S.st, grid_per_shard(E, 1));
    // links inside the subgroup only: rank g's neighbours g-1 / g+1 (link a joins ranks a
    // and a+1 on the communicators of rccl_xfers)
    std::vector<Xfer> xs;
    auto add = [&](Front* f, bool recv, int peer, ncclComm_t c) {
        Xfer x;
        x.device = E.device;
        x.src = f;
        x.recv = recv;
        x.peer = peer;
        x.comm = c;
        x.dst = recv ? (int32_t*)f->left_in.p : nullptr;
        x.dst_e = recv ? (int32_t*)f->left_in_e.p : nullptr;
        x.flag = recv ? (uint32_t*)f->left_flag.p : nullptr;
        x.h = f->h;
        xs.push_back(x);
    };
    const int g = R.rank;
    if (has_left) {
        add(&S.top, true, g - 1, R.comm[(g - 1) % 2]);
        add(&S.bot, false, g - 1, R.comm[2 + (g - 1) % 2]);
    }
    if (has_right) {
        add(&S.top, false, g + 1, R.comm[g % 2]);
        add(&S.bot, true, g + 1, R.comm[2 + g % 2]);
    }
    std::vector<std::thread> th = start_xfers(xs);
    bool ok = true;
    std::string err;
    try {
        wait_stream(S.st, 300.0, "sharded construct level");
        fill_finish(S.fc);
    } catch (const Failure& f) {
        ok = false;
        err = f.msg;
    }
    finish_xfers(th, xs, {&S}, ok);
    if (!ok) fail("%s", err.c_str());
    for (hipStream_t t : {S.top.s_send, S.top.s_recv, S.bot.s_send, S.bot.s_recv})
        if (t) wait_stream(t, 60.0, "shard transport");
    part_finish(S, J);
}

}  // namespace
}  // namespace host
}  // namespace anyseq

using namespace anyseq::host;

extern "C" {

int anyseq_shard_unique_ids(void* out, int count) {
    try {
        for (int i = 0; i < count; ++i) {
            ncclUniqueId id;
            NCCLCHECK(ncclGetUniqueId(&id));
            memcpy((char*)out + (size_t)i * NCCL_UNIQUE_ID_BYTES, &id, NCCL_UNIQUE_ID_BYTES);
        }
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_init(int rank, int world, const void* ids, int count) {
    try {
        if (count < kComms) fail("anyseq_shard_init needs %d unique ids, got %d", kComms, count);
        if (world < 1 || rank < 0 || rank >= world) fail("bad rank %d / world %d", rank, world);
        engine();   // selects the device
        g_rccl.reset(new RcclState);
        g_rccl->rank = rank;
        g_rccl->world = world;
        for (int i = 0; i < kComms; ++i) {
            ncclUniqueId id;
            memcpy(&id, (const char*)ids + (size_t)i * NCCL_UNIQUE_ID_BYTES, NCCL_UNIQUE_ID_BYTES);
            NCCLCHECK(ncclCommInitRank(&g_rccl->comm[i], world, id, rank));
        }
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_load(const char* query, int lenq, const char* subject_block, int w, int c0, int lens) {
    try {
        if (!g_rccl || g_rccl->rank < 0) fail("anyseq_shard_init has not been called");
        RcclState& R = *g_rccl;
        if (c0 != block_c0(R.rank, R.world, lens) || w != block_c0(R.rank + 1, R.world, lens) - c0)
            fail("rank %d must own columns [%d, %d) of %d", R.rank, block_c0(R.rank, R.world, lens),
                 block_c0(R.rank + 1, R.world, lens), lens);
        Engine& E = engine();
        std::lock_guard<std::mutex> lk(E.mu);
        HIPCHECK(hipMemcpy(R.q.get((size_t)lenq), query, (size_t)lenq, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(R.s.get((size_t)w), subject_block, (size_t)w, hipMemcpyHostToDevice));
        R.n = lenq;
        R.m = lens;
        R.c0 = c0;
        R.w = w;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_score(int kind, const anyseq_scoring* sc, int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : anyseq_scoring{2, -1, 0, -1};
        const int64_t v = shard_score_rccl(kind, s);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        if (g_rccl)
            for (auto& c : g_rccl->comm)
                if (c) ncclCommAbort(c), c = nullptr;
        return -1;
    }
}

int anyseq_shard_finalize(void) {
    if (g_rccl) {
        for (auto& c : g_rccl->comm)
            if (c) ncclCommDestroy(c), c = nullptr;
        g_rccl.reset();
    }
    return 0;
}

// Sharded affine construct.  Every rank passes the whole pair; the
// result (score, both strings) is returned on every rank.
static int64_t sharded_construct(int kind, const anyseq_scoring& s, const char* query, int lenq, const char* subject,
                                 int lens, char* alq, char* als, const ConstructShards& shards) {
    check_scoring(kind, s);
    check_value_range(s, lenq, lens);
    if (s.gap_open == 0) fail("sharded construct: affine gaps only (gap_open < 0)");
    if (lenq < 0 || lens < 0) fail("negative sequence length");
    // the ranks' strings merge by a byte-wise MAX over a ' ' prefill: every written
    // byte must sort above ' ' ('_' does), so sequence bytes <= 0x20 are refused
    if (shards.world > 1) {
        for (int i = 0; i < lenq; ++i)
            if ((unsigned char)query[i] <= 0x20) fail("sharded construct: query byte %d is <= 0x20 (0x%02x)", i,
                                                      (unsigned char)query[i]);
        for (int i = 0; i < lens; ++i)
            if ((unsigned char)subject[i] <= 0x20) fail("sharded construct: subject byte %d is <= 0x20 (0x%02x)", i,
                                                        (unsigned char)subject[i]);
    }
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    hipStream_t st = E.stream;
    const size_t L = (size_t)lenq + (size_t)lens;
    uint8_t* dq = (uint8_t*)E.q.get((size_t)std::max(lenq, 1));
    uint8_t* ds = (uint8_t*)E.s.get((size_t)std::max(lens, 1));
    if (lenq > 0) HIPCHECK(hipMemcpyAsync(dq, query, (size_t)lenq, hipMemcpyHostToDevice, st));
    if (lens > 0) HIPCHECK(hipMemcpyAsync(ds, subject, (size_t)lens, hipMemcpyHostToDevice, st));
    uint8_t* d_alq = (uint8_t*)E.alq.get(std::max<size_t>(L, 1));
    uint8_t* d_als = (uint8_t*)E.als.get(std::max<size_t>(L, 1));
    const int64_t v = construct_affine_dev(E, kind, s, dq, lenq, ds, lens, d_alq, d_als, st, &shards);
    if (L) {
        HIPCHECK(hipMemcpyAsync(alq, d_alq, L, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(als, d_als, L, hipMemcpyDeviceToHost, st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    return v;
}

int anyseq_construct_local_sharded(int kind, const anyseq_scoring* sc, const char* query, int lenq,
                                   const char* subject, int lens, int nshards, char* alQuery, char* alSubject,
                                   int64_t* score) {
    try {
        if (nshards < 1 || nshards > 64) fail("sharded construct: 1..64 local shards (level 1 column-blocked when the "
                                              "device and GPU_MAX_HW_QUEUES allow it, else round-robin)");
        ConstructShards cs;
        cs.world = nshards;
        cs.local = true;
        if (level1_local_possible(nshards, engine().num_cus))
            cs.blocked = [nshards](const ShardLevel& J) { blocked_local(J, nshards); };
        const int64_t v = sharded_construct(kind, sc ? *sc : anyseq_scoring{2, -1, -2, -1}, query, lenq, subject,
                                            lens, alQuery, alSubject, cs);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_construct(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject,
                           int lens, char* alQuery, char* alSubject, int64_t* score) {
    try {
        if (!g_rccl || g_rccl->rank < 0) fail("anyseq_shard_init has not been called");
        ncclComm_t comm = g_rccl->comm[0];
        ConstructShards cs;
        cs.rank = g_rccl->rank;
        cs.world = g_rccl->world;
        cs.sum_i32 = [comm](int32_t* p, size_t n, hipStream_t st) {
            NCCLCHECK(ncclAllReduce(p, p, n, ncclInt32, ncclSum, comm, st));
        };
        cs.max_i32 = [comm](int32_t* p, size_t n, hipStream_t st) {
            NCCLCHECK(ncclAllReduce(p, p, n, ncclInt32, ncclMax, comm, st));
        };
        cs.max_u8 = [comm](uint8_t* p, size_t n, hipStream_t st) {
            NCCLCHECK(ncclAllReduce(p, p, n, ncclUint8, ncclMax, comm, st));
        };
        if (level1_rccl_possible(cs.world)) cs.blocked = [](const ShardLevel& J) { blocked_rccl(J); };
        const int64_t v = sharded_construct(kind, sc ? *sc : anyseq_scoring{2, -1, -2, -1}, query, lenq, subject,
                                            lens, alQuery, alSubject, cs);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_construct_hostcoll(int kind, const anyseq_scoring* sc, const char* query, int lenq,
                                    const char* subject, int lens, int rank, int world,
                                    anyseq_host_allreduce_fn reduce, void* user, char* alQuery, char* alSubject,
                                    int64_t* score) {
    try {
        if (world < 2 || rank < 0 || rank >= world) fail("host-collective construct: rank %d of world %d", rank, world);
        if (!reduce) fail("host-collective construct: no reduce callback");
        // each reduction: the stream drained, the device buffer down, the ranks' host
        // all-reduce, the result back up -- the RCCL branch's data flow, host transport
        auto red = [reduce, user](void* p, size_t count, size_t esz, int dtype, int op, hipStream_t st) {
            std::vector<uint8_t> h(std::max<size_t>(count * esz, 1));
            HIPCHECK(hipMemcpyAsync(h.data(), p, count * esz, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipStreamSynchronize(st));
            if (reduce(h.data(), (int64_t)count, dtype, op, user) != 0) fail("host all-reduce callback failed");
            HIPCHECK(hipMemcpyAsync(p, h.data(), count * esz, hipMemcpyHostToDevice, st));
            HIPCHECK(hipStreamSynchronize(st));
        };
        ConstructShards cs;
        cs.rank = rank;
        cs.world = world;
        cs.sum_i32 = [red](int32_t* p, size_t n, hipStream_t st) { red(p, n, 4, 0, 0, st); };
        cs.max_i32 = [red](int32_t* p, size_t n, hipStream_t st) { red(p, n, 4, 0, 1, st); };
        cs.max_u8 = [red](uint8_t* p, size_t n, hipStream_t st) { red(p, n, 1, 1, 1, st); };
        const int64_t v = sharded_construct(kind, sc ? *sc : anyseq_scoring{2, -1, -2, -1}, query, lenq, subject,
                                            lens, alQuery, alSubject, cs);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

int anyseq_shard_score_local(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject,
                             int lens, int nshards, int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : anyseq_scoring{2, -1, 0, -1};
        const int64_t v = shard_score_local(kind, s, query, lenq, subject, lens, nshards);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        set_last_error(f.msg);
        return -1;
    }
}

}  // extern "C"
