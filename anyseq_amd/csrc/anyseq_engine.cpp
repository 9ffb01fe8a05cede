// anyseq_engine.cpp — host side of the MI355X AnySeq engine: per-device state,
// the score driver (align.impala:218-235) and the linear-space construct driver
// (the reference's column-split Hirschberg, align.impala:237-311,
// traceback_lintime.impala:1-148) over the HIP kernels of anyseq_kernels.hip.
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/anyseq.h"
#include "anyseq_host.h"
#include "anyseq_internal.h"

using namespace anyseq;

extern "C" {
hipError_t anyseq_launch_fill(int R, int CH, int NW, const DPProblem* probs, const GroupRef* groups, int ngroups,
                              uint32_t* dq, uint32_t* err, const FillParams* fp, int grid, hipStream_t st);
hipError_t anyseq_launch_fill_affine(int NW, const DPProblem* probs, const GroupRef* groups, int ngroups,
                                     uint32_t* dq, uint32_t* err, const FillParams* fp, int grid, hipStream_t st);
hipError_t anyseq_launch_aff_reduce(int kind, int two, const void* rowF, int h1, const void* rowB, int h2, int m,
                                    int go, int ge, const int32_t* colF, const int32_t* colB, int32_t* out,
                                    hipStream_t st);
hipError_t anyseq_launch_semiglobal_reduce(const int32_t* row_g, int m, const int32_t* col_h, int n, int ng,
                                           int32_t* out, hipStream_t st);
hipError_t anyseq_launch_front_combine(int kind, const int32_t* rowF, int h1, const int32_t* rowB, int h2, int m,
                                       int gap, const int32_t* colF, const int32_t* colB, int32_t* out,
                                       hipStream_t st);
hipError_t anyseq_launch_hb_sum(const void* parts, int nparts, int bpp, int half, const int32_t* L, const int32_t* R,
                                int kind, int gap, int32_t* bmax, int32_t* bind, int32_t* splits, hipStream_t st);
hipError_t anyseq_launch_pred(const void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S, uint8_t* pred,
                              const FillParams* fp, hipStream_t st);
hipError_t anyseq_launch_walk(const void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S,
                              const uint8_t* pred, int kind, uint8_t* alq, uint8_t* als, hipStream_t st);
hipError_t anyseq_launch_fulltb(const uint8_t* Q, int n, const uint8_t* S, int m, uint8_t* pred, int32_t* cols,
                                uint32_t* ticket, uint32_t* err, int match, int mismatch, int gap, uint8_t* alq,
                                uint8_t* als, hipStream_t st);
hipError_t anyseq_launch_aff_hb_join(const void* parts, int nparts, int half, const int32_t* LH, const int32_t* LE,
                                     const int32_t* RH, const int32_t* RE, const int32_t* pbest, int go, int ge,
                                     int32_t* splits, int32_t* types, int32_t* score, hipStream_t st);
hipError_t anyseq_launch_aff_row_to_col(const void* jobs, int njobs, int maxn, int nge, hipStream_t st);
hipError_t anyseq_launch_i32_jobs(const void* jobs, int njobs, int maxn, hipStream_t st);
hipError_t anyseq_launch_fill_prep(uint32_t* zero, int nzero, int32_t* init, int ninit, int32_t init_value,
                                   void* sent, size_t sent_bytes, uint32_t sent_value, const void* up_src, void* up_dst,
                                   size_t up_bytes, hipStream_t st);
hipError_t anyseq_launch_aff_hb_join2(const void* parts, int nparts, int maxlen, int half, const int32_t* LH,
                                      const int32_t* LE, const int32_t* RH, const int32_t* RE, const int32_t* pbest,
                                      int go, int ge, void* partial, int32_t* splits, int32_t* types, int32_t* score,
                                      hipStream_t st);
hipError_t anyseq_launch_view_reduce_i32(int32_t* base, size_t stride, int nviews, size_t n, int op, hipStream_t st);
hipError_t anyseq_launch_view_max_u8(uint8_t* dst, const uint8_t* others, size_t stride, int nothers, size_t n,
                                     hipStream_t st);
hipError_t anyseq_launch_seq_codes(const uint8_t* q, int n, const uint8_t* s, int m, uint32_t* mask, uint8_t* table,
                                   int32_t* alpha, uint8_t* out, uint8_t* fill0, uint8_t* fill1, size_t fill_len,
                                   hipStream_t st);
hipError_t anyseq_launch_aff_predwalk(void* blocks, int nblocks, const uint8_t* Q, const uint8_t* S, uint8_t* pred,
                                      int match, int mismatch, int go, int ge, uint8_t* alq, uint8_t* als, int lds_rows,
                                      hipStream_t st);
hipError_t anyseq_launch_aff_level_plan(const AffLevelPlan* plan, hipStream_t st);
hipError_t anyseq_launch_aff_final(const AffFinalPlan* plan, const uint8_t* Q, const uint8_t* S, uint8_t* pred,
                                   int match, int mismatch, int go, int ge, uint8_t* alq, uint8_t* als,
                                   hipStream_t st);
hipError_t anyseq_launch_aff_level_tail(const void* tail, int fill_groups, hipStream_t st);
hipError_t anyseq_launch_rows_check(const void* rows, size_t nwords, uint32_t sentinel, const void* probs, int nprobs,
                                    uint32_t* out, int inject, hipStream_t st);
hipError_t anyseq_launch_aff_scode(const void* probs, int nprobs, int64_t max_w, hipStream_t st);
}

namespace anyseq {
namespace host {

constexpr int32_t SPLIT_UNSET = 0x7fff0000;
constexpr int MIN_PART_WIDTH_HB = 128;             // align.impala:18
constexpr int CPU_BLOCK_WIDTH = 1024;              // iteration_cpu.impala:1 (hb_sum stride)

thread_local std::string g_last_error;
thread_local double g_fill_ms = 0.0;
thread_local int g_fill_launches = 0;
thread_local int g_fill_r2 = 0;     // affine launches with >= 2 rows per lane (anyseq_last_fill_multi_row_launches)
thread_local int g_fill_rmax = 1;   // the most rows per lane among them
thread_local int g_fill_stages = 0;
thread_local int g_shard_blocked_levels = 0;   // anyseq_last_shard_plan
thread_local int64_t g_fill_cells = 0;
thread_local int64_t g_inherit_stats[2] = {0, 0};   // split halves, reused halves (anyseq_last_inherit_stats)

int env_int_early(const char* name) {
    const char* v = getenv(name);
    return v ? atoi(v) : 0;
}
void set_last_error(const std::string& m) { g_last_error = m; }
// diagnostics (ANYSEQ_HOST_STAMPS=1): host-side phase stamps of one construct call,
// printed to stderr at its end (where the host, not the GPU, sits on the critical path)
const int g_host_stamps = env_int_early("ANYSEQ_HOST_STAMPS");
thread_local std::vector<std::pair<const char*, double>> g_hs;
double host_now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline void hstamp(const char* what) {
    if (g_host_stamps) g_hs.emplace_back(what, host_now_us());
}
void hstamp_print() {
    if (!g_host_stamps || g_hs.empty()) return;
    fprintf(stderr, "host stamps:");
    for (size_t i = 1; i < g_hs.size(); ++i) fprintf(stderr, " %s %.1f", g_hs[i].first, g_hs[i].second - g_hs[i - 1].second);
    fprintf(stderr, " | total %.1f us\n", g_hs.back().second - g_hs.front().second);
    g_hs.clear();
}

[[noreturn]] void fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw Failure{buf};
}

// ------------------------------------------------------------- buffers --
// Live allocations (for the ANYSEQ_CHECK_PTRS audit) and retired ones (freed by
// release_retired at a point where nothing of ours is in flight).
namespace {
struct Alloc {
    const void* owner;
    uintptr_t lo, hi;
};
std::mutex g_alloc_mu;
std::vector<Alloc> g_live;                   // owner -> current block
std::vector<std::pair<void*, bool>> g_retired;   // (block, pinned)
std::vector<std::pair<uintptr_t, uintptr_t>> g_extern;   // caller buffers of the current call

void note_live(const void* owner, void* p, size_t cap) {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    for (Alloc& a : g_live)
        if (a.owner == owner) {
            a.lo = (uintptr_t)p;
            a.hi = (uintptr_t)p + cap;
            return;
        }
    g_live.push_back(Alloc{owner, (uintptr_t)p, (uintptr_t)p + cap});
}
void retire(const void* owner, void* p, bool pinned) {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    if (p) g_retired.emplace_back(p, pinned);
    for (size_t i = 0; i < g_live.size(); ++i)
        if (g_live[i].owner == owner) {
            g_live.erase(g_live.begin() + (long)i);
            break;
        }
}
}  // namespace

void release_retired() {
    std::vector<std::pair<void*, bool>> r;
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        if (g_retired.empty()) return;
        r.swap(g_retired);
    }
    // (an API entry: none of this library's work is in flight; the device-wide wait
    // also covers a caller's stream that may still read a retired block)
    (void)hipDeviceSynchronize();
    for (auto& b : r) {
        if (b.second) (void)hipHostFree(b.first);
        else (void)hipFree(b.first);
    }
}

bool check_ptrs_enabled() {
    static const int on = env_int("ANYSEQ_CHECK_PTRS", 0);
    return on != 0;
}
void register_static_range(const void* p, size_t bytes) { note_live(p, const_cast<void*>(p), bytes); }
void register_extern_range(const void* p, size_t bytes) {
    if (!p || !check_ptrs_enabled()) return;
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_extern.emplace_back((uintptr_t)p, (uintptr_t)p + bytes);
}
void clear_extern_ranges() {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_extern.clear();
}
void check_range(const void* p, size_t bytes, const char* what) {
    if (!p) return;
    const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    for (const Alloc& a : g_live)
        if (lo >= a.lo && hi <= a.hi) return;
    for (const auto& e : g_extern)
        if (lo >= e.first && hi <= e.second) return;
    fail("pointer audit: %s %p + %zu bytes lies outside every live allocation", what, p, bytes);
}

void* DevBuf::get(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
        retire(this, p, false);
        p = nullptr;
        size_t c = std::max(bytes, cap * 3 / 2);
        c = (c + 255) & ~size_t(255);
        if (uncached) HIPCHECK(hipExtMallocWithFlags(&p, c, hipDeviceMallocUncached));
        else HIPCHECK(hipMalloc(&p, c));
        cap = c;
        note_live(this, p, c);
    }
    return p;
}

void* PinBuf::get(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
        retire(this, p, true);
        p = nullptr;
        size_t c = std::max(bytes, cap * 3 / 2);
        c = (c + 4095) & ~size_t(4095);
        HIPCHECK(hipHostMalloc(&p, c, hipHostMallocCoherent));
        cap = c;
        note_live(this, p, c);
    }
    return p;
}

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// H2D upload through a pinned staging buffer (never from pageable memory, which the
// runtime may read after the call returns).  `pb` must not be rewritten before the
// stream has passed the copy: every call site reuses it only after a synchronisation.
void upload_pinned(PinBuf& pb, void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (!bytes) return;
    void* h = pb.get(bytes);
    memcpy(h, src, bytes);
    HIPCHECK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st));
}

void FillCtx::init() {
    if (!ev0) HIPCHECK(hipEventCreate(&ev0));
    if (!ev1) HIPCHECK(hipEventCreate(&ev1));
    if (!ev2) HIPCHECK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
}

// Diagnostics (ANYSEQ_FAULT_INFO=1): report the address of a GPU memory fault and the
// engine buffer it falls in or next to (the HIP runtime itself prints no address).
namespace {
struct NamedBuf {
    const char* name;
    const DevBuf* buf;
};
std::vector<NamedBuf> g_named;

hsa_status_t fault_handler(const hsa_amd_event_t* ev, void*) {
    if (ev->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
    const uint64_t a = ev->memory_fault.virtual_address;
    fprintf(stderr, "anyseq: GPU memory fault at 0x%llx, reason mask 0x%x\n", (unsigned long long)a,
            ev->memory_fault.fault_reason_mask);
    for (const NamedBuf& nb : g_named) {
        const uint64_t p = (uint64_t)(size_t)nb.buf->p;
        if (!p) continue;
        const long long d = (long long)(a - p);
        if (d >= -(1ll << 16) && d < (long long)nb.buf->cap + (1ll << 16))
            fprintf(stderr, "anyseq:   %-8s %p + %zu: fault at offset %lld\n", nb.name, nb.buf->p, nb.buf->cap, d);
    }
    return HSA_STATUS_SUCCESS;
}
std::mutex g_named_mu;
}  // namespace

void register_fault_buf(const char* name, const DevBuf* b) {
    if (!env_int("ANYSEQ_FAULT_INFO", 0)) return;
    std::lock_guard<std::mutex> lk(g_named_mu);
    g_named.push_back(NamedBuf{name, b});
}

Engine::Engine(int dev) : device(dev) {
    if (env_int("ANYSEQ_FAULT_INFO", 0)) {
        const NamedBuf nb[] = {{"q", &q},       {"s", &s},         {"outcol", &outcol}, {"outrow", &outrow},
                               {"L", &L},       {"R", &R},         {"LE", &LE},         {"RE", &RE},
                               {"spl", &spl},   {"typ", &typ},     {"parts", &parts},   {"bmax", &bmax},
                               {"bind", &bind}, {"blocks", &blocks}, {"pred", &pred},   {"alq", &alq},
                               {"als", &als},   {"pos", &pos},     {"jobs", &jobs},     {"fc.probs", &fc.probs},
                               {"fc.groups", &fc.groups}, {"fc.rowbuf", &fc.rowbuf}, {"fc.flags", &fc.flags},
                               {"fc.ctr", &fc.ctr}};
        std::lock_guard<std::mutex> lk(g_named_mu);
        g_named.insert(g_named.end(), std::begin(nb), std::end(nb));
        hsa_amd_register_system_event_handler(fault_handler, nullptr);
    }
    HIPCHECK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, dev));
    num_cus = prop.multiProcessorCount;
    HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIPCHECK(hipEventCreateWithFlags(&ev_order, hipEventDisableTiming));
    fc.init();
}

std::mutex g_engines_mu;
std::vector<std::unique_ptr<Engine>> g_engines;
int g_device = -1;
Tuning g_tuning;
bool g_tuning_init = false;

// Tuning knobs from the environment, once, before the first use or change.
void init_tuning_locked() {
    if (g_tuning_init) return;
    g_tuning.R = env_int("ANYSEQ_R", g_tuning.R);
    g_tuning.NW = env_int("ANYSEQ_NW", g_tuning.NW);
    g_tuning.CH = env_int("ANYSEQ_CH", g_tuning.CH);
    g_tuning.grid = env_int("ANYSEQ_GRID", g_tuning.grid);
    g_tuning.fronts = env_int("ANYSEQ_FRONTS", g_tuning.fronts);
    g_tuning.affasm = env_int("ANYSEQ_AFFINE_ASM", g_tuning.affasm);
    g_tuning.afft = env_int("ANYSEQ_AFFINE_TRANSPOSE", g_tuning.afft);
    g_tuning.prio = env_int("ANYSEQ_PRIO", g_tuning.prio);
    g_tuning.thr = env_int("ANYSEQ_THROTTLE", g_tuning.thr);
    g_tuning.NWa = env_int("ANYSEQ_NWA", g_tuning.NWa);
    g_tuning.arows = env_int("ANYSEQ_AFF_ROWS", g_tuning.arows);
    g_tuning.selffwd = env_int("ANYSEQ_SELF_FWD", g_tuning.selffwd);
    g_tuning.linaff = env_int("ANYSEQ_LIN_AFF", g_tuning.linaff);
    g_tuning.linloop = env_int("ANYSEQ_LIN_LOOP", g_tuning.linloop);
    g_tuning.iofirst = env_int("ANYSEQ_IO_FIRST", g_tuning.iofirst);
    g_tuning.forcelb = env_int("ANYSEQ_FORCE_LB", g_tuning.forcelb);
    g_tuning.grida = env_int("ANYSEQ_GRIDA", g_tuning.grida);
    g_tuning.afflut = env_int("ANYSEQ_AFFINE_LUT", g_tuning.afflut);
    g_tuning.slack = env_int("ANYSEQ_SLACK", g_tuning.slack);
    g_tuning.slack_io = env_int("ANYSEQ_SLACK_IO", g_tuning.slack_io);
    g_tuning.io_stage = env_int("ANYSEQ_IO_STAGE", g_tuning.io_stage);
    g_tuning.io_skew = env_int("ANYSEQ_IO_SKEW", g_tuning.io_skew);
    g_tuning.io_poll2 = env_int("ANYSEQ_IO_POLL2", g_tuning.io_poll2);
    g_tuning.io_fwd = env_int("ANYSEQ_IO_FWD", g_tuning.io_fwd);
    g_tuning.fill_events = env_int("ANYSEQ_FILL_EVENTS", g_tuning.fill_events);
    g_tuning.virtbest = env_int("ANYSEQ_VIRT_BEST", g_tuning.virtbest);
    g_tuning.devplan = env_int("ANYSEQ_AFF_DEVPLAN", g_tuning.devplan);
    g_tuning.devfinal = env_int("ANYSEQ_AFF_DEVFINAL", g_tuning.devfinal);
    g_tuning.xcdq = env_int("ANYSEQ_XCD_GROUPS", g_tuning.xcdq);
    g_tuning.ctrue = env_int("ANYSEQ_CONSTRUCT_TRUE", g_tuning.ctrue);
    g_tuning.inherit = env_int("ANYSEQ_INHERIT", g_tuning.inherit);
    g_tuning.inherit_depth = env_int("ANYSEQ_INHERIT_DEPTH", g_tuning.inherit_depth);
    g_tuning_init = true;
}

int process_hw_queues() {
    static const int q = env_int("GPU_MAX_HW_QUEUES", 4);
    return q;
}

Engine& engine() {
    std::lock_guard<std::mutex> lk(g_engines_mu);
    init_tuning_locked();
    (void)process_hw_queues();   // (the snapshot, before this library's first HIP call)
    if (g_device < 0) g_device = env_int("ANYSEQ_DEVICE", 0);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) fail("no HIP device available (hipGetDeviceCount)");
    if (g_device >= ndev) fail("device %d out of range (%d devices)", g_device, ndev);
    if ((int)g_engines.size() < ndev) g_engines.resize(ndev);
    if (!g_engines[g_device]) g_engines[g_device].reset(new Engine(g_device));
    HIPCHECK(hipSetDevice(g_device));
    release_retired();
    return *g_engines[g_device];
}

// A caller's stream runs the engine's work for the device API: it first waits for
// everything already queued on the engine's own stream (explicit order instead of
// the assumption that the previous call drained it), and the caller's buffers are
// registered for the pointer audit.
hipStream_t caller_stream(Engine& E, void* stream) {
    if (!stream || (hipStream_t)stream == E.stream) return E.stream;
    HIPCHECK(hipEventRecord(E.ev_order, E.stream));
    HIPCHECK(hipStreamWaitEvent((hipStream_t)stream, E.ev_order, 0));
    return (hipStream_t)stream;
}

int rows_per_lane() { return g_tuning.R == 2 ? 2 : (g_tuning.R >= 4 ? 4 : 1); }
int waves_per_group() {
    const int nw = g_tuning.NW;
    return (nw == 3 || nw == 4 || nw == 7) ? nw : 8;
}
// affine fill: 3 or 4 compute waves per workgroup (one per SIMD), or 7 (two per SIMD
// beside the I/O wave: the steady state fits 256 VGPRs)
int aff_waves_per_group() {
    const int nw = g_tuning.NWa;
    return (nw == 3 || nw == 7) ? nw : 4;
}

// Affine fill, waves per workgroup of one launch: a launch is bound by
// its longest band chain (chain_steps = w + 1.28 h of its tallest problem, one step per
// wave step) or by its total work (wave_steps over the grid's compute waves).  One
// compute wave per SIMD (NW 4) runs a wave step in ~63 cycles; two per SIMD (NW 7) share
// the SIMD's VALU at ~100 cycles each: 1.26x the throughput, 1.55x the chain step
// (measured, tools/micro/aff_loop_micro.hip, profiles/r04_ab_nw_st.json).  Chain-bound
// launches (every configs[2] Hirschberg level) keep 4; throughput-bound ones (the
// genome-length fills, bands >> waves) take 7.  An explicit affine_waves_per_group wins.
// Round 5: the throughput-bound launches run 8 compute waves and no I/O wave when
// `affine_self_forward` is on (each group's first band forwards its own input row), so no
// compute wave runs alone beside the I/O wave on its SIMD.
int aff_waves_for(int64_t chain_steps, int64_t wave_steps, int grid) {
    if (g_tuning.NWa == 3 || g_tuning.NWa == 4 || g_tuning.NWa == 7 || g_tuning.NWa == 8) return g_tuning.NWa;
    const double g = (double)std::max(grid, 1);
    const double t4 = std::max((double)chain_steps, (double)wave_steps / (4.0 * g));
    const double t7 = 1.55 * std::max((double)chain_steps, (double)wave_steps / (7.0 * g));
    return t7 < 0.9 * t4 ? (g_tuning.selffwd ? 8 : 7) : 4;
}

// Affine fill, rows per lane of one launch (round 5): R rows per lane share
// the step's lane shifts, so a wave covers 64 R rows per step at s_R times the one-row step
// time at two waves per SIMD: s_2 = 1.5 (124.9 against 83.3 cycles per wave, tools/micro/
// mix_micro.hip R2FULL / FULL, profiles/r05aa_mix_micro_r2.txt), s_3 = 2.13 (the projection
// says 2.01, R3FULL 167.6; the product measures 1.054x over two rows at configs[4], 1.063x at
// configs[3], gpurun_out/r05af / r05ag).  The throughput gains, but the band chain steps at
// s_R for a hop over 64 R rows (chain_R = w + 1.28 h / R), and a column-block pipeline's
// ranks start one band sweep of the block (w steps) after each other (g_fill_stages: the
// pipeline's stages).  NW 7 / 8 launches take the R
// with the least model time when it gains >= 10 % over one row; an explicit
// affine_rows_per_lane wins (2 and 3 need NW 4, 7 or 8).
int aff_rows_for(int NW, const int64_t (&chain)[3], int64_t work, int grid, int64_t wmax) {
    if (g_tuning.arows >= 1 && g_tuning.arows <= 3)
        return g_tuning.arows == 1 || NW == 4 || NW == 7 || NW == 8 ? g_tuning.arows : 1;
    if (NW != 7 && NW != 8) return 1;
    const double g = (double)std::max(grid, 1), s[3] = {1.0, 1.5, 2.13};
    double t[3];
    for (int r = 0; r < 3; ++r)
        t[r] = s[r] * (std::max((double)chain[r], (double)work / ((double)NW * (r + 1) * g)) +
                       (double)g_fill_stages * (double)wmax);
    const int best = t[2] < t[1] ? 3 : 2;
    return t[best - 1] < 0.9 * t[0] ? best : 1;
}

namespace {
// chain[r]: the longest band chain with r+1 rows per lane, w + 1.28 h / (r+1) steps; work:
// one-row wave steps of the launch
void aff_launch_model(const std::vector<DPProblem>& probs, int64_t (&chain)[3], int64_t& work, int64_t& wmax) {
    chain[0] = chain[1] = chain[2] = 0;
    work = 0;
    wmax = 0;
    for (const DPProblem& P : probs) {
        if (P.h <= 0 || P.w <= 0) continue;
        wmax = std::max<int64_t>(wmax, P.w);
        for (int r = 0; r < 3; ++r) chain[r] = std::max(chain[r], (int64_t)P.w + (int64_t)P.h * 128 / (100 * (r + 1)));
        work += (int64_t)((P.h + 63) / 64) * ((int64_t)P.w + 64);
    }
}
}  // namespace

// ---------------------------------------------------------------- fill --
// Prepares one batched fill launch over `probs` (host copies; device pointers set):
// every allocation, upload and sentinel fill, enqueued on st.  No kernel yet.
// ANYSEQ_CHECK_PTRS: every pointer of every descriptor, with the extent the fill
// kernels address through it, inside a live allocation.
void audit_probs(const std::vector<DPProblem>& probs, bool aff) {
    const size_t vb = aff ? 8 : 4;   // bytes per hand-off row element
    for (const DPProblem& P : probs) {
        const int64_t qlo = std::min<int64_t>(P.q_off, P.q_off + (int64_t)P.q_step * (P.h - 1));
        const int64_t slo = std::min<int64_t>(P.s_off, P.s_off + (int64_t)P.s_step * (P.w - 1));
        if (P.h > 0) check_range(P.q + qlo, (size_t)P.h, "query rows");
        if (P.w > 0) check_range(P.s + slo, (size_t)P.w, "subject columns");
        check_range(P.out_col, (size_t)P.h * 4, "out_col");
        check_range(P.out_col_e, (size_t)P.h * 4, "out_col_e");
        check_range(P.out_row, (size_t)P.wpad * vb, "out_row");
        if (P.ngroups > 1) check_range(P.rowbuf, (size_t)P.nslots * P.wpad * vb, "hand-off rows");
        check_range(P.flags, (size_t)P.ngroups * 4, "group flags");
        check_range(P.best, 4, "best cell");
        check_range(P.left_in, (size_t)P.h * 4, "left_in");
        check_range(P.left_in_e, (size_t)P.h * 4, "left_in_e");
        check_range(P.out_f_last, 4, "out_f_last");
        if (P.left_flag && P.left_chunk > 0)
            check_range(P.left_flag, (size_t)((P.h + P.left_chunk - 1) / P.left_chunk) * 4, "left_flag");
        check_range(P.progress, 4, "progress");
        if (P.scode) check_range(P.scode, (size_t)(4 * scode_len(P.w)), "subject-code rows");
    }
}

// XCD-local groups (FillParams::xq): the affine fill of a single-GPU
// launch (no concurrent shard fill it could wait on: a shard launch passes its own grid)
// of a multiple of 8 workgroups, dealt grid / 8 per XCD, when the tuning asks for it;
// returns the run of consecutive groups per XCD, or 0 (one queue).  Off by default and UNSAFE under shared CUs:
// an XCD with no resident workgroup leaves its queue's groups undealt while others wait on them.
int xcd_run(const Engine& E, int grid, bool aff, int grid_req = 0) {
    if (!aff || !g_tuning.xcdq || grid_req > 0 || grid > E.num_cus || grid < kXcds || grid % kXcds != 0) return 0;
    return grid / kXcds;
}

void fill_prepare(Engine& E, FillCtx& C, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st,
                  int grid_req, const void* extra, size_t extra_bytes, int32_t* init, int init_words,
                  int32_t init_value) {
    C.init();
    C.pending = false;
    const bool aff = fp.affine != 0;
    // the affine fill has one row per lane and hands (G, F) pairs over (twice the row bytes)
    int NW = waves_per_group();
    int R = aff ? 1 : rows_per_lane();
    if (aff) {
        int64_t chain[3], work, wmax;
        aff_launch_model(probs, chain, work, wmax);
        const int g0 = grid_req > 0 ? grid_req : (g_tuning.grida > 0 ? g_tuning.grida : E.num_cus);
        NW = aff_waves_for(chain[0], work, g0);
        R = aff_rows_for(NW, chain, work, g0, wmax);   // (affine bands: 64 R rows)
    }
    const int vpc = aff ? 2 : 1;
    // Persistent grid: at most `grid` groups are in flight, and a group finishes only after
    // its predecessor in the same problem (it consumes that group's last chunk), so the
    // groups of a problem in flight when group k starts are within [k-grid+1, k].  Hand-off
    // rows therefore live in a ring of nslots >= 2*grid+2 rows per problem (group k writes
    // slot k % nslots, the reader puts the sentinel back): O(grid * w) memory instead of
    // O(h/64 * w), which is what makes genome-length matrices fit.
    int max_groups = 0;
    size_t total_groups = 0;
    for (auto& P : probs) {
        P.nbands = (P.h + 64 * R - 1) / (64 * R);
        P.ngroups = (P.nbands + NW - 1) / NW;
        P.wpad = (P.w + 63) & ~63;
        max_groups = std::max(max_groups, P.ngroups);
        total_groups += (size_t)P.ngroups;
    }
    int grid = aff ? (g_tuning.grida > 0 ? g_tuning.grida : E.num_cus) : (g_tuning.grid > 0 ? g_tuning.grid : E.num_cus);
    if (grid_req > 0) grid = grid_req;
    grid = (int)std::min<size_t>((size_t)grid, std::max<size_t>(total_groups, 1));
    const int min_slots = 2 * grid + 2;
    const int want_slots = std::max(g_tuning.ring_slots > 0 ? g_tuning.ring_slots : 2 * min_slots, min_slots);
    size_t rowbuf_ints = 0, flag_words = 0;
    C.cells = 0;
    for (auto& P : probs) {
        C.cells += (int64_t)P.h * P.w;
        P.nslots = std::max(1, std::min(P.ngroups - 1, want_slots));
        rowbuf_ints += (size_t)(P.ngroups > 1 ? P.nslots : 0) * P.wpad * vpc;
        flag_words += P.ngroups;
    }
    int32_t* rowbuf = (int32_t*)C.rowbuf.get(rowbuf_ints * 4);
    // group table: round-robin over problems so every sub-problem progresses
    std::vector<GroupRef>& groups = C.h_groups;
    groups.clear();
    for (int k = 0; k < max_groups; ++k)
        for (size_t p = 0; p < probs.size(); ++p)
            if (k < probs[p].ngroups) groups.push_back(GroupRef{(int32_t)p, k, 0, 0});
    // XCD-local groups (FillParams::xq; a launch over the whole chip only): the table
    // stably partitioned by XCD, its 9 offsets uploaded right behind it
    const int xrun = xcd_run(E, grid, aff, grid_req);
    uint32_t xoff[kXcds + 1] = {0};
    if (xrun > 0) {
        std::vector<int64_t> first(probs.size(), 0);   // problem-major index of each problem's group 0
        for (size_t p = 1; p < probs.size(); ++p) first[p] = first[p - 1] + probs[p - 1].ngroups;
        std::vector<GroupRef> byx[kXcds];
        for (const GroupRef& g : groups) byx[xcd_of_group(first[g.prob] + g.group, xrun)].push_back(g);
        groups.clear();
        for (int x = 0; x < kXcds; ++x) {
            xoff[x] = (uint32_t)groups.size();
            groups.insert(groups.end(), byx[x].begin(), byx[x].end());
        }
        xoff[kXcds] = (uint32_t)groups.size();
    }
    // ONE device block per launch: [counters (32 words) | group flags | descriptors |
    // group table (+ XCD offsets) | caller's extra payload], so the launch costs one
    // upload and one memset besides the hand-off rows' sentinel fill
    const size_t zb = ((32 + flag_words) * 4 + 255) & ~(size_t)255;
    const size_t pb = probs.size() * sizeof(DPProblem),
                 gb = groups.size() * sizeof(GroupRef) + (xrun > 0 ? sizeof xoff : 0);
    const size_t eoff = (pb + gb + 15) & ~(size_t)15;
    const size_t ub = eoff + extra_bytes;
    char* meta = (char*)C.probs.get(zb + ub);
    uint32_t* ctr = (uint32_t*)meta;   // [0] dequeue counter, [1] error word
    uint32_t* flags = ctr + 32;
    DPProblem* d_probs = (DPProblem*)(meta + zb);
    GroupRef* d_groups = (GroupRef*)(meta + zb + pb);
    C.d_extra = extra_bytes ? meta + zb + eoff : nullptr;
    size_t ro = 0, fo = 0;
    static std::atomic<int32_t> g_epoch{0};
    const int32_t epoch = (g_epoch.fetch_add(1) + 1) & 0x7ffff;
    for (auto& g : groups) {
        g.epoch = epoch;
        g.check = group_check(g.prob, g.group, epoch);
    }
    for (auto& P : probs) {
        P.rowbuf = rowbuf + ro;
        P.flags = flags + fo;
        ro += (size_t)(P.ngroups > 1 ? P.nslots : 0) * P.wpad * vpc;
        fo += P.ngroups;
    }
    // affine: every problem's subject-code rows (DPProblem::scode), built on the device
    // right after the descriptors land (aff_scode_kernel)
    int64_t scode_max_w = 0;
    if (aff) {
        size_t sb = 0;
        for (const auto& P : probs)
            if (P.h > 0 && P.w > 0) sb += (size_t)(4 * scode_len(P.w));
        uint8_t* sc = (uint8_t*)C.scode.get(std::max<size_t>(sb, 16));
        size_t so = 0;
        for (auto& P : probs) {
            P.scode = nullptr;
            if (P.h <= 0 || P.w <= 0) continue;
            P.scode = sc + so;
            so += (size_t)(4 * scode_len(P.w));
            scode_max_w = std::max<int64_t>(scode_max_w, P.w);
        }
    }
    // the digest covers every word of the final descriptor (pointers included)
    for (size_t i = 0; i < probs.size(); ++i) {
        probs[i].pad_ = 0;
        probs[i].magic = prob_magic(&probs[i], (int)i, epoch);
    }
    if (check_ptrs_enabled()) audit_probs(probs, aff);
    C.R = R;
    C.NW = NW;
    C.h_probs = probs;
    // staged in pinned memory (a truly asynchronous copy); the previous launch of this
    // context has completed (fill_finish / fill_collect), so the staging area is free.
    // (Coherent allocation + the kernel's descriptor digest guard against the round-start
    // fault's suspected mechanism, a stale cached staging line; that mechanism is an
    // unproven inference)
    char* pin = (char*)C.pin.get(64 + ub + 16);
    C.err_host = (uint32_t*)pin;
    memcpy(pin + 64, C.h_probs.data(), pb);
    memcpy(pin + 64 + pb, groups.data(), groups.size() * sizeof(GroupRef));
    if (xrun > 0) memcpy(pin + 64 + pb + groups.size() * sizeof(GroupRef), xoff, sizeof xoff);
    if (extra_bytes) memcpy(pin + 64 + eoff, extra, extra_bytes);
    if (groups.empty()) {
        if (ub) HIPCHECK(hipMemcpyAsync(meta + zb, pin + 64, ub, hipMemcpyHostToDevice, st));
        if (init_words) HIPCHECK(hipMemsetD32Async(init, init_value, (size_t)init_words, st));
        if (C.err_host) *C.err_host = 0u;   // (no copy targets it: the previous launch has completed)
        C.timed = true;
        HIPCHECK(hipEventRecord(C.ev0, st));
        HIPCHECK(hipEventRecord(C.ev1, st));
        HIPCHECK(hipEventRecord(C.ev2, st));
        return;
    }
    // counters and flags to 0, the caller's best cells to init_value, and the group ->
    // group hand-off rows to the sentinel the consumer polls the data against (-1 for
    // linear, 0x80808080 for affine): one launch
    // (the kernel also copies the descriptors in from the pinned staging area)
    HIPCHECK(anyseq_launch_fill_prep(ctr, (int)(32 + flag_words), init, init_words, init_value, rowbuf,
                                     rowbuf_ints * 4, aff ? 0x80808080u : 0xffffffffu, pin + 64, meta + zb, ub, st));
    if (aff) HIPCHECK(anyseq_launch_aff_scode(d_probs, (int)probs.size(), scode_max_w, st));
    FillParams fpl = fp;
    fpl.epoch = epoch;
    fpl.arows = aff ? R : 0;
    fpl.xq = xrun > 0 ? reinterpret_cast<const uint32_t*>(d_groups + groups.size()) : nullptr;
    fpl.prio = fill_prio(aff);
    fpl.throttle = g_tuning.thr;
    fpl.slack = g_tuning.slack;
    fpl.slack_io = g_tuning.slack_io;
    unsigned long long* dbg = nullptr;
    static DevBuf stamp_buf;
    if (getenv("ANYSEQ_STAMPS")) {
        // [header 16 | timeline 4/band | hand-off events 16/band | clock 4/band] x 4096 bands
        dbg = (unsigned long long*)stamp_buf.get(8 * (16 + 24 * 4096));
        HIPCHECK(hipMemsetAsync(dbg, 0, 8 * (16 + 24 * 4096), st));
        fpl.dbg = dbg;
    }
    C.stamps = dbg;
    C.pending = true;
    C.aff = aff;
    C.d_probs = d_probs;
    C.d_groups = d_groups;
    C.ngroups = (int)groups.size();
    C.grid = grid;
    C.fp = fpl;
    C.st = st;
}

void fill_launch(FillCtx& C) {
    if (!C.pending) return;   // nothing to compute (events already recorded)
    C.pending = false;
    uint32_t* ctr = (uint32_t*)C.probs.p;   // the launch block's counters (fill_prepare)
    C.timed = g_tuning.fill_events != 0;
    if (C.timed) HIPCHECK(hipEventRecord(C.ev0, C.st));
    if (C.aff)
        HIPCHECK(anyseq_launch_fill_affine(C.NW, C.d_probs, C.d_groups, C.ngroups, ctr, ctr + 1, &C.fp, C.grid, C.st));
    else
        HIPCHECK(anyseq_launch_fill(C.R, g_tuning.CH, C.NW, C.d_probs, C.d_groups, C.ngroups, ctr, ctr + 1, &C.fp,
                                    C.grid, C.st));
    if (C.timed) HIPCHECK(hipEventRecord(C.ev1, C.st));
    // ANYSEQ_CHECK_ROWS (host-built affine launches, round 5): every ring that is reused
    // within the launch (nslots < ngroups - 1: each reader puts the sentinel back) must
    // be all sentinel again afterwards, as the device-planned levels' rows;
    // 2 plants one stale word past w in the first such ring (the check's own test)
    C.rows_checked = false;
    const int check_rows = C.aff ? env_int("ANYSEQ_CHECK_ROWS", 0) : 0;
    if (check_rows) {
        uint32_t* w = (uint32_t*)C.rcheck.get(64);
        HIPCHECK(hipMemsetAsync(w, 0, 64, C.st));
        bool injected = false;
        for (size_t i = 0; i < C.h_probs.size(); ++i) {
            const DPProblem& P = C.h_probs[i];
            if (P.ngroups <= 1 || P.nslots >= P.ngroups - 1) continue;
            const bool inject = check_rows == 2 && !injected;
            injected |= inject;
            HIPCHECK(anyseq_launch_rows_check(P.rowbuf, (size_t)P.nslots * P.wpad * 2, 0x80808080u, C.d_probs + i, 1,
                                              w, inject, C.st));
            C.rows_checked = true;
        }
    }
    HIPCHECK(hipMemcpyAsync(C.err_host, ctr + 1, 4, hipMemcpyDeviceToHost, C.st));
    HIPCHECK(hipEventRecord(C.ev2, C.st));
}

void fill_async(Engine& E, FillCtx& C, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st,
                int grid_req, const void* extra, size_t extra_bytes, int32_t* init, int init_words,
                int32_t init_value) {
    fill_prepare(E, C, probs, fp, st, grid_req, extra, extra_bytes, init, init_words, init_value);
    fill_launch(C);
}

// Launch context for error messages: the stage label and the shapes of the launch's
// first problems, so a device fault names what was running.
thread_local const char* g_stage = "fill";
thread_local int g_stage_level = -1;

std::string fill_summary(const FillCtx& C) {
    char buf[160];
    snprintf(buf, sizeof buf, "%s level %d, %s fill of %zu problem(s), grid %d:", g_stage, g_stage_level,
             C.aff ? "affine" : "linear", C.h_probs.size(), C.grid);
    std::string s = buf;
    snprintf(buf, sizeof buf, " buffers: probs %p groups %p rowbuf %p+%zu flags %p ctr %p;", C.probs.p, C.groups.p,
             C.rowbuf.p, C.rowbuf.cap, C.flags.p, C.ctr.p);
    s += buf;
    for (size_t i = 0; i < C.h_probs.size() && i < 6; ++i) {
        const DPProblem& P = C.h_probs[i];
        snprintf(buf, sizeof buf, " [%dx%d q%+d@%d s%+d@%d bm%d am%d]", P.h, P.w, P.q_step, P.q_off, P.s_step,
                 P.s_off, P.bmode, P.amode);
        s += buf;
    }
    return s;
}

// The level's only synchronisation: poll the stream instead of a blocking wait, whose
// wake-up (tens of microseconds) would sit between every two Hirschberg levels.
hipError_t stream_wait_spin(hipStream_t st) {
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e == hipSuccess ? hipStreamSynchronize(st) : e;
    }
}

void stage_check(hipStream_t st, const char* what) {
    static const int on = env_int("ANYSEQ_DEBUG_SYNC", 0);
    if (!on) return;
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) fail("%s (%s level %d) failed: %s", what, g_stage, g_stage_level, hipGetErrorString(e));
}

void fill_finish(FillCtx& C) {
    {
        const hipError_t e = hipEventSynchronize(C.timed ? C.ev1 : C.ev2);
        if (e != hipSuccess) fail("fill failed: %s (%s)", hipGetErrorString(e), fill_summary(C).c_str());
    }
    fill_collect(C);
}

void fill_collect(FillCtx& C) {
    const int R = C.R, NW = C.NW;
    unsigned long long* dbg = C.stamps;
    {
        const hipError_t e = hipEventSynchronize(C.ev2);
        if (e != hipSuccess) {
            if (const char* path = getenv("ANYSEQ_FAIL_DUMP")) {   // every problem of the failed launch
                if (FILE* f = fopen(path, "w")) {
                    fprintf(f, "# %s\n", fill_summary(C).c_str());
                    for (const DPProblem& P : C.h_probs)
                        fprintf(f, "%d %d q=%p %d %d s=%p %d %d bm=%d am=%d out_row=%p out_col=%p out_col_e=%p best=%p "
                                   "rowbuf=%p nslots=%d wpad=%d nbands=%d ngroups=%d\n",
                                P.h, P.w, (const void*)P.q, P.q_off, P.q_step, (const void*)P.s, P.s_off, P.s_step,
                                P.bmode, P.amode, (void*)P.out_row, (void*)P.out_col, (void*)P.out_col_e,
                                (void*)P.best, (void*)P.rowbuf, P.nslots, P.wpad, P.nbands, P.ngroups);
                    fclose(f);
                }
            }
            fail("fill failed: %s (%s)", hipGetErrorString(e), fill_summary(C).c_str());
        }
    }
    float ms = 0.f;
    if (C.timed) HIPCHECK(hipEventElapsedTime(&ms, C.ev0, C.ev1));
    g_fill_ms += ms;
    g_fill_launches += 1;
    g_fill_cells += C.cells;
    if (C.aff && C.R >= 2) {
        g_fill_r2 += 1;
        g_fill_rmax = std::max(g_fill_rmax, C.R);
    }
    const uint32_t err = C.err_host ? *(volatile uint32_t*)C.err_host : 0u;
    if (C.rows_checked && !err) {
        uint32_t c[8];
        HIPCHECK(hipMemcpy(c, C.rcheck.p, sizeof c, hipMemcpyDeviceToHost));
        if (c[0])
            fail("hand-off row invariant broken after a host-built fill: %u non-sentinel word(s), the first in a ring "
                 "at word %u = ring slot %d, column %d (width %d)", c[0], c[1], (int)c[3], (int)c[4], (int)c[5]);
    }
    if (dbg) {
        unsigned long long h[16];
        HIPCHECK(hipMemcpy(h, dbg, sizeof h, hipMemcpyDeviceToHost));
        const double nb = (double)std::max(1ull, h[6]);
        fprintf(stderr,
                "anyseq stamps: %.3f ms R=%d NW=%d bands=%llu blocks=%llu | per band: total %.0f cyc, compute %.0f, "
                "wait_in %.0f, wait_s %.0f, wait_out %.0f | compute/block %.1f cyc | polls/block: subject %.2f "
                "in %.2f out %.2f\n",
                ms, R, NW, h[5], h[6], (double)h[0] / h[5], (double)h[1] / h[5], (double)h[2] / h[5],
                (double)h[3] / h[5], (double)h[4] / h[5], (double)h[1] / nb, h[10] / nb, h[11] / nb, h[12] / nb);
        if (const char* tl = getenv("ANYSEQ_TIMELINE")) {
            std::vector<unsigned long long> t(4 * 4096);
            HIPCHECK(hipMemcpy(t.data(), dbg + 16, t.size() * 8, hipMemcpyDeviceToHost));
            FILE* f = fopen(tl, "a");
            if (f) {
                fprintf(f, "# launch %.3f ms R=%d NW=%d\n", ms, R, NW);
                unsigned long long t0 = ~0ull;
                for (size_t i = 0; i < t.size(); i += 4) if (t[i] && t[i] < t0) t0 = t[i];
                // clock per band (round 5): shader cycles / 100 MHz ticks over the band's loop
                std::vector<unsigned long long> ck(4 * 4096);
                HIPCHECK(hipMemcpy(ck.data(), dbg + 16 + 20 * 4096, ck.size() * 8, hipMemcpyDeviceToHost));
                if (FILE* g = fopen((std::string(tl) + ".clk").c_str(), "a")) {
                    fprintf(g, "# launch: band shader_cycles ticks_100MHz\n");
                    for (size_t i = 0; i < ck.size(); i += 4)
                        if (ck[i] && ck[i + 2] > ck[i] && ck[i + 3] > ck[i + 1])
                            fprintf(g, "%zu %llu %llu\n", i / 4, ck[i + 2] - ck[i], ck[i + 3] - ck[i + 1]);
                    fclose(g);
                }
                for (size_t i = 0; i < t.size(); i += 4)
                    if (t[i]) fprintf(f, "%zu %.2f %.2f %.2f %.2f\n", i / 4, (t[i] - t0) / 100.0,
                                      t[i + 1] ? (t[i + 1] - t0) / 100.0 : -1.0, (t[i + 2] - t0) / 100.0,
                                      t[i + 3] && t[i + 3] >= t0 ? (t[i + 3] - t0) / 100.0
                                                                 : (t[i + 3] < (1ull << 32) ? -2.0 - (double)t[i + 3] : -1.0));
                fclose(f);
            }
            // hand-off events of one block per band (affine asm, diagnostic build): 16 per band
            std::vector<unsigned long long> ev(16 * 4096);
            HIPCHECK(hipMemcpy(ev.data(), dbg + 16 + 4 * 4096, ev.size() * 8, hipMemcpyDeviceToHost));
            if (FILE* g = fopen((std::string(tl) + ".ev").c_str(), "a")) {
                fprintf(g, "# launch\n");
                for (size_t i = 0; i < ev.size(); i += 16) {
                    if (!ev[i + 3] && !ev[i]) continue;
                    fprintf(g, "%zu", i / 16);
                    for (int k = 0; k < 15; ++k) fprintf(g, " %llu", ev[i + k]);
                    fprintf(g, "\n");
                }
                fclose(g);
            }
        }
    }
    if (err & ERR_BAD_DESC) fail("fill kernel read a corrupt problem descriptor (error %u; %s)", err, fill_summary(C).c_str());
    if (err) fail("fill kernel reported error %u (spin timeout)", err);
}

void run_fill(Engine& E, std::vector<DPProblem>& probs, const FillParams& fp, hipStream_t st) {
    fill_async(E, E.fc, probs, fp, st);
    fill_finish(E.fc);
}

// Alphabet codes of the pair: q ++ s recoded into E.codes (n + m
// bytes), the symbol count in device memory.  The affine fills compare codes; the
// kernel reads the count itself (no host synchronisation).
SeqCodes prepare_codes(Engine& E, const uint8_t* dq, int n, const uint8_t* ds, int m, hipStream_t st,
                       uint8_t* fill0, uint8_t* fill1, size_t fill_len) {
    const bool fresh = E.codemeta.p == nullptr;
    char* meta = (char*)E.codemeta.get(512);
    uint32_t* mask = (uint32_t*)meta;   // (+ the recode kernel's block counter at word 8)
    uint8_t* table = (uint8_t*)(meta + 64);
    int32_t* alpha = (int32_t*)(meta + 320);
    if (fresh) HIPCHECK(hipMemsetAsync(mask, 0, 64, st));   // (the recode kernel clears them after each use)
    uint8_t* out = (uint8_t*)E.codes.get((size_t)std::max(n, 0) + (size_t)std::max(m, 0) + 16);
    HIPCHECK(anyseq_launch_seq_codes(dq, std::max(n, 0), ds, std::max(m, 0), mask, table, alpha, out, fill0, fill1,
                                     fill_len, st));
    return SeqCodes{out, out + std::max(n, 0), alpha};
}

FillParams make_params(int kind, const anyseq_scoring& sc) {
    FillParams fp;
    memset(&fp, 0, sizeof fp);
    fp.kind = kind;
    fp.match = sc.match;
    fp.mismatch = sc.mismatch;
    fp.gap = sc.gap_extend;
    fp.gap_open = sc.gap_open;
    fp.gap_extend = sc.gap_extend;
    fp.affine = sc.gap_open != 0;
    fp.dbg = nullptr;
    // affine_asm bit 0: asm steady state, bit 1: scalar row stores (diagnostics)
    fp.pad = ((g_tuning.affasm & 1) ? 0 : 1) | (g_tuning.affasm & 2) | (g_tuning.affasm & 12) | (g_tuning.affasm & 96);
    // the LUT weights (G space sub - 2 ge, X space sub - ge) must fit int8
    const int nge = -sc.gap_extend;
    const int ws[4] = {sc.match + 2 * nge, sc.mismatch + 2 * nge, sc.match + nge, sc.mismatch + nge};
    fp.lut_ok = g_tuning.afflut ? 1 : 0;
    for (int w : ws)
        if (w < -128 || w > 127) fp.lut_ok = 0;
    // bit 4: a NORMAL-border best of every cell may run the virtual prologue (its column
    // -1 border cells, at most go + ge, never exceed cell (0,0) >= min(match, mismatch))
    if (g_tuning.virtbest && std::min(sc.match, sc.mismatch) >= sc.gap_open + sc.gap_extend) fp.pad |= 16;
    // bit 7: gap open 0 through the affine loop, not the linear one (A/B)
    if (!g_tuning.linloop) fp.pad |= 128;
    // bit 8: the affine I/O wave on the first hardware wave (A/B)
    if (g_tuning.iofirst) fp.pad |= 256;
    // bit 9: a zero-open left border through the C++ blocks, not the forcing prologue (A/B)
    if (!g_tuning.forcelb) fp.pad |= 512;
    fp.alpha = nullptr;
    fp.io_stage = g_tuning.io_stage;
    fp.io_skew = g_tuning.io_skew;
    fp.io_poll2 = g_tuning.io_poll2;
    fp.io_fwd = g_tuning.io_fwd;
    return fp;
}

void set_aff_kind(DPProblem& P, int kind) {
    P.bmode = kind == KIND_GLOBAL ? BM_NORMAL : kind == KIND_SEMIGLOBAL ? BM_FREE_SEMI_OPEN : BM_FREE_LOCAL;
    P.amode = kind == KIND_LOCAL ? (AM_CLAMP | AM_BEST_ALL) : 0;
}

// The kernels keep every DP value in int32 with -2^29 as "minus infinity", and the
// G-space shift (r + c + 2)·|gap| grows with the matrix: reject problems whose values
// could come near it (a silently wrong score otherwise).
void check_value_range(const anyseq_scoring& sc, int64_t n, int64_t m) {
    const int64_t per = std::llabs(sc.match) + std::llabs(sc.mismatch) + std::llabs(sc.gap_open) +
                        2 * std::llabs(sc.gap_extend);
    if ((n + m + 2) * per >= (int64_t(1) << 28))
        fail("%lld x %lld with these scores (sum of |match|, |mismatch|, |gap open|, 2|gap extend| = %lld) can "
             "exceed the kernels' int32 value range: (n + m + 2) x that sum must stay below 2^28",
             (long long)n, (long long)m, (long long)per);
}

void check_scoring(int kind, const anyseq_scoring& sc) {
    if (kind < 0 || kind > 2) fail("invalid alignment kind %d", kind);
    if (sc.gap_extend >= 0) fail("gap_extend must be negative (got %d)", sc.gap_extend);
    if (sc.gap_open > 0) fail("gap_open must be <= 0 (got %d)", sc.gap_open);
    // |scores| stay far from the kernels' -2^29 "minus infinity" and int32 range
    const long long mx = std::max({std::llabs(sc.match), std::llabs(sc.mismatch), std::llabs(sc.gap_open),
                                   std::llabs(sc.gap_extend)});
    if (mx > 1024) fail("scoring parameters must be within [-1024, 1024]");
}

namespace {

// Score of an empty matrix (reference semantics with benchmark restored).
int64_t empty_score(int kind, int n, int m, const anyseq_scoring& sc) {
    if (kind == KIND_GLOBAL) {
        const int len = n > 0 ? n : m;
        if (len <= 0) return 0;
        return (int64_t)sc.gap_open + (int64_t)len * sc.gap_extend;  // init(n-1) or init(m-1)
    }
    if (kind == KIND_SEMIGLOBAL) return 0;
    return SCORE_MIN_VALUE;  // local: no slot is ever written
}

// Fill-based score on device-resident sequences (align.impala:218-235).
// Matrices with enough rows run as two fronts (top half forward, bottom half on
// reversed sequences) in ONE launch and are combined by a row split
// (front_combine_kernel): the pipeline depth of the band wavefront halves.
int64_t score_dev_affine(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n, const uint8_t* ds,
                         int m, hipStream_t st);

int64_t score_dev(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n, const uint8_t* ds, int m,
                  hipStream_t st) {
    if (n <= 0 || m <= 0) return empty_score(kind, n, m, sc);
    // a linear score runs through the affine fill with gap open 0 (round 5):
    // its linear loop on the affine kernel's code rows, lean blocks and half-chunk hand-off
    // (semiglobal with its zero-open left border forced at column -1, the `pro` prologue)
    const bool via_aff = g_tuning.linaff != 0;
    if (sc.gap_open != 0 || via_aff) return score_dev_affine(E, kind, sc, dq, n, ds, m, st);
    const FillParams fp = make_params(kind, sc);
    const int wpad = (m + 63) & ~63;
    int32_t* res = (int32_t*)E.fc.ctr.get(128) + 4;
    HIPCHECK(hipMemsetAsync(res, kind == KIND_LOCAL ? 0 : 0x80, 4, st));  // local: 0; else ~INT_MIN
    const bool two_fronts = g_tuning.fronts > 1 && n >= 2 * 64 * rows_per_lane() * waves_per_group();
    std::vector<DPProblem> probs;
    DPProblem P;
    memset(&P, 0, sizeof P);
    P.q = dq;
    P.s = ds;
    P.q_step = 1;
    P.s_step = 1;
    P.w = m;
    if (!two_fronts) {
        P.h = n;
        if (kind != KIND_LOCAL) P.out_col = (int32_t*)E.outcol.get((size_t)n * 4);
        if (kind == KIND_SEMIGLOBAL) P.out_row = (int32_t*)E.outrow.get((size_t)wpad * 4);
        if (kind == KIND_LOCAL) P.best = res;
        probs.push_back(P);
        run_fill(E, probs, fp, st);
        int32_t v = 0;
        if (kind == KIND_GLOBAL) {
            HIPCHECK(hipMemcpyAsync(&v, P.out_col + (n - 1), 4, hipMemcpyDeviceToHost, st));
        } else if (kind == KIND_SEMIGLOBAL) {
            HIPCHECK(hipMemsetAsync(res, 0, 4, st));
            HIPCHECK(anyseq_launch_semiglobal_reduce(P.out_row, m, P.out_col, n, -sc.gap_extend, res, st));
            HIPCHECK(hipMemcpyAsync(&v, res, 4, hipMemcpyDeviceToHost, st));
        } else {
            HIPCHECK(hipMemcpyAsync(&v, res, 4, hipMemcpyDeviceToHost, st));
        }
        HIPCHECK(hipStreamSynchronize(st));
        return v;
    }
    const int h1 = n / 2, h2 = n - h1;
    int32_t* rows = (int32_t*)E.outrow.get((size_t)2 * wpad * 4);
    int32_t* cols = kind == KIND_SEMIGLOBAL ? (int32_t*)E.outcol.get((size_t)n * 4) : nullptr;
    // top front: rows [0, h1) forward
    P.h = h1;
    P.out_row = rows;
    P.out_col = cols;
    if (kind == KIND_LOCAL) P.best = res;
    probs.push_back(P);
    // bottom front: rows [h1, n) with query and subject reversed
    P.q_off = n - 1;
    P.q_step = -1;
    P.s_off = m - 1;
    P.s_step = -1;
    P.h = h2;
    P.out_row = rows + wpad;
    P.out_col = cols ? cols + h1 : nullptr;
    probs.push_back(P);
    run_fill(E, probs, fp, st);
    HIPCHECK(anyseq_launch_front_combine(kind, rows, h1, rows + wpad, h2, m, sc.gap_extend, cols,
                                         cols ? cols + h1 : nullptr, res, st));
    int32_t v = 0;
    HIPCHECK(hipMemcpyAsync(&v, res, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    return v;
}

// Affine (Gotoh) score: the same one- or two-front scheme as score_dev over
// fill_affine_kernel; rows are (G, F) pairs, so the combine also joins a vertical
// gap that crosses the split row (aff_reduce_kernel).
int64_t score_dev_affine(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq_raw, int n,
                         const uint8_t* ds_raw, int m, hipStream_t st) {
    FillParams fp = make_params(kind, sc);
    fp.affine = 1;   // (also a linear score: gap open 0)
    const SeqCodes cd = prepare_codes(E, dq_raw, n, ds_raw, m, st);
    fp.alpha = cd.alpha;
    const uint8_t *dq = cd.q, *ds = cd.s;
    const int wpad = (m + 63) & ~63;
    const int NW = aff_waves_per_group();
    int32_t* res = (int32_t*)E.fc.ctr.get(128) + 4;
    HIPCHECK(hipMemsetAsync(res, kind == KIND_LOCAL ? 0 : 0x80, 4, st));
    const bool two = g_tuning.fronts > 1 && n >= 2 * 64 * NW;
    std::vector<DPProblem> probs;
    DPProblem P;
    memset(&P, 0, sizeof P);
    P.q = dq;
    P.s = ds;
    P.q_step = 1;
    P.s_step = 1;
    P.w = m;
    set_aff_kind(P, kind);
    const int h1 = two ? n / 2 : n, h2 = n - h1;
    int32_t* rows = (int32_t*)E.outrow.get((size_t)2 * 2 * wpad * 4);
    int32_t* cols = kind != KIND_LOCAL ? (int32_t*)E.outcol.get((size_t)n * 4) : nullptr;
    P.h = h1;
    P.out_row = (kind != KIND_GLOBAL || two) ? rows : nullptr;
    P.out_col = cols;
    if (kind == KIND_LOCAL) P.best = res;
    probs.push_back(P);
    if (two) {
        P.q_off = n - 1;
        P.q_step = -1;
        P.s_off = m - 1;
        P.s_step = -1;
        P.h = h2;
        P.out_row = rows + 2 * wpad;
        P.out_col = cols ? cols + h1 : nullptr;
        probs.push_back(P);
    }
    run_fill(E, probs, fp, st);
    int32_t v = 0;
    if (!two && kind == KIND_GLOBAL) {
        HIPCHECK(hipMemcpyAsync(&v, cols + (n - 1), 4, hipMemcpyDeviceToHost, st));
    } else {
        if (two || kind == KIND_SEMIGLOBAL)
            HIPCHECK(anyseq_launch_aff_reduce(kind, two ? 1 : 0, rows, h1, rows + 2 * wpad, h2, m, sc.gap_open,
                                              sc.gap_extend, cols, cols ? cols + h1 : nullptr, res, st));
        HIPCHECK(hipMemcpyAsync(&v, res, 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    return v;
}

int64_t score_host(int kind, const anyseq_scoring& sc, const char* q, int n, const char* s, int m) {
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    if (n <= 0 || m <= 0) return empty_score(kind, n, m, sc);
    uint8_t* dq = (uint8_t*)E.q.get((size_t)n);
    uint8_t* ds = (uint8_t*)E.s.get((size_t)m);
    HIPCHECK(hipMemcpyAsync(dq, q, (size_t)n, hipMemcpyHostToDevice, E.stream));
    HIPCHECK(hipMemcpyAsync(ds, s, (size_t)m, hipMemcpyHostToDevice, E.stream));
    return score_dev(E, kind, sc, dq, n, ds, m, E.stream);
}

// ------------------------------------------------------------- construct --
int next_pow_2(int i) {  // utils.impala:19-28
    if (i == 0) return 0;
    int n = i - 1, r = 1;
    while (n > 0) {
        n >>= 1;
        r <<= 1;
    }
    return r;
}

struct HostSplits {  // traceback_lintime.impala:1-42 (logical index -1 at storage 0)
    std::vector<int32_t> v;
    int nb = 0, bpp = 0;
    int32_t at(int idx) const {
        const int32_t x = v[idx + 1];
        if (x == SPLIT_UNSET) fail("internal: split %d read before being set", idx);
        return x;
    }
    void dims(int part, int& off, int& h) const {
        const int start = part * bpp - 1;
        const int end = std::min((part + 1) * bpp - 1, nb - 1);
        off = at(start);
        h = at(end) - off;
    }
};

// Linear-space construct (traceback_lintime, align.impala:237-311) on the GPU, on
// device-resident sequences, into device strings d_alq/d_als of n+m bytes (the
// sparse i+j+1 layout, blanks first).  Enqueued on st; returns after the last
// kernel has been enqueued (the level loop syncs on the split vector).
void construct_dev(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n, const uint8_t* ds, int m,
                   uint8_t* d_alq, uint8_t* d_als, hipStream_t st) {
    const size_t L = (size_t)n + (size_t)m;
    if (L == 0) return;
    HIPCHECK(hipMemsetAsync(d_alq, ' ', L, st));
    HIPCHECK(hipMemsetAsync(d_als, ' ', L, st));
    if (m <= 0) return;  // no 128-column block: the reference writes only blanks
    const FillParams fp = make_params(kind, sc);

    HostSplits sp;
    sp.nb = (m + MIN_PART_WIDTH_HB - 1) / MIN_PART_WIDTH_HB;
    sp.v.assign((size_t)sp.nb + 1, SPLIT_UNSET);
    int pw = next_pow_2(m);
    sp.bpp = pw / MIN_PART_WIDTH_HB;
    sp.v[0] = 0;
    sp.v[sp.nb] = n;
    int32_t* d_spl = (int32_t*)E.spl.get(sp.v.size() * 4);
    upload_pinned(E.pin_down, d_spl, sp.v.data(), sp.v.size() * 4, st);
    int32_t* dL = (int32_t*)E.L.get((size_t)std::max(n, 1) * 4);
    int32_t* dR = (int32_t*)E.R.get((size_t)std::max(n, 1) * 4);

    while (pw > MIN_PART_WIDTH_HB) {  // traceback_lintime_step, align.impala:273-290
        const int half = pw / 2;
        const int parts = (m + half - 1) / pw;
        std::vector<DPProblem> probs;
        std::vector<PartInfo> pinfo;
        for (int p = 0; p < parts; ++p) {
            int hoi, hh;
            sp.dims(p, hoi, hh);
            const int hoj_l = p * pw, hoj_r = p * pw + half;
            const int hw = std::min(half, m - hoj_r);
            PartInfo pi;
            pi.off = hoi;
            pi.len = hh;
            pi.rhw = hw;
            pi.split_index = p * sp.bpp + sp.bpp / 2 - 1;
            pinfo.push_back(pi);
            if (hh <= 0) continue;
            DPProblem P;
            memset(&P, 0, sizeof P);
            P.q = dq;
            P.s = ds;
            P.h = hh;
            // left half: forward
            P.q_off = hoi;
            P.q_step = 1;
            P.s_off = hoj_l;
            P.s_step = 1;
            P.w = half;
            P.out_col = dL + hoi;
            probs.push_back(P);
            // right half: query rows and subject columns reversed (get_sequence_acc_half)
            P.q_off = hoi + hh - 1;
            P.q_step = -1;
            P.s_off = hoj_r + hw - 1;
            P.s_step = -1;
            P.w = hw;
            P.out_col = dR + hoi;
            probs.push_back(P);
        }
        run_fill(E, probs, fp, st);
        // hb_sum (traceback_lintime.impala:44-135), CPU BLOCK_WIDTH candidate order
        const int bwh = std::min(CPU_BLOCK_WIDTH, half * 2);
        const int bpp_h = half * 2 / bwh;
        PartInfo* d_parts = (PartInfo*)E.parts.get(pinfo.size() * sizeof(PartInfo));
        upload_pinned(E.pin_up, d_parts, pinfo.data(), pinfo.size() * sizeof(PartInfo), st);
        int32_t* d_bmax = (int32_t*)E.bmax.get((size_t)parts * bpp_h * 4);
        int32_t* d_bind = (int32_t*)E.bind.get((size_t)parts * bpp_h * 4);
        HIPCHECK(anyseq_launch_hb_sum(d_parts, parts, bpp_h, half, dL, dR, kind, sc.gap_extend, d_bmax, d_bind, d_spl,
                                      st));
        HIPCHECK(hipMemcpyAsync(sp.v.data(), d_spl, sp.v.size() * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        pw /= 2;
        sp.bpp /= 2;
    }

    // final level: blockwise predecessors + per-block walk (align.impala:292-311)
    std::vector<BlockInfo>& blocks = E.host_blocks;   // outlives the async upload
    blocks.assign((size_t)sp.nb, BlockInfo{});
    int64_t pred_bytes = 0;
    for (int b = 0; b < sp.nb; ++b) {
        BlockInfo& bi = blocks[b];
        sp.dims(b, bi.oi, bi.h);
        bi.oj = b * MIN_PART_WIDTH_HB;
        bi.w = std::min(MIN_PART_WIDTH_HB, m - bi.oj);
        bi.pred_base = pred_bytes;
        if (bi.h > 0) pred_bytes += (int64_t)(bi.h + 127) * 128;
    }
    BlockInfo* d_blocks = (BlockInfo*)E.blocks.get(blocks.size() * sizeof(BlockInfo));
    upload_pinned(E.pin_blocks, d_blocks, blocks.data(), blocks.size() * sizeof(BlockInfo), st);
    uint8_t* d_pred = (uint8_t*)E.pred.get((size_t)std::max<int64_t>(pred_bytes, 16));
    HIPCHECK(anyseq_launch_pred(d_blocks, sp.nb, dq, ds, d_pred, &fp, st));
    HIPCHECK(anyseq_launch_walk(d_blocks, sp.nb, dq, ds, d_pred, kind, d_alq, d_als, st));
}

void construct_host(int kind, const anyseq_scoring& sc, const char* q, int n, const char* s, int m, char* alq,
                    char* als) {
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    hipStream_t st = E.stream;
    const size_t L = (size_t)n + (size_t)m;
    if (L == 0) return;
    uint8_t* dq = (uint8_t*)E.q.get((size_t)std::max(n, 1));
    uint8_t* ds = (uint8_t*)E.s.get((size_t)std::max(m, 1));
    if (n > 0) HIPCHECK(hipMemcpyAsync(dq, q, (size_t)n, hipMemcpyHostToDevice, st));
    if (m > 0) HIPCHECK(hipMemcpyAsync(ds, s, (size_t)m, hipMemcpyHostToDevice, st));
    uint8_t* d_alq = (uint8_t*)E.alq.get(L);
    uint8_t* d_als = (uint8_t*)E.als.get(L);
    construct_dev(E, kind, sc, dq, n, ds, m, d_alq, d_als, st);
    HIPCHECK(hipMemcpyAsync(alq, d_alq, L, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(als, d_als, L, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
}

// ------------------------------------------------------ affine construct --
// Build-defined linear-space affine alignment (semantics =
// oracle_affine_construct): ONE column-split Hirschberg over the whole matrix.
// Every split boundary carries a row and a type (T_H / T_E crossings, T_BEFORE:
// the path ended left of it, T_AFTER: it starts right of it), so local and
// semiglobal ends are found by the levels themselves (a part's start or end is
// free until a level pins it) instead of by separate end / start searches.  Each
// level is ONE fill launch over every part's two halves, whatever their border
// modes (fill_affine_kernel reads them per problem), then one join launch.
DPProblem aff_problem(const uint8_t* dq, int q_off, int q_step, int h, const uint8_t* ds, int s_off, int s_step, int w) {
    DPProblem P;
    memset(&P, 0, sizeof P);
    P.q = dq;
    P.s = ds;
    P.q_off = q_off;
    P.q_step = q_step;
    P.s_off = s_off;
    P.s_step = s_step;
    P.h = h;
    P.w = w;
    return P;
}

// Border mode of a free start / end (oracle free_bm): local clamps everywhere,
// semiglobal opens the side border only at the matrix edge.
int free_bm(int kind, bool at_edge) { return aff_free_bm(kind, at_edge); }

// The same borders with query and subject swapped (a transposed half).
int transposed_bm(int bm) { return aff_transposed_bm(bm); }

using RowToColJob = RowToCol;   // anyseq_internal.h

// One Hirschberg half: rows qoff + qstep*r (r < h) of the query against columns
// soff + sstep*c (c < w) of the subject, border mode bm, kind bits amode; its last
// column goes to H / E (h each).  A half taller than wide runs TRANSPOSED (subject
// bytes as rows): its band chain then follows the shorter side (h/64 bands of lag
// + w steps becomes w/64 + h), and its bottom row (G, F-down) is the last column
// (H, E-right) -- the join decisions are unchanged (aff_row_to_col_kernel).  The
// values are those of the untransposed DP, so parity is unaffected.
void add_half(std::vector<DPProblem>& probs, std::vector<RowToColJob>& jobs, int32_t*& rowpool, const uint8_t* dq,
              int qoff, int qstep, int h, const uint8_t* ds, int soff, int sstep, int w, int bm, int amode,
              int32_t* best, int32_t* H, int32_t* E) {
    if (g_tuning.afft && h > w) {
        DPProblem P = aff_problem(ds, soff, sstep, w, dq, qoff, qstep, h);
        P.bmode = transposed_bm(bm);
        // the original's last row is the transposed problem's last column
        P.amode = (amode & AM_CLAMP) | ((amode & AM_BEST_LASTCOL) == AM_BEST_LAST ? AM_BEST_LASTCOL
                                                                                   : (amode & AM_BEST_LASTCOL));
        P.best = best;
        P.out_row = rowpool;
        rowpool += (size_t)((h + 63) & ~63) * 2;
        probs.push_back(P);
        jobs.push_back(RowToColJob{P.out_row, H, E, h, w - 1, P.amode != 0 ? 1 : 0, 0});
        return;
    }
    DPProblem P = aff_problem(dq, qoff, qstep, h, ds, soff, sstep, w);
    P.bmode = bm;
    P.amode = amode;
    P.best = best;
    P.out_col = H;
    P.out_col_e = E;
    probs.push_back(P);
}

// Hirschberg levels + final blocks into d_alq / d_als (n+m bytes, already blank).
// Returns the level-1 join value (the optimal score) or INT64_MIN if m <= 128
// (no level).  kind != global with a level-1 value <= 0 stops there (empty
// alignment).
//
// Sharded: the half fills of every level and the final blocks are
// dealt round-robin to `world` ranks.  A rank fills only its halves into ZEROED level
// columns, the columns are SUM-reduced and the free-end best cells MAX-reduced over the
// ranks (rows a rank did not fill are 0), so every rank joins every part; a rank walks
// only its final blocks into ' '-filled strings, which merge by a byte-wise MAX.  The
// RCCL path holds one rank view per process and reduces with RCCL; local mode holds
// all `world` views in this process (each with its own columns, best cells and
// strings) and reduces them with device kernels -- the same data flow on one GPU.
// `clear`: the strings' ' ' prefill (n+m bytes each) is this call's job (it rides in the
// alphabet-coding launch: one launch fewer in front of level 1's fill)
int64_t aff_construct_hb(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n, const uint8_t* ds,
                         int m, uint8_t* d_alq, uint8_t* d_als, hipStream_t st, const ConstructShards* shards,
                         bool clear) {
    FillParams fp = make_params(KIND_GLOBAL, sc);
    // the affine fill for every level, gap open 0 included (its linear loop): make_params
    // marks open 0 as a linear fill, which would send the host-built levels' affine problems
    // to fill_kernel (round 6: wrong linear true constructs there, tools/lin_host_probe.py)
    fp.affine = 1;
    hstamp("enter");
    // the level fills compare alphabet codes; the final blocks emit the raw bytes (the
    // strings' prefill rides in the coding launch)
    const SeqCodes cd = prepare_codes(E, dq, n, ds, m, st, clear ? d_alq : nullptr, clear ? d_als : nullptr,
                                      (size_t)n + (size_t)m);
    hstamp("codes");
    fp.alpha = cd.alpha;
    const uint8_t *cq = cd.q, *cs = cd.s;
    const int world = shards ? shards->world : 1;
    const bool sharded = world > 1;
    const bool emulate = shards && shards->local && sharded;   // all ranks' views in this process
    const int nviews = emulate ? world : 1;
    const int my_rank = shards && !shards->local ? shards->rank : 0;
    auto owner = [&](int idx) { return idx % world; };
    auto view_rank = [&](int v) { return emulate ? v : my_rank; };
    const bool local = kind == KIND_LOCAL;
    HostSplits sp;
    sp.nb = (m + MIN_PART_WIDTH_HB - 1) / MIN_PART_WIDTH_HB;
    sp.v.assign((size_t)sp.nb + 1, SPLIT_UNSET);
    std::vector<int32_t> typ((size_t)sp.nb + 1, T_H);
    // levels: P = 1, 2, 4, .. < nb parts, each split at its middle block (aff_part_geo)
    sp.bpp = 0;
    // the widest half of the level with P parts (ceil(ceil(nb / P) / 2) blocks)
    auto level_half = [&](int P) { return MIN_PART_WIDTH_HB * (((sp.nb + P - 1) / P + 1) / 2); };
    sp.v[0] = 0;
    sp.v[sp.nb] = n;
    if (kind != KIND_GLOBAL) {
        typ[0] = T_AFTER;
        typ[sp.nb] = T_BEFORE;
    }
    // one device status block per construct: splits | types | level-1 score, downloaded
    // in one copy per level into pinned memory (the level's only synchronisation)
    const size_t nsv = sp.v.size();
    // (+ the device-planned levels' tail words at tail_off, downloaded in the same copy)
    const size_t tail_off = (2 * nsv + 4 + 3) & ~(size_t)3, tail_cap = 32 * 17 + 1 + 3;
    int32_t* d_status = (int32_t*)E.status.get((tail_off + tail_cap) * 4);
    int32_t* d_spl = d_status;
    int32_t* d_typ = d_status + nsv;
    int32_t* d_score = d_status + 2 * nsv;
    int32_t* h_status = (int32_t*)E.pin_down.get((tail_off + tail_cap) * 4);
    // the initial split table: uploaded by the host-built levels below; the device-planned
    // levels set its two ends in level 1's plan launch (the rest is written level by level)
    auto upload_status = [&]() {
        memcpy(h_status, sp.v.data(), nsv * 4);
        memcpy(h_status + nsv, typ.data(), nsv * 4);
        HIPCHECK(hipMemcpyAsync(d_status, h_status, 2 * nsv * 4, hipMemcpyHostToDevice, st));
    };
    // level columns: view v's LH / LE / RH / RE at + v * nn
    const size_t nn = (size_t)std::max(n, 1);
    int32_t *LH0 = (int32_t*)E.L.get(nviews * nn * 4), *LE0 = (int32_t*)E.LE.get(nviews * nn * 4);
    int32_t *RH0 = (int32_t*)E.R.get(nviews * nn * 4), *RE0 = (int32_t*)E.RE.get(nviews * nn * 4);
    // emulated ranks' strings (view 0 writes the output itself)
    const size_t L = (size_t)n + (size_t)m;
    uint8_t* vstr = nullptr;
    if (emulate) {
        vstr = (uint8_t*)E.vstr.get((size_t)(nviews - 1) * 2 * std::max<size_t>(L, 1));
        HIPCHECK(hipMemsetAsync(vstr, ' ', (size_t)(nviews - 1) * 2 * L, st));
    }
    auto view_str = [&](int v, uint8_t*& aq, uint8_t*& as) {
        if (v == 0) {
            aq = d_alq;
            as = d_als;
        } else {
            aq = vstr + (size_t)(v - 1) * 2 * L;
            as = aq + L;
        }
    };
    // (the host-built levels rewrite h_status in their first download: they synchronise
    // with its upload first, below; the device-planned levels download it at the end)
    auto tp = [&](int idx) { return typ[idx + 1]; };
    int64_t score = INT64_MIN;
    bool level1 = true;
    struct StageScope {
        StageScope() { g_stage = "affine construct", g_stage_level = 0; }
        ~StageScope() { g_stage = "fill", g_stage_level = -1; }
    } stage_scope;
    static const int level_timing = env_int("ANYSEQ_LEVEL_TIMING", 0);   // diagnostics: host phases per level
    auto now_us = [] {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    double t_wake = now_us();
    // the device plan sizes the hand-off rows for the worst split of every level; past a
    // few GB (genome-length halves) the host-built levels keep the exact sizes
    // a planned level's waves per workgroup, from its nominal shape (parts of n/parts rows;
    // halves of `half` columns, transposed when taller than wide)
    auto level_nw = [&](int half, int parts) {
        const int64_t rows = std::max<int64_t>(1, (int64_t)n / std::max(parts, 1));
        const bool tr = g_tuning.afft && rows > half;
        const int64_t h = tr ? half : rows, w = tr ? rows : half;
        const int64_t chain = w + h * 128 / 100, work = 2 * (int64_t)parts * ((h + 63) / 64) * (w + 64);
        const int g0 = g_tuning.grida > 0 ? g_tuning.grida : E.num_cus;
        return aff_waves_for(chain, work, g0);
    };
    auto plan_rowbuf_bytes = [&]() {
        size_t mx = 0;
        for (int parts = 1; parts < sp.nb; parts *= 2) {
            const int h2 = level_half(parts);
            const int NWa = level_nw(h2, parts);
            const int maxh = g_tuning.afft ? h2 : std::max(h2, n);
            const int bound = std::max(1, ((maxh + 63) / 64 + NWa - 1) / NWa);
            const int grid = std::max(1, std::min(g_tuning.grida > 0 ? g_tuning.grida : E.num_cus, 2 * parts * bound));
            const int want = std::max(g_tuning.ring_slots > 0 ? g_tuning.ring_slots : 4 * grid + 4, 2 * grid + 2);
            const int64_t cols = std::min<int64_t>((int64_t)n + (int64_t)parts * h2, (int64_t)parts * std::max(n, h2)) +
                                 64 * (int64_t)parts;
            mx = std::max(mx, (size_t)std::min(bound - 1, want) * 2 * (size_t)cols * 2 * 4);
        }
        return mx;
    };
    bool planned = false, dev_final = false;
    const bool plan_ok = g_tuning.devplan && plan_rowbuf_bytes() <= ((size_t)8 << 30) && n < 8192 * 4096 - 1;
    // Device-planned levels: every level from the one with P0 parts on is
    // enqueued up front -- plan (aff_level_plan_kernel builds the level from the splits on
    // the device), prep, fill, row-to-column, join -- and the splits come back in ONE
    // download after the last level, instead of a download and a host rebuild per level.
    // Sharded (round 5): the levels the host loop does not column-block (the halves dealt
    // round-robin) go the same way, each rank's fill running only its own halves (emulated
    // ranks: every half, into its owner's view), the level's columns, transposed bottom
    // rows and best cells reduced over the ranks between the fill and the tail.
    auto run_planned = [&](int P0) {
        const int lev0 = [&] { int k = 0; while ((1 << k) < P0) ++k; return k; }();   // levels before P0
        struct Lev {
            int half, parts, bound, nh, slots, grid, want, nw;   // half: the level's widest half
            size_t rowbuf_bytes;
        };
        std::vector<Lev> lv;
        size_t max_meta = 0, max_rowbuf = 0, max_rowpool = 0, max_joinbuf = 0;
        int max_parts = 1;
        const int nsl = std::max(1, (n + 1 + 4095) / 4096);   // join slices of the longest possible part
        for (int P = P0; P < sp.nb; P *= 2) {
            Lev L;
            L.half = level_half(P);
            L.parts = P;
            // a half runs at most `half` rows (taller ones transposed), else up to n
            const int maxh = g_tuning.afft ? L.half : std::max(L.half, n);
            L.nw = level_nw(L.half, L.parts);
            const int NWa = L.nw;
            L.bound = std::max(1, ((maxh + 63) / 64 + NWa - 1) / NWa);
            L.nh = 2 * L.parts;
            L.slots = L.nh * L.bound;
            const int grid0 = g_tuning.grida > 0 ? g_tuning.grida : E.num_cus;
            L.grid = std::max(1, std::min(grid0, L.slots));
            const int min_slots = 2 * L.grid + 2;
            L.want = std::max(g_tuning.ring_slots > 0 ? g_tuning.ring_slots : 2 * min_slots, min_slots);
            // hand-off rows: a half's pitch is max(len, width) rounded up, Sum max(len_p, half)
            // <= min(n + parts*half, parts*max(n, half))
            const int64_t cols = std::min<int64_t>((int64_t)n + (int64_t)L.parts * L.half,
                                                   (int64_t)L.parts * std::max(n, L.half)) +
                                 64 * (int64_t)L.parts;
            L.rowbuf_bytes = (size_t)std::min(L.bound - 1, L.want) * 2 * (size_t)cols * 2 * 4;
            const size_t meta = (((32 + (size_t)L.slots) * 4 + 255) & ~(size_t)255) +
                                (size_t)L.nh * sizeof(DPProblem) + (size_t)L.slots * sizeof(GroupRef) +
                                (kXcds + 1) * 4;   // (+ the XCD offsets of FillParams::xq)
            max_meta = std::max(max_meta, meta);
            max_rowbuf = std::max(max_rowbuf, L.rowbuf_bytes);
            max_rowpool = std::max(max_rowpool, (size_t)2 * ((size_t)n + 64 * (size_t)L.parts) * 2 * 4);
            // (the tail's join: at most ~256 workgroups, nslices = min(nsl, 256 / parts) per part)
            max_joinbuf = std::max(max_joinbuf, (size_t)L.parts * std::max(1, std::min(nsl, (256 + L.parts - 1) / L.parts)) * 8);
            max_parts = std::max(max_parts, L.parts);
            lv.push_back(L);
        }
        const int nlev = (int)lv.size();
        // every allocation before the first enqueue (growth may synchronise the device)
        char* meta = (char*)E.pl_meta.get(std::max<size_t>(max_meta, 256));
        // hand-off rows: every planned fill puts the sentinel back after each read, so the
        // buffer stays all sentinel between launches; it is filled once per allocation
        // (and again after a failed call)
        void* const rb_prev = E.pl_rowbuf.p;
        int32_t* rowbuf = (int32_t*)E.pl_rowbuf.get(std::max<size_t>(max_rowbuf, 16));
        if (rowbuf != rb_prev || E.pl_dirty)
            HIPCHECK(hipMemsetD32Async(rowbuf, 0x80808080, E.pl_rowbuf.cap / 4, st));
        E.pl_dirty = true;   // until this call has checked its error words
        int32_t* rowpool = (int32_t*)E.outrow.get(std::max<size_t>(max_rowpool, 16));
        // subject-code rows of a level's halves: sum of 4 scode_len(w) <= 4 (2n + m + 192 halves)
        // (a half's w is its part's rows or its width; the parts' rows and widths are disjoint)
        const size_t scode_cap = 4 * ((size_t)2 * n + (size_t)m + 192 * (size_t)(2 * max_parts)) + 16;
        uint8_t* scode_rows = (uint8_t*)E.pl_scode.get(scode_cap);
        PartInfo* d_parts = (PartInfo*)E.pl_parts.get((size_t)max_parts * sizeof(PartInfo));
        RowToCol* d_jobs = (RowToCol*)E.pl_jobs.get((size_t)2 * max_parts * sizeof(RowToCol));
        // best cells: 2 per part and view (view v at + v * pstride)
        const int64_t pstride = 2 * (int64_t)max_parts;
        int32_t* pbest = (int32_t*)E.bmax.get((size_t)nviews * pstride * 4);
        const int ninit_best = (int)(nviews * pstride);
        void* partial = E.joinbuf.get(std::max<size_t>(max_joinbuf, 16));
        // per level: header (8 words: sentinel uint4s, bound check, cells (u64), tail counter)
        // then one error word per level
        // + with ANYSEQ_CHECK_ROWS, 8 words per level of the hand-off row check
        const int check_rows = env_int("ANYSEQ_CHECK_ROWS", 0);   // (read per call: tests toggle it)
        // + one word: the final level's split-table check (aff_final_blocks_kernel)
        const size_t tail_words = (size_t)std::max(nlev, 1) * (check_rows ? 17 : 9) + 1;
        if (tail_words > tail_cap) fail("internal: %d planned levels", nlev);
        // (in the status block, so one download carries the splits, the score and these)
        uint32_t* d_tail = reinterpret_cast<uint32_t*>(d_status + tail_off);
        uint32_t* d_hdr = d_tail;
        uint32_t* d_err = d_tail + 8 * nlev;
        uint32_t* h_tail = reinterpret_cast<uint32_t*>(h_status + tail_off);
        // the final level on the device too, right behind the levels (no host round trip):
        // its block table, list of tall blocks and (worst case) HBM slab
        const int64_t slab_bound = ((int64_t)n + 127 * (int64_t)sp.nb) * 128;
        dev_final = g_tuning.devfinal && slab_bound <= ((int64_t)4 << 30);
        BlockInfo* d_fblocks = nullptr;
        int32_t* d_tall = nullptr;
        uint8_t* d_fpred = nullptr;
        if (dev_final) {   // (a block table and tall list per view)
            d_fblocks = (BlockInfo*)E.blocks.get((size_t)nviews * sp.nb * sizeof(BlockInfo));
            d_tall = (int32_t*)E.tall.get((size_t)nviews * ((size_t)sp.nb + 1) * 4);
            d_fpred = (uint8_t*)E.pred.get((size_t)std::max<int64_t>(slab_bound, 16));
        }
        const bool timed = g_tuning.fill_events != 0;   // (events around each planned fill: last_fill_stats)
        while ((int)E.pl_ev.size() < 2 * nlev) {
            hipEvent_t ev;
            HIPCHECK(hipEventCreate(&ev));
            E.pl_ev.push_back(ev);
        }
        if (check_ptrs_enabled()) {
            register_static_range(meta, max_meta);
            register_static_range(rowbuf, max_rowbuf);
            register_static_range(rowpool, max_rowpool);
        }
        // (every level's header and error word are zeroed by level 1's plan launch; the
        // final level's check word is written by aff_final_blocks_kernel)
        uint32_t* d_rchk = d_tail + 9 * (size_t)nlev;   // check words of level li at + 8 * li
        if (check_rows) HIPCHECK(hipMemsetD32Async(d_rchk, 0xffffffffu, 8 * (size_t)nlev, st));
        // diagnostics: the tail launches' phases (aff_level_tail_kernel stamps, 8 words a level)
        static const int tail_stamps = env_int("ANYSEQ_TAIL_STAMPS", 0);
        unsigned long long* d_tst = nullptr;
        if (tail_stamps) {
            d_tst = (unsigned long long*)E.tst.get((size_t)16 * std::max(nlev, 1) * 8);
            std::vector<unsigned long long> init((size_t)16 * std::max(nlev, 1), 0ull);
            for (size_t i = 0; i < init.size(); i += 16) init[i] = ~0ull;
            HIPCHECK(hipMemcpyAsync(d_tst, init.data(), init.size() * 8, hipMemcpyHostToDevice, st));
            HIPCHECK(hipStreamSynchronize(st));
        }
        static std::atomic<int32_t> g_plan_epoch{0x40000};
        uint32_t* ctr = (uint32_t*)meta;
        std::vector<AffLevelPlan> plans((size_t)nlev);
        std::vector<int32_t> epochs((size_t)nlev);
        for (int li = 0; li < nlev; ++li) {
            const Lev& L = lv[li];
            const size_t zb = ((32 + (size_t)L.slots) * 4 + 255) & ~(size_t)255;
            DPProblem* d_probs = (DPProblem*)(meta + zb);
            GroupRef* d_groups = (GroupRef*)(meta + zb + (size_t)L.nh * sizeof(DPProblem));
            const int32_t epoch = (g_plan_epoch.fetch_add(1) + 1) & 0x7ffff;
            epochs[li] = epoch;
            AffLevelPlan& A = plans[li];
            A = AffLevelPlan{};
            A.parts = L.parts;
            A.bpp = 0;
            A.nb = sp.nb;
            A.half = L.half;
            A.pw = 0;
            A.m = m;
            A.n = n;
            A.kind = kind;
            A.best_bits = local ? AM_BEST_ALL : AM_BEST_LAST;
            A.afft = g_tuning.afft ? 1 : 0;
            A.NW = L.nw;
            A.want_slots = L.want;
            A.bound = L.bound;
            A.epoch = epoch;
            A.q = cq;
            A.s = cs;
            A.LH = LH0;
            A.LE = LE0;
            A.RH = RH0;
            A.RE = RE0;
            A.pbest = pbest;
            A.rowpool = rowpool;
            A.rowbuf = rowbuf;
            A.flags = ctr + 32;
            A.spl = d_spl;
            A.typ = d_typ;
            A.score = li == 0 && P0 == 1 ? nullptr : d_score;   // (level 1's own value: its tail)
            A.parts_out = d_parts;
            A.probs = d_probs;
            A.groups = d_groups;
            A.jobs = d_jobs;
            A.hdr = d_hdr + 8 * li;
            A.xrun = xcd_run(E, L.grid, true);
            A.xq = reinterpret_cast<uint32_t*>(d_groups + L.slots);
            A.scode = scode_rows;
            A.scode_cap = (int64_t)scode_cap;
            A.world = sharded ? world : 1;
            A.rank = emulate ? -1 : my_rank;
            A.vstride = (int64_t)nn;
            A.pstride = pstride;
        }
        // level 1: plan + prep; every level: fill, then one tail launch (join, next level's
        // sentinel rows, counters, best cells and plan)
        if (nlev == 0) upload_status();   // (no level: the table's ends come from the host)
        hstamp("plan setup");
        if (nlev > 0) {
            plans[0].zero_init = d_tail;
            plans[0].nzero_init = 9 * nlev;
            plans[0].init_ends = 1;
            // (the fill prep's work too: level 1's counters and best cells; the hand-off
            // rows are all sentinel already)
            plans[0].zero2 = ctr;
            plans[0].nzero2 = 32 + lv[0].slots;
            plans[0].init2 = pbest;
            plans[0].ninit2 = ninit_best;
            plans[0].init2_value = kAffNegH;
            HIPCHECK(anyseq_launch_aff_level_plan(&plans[0], st));
        }
        for (int li = 0; li < nlev; ++li) {
            const Lev& L = lv[li];
            const AffLevelPlan& A = plans[li];
            g_stage_level = lev0 + li + 1;
            if (sharded) {   // rows and best cells a rank does not fill are zero / -inf in the reductions
                for (int32_t* b : {LH0, LE0, RH0, RE0}) HIPCHECK(hipMemsetAsync(b, 0, nviews * nn * 4, st));
                if (!emulate) HIPCHECK(hipMemsetAsync(rowpool, 0, max_rowpool, st));
            }
            DPProblem* d_probs = A.probs;
            GroupRef* d_groups = A.groups;
            FillParams fpl = fp;
            fpl.epoch = epochs[li];
            fpl.prio = fill_prio(true);
            fpl.throttle = g_tuning.thr;
            fpl.slack = g_tuning.slack;
            fpl.slack_io = g_tuning.slack_io;
            fpl.dbg = nullptr;
            fpl.xq = A.xrun > 0 ? A.xq : nullptr;
            // the level's subject-code rows, from the descriptors its plan just wrote
            HIPCHECK(anyseq_launch_aff_scode(d_probs, L.nh, std::max(n, m), st));
            if (timed) HIPCHECK(hipEventRecord(E.pl_ev[2 * li], st));
            HIPCHECK(anyseq_launch_fill_affine(L.nw, d_probs, d_groups, L.slots, ctr, d_err + li, &fpl, L.grid, st));
            if (li == 0) hstamp("first fill");
            if (timed) HIPCHECK(hipEventRecord(E.pl_ev[2 * li + 1], st));
            if (check_rows) {
                // the invariant the next launch relies on: every hand-off row word is the
                // sentinel again (ANYSEQ_CHECK_ROWS=2 first leaves a stale word past w in
                // level 1's first half with a ring, and puts it back once found: the check's
                // own test, the construct then fails with the check's message)
                uint32_t* w = d_rchk + 8 * (size_t)li;
                HIPCHECK(hipMemsetAsync(w, 0, 4, st));
                const int inject = check_rows == 2 && li == 0;
                HIPCHECK(anyseq_launch_rows_check(rowbuf, max_rowbuf / 4, 0x80808080u, d_probs, L.nh, w, inject, st));
            }
            if (sharded) {   // every rank gets every half's columns, bottom rows and best cells
                if (emulate) {
                    for (int32_t* b : {LH0, LE0, RH0, RE0})
                        HIPCHECK(anyseq_launch_view_reduce_i32(b, nn, nviews, nn, 0, st));
                    HIPCHECK(anyseq_launch_view_reduce_i32(pbest, (size_t)pstride, nviews, (size_t)2 * L.parts, 1, st));
                } else {
                    for (int32_t* b : {LH0, LE0, RH0, RE0}) shards->sum_i32(b, (size_t)n, st);
                    shards->sum_i32(rowpool, max_rowpool / 4, st);
                    shards->max_i32(pbest, (size_t)2 * L.parts, st);
                }
                stage_check(st, "sharded level reductions (device plan)");
            }
            AffLevelTail T{};
            T.parts = d_parts;
            T.jobs = d_jobs;
            T.LH = LH0;
            T.LE = LE0;
            T.RH = RH0;
            T.RE = RE0;
            T.pbest = pbest;
            T.nparts = L.parts;
            T.half = L.half;
            // ~256 join workgroups: few long parts split into slices, many short ones whole
            T.nslices = std::max(1, std::min(nsl, (256 + L.parts - 1) / L.parts));
            T.slice_len = (n + 1 + T.nslices - 1) / T.nslices;
            T.go = sc.gap_open;
            T.ge = sc.gap_extend;
            T.partial = partial;
            T.splits = d_spl;
            T.types = d_typ;
            T.score = li == 0 && P0 == 1 ? d_score : nullptr;
            T.done = d_hdr + 8 * li + 4;
            T.stamps = d_tst ? d_tst + 16 * li : nullptr;
            T.has_next = li + 1 < nlev;
            if (T.has_next) {
                const Lev& N = lv[li + 1];
                T.sent = rowbuf;
                T.nsent16 = 0;   // (the rows are sentinel already)
                T.zero = ctr;
                T.nzero = 32 + N.slots;
                T.init = pbest;
                T.ninit = ninit_best;
                T.next = plans[li + 1];
            }
            HIPCHECK(anyseq_launch_aff_level_tail(&T, T.has_next && T.nsent16 ? 1024 : 1, st));
            stage_check(st, "affine level (device plan)");
        }
        uint32_t* d_ferr = d_tail + tail_words - 1;
        if (dev_final) {
            // sharded: each view walks its blocks (b % world == rank) into its own strings,
            // which merge by the byte-wise MAX of the host-built final level
            for (int v = 0; v < nviews; ++v) {
                AffFinalPlan F{};
                F.spl = d_spl;
                F.typ = d_typ;
                // (no level, m <= 128: nothing writes d_score; the caller checked score > 0)
                F.score = lev0 + nlev > 0 ? d_score : nullptr;
                F.blocks = d_fblocks + (size_t)v * sp.nb;
                F.tall = d_tall + (size_t)v * (sp.nb + 1);
                F.err = d_ferr;
                F.nb = sp.nb;
                F.n = n;
                F.m = m;
                F.kind = kind;
                F.small_rows = kPredSmallRows;
                F.world = sharded ? world : 1;
                F.rank = view_rank(v);
                g_stage_level = lev0 + nlev + 1;
                uint8_t *aq, *as;
                view_str(v, aq, as);
                HIPCHECK(anyseq_launch_aff_final(&F, dq, ds, d_fpred, sc.match, sc.mismatch, sc.gap_open,
                                                 sc.gap_extend, aq, as, st));
                stage_check(st, "aff_final (device plan)");
            }
            if (sharded) {
                if (emulate) {
                    HIPCHECK(anyseq_launch_view_max_u8(d_alq, vstr, 2 * L, nviews - 1, L, st));
                    HIPCHECK(anyseq_launch_view_max_u8(d_als, vstr + L, 2 * L, nviews - 1, L, st));
                } else {
                    shards->max_u8(d_alq, L, st);
                    shards->max_u8(d_als, L, st);
                }
            }
        }
        HIPCHECK(hipMemcpyAsync(h_status, d_status, (tail_off + tail_words) * 4, hipMemcpyDeviceToHost, st));
        hstamp("enqueued");
        {
            const hipError_t e = stream_wait_spin(st);
            hstamp("wait");
            if (e != hipSuccess) fail("affine construct levels failed: %s", hipGetErrorString(e));
        }
        if (d_tst) {
            std::vector<unsigned long long> h((size_t)16 * nlev);
            HIPCHECK(hipMemcpy(h.data(), d_tst, h.size() * 8, hipMemcpyDeviceToHost));
            for (int li = 0; li < nlev; ++li) {
                const unsigned long long* q = h.data() + 16 * li;
                auto d = [&](int a, int b) { return q[a] && q[b] ? ((double)q[b] - (double)q[a]) / 100.0 : 0.0; };
                fprintf(stderr, "tail %d: join %.2f us, final pass %.2f, counters %.2f, plan %.2f | plan: enter %.2f, "
                        "parts %.2f, scans %.2f, halves %.2f, groups %.2f, end %.2f\n",
                        lev0 + li + 1, d(0, 1), d(1, 2), d(2, 3), d(3, 4), d(3, 8), d(8, 9), d(9, 10), d(10, 11),
                        d(11, 12), d(12, 4));
            }
        }
        bool any_err = false;
        for (int li = 0; li < nlev; ++li) any_err |= h_tail[8 * nlev + li] != 0;
        for (int li = 0; check_rows && li < nlev; ++li) any_err |= h_tail[9 * nlev + 8 * li] != 0;
        E.pl_dirty = any_err;
        for (int li = 0; check_rows && li < nlev; ++li) {
            const uint32_t* c = h_tail + 9 * nlev + 8 * li;
            if (c[0])
                fail("hand-off row invariant broken after planned level %d: %u non-sentinel word(s), the first at "
                     "word %u = half %d, ring slot %d, column %d (half width %d)", lev0 + li + 1, c[0], c[1], (int)c[2],
                     (int)c[3], (int)c[4], (int)c[5]);
        }
        for (int li = 0; li < nlev; ++li) {
            const uint32_t err = h_tail[8 * nlev + li];
            g_stage_level = lev0 + li + 1;
            if (err & ERR_BAD_DESC) fail("fill kernel read a corrupt problem descriptor (error %u; planned level %d)", err, lev0 + li + 1);
            if (err) fail("fill kernel reported error %u (spin timeout; planned level %d)", err, lev0 + li + 1);
            if (h_tail[8 * li + 1]) fail("internal: planned level %d: a half exceeds its group slots", lev0 + li + 1);
            float ms = 0.f;
            if (timed) HIPCHECK(hipEventElapsedTime(&ms, E.pl_ev[2 * li], E.pl_ev[2 * li + 1]));
            g_fill_ms += ms;
            g_fill_launches += 1;
            uint64_t cells;
            memcpy(&cells, h_tail + 8 * li + 2, 8);
            g_fill_cells += (int64_t)cells;
        }
        memcpy(sp.v.data(), h_status, nsv * 4);
        memcpy(typ.data(), h_status + nsv, nsv * 4);
        // the splits run from 0 to n, in order, each with a known type
        for (size_t i = 1; i < nsv; ++i)
            if (sp.v[i] < sp.v[i - 1] || sp.v[i] > n || typ[i] < T_H || typ[i] > T_AFTER)
                fail("internal: planned levels left split %zu = %d (type %d)", i - 1, sp.v[i], typ[i]);
        if (dev_final && h_tail[tail_words - 1])
            fail("internal: the device final level found a bad split table (the host check passed)");
        if (nlev > 0 && P0 == 1) {   // (P0 > 1: the host's level 1 set it)
            const int32_t s32 = h_status[2 * nsv];
            score = kind == KIND_SEMIGLOBAL ? std::max(s32, 0) : s32;
        }
        planned = true;   // (the host loop has nothing left)
        hstamp("checks");
    };
    if (!sharded && plan_ok) run_planned(1);
    if (planned && kind != KIND_GLOBAL && score <= 0) return score;   // the empty alignment
    if (!planned) {
        upload_status();
        HIPCHECK(hipStreamSynchronize(st));   // h_status: its upload before the first download
    }
    int handover = 0;
    // Inherited halves (one GPU, global / semiglobal): a half of a
    // throughput-bound level may run as column blocks cut at its next descendants' splits --
    // a block's last column (H, E) is then also that descendant half's last column on the
    // descendant's rows (same anchor, same borders, a prefix of the columns and rows), so
    // at that level the descendant half is a copy instead of a fill.  A left half's line is
    // its leftmost descendants' left halves, a right half's its rightmost descendants' right
    // halves.  ch*_prev: per part of the previous level, the recorded chain its child half
    // takes (left halves' columns by query row, right halves' by n-1-row).
    const bool inh_on = !sharded && g_tuning.inherit > 0 && !local;
    // cap[side][d][0/1]: the depth-d recorded column (H / E by query row; d = 1: the
    // child's, d = 2: the grandchild's, ...), side 0 left halves, 1 right halves
    constexpr int kInhMax = 4;
    const int inh_depth = std::max(1, std::min(kInhMax, g_tuning.inherit_depth));
    struct InhChain {
        int j = 0, mx = 0, base = 0;   // depth of the child half's column (0: none), deepest recorded, column offset
    };
    std::vector<InhChain> chL_prev, chR_prev;
    int32_t* cap[2][kInhMax + 1][2] = {};
    if (inh_on && !planned) {
        for (int side = 0; side < 2; ++side) {
            int32_t* b = (int32_t*)(side ? E.capR : E.capL).get((size_t)inh_depth * 2 * nn * 4);
            for (int d = 1; d <= inh_depth; ++d)
                for (int k = 0; k < 2; ++k) cap[side][d][k] = b + ((size_t)(d - 1) * 2 + k) * nn;
        }
    }
    const int inh_nge = -sc.gap_extend;
    for (int parts = 1; !planned && parts < sp.nb; parts *= 2) {
        ++g_stage_level;
        // free-end best cells, 2 per part, per view
        int32_t* pbest0 = (int32_t*)E.bmax.get((size_t)nviews * 2 * parts * 4);
        std::vector<std::vector<DPProblem>> probs_of((size_t)nviews);
        std::vector<PartInfo>& pinfo = E.host_parts;
        pinfo.assign((size_t)parts, PartInfo{});
        std::vector<RowToColJob> jobs;
        int half_index = 0;   // the level's half fills in part order: left 2k, right 2k+1
        ShardLevel lvl;
        bool blocked = false;
        if (sharded) {   // rows a rank does not fill are zero in the SUM reduction
            for (int32_t* b : {LH0, LE0, RH0, RE0}) HIPCHECK(hipMemsetAsync(b, 0, nviews * nn * 4, st));
        }
        // transposed halves' bottom rows: sum of part heights <= n (parts' rows are disjoint)
        int32_t* rowpool = (int32_t*)E.outrow.get((size_t)2 * ((size_t)n + 64 * (size_t)parts) * 2 * 4);
        const int best_bits = local ? AM_BEST_ALL : AM_BEST_LAST;
        for (int p = 0; p < parts; ++p) {
            const AffPartGeo pg = aff_part_geo(sp.nb, m, parts, p);
            const int sb = pg.sb, eb = pg.eb;
            PartInfo& pi = pinfo[p];
            pi.split_index = pg.mid;
            pi.lhw = pg.lw;
            if (pg.lw <= 0 || pg.hw <= 0) {   // a one-block part: no split
                pi.flags = 8;
                continue;
            }
            const int ts = tp(sb), te = tp(eb);
            if (ts == T_BEFORE || te == T_AFTER) {   // empty part: so are both halves
                pi.flags = 4;
                pi.empty_type = ts == T_BEFORE ? T_BEFORE : T_AFTER;
                pi.off = sp.at(sb);
                continue;
            }
            const int off = sp.at(sb), len = sp.at(eb) - off;
            const int hoj_l = pg.hoj_l, hoj_r = pg.hoj_r, hw = pg.hw;
            const bool sfree = ts == T_AFTER, efree = te == T_BEFORE;
            pi.off = off;
            pi.len = len;
            pi.rhw = hw;
            pi.smode = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : free_bm(kind, hoj_l == 0);
            pi.emode = te == T_H ? BM_NORMAL : te == T_E ? BM_EPAID : free_bm(kind, hoj_r + hw == m);
            pi.flags = (sfree ? 1 : 0) | (efree ? 2 : 0);
        }
        // Column-blocked level: with world >= 2 * parts every part runs
        // over its own subgroup of ranks (both halves transposed, each rank a block of
        // the part's query rows); else the halves are dealt round-robin.
        if (sharded && shards->blocked && world >= 2 * parts && g_tuning.afft && env_int("ANYSEQ_SHARD_L1", 1) != 0) {
            blocked = true;
            for (int p = 0; p < parts; ++p) {
                const PartInfo& pi = pinfo[p];
                const int r0 = (int)((int64_t)p * world / parts), G = (int)((int64_t)(p + 1) * world / parts) - r0;
                if ((pi.flags & 12) == 0 && pi.len > 0 && pi.len < G) blocked = false;
            }
        }
        if (sharded && plan_ok && !blocked && env_int("ANYSEQ_SHARD_DEVPLAN", 1) != 0) {
            handover = parts;   // this level and the rest: device-planned
            break;
        }
        if (blocked) {
            auto tam = [](int am) {
                return (am & AM_CLAMP) |
                       ((am & AM_BEST_LASTCOL) == AM_BEST_LAST ? AM_BEST_LASTCOL : (am & AM_BEST_LASTCOL));
            };
            lvl.kind = kind;
            lvl.sc = sc;
            lvl.fp = fp;
            lvl.LH = LH0;
            lvl.LE = LE0;
            lvl.RH = RH0;
            lvl.RE = RE0;
            lvl.nn = nn;
            lvl.pstride = (size_t)2 * parts;
            lvl.st = st;
            lvl.E = &E;
            for (int p = 0; p < parts; ++p) {
                const PartInfo& pi = pinfo[p];
                if ((pi.flags & 12) || pi.len <= 0) continue;   // no halves: the part's ranks idle
                const AffPartGeo pg = aff_part_geo(sp.nb, m, parts, p);
                const bool sfree = pi.flags & 1, efree = pi.flags & 2;
                ShardPart T;
                T.cq = cq;
                T.cs = cs;
                T.off = pi.off;
                T.len = pi.len;
                T.soff = pg.hoj_l;
                T.mw = pg.lw + pg.hw;
                T.half = pg.lw;
                T.bm_l = transposed_bm(pi.smode);
                T.am_l = tam((pi.smode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (efree ? best_bits : 0));
                T.bm_r = transposed_bm(pi.emode);
                T.am_r = tam((pi.emode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (sfree ? best_bits : 0));
                T.pbest = pbest0 + 2 * p;
                T.r0 = (int)((int64_t)p * world / parts);
                T.G = (int)((int64_t)(p + 1) * world / parts) - T.r0;
                lvl.parts.push_back(T);
            }
            if (g_shard_blocked_levels == g_stage_level - 1) g_shard_blocked_levels = g_stage_level;
        }
        // inherited halves of this level: split halves' later blocks (a launch each, after the
        // first blocks), the copies of the reused halves (before the fills) and the frame
        // corrections of the later blocks' columns (after them)
        const bool inh_level = inh_on && 2 * parts < sp.nb &&
                               (g_tuning.inherit >= 2 || [&] {
                                   const int64_t rows = std::max<int64_t>(1, (int64_t)n / parts), w = level_half(parts);
                                   const int64_t chain = w + rows * 128 / 100,
                                                 work = 2 * (int64_t)parts * ((rows + 63) / 64) * (w + 64);
                                   return aff_waves_for(chain, work, g_tuning.grida > 0 ? g_tuning.grida : E.num_cus) >= 7;
                               }());
        std::vector<InhChain> chL_cur(inh_on ? (size_t)parts : 0), chR_cur(inh_on ? (size_t)parts : 0);
        std::vector<std::vector<DPProblem>> later;   // split halves' blocks 2, 3, .. (one launch each, in order)
        std::vector<I32Job> copy_jobs, shift_jobs;
        int64_t n_split = 0, n_reused = 0;
        // a half as column blocks cut at `cuts` (ascending): block i < last records its last
        // column into caps[i] (the deepest descendant's first), block i > 0 takes block i-1's
        // as its complete left border (the sharded score's left_in) in its own frame, moved
        // by the top border's slope (NORMAL / EFREE: |ge| per column of the block's start;
        // the free borders are flat) and moved back by a job after the level's last launch;
        // a best cell is shared (flat frames only)
        auto split_half = [&](int qoff, int qstep, int h, int soff, int sstep, int w, const std::vector<int>& cuts,
                              int bm, int am, int32_t* best, const std::vector<std::pair<int32_t*, int32_t*>>& caps,
                              int32_t* H, int32_t* Ecol) {
            const bool flat = !(bm == BM_NORMAL || bm == BM_EFREE);
            const int nbk = (int)cuts.size() + 1;
            for (int i = 0; i < nbk; ++i) {
                const int s0 = i == 0 ? 0 : cuts[i - 1], e0 = i + 1 < nbk ? cuts[i] : w;
                DPProblem P = aff_problem(cq, qoff, qstep, h, cs, soff + sstep * s0, sstep, e0 - s0);
                P.bmode = bm;
                P.amode = am;
                P.best = best;
                int32_t* oh = i + 1 < nbk ? caps[i].first : H;
                int32_t* oe = i + 1 < nbk ? caps[i].second : Ecol;
                P.out_col = oh;
                P.out_col_e = oe;
                if (i > 0) {
                    P.left_in = caps[i - 1].first;
                    P.left_in_e = caps[i - 1].second;
                    const int sp0 = i >= 2 ? cuts[i - 2] : 0;   // block i-1's first column (its frame)
                    P.left_shift = flat ? 0 : (s0 - sp0) * inh_nge;
                }
                if (i == 0) {
                    probs_of[0].push_back(P);
                } else {
                    if ((int)later.size() < i) later.resize(i);
                    later[i - 1].push_back(P);
                }
                if (!flat && s0 > 0) {
                    shift_jobs.push_back(I32Job{oh, oh, h, -s0 * inh_nge});
                    shift_jobs.push_back(I32Job{oe, oe, h, -s0 * inh_nge});
                }
            }
            ++n_split;
        };
        // the columns a half of part p can record: its leftmost (side 0) / rightmost (1)
        // descendant's half width at each of the next inh_depth levels, while they split
        auto desc_cuts = [&](int p, int side, int width) {
            std::vector<int> c;
            int prev = width;
            for (int d = 1; d <= inh_depth; ++d) {
                const int64_t P2 = (int64_t)parts << d;
                if (P2 >= sp.nb) break;
                const int q = side == 0 ? (int)((int64_t)p << d) : (int)(((int64_t)(p + 1) << d) - 1);
                const AffPartGeo g = aff_part_geo(sp.nb, m, (int)P2, q);
                const int cw = side == 0 ? g.lw : g.hw;
                if (g.lw <= 0 || g.hw <= 0 || cw <= 0 || cw >= prev) break;
                c.push_back(cw);
                prev = cw;
            }
            std::reverse(c.begin(), c.end());   // ascending: the deepest descendant's first
            return c;
        };
        // may the half (border mode bm, kind bits am) run split?  No clamp, no EPAID
        // corner (the shard frame's corner is go only under NORMAL), a best only in a flat frame
        auto splittable = [&](int bm, int am) {
            if (am & AM_CLAMP) return false;
            if (bm == BM_EPAID || bm == BM_FREE_LOCAL) return false;
            // (a best of the last row: the blocks' last rows are the half's; not of every cell)
            if ((am & AM_BEST_LASTCOL) != 0 && (am & AM_BEST_LASTCOL) != AM_BEST_LAST) return false;
            return (am & AM_BEST_LASTCOL) == 0 || !(bm == BM_NORMAL || bm == BM_EFREE);
        };
        for (int p = 0; p < parts && !blocked; ++p) {
            const PartInfo& pi = pinfo[p];
            if ((pi.flags & 12) || pi.len <= 0) continue;
            const AffPartGeo pg = aff_part_geo(sp.nb, m, parts, p);
            const int off = pi.off, len = pi.len, half = pg.lw, hoj_l = pg.hoj_l, hoj_r = pg.hoj_r, hw = pg.hw;
            const bool sfree = pi.flags & 1, efree = pi.flags & 2;
            // (half_index advances on every rank, so all ranks agree on the owners)
            const int ol = owner(half_index++), orr = owner(half_index++);
            if (inh_on) {   // (one view: not sharded)
                int32_t* pb = pbest0;
                const int am_l = (pi.smode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (efree ? best_bits : 0);
                const int am_r = (pi.emode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (sfree ? best_bits : 0);
                // One side's half: the chain it inherits (the leftmost / rightmost descendant
                // line of a half that recorded columns), then copy it (no best cell of its
                // own), split it (recording its own descendants' columns), or fill it whole
                // and pass the inherited chain on to its child.
                auto side_half = [&](int side, const InhChain& in, int am, int bm, int width, int qoff, int qstep,
                                     int soff, int sstep, int32_t* best, int32_t* H, int32_t* Ecol) {
                    InhChain out;
                    if (in.j > 0 && am == 0) {
                        copy_jobs.push_back(I32Job{cap[side][in.j][0] + in.base, H, len, 0});
                        copy_jobs.push_back(I32Job{cap[side][in.j][1] + in.base, Ecol, len, 0});
                        ++n_reused;
                        if (in.j < in.mx) out = InhChain{in.j + 1, in.mx, in.base};
                        return out;
                    }
                    const std::vector<int> cuts =
                        inh_level && splittable(bm, am) ? desc_cuts(p, side, width) : std::vector<int>();
                    if (!cuts.empty()) {
                        const int D = (int)cuts.size();
                        // recorded columns by query row: a left half's rows from `off` up, a right
                        // half's (reversed) from its last row down, at n-1-row -- so the columns of
                        // different parts never overlap, whatever the levels between write
                        const int base = side == 0 ? off : n - (off + len);
                        std::vector<std::pair<int32_t*, int32_t*>> caps;
                        for (int i = 0; i < D; ++i)   // cuts[i] is the depth D - i descendant's width
                            caps.emplace_back(cap[side][D - i][0] + base, cap[side][D - i][1] + base);
                        split_half(qoff, qstep, len, soff, sstep, width, cuts, bm, am, best, caps, H, Ecol);
                        return InhChain{1, D, base};
                    }
                    add_half(probs_of[0], jobs, rowpool, cq, qoff, qstep, len, cs, soff, sstep, width, bm, am, best, H,
                             Ecol);
                    if (in.j > 0 && in.j < in.mx) out = InhChain{in.j + 1, in.mx, in.base};
                    return out;
                };
                const InhChain none;
                chL_cur[p] = side_half(0, p % 2 == 0 && parts > 1 ? chL_prev[p / 2] : none, am_l, pi.smode, half,
                                       off, 1, hoj_l, 1, efree ? pb + 2 * p : nullptr, LH0 + off, LE0 + off);
                chR_cur[p] = side_half(1, p % 2 == 1 ? chR_prev[p / 2] : none, am_r, pi.emode, hw, off + len - 1,
                                       -1, hoj_r + hw - 1, -1, sfree ? pb + 2 * p + 1 : nullptr, RH0 + off,
                                       RE0 + off);
                continue;
            }
            for (int v = 0; v < nviews; ++v) {
                const size_t vo = (size_t)v * nn;
                int32_t* pb = pbest0 + (size_t)v * 2 * parts;
                if (!sharded || ol == view_rank(v))
                    add_half(probs_of[v], jobs, rowpool, cq, off, 1, len, cs, hoj_l, 1, half, pi.smode,
                             (pi.smode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (efree ? best_bits : 0),
                             efree ? pb + 2 * p : nullptr, LH0 + vo + off, LE0 + vo + off);
                if (!sharded || orr == view_rank(v))
                    add_half(probs_of[v], jobs, rowpool, cq, off + len - 1, -1, len, cs, hoj_r + hw - 1, -1, hw,
                             pi.emode, (pi.emode == BM_FREE_LOCAL ? AM_CLAMP : 0) | (sfree ? best_bits : 0),
                             sfree ? pb + 2 * p + 1 : nullptr, RH0 + vo + off, RE0 + vo + off);
            }
        }
        // the level's parts and row-to-column jobs, staged together in pinned memory
        // (the jobs hold pointers: they start 16-byte aligned)
        const size_t jb = jobs.size() * sizeof(RowToColJob), pb = (pinfo.size() * sizeof(PartInfo) + 15) & ~(size_t)15;
        char* up = (char*)E.pin_up.get(jb + pb + 16);
        memcpy(up, pinfo.data(), pinfo.size() * sizeof(PartInfo));
        memcpy(up + pb, jobs.data(), jb);
        // one fill launch per view with work; all but the last complete in turn (they share
        // the fill context), the last is collected after the level's single synchronisation.
        // A single launch carries the parts and jobs in its own upload (one copy per level).
        int nl = 0;
        for (const auto& probs : probs_of) nl += probs.empty() ? 0 : 1;
        bool pending_fill = false;
        const char* d_up = nullptr;
        const double t_built = now_us();
        // inherited halves: the copy and frame jobs in one upload, the copies before the fills
        const char* d_aux = nullptr;
        if (!copy_jobs.empty() || !shift_jobs.empty()) {
            const size_t nb_aux = (copy_jobs.size() + shift_jobs.size()) * sizeof(I32Job);
            char* ha = (char*)E.pin_aux.get(nb_aux);
            memcpy(ha, copy_jobs.data(), copy_jobs.size() * sizeof(I32Job));
            memcpy(ha + copy_jobs.size() * sizeof(I32Job), shift_jobs.data(), shift_jobs.size() * sizeof(I32Job));
            char* da = (char*)E.auxjobs.get(nb_aux);
            HIPCHECK(hipMemcpyAsync(da, ha, nb_aux, hipMemcpyHostToDevice, st));
            d_aux = da;
        }
        auto run_jobs = [&](const std::vector<I32Job>& J, const char* d) {
            int maxn = 0;
            for (const I32Job& j : J) maxn = std::max(maxn, j.n);
            HIPCHECK(anyseq_launch_i32_jobs(d, (int)J.size(), maxn, st));
        };
        if (!copy_jobs.empty()) run_jobs(copy_jobs, d_aux);
        if (!later.empty()) {
            // split halves: their first blocks (with the unsplit halves), then each further
            // block in its own launch behind the one before; the last carries the level's
            // upload (one view: not sharded)
            fill_async(E, E.fc, probs_of[0], fp, st, 0, nullptr, 0, pbest0, 2 * parts, kAffNegH);
            for (size_t i = 0; i < later.size(); ++i) {
                fill_finish(E.fc);
                const bool last = i + 1 == later.size();
                fill_async(E, E.fc, later[i], fp, st, 0, last ? up : nullptr, last ? pb + jb : 0, nullptr, 0, 0);
            }
            d_up = (const char*)E.fc.d_extra;
            pending_fill = true;
        }
        for (int v = 0; v < nviews && later.empty(); ++v) {
            auto& probs = probs_of[v];
            int32_t* pbv = pbest0 + (size_t)v * 2 * parts;
            if (probs.empty()) {
                HIPCHECK(hipMemsetD32Async(pbv, kAffNegH, (size_t)2 * parts, st));
                continue;
            }
            if (pending_fill) fill_finish(E.fc);
            if (nl == 1) {
                fill_async(E, E.fc, probs, fp, st, 0, up, pb + jb, pbv, 2 * parts, kAffNegH);
                d_up = (const char*)E.fc.d_extra;
            } else {
                fill_async(E, E.fc, probs, fp, st, 0, nullptr, 0, pbv, 2 * parts, kAffNegH);
            }
            pending_fill = true;
        }
        if (blocked) {   // (every view's best cells were reset above: no view has probs)
            shards->blocked(lvl);
            stage_check(st, "sharded column-blocked level");
        }
        if (!d_up) {
            char* d = (char*)E.parts.get(pb + jb + 16);
            HIPCHECK(hipMemcpyAsync(d, up, pb + jb, hipMemcpyHostToDevice, st));
            d_up = d;
        }
        stage_check(st, "affine fill");
        const double t_launched = now_us();
        if (!jobs.empty()) {
            int maxn = 0;
            for (const auto& J : jobs) maxn = std::max(maxn, J.n);
            HIPCHECK(anyseq_launch_aff_row_to_col(d_up + pb, (int)jobs.size(), maxn, -sc.gap_extend, st));
            stage_check(st, "aff_row_to_col");
        }
        if (!shift_jobs.empty()) {   // split halves' second blocks: their columns back to the half's frame
            run_jobs(shift_jobs, d_aux + copy_jobs.size() * sizeof(I32Job));
            stage_check(st, "inherited halves: frames");
        }
        if (sharded) {   // every rank gets every part's columns and best cells
            if (emulate) {
                for (int32_t* b : {LH0, LE0, RH0, RE0})
                    HIPCHECK(anyseq_launch_view_reduce_i32(b, nn, nviews, nn, 0, st));
                HIPCHECK(anyseq_launch_view_reduce_i32(pbest0, (size_t)2 * parts, nviews, (size_t)2 * parts, 1, st));
            } else {
                for (int32_t* b : {LH0, LE0, RH0, RE0}) shards->sum_i32(b, (size_t)n, st);
                shards->max_i32(pbest0, (size_t)2 * parts, st);
            }
        }
        const PartInfo* d_parts = (const PartInfo*)d_up;
        int maxlen = 0;
        for (const PartInfo& q : pinfo) maxlen = std::max(maxlen, (q.flags & 4) ? 0 : q.len);
        const size_t nsl = (size_t)std::max(1, (maxlen + 1 + 4095) / 4096);
        void* partial = E.joinbuf.get((size_t)parts * nsl * 8);
        // (view 0's columns: after the reduction every view holds the same)
        HIPCHECK(anyseq_launch_aff_hb_join2(d_parts, parts, maxlen, 0, LH0, LE0, RH0, RE0, pbest0, sc.gap_open,
                                            sc.gap_extend, partial, d_spl, d_typ, level1 ? d_score : nullptr, st));
        stage_check(st, "aff_hb_join");
        HIPCHECK(hipMemcpyAsync(h_status, d_status, (2 * nsv + (level1 ? 1 : 0)) * 4, hipMemcpyDeviceToHost, st));
        {
            const double t_enq = now_us();
            const hipError_t e = stream_wait_spin(st);
            const double t_w = now_us();
            if (level_timing)
                fprintf(stderr, "level %d: build %.1f us, fill launch %.1f us, join enqueue %.1f us, wait %.1f us\n",
                        g_stage_level, t_built - t_wake, t_launched - t_built, t_enq - t_launched, t_w - t_enq);
            t_wake = t_w;
            if (e != hipSuccess && pending_fill)
                fail("fill failed: %s (%s)", hipGetErrorString(e), fill_summary(E.fc).c_str());
            HIPCHECK(e);
        }
        if (pending_fill) fill_collect(E.fc);
        memcpy(sp.v.data(), h_status, nsv * 4);
        memcpy(typ.data(), h_status + nsv, nsv * 4);
        const int32_t s32 = level1 ? h_status[2 * nsv] : 0;
        // every split this level set lies inside its part and has a known type (the
        // next level's sub-problems are built from them)
        for (int p = 0; p < parts; ++p) {
            if (pinfo[p].flags & 8) continue;   // a one-block part: nothing split
            const int si = pinfo[p].split_index + 1;
            const int lo = pinfo[p].off, hi = (pinfo[p].flags & 4) ? lo : lo + std::max(pinfo[p].len, 0);
            if (sp.v[si] < lo || sp.v[si] > hi || typ[si] < T_H || typ[si] > T_AFTER)
                fail("internal: level %d part %d split %d (type %d) outside rows [%d, %d]", g_stage_level, p,
                     sp.v[si], typ[si], lo, hi);
        }
        if (level1) {
            // semiglobal: the empty alignment (a border cell, 0) is a candidate too
            score = kind == KIND_SEMIGLOBAL ? std::max(s32, 0) : s32;
            level1 = false;
            if (kind != KIND_GLOBAL && score <= 0) return score;   // the empty alignment
        }
        if (inh_on) {
            chL_prev.swap(chL_cur);
            chR_prev.swap(chR_cur);
            g_inherit_stats[0] += n_split;
            g_inherit_stats[1] += n_reused;
        }
    }
    if (handover > 0) {
        run_planned(handover);
        if (kind != KIND_GLOBAL && score <= 0) return score;   // (checked by the host's level 1 already)
    }
    if (dev_final) return score;   // (the final level is done: enqueued behind the levels)
    // final 128-column blocks: each view walks its own into its strings
    std::vector<BlockInfo>& blocks = E.host_blocks;   // outlives the async upload
    blocks.clear();
    std::vector<int> vbeg((size_t)nviews + 1, 0);
    int64_t pred_bytes = 0;
    int lds_rows = 1;   // the tallest block, up to kPredLdsMaxRows (its predecessors fit in LDS)
    for (int b = 0; b < sp.nb; ++b)
        if (!(tp(b - 1) == T_BEFORE || tp(b) == T_AFTER))
            lds_rows = std::max(lds_rows, std::min(kPredLdsMaxRows, sp.at(b) - sp.at(b - 1)));
    for (int v = 0; v < nviews; ++v) {
        vbeg[v] = (int)blocks.size();
        for (int b = 0; b < sp.nb; ++b) {
            const int ts = tp(b - 1), te = tp(b);
            if (ts == T_BEFORE || te == T_AFTER) continue;        // the path does not touch the block
            if (sharded && owner(b) != view_rank(v)) continue;    // another rank walks it
            BlockInfo bi{};
            bi.oi = sp.at(b - 1);
            bi.h = sp.at(b) - bi.oi;
            bi.oj = b * MIN_PART_WIDTH_HB;
            bi.w = std::min(MIN_PART_WIDTH_HB, m - bi.oj);
            bi.pred_base = pred_bytes;
            bi.smode = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : free_bm(kind, bi.oj == 0);
            bi.e_end = te == T_H ? 0 : te == T_E ? 1 : 2;
            bi.flags = (local ? 1 : 0) | (bi.oj + bi.w == m ? 2 : 0);
            if (bi.h > lds_rows) pred_bytes += (int64_t)(bi.h + 127) * 128;   // (shorter blocks: LDS)
            blocks.push_back(bi);
        }
    }
    vbeg[nviews] = (int)blocks.size();
    if (!blocks.empty()) {
        BlockInfo* d_blocks = (BlockInfo*)E.blocks.get(blocks.size() * sizeof(BlockInfo));
        upload_pinned(E.pin_blocks, d_blocks, blocks.data(), blocks.size() * sizeof(BlockInfo), st);
        uint8_t* d_pred = (uint8_t*)E.pred.get((size_t)std::max<int64_t>(pred_bytes, 16));
        for (int v = 0; v < nviews; ++v) {
            const int nb = vbeg[v + 1] - vbeg[v];
            if (nb <= 0) continue;
            uint8_t *aq, *as;
            view_str(v, aq, as);
            HIPCHECK(anyseq_launch_aff_predwalk(d_blocks + vbeg[v], nb, dq, ds, d_pred, sc.match, sc.mismatch,
                                                sc.gap_open, sc.gap_extend, aq, as, lds_rows, st));
            stage_check(st, "aff_predwalk");
        }
    }
    if (sharded) {
        // blocks write disjoint positions over a ' ' prefill, and every written byte
        // ('_' or a symbol; sharded_construct refuses bytes <= ' ') is above ' ': a
        // byte-wise MAX merges the ranks' strings
        if (emulate) {
            HIPCHECK(anyseq_launch_view_max_u8(d_alq, vstr, 2 * L, nviews - 1, L, st));
            HIPCHECK(anyseq_launch_view_max_u8(d_als, vstr + L, 2 * L, nviews - 1, L, st));
        } else {
            shards->max_u8(d_alq, L, st);
            shards->max_u8(d_als, L, st);
        }
    }
    return score;
}


// Affine construct on device-resident sequences into device strings (n+m bytes);
// returns the optimal score.
}  // namespace

int64_t construct_affine_dev(Engine& E, int kind, const anyseq_scoring& sc, const uint8_t* dq, int n,
                             const uint8_t* ds, int m, uint8_t* d_alq, uint8_t* d_als, hipStream_t st,
                             const ConstructShards* shards) {
    const size_t L = (size_t)n + (size_t)m;
    if (L == 0) return empty_score(kind, n, m, sc);
    // the strings' ' ' prefill: here for the degenerate shapes, else inside the construct
    // (in its alphabet-coding launch)
    bool clear = true;
    if (n <= 0 || m <= 0) {
        HIPCHECK(hipMemsetAsync(d_alq, ' ', L, st));
        HIPCHECK(hipMemsetAsync(d_als, ' ', L, st));
        clear = false;
        if (kind == KIND_GLOBAL && m <= 0 && n > 0) {   // all query rows against gaps, down the left border
            HIPCHECK(hipMemcpyAsync(d_alq, dq, (size_t)n, hipMemcpyDeviceToDevice, st));
            HIPCHECK(hipMemsetAsync(d_als, '_', (size_t)n, st));
        }
        if (kind != KIND_GLOBAL || m <= 0) return empty_score(kind, n, m, sc);
    }
    if (m <= MIN_PART_WIDTH_HB) {   // no Hirschberg level: the score from a (small) fill
        const int64_t score = score_dev(E, kind, sc, dq, n, ds, m, st);
        if (kind != KIND_GLOBAL && score <= 0) {
            if (clear) {
                HIPCHECK(hipMemsetAsync(d_alq, ' ', L, st));
                HIPCHECK(hipMemsetAsync(d_als, ' ', L, st));
            }
            return score;
        }
        aff_construct_hb(E, kind, sc, dq, n, ds, m, d_alq, d_als, st, shards, clear);
        return score;
    }
    return aff_construct_hb(E, kind, sc, dq, n, ds, m, d_alq, d_als, st, shards, clear);
}

namespace {

int64_t construct_affine_host(int kind, const anyseq_scoring& sc, const char* q, int n, const char* s, int m,
                              char* alq, char* als) {
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    hipStream_t st = E.stream;
    const size_t L = (size_t)n + (size_t)m;
    if (L == 0) return empty_score(kind, n, m, sc);
    uint8_t* dq = (uint8_t*)E.q.get((size_t)std::max(n, 1));
    uint8_t* ds = (uint8_t*)E.s.get((size_t)std::max(m, 1));
    if (n > 0) HIPCHECK(hipMemcpyAsync(dq, q, (size_t)n, hipMemcpyHostToDevice, st));
    if (m > 0) HIPCHECK(hipMemcpyAsync(ds, s, (size_t)m, hipMemcpyHostToDevice, st));
    uint8_t* d_alq = (uint8_t*)E.alq.get(L);
    uint8_t* d_als = (uint8_t*)E.als.get(L);
    const int64_t score = construct_affine_dev(E, kind, sc, dq, n, ds, m, d_alq, d_als, st);
    HIPCHECK(hipMemcpyAsync(alq, d_alq, L, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(als, d_als, L, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    return score;
}

// construct_*_alignment_fulltb: full-matrix predecessors + one walk (align.impala:190-216),
// global scheme for all three exports (export.impala:52,108,165).  Returns H[n-1][m-1].
int64_t construct_fulltb_host(const anyseq_scoring& sc, const char* q, int n, const char* s, int m, char* alq,
                              char* als) {
    if (sc.gap_open != 0) fail("fulltb: linear gaps only (the reference's traceback_full)");
    Engine& E = engine();
    std::lock_guard<std::mutex> lk(E.mu);
    hipStream_t st = E.stream;
    const size_t L = (size_t)n + (size_t)m;
    if (L == 0) return 0;
    const int nstrips = (m + 127) / 128;
    const size_t pred_bytes = (size_t)nstrips * (size_t)(n + 127) * 128;
    if (pred_bytes > ((size_t)16 << 30))
        fail("fulltb: %d x %d needs %.1f GB of predecessors (limit 16 GB; the reference's own limit is "
             "n*m < 2^31, use construct_* for long sequences)", n, m, pred_bytes / 1e9);
    uint8_t* dq = (uint8_t*)E.q.get((size_t)std::max(n, 1));
    uint8_t* ds = (uint8_t*)E.s.get((size_t)std::max(m, 1));
    if (n > 0) HIPCHECK(hipMemcpyAsync(dq, q, (size_t)n, hipMemcpyHostToDevice, st));
    if (m > 0) HIPCHECK(hipMemcpyAsync(ds, s, (size_t)m, hipMemcpyHostToDevice, st));
    uint8_t* d_pred = (uint8_t*)E.pred.get(std::max<size_t>(pred_bytes, 16));
    const size_t col_ints = (size_t)std::max(nstrips - 1, 1) * (size_t)std::max(n, 1);
    int32_t* cols = (int32_t*)E.outcol.get(col_ints * 4);
    HIPCHECK(hipMemsetAsync(cols, 0x80, col_ints * 4, st));
    uint32_t* ctr = (uint32_t*)E.fc.ctr.get(128) + 8;   // [0] ticket, [1] error word
    HIPCHECK(hipMemsetAsync(ctr, 0, 8, st));
    uint8_t* d_alq = (uint8_t*)E.alq.get(L);
    uint8_t* d_als = (uint8_t*)E.als.get(L);
    HIPCHECK(hipMemsetAsync(d_alq, ' ', L, st));
    HIPCHECK(hipMemsetAsync(d_als, ' ', L, st));
    HIPCHECK(anyseq_launch_fulltb(dq, n, ds, m, d_pred, cols, ctr, ctr + 1, sc.match, sc.mismatch, sc.gap_extend,
                                  d_alq, d_als, st));
    HIPCHECK(hipMemcpyAsync(alq, d_alq, L, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(als, d_als, L, hipMemcpyDeviceToHost, st));
    uint32_t err = 0;
    HIPCHECK(hipMemcpyAsync(&err, ctr + 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (err) fail("fulltb kernel reported error %u (spin timeout)", err);
    if (n <= 0 || m <= 0) return empty_score(KIND_GLOBAL, n, m, sc);
    return score_dev(E, KIND_GLOBAL, sc, dq, n, ds, m, st);
}

const anyseq_scoring kAbiScoring = {2, -1, 0, -1};  // linear_scoring_scheme(2,-1,-1)

// The caller's device buffers of one device-API call, registered for the pointer
// audit while the call runs.
struct ExternRanges {
    explicit ExternRanges(std::initializer_list<std::pair<const void*, size_t>> r) {
        for (const auto& x : r) register_extern_range(x.first, x.second);
    }
    ~ExternRanges() { clear_extern_ranges(); }
};

int64_t abi_score(int kind, const char* q, int n, const char* s, int m) {
    try {
        return score_host(kind, kAbiScoring, q, n, s, m);
    } catch (const Failure& f) {
        g_last_error = f.msg;
        fprintf(stderr, "anyseq: %s\n", f.msg.c_str());
        return INT64_MIN;
    }
}

int64_t abi_construct(int kind, const char* q, int n, const char* s, int m, char* alq, char* als) {
    try {
        construct_host(kind, kAbiScoring, q, n, s, m, alq, als);
        if (env_int("ANYSEQ_CONSTRUCT_TRUE_SCORE", 0)) return score_host(kind, kAbiScoring, q, n, s, m);
        // the reference's literal return (scoring object never relaxed)
        if (kind == KIND_GLOBAL) return (int64_t)n * kAbiScoring.gap_extend;
        if (kind == KIND_SEMIGLOBAL) return 0;
        return SCORE_MIN_VALUE;
    } catch (const Failure& f) {
        g_last_error = f.msg;
        fprintf(stderr, "anyseq: %s\n", f.msg.c_str());
        return INT64_MIN;
    }
}

}  // namespace
}  // namespace host
}  // namespace anyseq

using namespace anyseq::host;

// ======================================================================= ABI
extern "C" {

int64_t global_alignment_score(const char* query, int lenq, const char* subject, int lens) {
    return abi_score(KIND_GLOBAL, query, lenq, subject, lens);
}
int64_t semiglobal_alignment_score(const char* query, int lenq, const char* subject, int lens) {
    return abi_score(KIND_SEMIGLOBAL, query, lenq, subject, lens);
}
int64_t local_alignment_score(const char* query, int lenq, const char* subject, int lens) {
    return abi_score(KIND_LOCAL, query, lenq, subject, lens);
}
int64_t construct_global_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                   char* alSubject) {
    return abi_construct(KIND_GLOBAL, query, lenq, subject, lens, alQuery, alSubject);
}
int64_t construct_semiglobal_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                       char* alSubject) {
    return abi_construct(KIND_SEMIGLOBAL, query, lenq, subject, lens, alQuery, alSubject);
}
int64_t construct_local_alignment(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                  char* alSubject) {
    return abi_construct(KIND_LOCAL, query, lenq, subject, lens, alQuery, alSubject);
}

// The reference's undeclared *_fulltb exports (export.impala:37-53,93-109,150-166):
// all three run the GLOBAL scheme (export.impala:52,108,165) -- reproduced as is.
static int64_t abi_fulltb(const char* q, int n, const char* s, int m, char* alq, char* als) {
    try {
        return construct_fulltb_host(kAbiScoring, q, n, s, m, alq, als);
    } catch (const Failure& f) {
        g_last_error = f.msg;
        fprintf(stderr, "anyseq: %s\n", f.msg.c_str());
        return INT64_MIN;
    }
}
int64_t construct_global_alignment_fulltb(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                          char* alSubject) {
    return abi_fulltb(query, lenq, subject, lens, alQuery, alSubject);
}
int64_t construct_semiglobal_alignment_fulltb(const char* query, int lenq, const char* subject, int lens,
                                              char* alQuery, char* alSubject) {
    return abi_fulltb(query, lenq, subject, lens, alQuery, alSubject);
}
int64_t construct_local_alignment_fulltb(const char* query, int lenq, const char* subject, int lens, char* alQuery,
                                         char* alSubject) {
    return abi_fulltb(query, lenq, subject, lens, alQuery, alSubject);
}

int anyseq_score(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject, int lens,
                 int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : kAbiScoring;
        check_scoring(kind, s);
        check_value_range(s, lenq, lens);
        const int64_t v = score_host(kind, s, query, lenq, subject, lens);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        g_last_error = f.msg;
        return -1;
    }
}

int anyseq_score_device(int kind, const anyseq_scoring* sc, const uint8_t* d_query, int lenq, const uint8_t* d_subject,
                        int lens, void* stream, int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : kAbiScoring;
        check_scoring(kind, s);
        check_value_range(s, lenq, lens);
        Engine& E = engine();
        std::lock_guard<std::mutex> lk(E.mu);
        hipStream_t st = caller_stream(E, stream);
        ExternRanges xr({{d_query, (size_t)std::max(lenq, 0)}, {d_subject, (size_t)std::max(lens, 0)}});
        const int64_t v = score_dev(E, kind, s, d_query, lenq, d_subject, lens, st);
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        g_last_error = f.msg;
        return -1;
    }
}

// The extended API's construct: the build-defined true global / semiglobal / local
// construct for affine gaps, and for linear gaps under construct_mode 1 (the affine
// construct with gap open 0); else the reference's compat construct.
static bool true_construct(const anyseq_scoring& s) {
    if (s.gap_open != 0) return true;
    std::lock_guard<std::mutex> lk(g_engines_mu);
    init_tuning_locked();
    return g_tuning.ctrue != 0;
}

int anyseq_construct(int kind, const anyseq_scoring* sc, const char* query, int lenq, const char* subject, int lens,
                     char* alQuery, char* alSubject, int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : kAbiScoring;
        check_scoring(kind, s);
        check_value_range(s, lenq, lens);
        if (true_construct(s)) {   // build-defined affine construct (true global / semiglobal / local)
            const int64_t v = construct_affine_host(kind, s, query, lenq, subject, lens, alQuery, alSubject);
            if (score) *score = v;
            return 0;
        }
        construct_host(kind, s, query, lenq, subject, lens, alQuery, alSubject);
        if (score) *score = score_host(kind, s, query, lenq, subject, lens);
        return 0;
    } catch (const Failure& f) {
        g_last_error = f.msg;
        return -1;
    }
}

int anyseq_construct_device(int kind, const anyseq_scoring* sc, const uint8_t* d_query, int lenq,
                            const uint8_t* d_subject, int lens, uint8_t* d_alQuery, uint8_t* d_alSubject, void* stream,
                            int64_t* score) {
    try {
        const anyseq_scoring s = sc ? *sc : kAbiScoring;
        check_scoring(kind, s);
        check_value_range(s, lenq, lens);
        if (lenq < 0 || lens < 0) fail("negative sequence length");
        hstamp("entry");
        Engine& E = engine();
        std::lock_guard<std::mutex> lk(E.mu);
        hipStream_t st = caller_stream(E, stream);
        const size_t L = (size_t)std::max(lenq, 0) + (size_t)std::max(lens, 0);
        ExternRanges xr({{d_query, (size_t)std::max(lenq, 0)}, {d_subject, (size_t)std::max(lens, 0)},
                         {d_alQuery, L}, {d_alSubject, L}});
        int64_t v;
        hstamp("setup");
        if (true_construct(s)) {
            v = construct_affine_dev(E, kind, s, d_query, lenq, d_subject, lens, d_alQuery, d_alSubject, st);
        } else {
            construct_dev(E, kind, s, d_query, lenq, d_subject, lens, d_alQuery, d_alSubject, st);
            v = lenq > 0 && lens > 0 ? score_dev(E, kind, s, d_query, lenq, d_subject, lens, st)
                                     : empty_score(kind, lenq, lens, s);
        }
        HIPCHECK(hipStreamSynchronize(st));
        hstamp("sync");
        hstamp_print();
        if (score) *score = v;
        return 0;
    } catch (const Failure& f) {
        g_last_error = f.msg;
        return -1;
    }
}

int anyseq_set_device(int device) {
    std::lock_guard<std::mutex> lk(g_engines_mu);
    g_device = device;
    return 0;
}

int anyseq_get_device(void) { return g_device < 0 ? env_int("ANYSEQ_DEVICE", 0) : g_device; }

const char* anyseq_last_error(void) { return g_last_error.c_str(); }

void anyseq_set_tuning(int rows_per_lane, int waves_per_group, int grid) {
    std::lock_guard<std::mutex> lk(g_engines_mu);
    init_tuning_locked();
    if (rows_per_lane > 0) g_tuning.R = rows_per_lane;
    if (waves_per_group > 0) g_tuning.NW = waves_per_group;
    if (grid >= 0) g_tuning.grid = grid;
}

int anyseq_set_option(const char* name, int value) {
    std::lock_guard<std::mutex> lk(g_engines_mu);
    init_tuning_locked();
    const std::string n = name ? name : "";
    if (n == "rows_per_lane") g_tuning.R = value;
    else if (n == "chunk") g_tuning.CH = value == 16 ? 16 : 32;
    else if (n == "waves_per_group") g_tuning.NW = value;
    else if (n == "grid") g_tuning.grid = value;
    else if (n == "fronts") g_tuning.fronts = value;
    else if (n == "affine_waves_per_group") g_tuning.NWa = value;
    else if (n == "affine_rows_per_lane") g_tuning.arows = value;
    else if (n == "affine_self_forward") g_tuning.selffwd = value;
    else if (n == "linear_via_affine") g_tuning.linaff = value;
    else if (n == "linear_affine_loop") g_tuning.linloop = value;
    else if (n == "affine_io_first") g_tuning.iofirst = value;
    else if (n == "affine_force_border") g_tuning.forcelb = value;
    else if (n == "affine_grid") g_tuning.grida = value;
    else if (n == "affine_asm") g_tuning.affasm = value;
    else if (n == "ring_slots") g_tuning.ring_slots = value;
    else if (n == "affine_transpose") g_tuning.afft = value;
    else if (n == "priority") g_tuning.prio = value;
    else if (n == "throttle") g_tuning.thr = value;
    else if (n == "affine_lut") g_tuning.afflut = value;
    else if (n == "slack") g_tuning.slack = value;
    else if (n == "slack_io") g_tuning.slack_io = value;
    else if (n == "io_stage") g_tuning.io_stage = value;
    else if (n == "io_skew") g_tuning.io_skew = value;
    else if (n == "io_poll2") g_tuning.io_poll2 = value;
    else if (n == "io_forward") g_tuning.io_fwd = value;
    else if (n == "fill_events") g_tuning.fill_events = value;
    else if (n == "virtual_best") g_tuning.virtbest = value;
    else if (n == "affine_device_plan") g_tuning.devplan = value;
    else if (n == "affine_device_final") g_tuning.devfinal = value;
    else if (n == "plan_hw_queues") g_tuning.plan_queues = value;
    else if (n == "xcd_groups") g_tuning.xcdq = value;
    else if (n == "construct_mode") g_tuning.ctrue = value;
    else if (n == "inherit_halves") g_tuning.inherit = value;
    else if (n == "inherit_depth") g_tuning.inherit_depth = value;
    else return -1;
    return 0;
}

void anyseq_last_fill_timing(double* ms, int* launches) {
    anyseq_last_fill_stats(ms, launches, nullptr);
}

void anyseq_last_fill_stats(double* ms, int* launches, int64_t* cells) {
    if (ms) *ms = g_fill_ms;
    if (launches) *launches = g_fill_launches;
    if (cells) *cells = g_fill_cells;
    g_fill_ms = 0.0;
    g_fill_launches = 0;
    g_fill_cells = 0;
}

int64_t anyseq_last_inherit_stats(int64_t* reused) {
    const int64_t v = g_inherit_stats[0];
    if (reused) *reused = g_inherit_stats[1];
    g_inherit_stats[0] = g_inherit_stats[1] = 0;
    return v;
}

int anyseq_last_fill_multi_row_launches(int* max_rows) {
    const int v = g_fill_r2;
    if (max_rows) *max_rows = g_fill_rmax;
    g_fill_r2 = 0;
    g_fill_rmax = 1;
    return v;
}

int anyseq_last_shard_plan(void) {
    const int v = g_shard_blocked_levels;
    g_shard_blocked_levels = 0;
    return v;
}

void anyseq_main_random_pair(int64_t minlen, int64_t maxlen, char* query, int64_t* lenq, char* subject,
                             int64_t* lens) {
    // main.cpp:90-120 (uniform_ACGT_distribution, random_string) and :207-209
    std::mt19937_64 urng;
    auto gen = [&](char* out) -> int64_t {
        const size_t len = std::uniform_int_distribution<size_t>{(size_t)minlen, (size_t)maxlen}(urng);
        std::uniform_int_distribution<char> d{0, 3};
        static const char acgt[4] = {'A', 'C', 'G', 'T'};
        for (size_t i = 0; i < len; ++i) {
            const int r = d(urng);
            out[i] = (r >= 0 && r < 4) ? acgt[r] : '_';
        }
        return (int64_t)len;
    };
    *lenq = gen(query);
    *lens = gen(subject);
}

}  // extern "C"
