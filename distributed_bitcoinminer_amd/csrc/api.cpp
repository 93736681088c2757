// api.cpp -- the hipminer C ABI (include/hipminer.h).
//
// Replaces, inside the Go miner process, the scan of evalRoutine
// (cmu440/bitcoin/miner/miner.go:46-59) and bitcoin.Hash
// (cmu440/bitcoin/hash.go:13-17).  Per device and per call:
//
//   host:  plan_message (midstate) -> plan_range (digit segments, layouts)
//   GPU :  per segment, on one of kStreams HIP streams
//            [tiled]   hm_tile_plan_kernel -> counter reset -> hm_tiled_kernel
//            [chained] hm_kw_table_kernel, hm_tile_plan_kernel -> hm_chained_kernel
//            [generic] hm_generic_kernel
//          -> hm_fold_kernel (per-wave candidates -> per-stream best)
//          -> join streams -> hm_fold_kernel (stream bests -> 16-B result)
//   multi-device: contiguous shards, then either a host merge of the 16-B
//          results or an RCCL all-gather of them (HM_OPT_MERGE_RCCL).
//   The scan kernels come from their own code object (scan_kernels.hip ->
//   align_loops.py -> hipminer_scan.hsaco, embedded by scan_blob.S), loaded
//   per device with hipModuleLoadData and launched with hipModuleLaunchKernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hipminer.h"
#include "build_id.h"  // generated: HM_BUILD_ID (distributed_bitcoinminer_amd/build_id.py)
#include "kernels.hpp"
#include "plan.hpp"

using namespace hm;

// The scan kernels' code object (scan_blob.S .incbin of hipminer_scan.hsaco).
extern "C" const unsigned char hm_scan_code_object[];
extern "C" const unsigned char hm_scan_code_object_end[];

namespace {

constexpr int kStreams = 4;
// Requests of at most this many nonces (≈3.6 ms of work) run their digit
// segments concurrently on all streams; larger ones use the dominant-stream
// order with tail filling (enqueue_device_batch).
constexpr uint64_t kConcurrentNonces = 1ull << 27;
// Workgroups per CU of a fused (small-request) launch: fewer waves per SIMD
// than occupancy allows (6), so a task's wall time, and with it the launch's
// tail, is about halved at < 1 % of issue rate; first tasks handed out by
// wave slot (no opening burst of queue atomics).  Interleaved A/B over
// flags x grids: profiles/r05/fused/fused_ab.jsonl.
constexpr int kFusedPerCu = 3;
constexpr uint32_t kFusedDefaultFlags = kFusedStaticFirst;
constexpr uint32_t kFusedDefaultParts = 1;  // tiled fused tasks: one tens digit (10 steps)
// Tasks one queue atomic fetches for a workgroup (scan_tasks.hpp lds_dequeue,
// log2): 4, and 16 for launches of at least kBigLaunchNonces nonces
// (HM_OPT_QUEUE_BATCH; configs[3]'s d = 12 launch: 9e11 nonces, ~24 s).
constexpr uint32_t kQueueShift = 2;
constexpr uint32_t kQueueShiftBig = 4;
constexpr uint64_t kBigLaunchNonces = 100000000000ull;
// Guided tail of a fused launch (HM_OPT_FUSED_TAIL): the tasks of the last,
// partial wave-round are cut into up to this many pieces each.
constexpr uint32_t kFusedDefaultTail = 2;

// No C++ exception crosses the C ABI (include/hipminer.h): the entry points
// run their bodies through guarded(), which maps an escaping exception
// (std::bad_alloc from the planner's vectors, anything else) to a return code.
template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return HM_ERR_NOMEM;
    } catch (...) {
        return HM_ERR_INTERNAL;
    }
}

struct Launch {
    hipEvent_t start, stop;
    uint64_t nonces;
    int kind;
    int grid;
    uint32_t compressions;
    double comp_eff;  // compressions per nonce the kernel executes (hm_stats)
    char kernel[64];  // kernel instantiation, as rocprofv3 names it (sans args)
};

void name_tiled(char* out, const SegPlan& s, bool csum) {
    snprintf(out, 64, "%s<%d, %s, %s>", csum ? "hm_tiled_csum_kernel" : "hm_tiled_kernel", s.W1,
             s.straddle ? "true" : "false", s.trailer ? "true" : "false");
}

struct Device {
    int ordinal = -1;
    int cus = 0;
    int prio_hi = 0, prio_lo = 0;  // stream priorities (stream 0 / streams 1..)
    // streams (and their buffers) made so far: stream 0 at hm_open, streams
    // 1.. on the first call that enqueues onto them (make_streams).  Each HIP
    // stream holds a hardware queue until the process exits, and the GPU
    // time-slices once a process set holds more than ~20, so a
    // context that only ever runs fused requests, or HM_OPT_STREAMS = 2,
    // never creates the others.
    int nmade = 0;
    hipStream_t stream[kStreams] = {};
    uint32_t* rec[kStreams] = {};
    uint32_t* kwt[kStreams] = {};
    uint32_t* aux[kStreams] = {};      // fused launches: s0 / trailer / K+W tables
    uint64_t kwt_rows[kStreams] = {};  // rows allocated (grown on demand, kw_table_rows)
    std::vector<uint32_t*> retired;    // tables replaced by larger ones, freed at hm_close
    uint64_t* cand[kStreams] = {};
    unsigned int* counter[kStreams] = {};
    uint64_t* sums[kStreams] = {};  // checked scans: per-wave (sum, count) slots
    uint64_t* acc = nullptr;        // checked scans: [kStreams][2] (sum, count)
    uint64_t* best = nullptr;      // [kMaxBatch][kStreams][2]: per request, per stream
    uint64_t* result = nullptr;    // [kMaxBatch][2]
    uint64_t* gathered = nullptr;  // [ndev][kMaxBatch][2] (RCCL merge)
    uint64_t* trace = nullptr;     // HM_OPT_FUSED_TRACE: 4 x u64 per wave slot of a fused launch
    int trace_waves = 0;           // wave slots of the last traced fused launch
    hm_result* host_out = nullptr; // pinned, fine-grained [kMaxBatch]: the 16-B readback slots
    uint64_t* host_dev = nullptr;  // host_out as the device addresses it
    hipEvent_t join[kStreams] = {};
    hipEvent_t gate = nullptr;     // stream 0 reached its last dominant segment
    hipEvent_t t0 = nullptr;       // timing origin of the current call
    std::vector<hipEvent_t> evpool;
    size_t evnext = 0;
    std::vector<Launch> launches;
    ncclComm_t comm = nullptr;
    hipModule_t mod = nullptr;  // scan kernels (hipminer_scan.hsaco)
    struct Fn { std::string sym; hipFunction_t fn; int blocks_per_cu; };
    std::deque<Fn> fns;         // resolved on first use (stable addresses)
};

bool debug_on() {
    static const bool on = getenv("HM_DEBUG") != nullptr;
    return on;
}

int hip_fail(hipError_t e, const char* what) {
    if (debug_on()) fprintf(stderr, "hipminer: %s: %s\n", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? HM_ERR_NOMEM : HM_ERR_HIP;
}

#define HIPCHK(expr)                                   \
    do {                                               \
        hipError_t e_ = (expr);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

}  // namespace

struct hm_ctx {
    mutable std::mutex mu;
    std::vector<Device> devs;
    bool force_generic = false;
    bool merge_rccl = false;
    int grid_per_cu = 0;
    int streams = kStreams;  // HM_OPT_STREAMS (tail filling by default)
    int table_digits = 0;    // HM_OPT_TABLE_DIGITS (test hook; 0 = default, -1 = off)
    uint64_t table_rows_cap = 0;  // HM_OPT_TABLE_ROWS_CAP (test hook; 0 = off)
    bool test_mid_sync = false;   // HM_OPT_TEST_MID_SYNC (test hook: a host wait mid-enqueue)
    bool fused = true;            // HM_OPT_FUSED: small requests in one launch
    uint32_t fused_flags = kFusedDefaultFlags;  // HM_OPT_FUSED_FLAGS (experiment hook)
    uint32_t fused_parts = kFusedDefaultParts;  // HM_OPT_FUSED_PARTS (experiment hook)
    uint32_t fused_tail = kFusedDefaultTail;    // HM_OPT_FUSED_TAIL (1 = no split)
    bool tail_fused = true;  // HM_OPT_TAIL_FUSED: a large request's tail segments in one fused launch
    // HM_OPT_HOST_RESULT (experiment hook, off): results stored to pinned host
    // memory by the last fold instead of a 16-B copy -- measured no faster
    // (config 1: 0.3591 vs 0.3595 ms, profiles/r06/experiments/host_result/)
    bool host_result = false;
    int queue_batch = 0;     // HM_OPT_QUEUE_BATCH: 0 = auto, else tasks per queue atomic (4..32)
    bool fused_trace = false; // HM_OPT_FUSED_TRACE (diagnostics): fused waves record their timeline
    // host waits on GPU work while the call is still enqueuing (hm_stats.mid_call_syncs)
    bool enqueuing = false;
    int32_t mid_syncs = 0;
    int32_t table_grows = 0;
    double enqueue_ms = 0;
    bool csum = false;  // inside hm_scan_checked: checked kernels + coverage sums
    // HM_OPT_DEADLINE_MS: 0 = none (the host blocks until the GPU is done),
    // > 0 = that many ms per call, -1 = auto (deadline_for).  Past the
    // deadline a call returns HM_ERR_TIMEOUT and the context is abandoned:
    // its queued work may still run, so no later call touches its devices
    // and hm_close leaks them rather than wait (SURVEY §8(b) liveness).
    int64_t deadline_opt = 0;
    bool has_deadline = false;
    std::chrono::steady_clock::time_point deadline_at{};
    double deadline_ms = 0;  // the current call's deadline (hm_stats.deadline_ms)
    bool abandoned = false;
    bool have_stats = false;
    int merge = HM_MERGE_NONE;  // how the current call merged device results
    hm_stats last{};
};

namespace {

int next_event(Device& dv, hipEvent_t* ev) {
    if (dv.evnext == dv.evpool.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        dv.evpool.push_back(e);
    }
    *ev = dv.evpool[dv.evnext++];
    return HM_OK;
}

// Create streams nmade..n-1 of dv and their per-stream buffers (device
// current).  Stream 0 (the dominant kernel's segments, fused launches) runs
// at the highest priority, the others at the lowest: their workgroups only
// fill what the dominant persistent launch leaves free, i.e. its tail.
// Neither hipStreamCreate nor hipMalloc waits for queued work, so a call may
// make streams while it enqueues.
int make_streams(Device& dv, int n) {
    for (int s = dv.nmade; s < n && s < kStreams; ++s) {
        HIPCHK(hipStreamCreateWithPriority(&dv.stream[s], hipStreamNonBlocking,
                                           s == 0 ? dv.prio_hi : dv.prio_lo));
        HIPCHK(hipMalloc(&dv.rec[s], (size_t)kMaxTilesPerLaunch * kRecWords * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&dv.cand[s], (size_t)kMaxCandWaves * 2 * sizeof(uint64_t)));
        HIPCHK(hipMalloc(&dv.kwt[s], (size_t)kMaxChainedTable * 64 * sizeof(uint32_t)));
        dv.kwt_rows[s] = kMaxChainedTable;
        HIPCHK(hipMalloc(&dv.aux[s], (size_t)kFusedAuxWords * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&dv.counter[s], sizeof(unsigned int)));
        HIPCHK(hipMalloc(&dv.sums[s], (size_t)kMaxCandWaves * 2 * sizeof(uint64_t)));
        HIPCHK(hipEventCreateWithFlags(&dv.join[s], hipEventDisableTiming));
        dv.nmade = s + 1;
    }
    return HM_OK;
}

int device_init(Device& dv, int ordinal) {
    dv.ordinal = ordinal;
    HIPCHK(hipSetDevice(ordinal));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, ordinal));
    dv.cus = prop.multiProcessorCount;
    HIPCHK(hipDeviceGetStreamPriorityRange(&dv.prio_lo, &dv.prio_hi));
    HIPCHK(hipModuleLoadData(&dv.mod, hm_scan_code_object));
    int rc = make_streams(dv, 1);
    if (rc) return rc;
    HIPCHK(hipEventCreateWithFlags(&dv.gate, hipEventDisableTiming));
    HIPCHK(hipEventCreate(&dv.t0));
    HIPCHK(hipMalloc(&dv.best, (size_t)kMaxBatch * kStreams * 2 * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&dv.acc, (size_t)kStreams * 2 * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&dv.result, (size_t)kMaxBatch * 2 * sizeof(uint64_t)));
    // fine-grained (coherent) pinned memory: the last fold kernel of a call
    // stores the results here with system-scope stores (HM_OPT_HOST_RESULT)
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&dv.host_out), kMaxBatch * sizeof(hm_result),
                         hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dv.host_dev), dv.host_out, 0));
    return HM_OK;
}

void device_free(Device& dv) {
    if (dv.ordinal < 0) return;
    (void)hipSetDevice(dv.ordinal);
    for (int s = 0; s < kStreams; ++s) {
        if (dv.stream[s]) (void)hipStreamSynchronize(dv.stream[s]);
    }
    if (dv.comm) ncclCommDestroy(dv.comm);
    for (int s = 0; s < kStreams; ++s) {
        if (dv.rec[s]) (void)hipFree(dv.rec[s]);
        if (dv.cand[s]) (void)hipFree(dv.cand[s]);
        if (dv.kwt[s]) (void)hipFree(dv.kwt[s]);
        if (dv.aux[s]) (void)hipFree(dv.aux[s]);
        if (dv.counter[s]) (void)hipFree(dv.counter[s]);
        if (dv.sums[s]) (void)hipFree(dv.sums[s]);
        if (dv.join[s]) (void)hipEventDestroy(dv.join[s]);
        if (s == 0 && dv.gate) (void)hipEventDestroy(dv.gate);
        if (s == 0 && dv.t0) (void)hipEventDestroy(dv.t0);
        if (dv.stream[s]) (void)hipStreamDestroy(dv.stream[s]);
    }
    for (uint32_t* t : dv.retired) (void)hipFree(t);
    dv.retired.clear();
    for (hipEvent_t e : dv.evpool) (void)hipEventDestroy(e);
    if (dv.mod) (void)hipModuleUnload(dv.mod);
    dv.fns.clear();
    if (dv.best) (void)hipFree(dv.best);
    if (dv.acc) (void)hipFree(dv.acc);
    if (dv.result) (void)hipFree(dv.result);
    if (dv.gathered) (void)hipFree(dv.gathered);
    if (dv.trace) (void)hipFree(dv.trace);
    if (dv.host_out) (void)hipHostFree(dv.host_out);
    dv.ordinal = -1;
}

// Mangled names of the scan kernels in hipminer_scan.hsaco (scan_kernels.hip).
std::string tiled_symbol(const SegPlan& s, bool csum) {
    char b[128];
    snprintf(b, sizeof b, "_ZN2hm%s_kernelILi%dELb%dELb%dEEEvNS_9TiledArgsE",
             csum ? "20hm_tiled_csum" : "15hm_tiled", s.W1, s.straddle ? 1 : 0,
             s.trailer ? 1 : 0);
    return b;
}
const char* chained_symbol(bool csum) {
    return csum ? "_ZN2hm22hm_chained_csum_kernelENS_11ChainedArgsE"
                : "_ZN2hm17hm_chained_kernelENS_11ChainedArgsE";
}
const char* fused_symbol(bool csum) {
    return csum ? "_ZN2hm20hm_fused_csum_kernelENS_9FusedArgsE"
                : "_ZN2hm15hm_fused_kernelENS_9FusedArgsE";
}
const char* generic_symbol(bool csum) {
    return csum ? "_ZN2hm22hm_generic_csum_kernelENS_11GenericArgsE"
                : "_ZN2hm17hm_generic_kernelENS_11GenericArgsE";
}

// Resolve a scan kernel of dv's module (cached with its occupancy).
int scan_fn(Device& dv, const std::string& sym, const Device::Fn** out) {
    for (const auto& f : dv.fns)
        if (f.sym == sym) { *out = &f; return HM_OK; }
    Device::Fn f{sym, nullptr, 0};
    HIPCHK(hipModuleGetFunction(&f.fn, dv.mod, sym.c_str()));
    HIPCHK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&f.blocks_per_cu, f.fn, kBlock, 0));
    dv.fns.push_back(f);
    *out = &dv.fns.back();
    return HM_OK;
}

// Launch a scan kernel with its argument block (the kernel's only, by-value
// parameter) on `grid` workgroups of kBlock threads.
template <typename Args>
int launch_scan(const Device::Fn& f, const Args& args, int grid, hipStream_t st) {
    if (grid < 1 || (uint32_t)grid * (kBlock / kWaveSize) > kMaxCandWaves)
        return hip_fail(hipErrorInvalidValue, "scan grid");
    size_t size = sizeof(Args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, const_cast<Args*>(&args),
                   HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    HIPCHK(hipModuleLaunchKernel(f.fn, (unsigned)grid, 1, 1, kBlock, 1, 1, 0, st, nullptr, cfg));
    return HM_OK;
}

// log2 of the tasks per queue atomic of a per-segment launch over `nonces`.
uint32_t queue_shift(const hm_ctx* ctx, uint64_t nonces) {
    if (ctx->queue_batch > 0) return (uint32_t)__builtin_ctz((unsigned)ctx->queue_batch);
    return nonces >= kBigLaunchNonces ? kQueueShiftBig : kQueueShift;
}

uint32_t count_compressions(const SegPlan& s) {
    // SHA-256 compressions per nonce after the host midstate (SURVEY §8d "C").
    return s.nb;
}

// Compressions per nonce the segment's scan kernel executes: the algorithmic
// C minus what is hoisted out of the per-nonce loop (hm_stats.dom_compressions_eff).
// The chained kernel's launches count their block-0 compressions exactly
// (one per task and lane, enqueue_chained), guided-split pieces included.
double executed_compressions(const SegPlan& s) {
    switch (s.kind) {
        case HM_KIND_TILED:  // a two-block tail's block 0 is compressed per tile by the planner
            return s.trailer ? 2.0 : 1.0;
        default:
            return (double)s.nb;
    }
}

int persistent_grid(const hm_ctx* ctx, const Device& dv, int per_cu_auto, uint64_t ntasks) {
    int per_cu = ctx->grid_per_cu > 0 ? ctx->grid_per_cu : per_cu_auto;
    if (per_cu <= 0) per_cu = 1;
    uint64_t grid = (uint64_t)per_cu * (uint64_t)dv.cus;
    const uint64_t waves_per_block = kBlock / kWaveSize;
    grid = std::min<uint64_t>(grid, (ntasks + waves_per_block - 1) / waves_per_block);
    grid = std::min<uint64_t>(grid, kMaxCandWaves / waves_per_block);
    return (int)std::max<uint64_t>(grid, 1);
}

// Guided task list of a persistent launch over `nunits` work units: the
// last ~one unit per wave of the grid is split into kSplit tasks.  Returns
// the task-id count; *nbig = units dequeued whole.
uint32_t guided_tasks(uint64_t nunits, int grid, uint32_t* nbig) {
    const uint64_t waves = (uint64_t)grid * (kBlock / kWaveSize);
    const uint64_t small = std::min<uint64_t>(nunits, waves);
    *nbig = (uint32_t)(nunits - small);
    return (uint32_t)(nunits - small + kSplit * small);
}

// Grid and guided task list of a persistent launch over `nunits` units: the
// split is planned against the occupancy-sized grid, then the grid is cut to
// the task count (one wave per task at most).  A launch with fewer units than
// the GPU has waves splits every unit, and sizing its grid by tasks rather
// than units gives each task its own wave: a segment of 10^4..10^7 nonces is
// latency-bound (one wave runs its tasks' SHA chains back to back), so this
// cuts such launches from ≈270-390 µs to tens of µs (config 1's request).
int plan_launch(const hm_ctx* ctx, const Device& dv, int per_cu_auto, uint64_t nunits,
                uint32_t* ntasks, uint32_t* nbig) {
    const int cap = persistent_grid(ctx, dv, per_cu_auto, 1ull << 40);  // occupancy-sized
    *ntasks = guided_tasks(nunits, cap, nbig);
    return persistent_grid(ctx, dv, per_cu_auto, *ntasks);
}

// Units of a launch over tiles [t, t+nt) (unit = lane chunk x `per_chunk`
// loop chunks; lane value v of a tile covers nonces base + v*step + [0, step)):
// the lane chunks of the first tile wholly below s.lo and of the last tile
// wholly above s.hi are skipped, so shards and segments that start or end
// inside a tile hash no out-of-range nonces beyond their edge chunks.
// *unit0 = the first unit kept, *nunits = the count kept.
void launch_units(const SegPlan& s, uint64_t t, uint64_t nt, uint64_t per_chunk, uint64_t step,
                  uint32_t* unit0, uint64_t* nunits) {
    const uint64_t P = s.pow10V;
    const uint64_t per_tile = (uint64_t)s.tpt * per_chunk;
    uint64_t first = 0, last = nt * per_tile - 1;
    const uint64_t b0 = t * P;  // <= s.hi: every tile of the launch meets [lo, hi]
    if (s.lo > b0) first = (s.lo - b0) / step / kWaveSize * per_chunk;
    const uint64_t bl = (t + nt - 1) * P;
    if (s.hi - bl < P - 1)
        last = (nt - 1) * per_tile + ((s.hi - bl) / step / kWaveSize + 1) * per_chunk - 1;
    *unit0 = (uint32_t)first;
    *nunits = last - first + 1;
}

// nonces of [t*P, (t+nt)*P - 1] ∩ [lo, hi] (P = nonces per tile)
uint64_t tile_span_nonces(const SegPlan& s, uint64_t t, uint64_t nt) {
    const uint64_t a = std::max(s.lo, t * s.pow10V);
    const bool wraps = (t + nt) > (~0ull) / s.pow10V;
    const uint64_t b = wraps ? s.hi : std::min(s.hi, (t + nt) * s.pow10V - 1);
    return b - a + 1;
}

// The host-blocking HIP calls of a scan call -- a stream wait and a
// synchronous readback -- go through these two helpers and nowhere else
// (device_free at hm_close is outside any call; tests/test_abi.py checks the
// sources for stray ones).  Each counts in hm_stats.mid_call_syncs when the
// call is still enqueuing work (on this or a later device): such a wait would
// hold back every launch after it.  No enqueue path calls them
// (HM_OPT_TEST_MID_SYNC makes one, so tests can see the counter work).  The
// enqueue path's only other host calls that are not async launches, event
// records or memsets are hipMalloc of a grown K+W table (hm_stats.table_grows)
// and of a context's streams 1.. on first use (make_streams), neither of
// which waits for queued work (tests/test_gpu_enqueue.py bounds enqueue_ms
// against the call's wall).  The library never calls hipFree during a call:
// it waits for the whole device, other contexts' work included.
//
// With a deadline (HM_OPT_DEADLINE_MS) the stream wait polls hipStreamQuery
// instead of blocking: spinning (yield) for the first 2 ms, then sleeping
// 100 us between queries.  Past the deadline it abandons the context and
// returns HM_ERR_TIMEOUT, so a hung or starved GPU scan cannot hold a miner
// whose LSP thread keeps heartbeating (lsp_client.cpp) -- the server would
// never reassign its chunk (server.go:326-376).
int host_wait(hm_ctx* ctx, hipStream_t st) {
    if (ctx->enqueuing) ++ctx->mid_syncs;
    if (!ctx->has_deadline) {
        HIPCHK(hipStreamSynchronize(st));
        return HM_OK;
    }
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return HM_OK;
        if (e != hipErrorNotReady) return hip_fail(e, "hipStreamQuery");
        const auto now = clk::now();
        if (now >= ctx->deadline_at) {
            ctx->abandoned = true;
            if (debug_on())
                fprintf(stderr, "hipminer: scan deadline of %.1f ms passed: context abandoned\n",
                        ctx->deadline_ms);
            return HM_ERR_TIMEOUT;
        }
        if (now - t0 < std::chrono::milliseconds(2)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}
int host_read(hm_ctx* ctx, void* dst, const void* src, size_t n) {
    if (ctx->enqueuing) ++ctx->mid_syncs;
    HIPCHK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
    return HM_OK;
}

// Make stream si's K+W table hold `rows` rows.  Grown once to the largest
// table used so far (10^5 .. 10^7 rows, up to 2.56 GB, for final blocks of
// >= 5 digits).  Work queued earlier on the stream may still read the old
// table, and hipFree would wait for the whole device (other contexts' work
// too), so the old table is retired and freed at hm_close.  Rows are powers
// of ten, so all tables a stream retires together hold < 1/9 of its current
// one (at most 0.28 GB beside a 2.56-GB table).
// Returns HM_ERR_NOMEM (with HIP's error state cleared, the old table kept)
// when the device cannot hold the table, or the HM_OPT_TABLE_ROWS_CAP test
// hook refuses it; the caller then plans smaller tables.
int kw_table_rows(hm_ctx* ctx, Device& dv, int si, uint64_t rows) {
    if (rows <= dv.kwt_rows[si]) return HM_OK;
    if (ctx->table_rows_cap && rows > ctx->table_rows_cap) return HM_ERR_NOMEM;
    uint32_t* t = nullptr;
    if (hipMalloc(&t, (size_t)rows * 64 * sizeof(uint32_t)) != hipSuccess) {
        (void)hipGetLastError();
        return HM_ERR_NOMEM;
    }
    if (dv.kwt[si]) dv.retired.push_back(dv.kwt[si]);
    dv.kwt[si] = t;
    dv.kwt_rows[si] = rows;
    ++ctx->table_grows;
    return HM_OK;
}

// One chained launch: tiles [t, t + nt) of segment s in epoch e (final-block
// values e * nloop + [0, nloop), K+W table already built on stream si).
int launch_chained_tiles(hm_ctx* ctx, Device& dv, const MsgPlan& mp, const SegPlan& s, int si,
                         uint64_t* best, uint64_t t, uint64_t nt, uint64_t e, uint64_t nep) {
    hipStream_t st = dv.stream[si];
    const uint64_t nloop = pow10_u64(s.fe);
    PlanArgs pa;
    pa.rec = dv.rec[si];
    pa.tile0 = t;
    pa.pow10V = s.pow10V;
    pa.total_bits = s.total_bits;
    pa.ntiles = (uint32_t)nt;
    pa.V = s.V;
    pa.d = s.d;
    pa.r = mp.r;
    pa.fb = 0;  // keep tail block 0 raw; its compression is per lane
    pa.nb = s.nb;
    memcpy(pa.pw, mp.pw, sizeof pa.pw);
    memcpy(pa.mid, mp.mid, sizeof pa.mid);
    HIPCHK(launch_tile_plan(pa, st));
    ChainedArgs ca;
    ca.rec = dv.rec[si];
    ca.kwt = dv.kwt[si];
    ca.counter = dv.counter[si];
    ca.cand = dv.cand[si];
    ca.sums = ctx->csum ? dv.sums[si] : nullptr;
    ca.tile0 = t;
    ca.pow10qf = s.pow10V;
    ca.pow10f = pow10_u64(s.f);
    ca.ebase = e * nloop;
    ca.nloop = (uint32_t)nloop;
    ca.seg_lo = s.lo;
    ca.seg_hi = s.hi;
    uint32_t unit0;
    uint64_t nunits;
    launch_units(s, t, nt, s.ntc, pow10_u64(s.f), &unit0, &nunits);
    ca.tpt = s.tpt;
    ca.ntc = s.ntc;
    ca.tch = s.tch;
    ca.vmax = (uint32_t)(pow10_u64(s.q) - 1);
    ca.q = s.q;
    ca.lds_shift = queue_shift(ctx, tile_span_nonces(s, t, nt) / nep);
    const Device::Fn* fn = nullptr;
    int rc = scan_fn(dv, chained_symbol(ctx->csum), &fn);
    if (rc) return rc;
    const int grid = plan_launch(ctx, dv, fn->blocks_per_cu, nunits, &ca.ntasks, &ca.nbig);
    // every task compresses its lanes' tail block 0 once; the final block
    // runs once per lane and loop value: nunits * tch values per lane
    const double block0_per_value = (double)ca.ntasks / ((double)nunits * (double)s.tch);
    // task ids start at unit0 (the queue counter too): the kernels map a
    // task below nbig to that unit, so the skipped units are never dequeued
    ca.ntasks += unit0;
    ca.nbig += unit0;
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)dv.counter[si], (int)unit0, 1, st));
    Launch L;
    rc = next_event(dv, &L.start);
    if (rc) return rc;
    rc = next_event(dv, &L.stop);
    if (rc) return rc;
    // the epochs split every lane value's nonces evenly (stats only)
    const uint64_t span = tile_span_nonces(s, t, nt);
    L.nonces = span / nep + (e + 1 == nep ? span % nep : 0);
    L.kind = HM_KIND_CHAINED;
    snprintf(L.kernel, sizeof L.kernel, ctx->csum ? "hm_chained_csum_kernel" : "hm_chained_kernel");
    L.grid = grid;
    L.compressions = count_compressions(s);
    L.comp_eff = 1.0 + block0_per_value;
    HIPCHK(hipEventRecord(L.start, st));
    rc = launch_scan(*fn, ca, grid, st);
    if (rc) return rc;
    HIPCHK(hipEventRecord(L.stop, st));
    HIPCHK(launch_fold(dv.cand[si], (uint32_t)grid * (kBlock / kWaveSize), best + 2 * si, st));
    if (ctx->csum)
        HIPCHK(launch_sum_fold(dv.sums[si], (uint32_t)grid * (kBlock / kWaveSize),
                               dv.acc + 2 * si, st));
    dv.launches.push_back(L);
    return HM_OK;
}

int enqueue_chained(hm_ctx* ctx, Device& dv, const MsgPlan& mp, const SegPlan& plan, int si,
                    uint64_t* best) {
    if (plan.fe < 1 || plan.fe > kMaxTableDigits || plan.fe > plan.f) return HM_ERR_INTERNAL;
    // a device short of memory for the planned table gets smaller tables and
    // more epochs: the same nonces on the same kernel, more launches
    SegPlan s = plan;
    int rc;
    while ((rc = kw_table_rows(ctx, dv, si, pow10_u64(s.fe))) == HM_ERR_NOMEM && s.fe > 1) {
        --s.fe;
        s.tch = (uint32_t)std::min<uint64_t>(s.tch, pow10_u64(s.fe));
        s.ntc = (uint32_t)(pow10_u64(s.fe) / s.tch);
    }
    if (rc) return rc;
    const uint64_t nloop = pow10_u64(s.fe);       // table rows = loop values per lane
    const uint64_t nep = pow10_u64(s.f - s.fe);   // epochs: the final block's high digits
    const uint64_t per_tile = (uint64_t)s.tpt * s.ntc;
    const uint64_t max_tiles = std::min<uint64_t>(kMaxTilesPerLaunch, 0x7fffffffull / per_tile);
    for (uint64_t e = 0; e < nep; ++e) {
        HIPCHK(launch_kw_table(dv.kwt[si], s.f, s.fe, e * nloop, s.total_bits, dv.stream[si]));
        for (uint64_t t = s.tile_lo; t <= s.tile_hi;) {
            const uint64_t nt = std::min<uint64_t>(max_tiles, s.tile_hi - t + 1);
            rc = launch_chained_tiles(ctx, dv, mp, s, si, best, t, nt, e, nep);
            if (rc) return rc;
            t += nt;
            if (t == 0) break;
        }
    }
    return HM_OK;
}

// Enqueue one segment on stream `si`; records its launches for stats.
// `best` = the request's [kStreams][2] running bests; this stream folds into best + 2*si.
int enqueue_segment(hm_ctx* ctx, Device& dv, const MsgPlan& mp, const SegPlan& s, int si,
                    uint64_t* best) {
    hipStream_t st = dv.stream[si];
    if (s.kind == HM_KIND_CHAINED) return enqueue_chained(ctx, dv, mp, s, si, best);
    if (s.kind == HM_KIND_TILED) {
        uint32_t kw[64] = {0};
        if (s.trailer) trailer_kw(s, kw);
        const uint64_t max_tiles =
            std::min<uint64_t>(kMaxTilesPerLaunch, (uint64_t)0x7fffffffu / s.tpt);
        for (uint64_t t = s.tile_lo; t <= s.tile_hi;) {
            const uint64_t nt = std::min<uint64_t>(max_tiles, s.tile_hi - t + 1);
            PlanArgs pa;
            pa.rec = dv.rec[si];
            pa.tile0 = t;
            pa.pow10V = s.pow10V;
            pa.total_bits = s.total_bits;
            pa.ntiles = (uint32_t)nt;
            pa.V = s.V;
            pa.d = s.d;
            pa.r = mp.r;
            pa.fb = s.fb;
            pa.nb = s.nb;
            memcpy(pa.pw, mp.pw, sizeof pa.pw);
            memcpy(pa.mid, mp.mid, sizeof pa.mid);
            HIPCHK(launch_tile_plan(pa, st));
            TiledArgs ta;
            ta.rec = dv.rec[si];
            ta.counter = dv.counter[si];
            ta.cand = dv.cand[si];
            ta.sums = ctx->csum ? dv.sums[si] : nullptr;
            ta.tile0 = t;
            ta.pow10V = s.pow10V;
            ta.seg_lo = s.lo;
            ta.seg_hi = s.hi;
            uint32_t unit0;
            uint64_t nunits;
            launch_units(s, t, nt, 1, 100, &unit0, &nunits);
            ta.tpt = s.tpt;
            ta.vmax = (uint32_t)(pow10_u64(s.q) - 1);
            ta.q = s.q;
            ta.lane_shift = s.lane_shift;
            ta.loop_shift = s.loop_shift;
            ta.lds_shift = queue_shift(ctx, tile_span_nonces(s, t, nt));
            memcpy(ta.trailer_kw, kw, sizeof kw);
            tiled_loop_sigma0(s, ta.s0_loop);
            const Device::Fn* fn = nullptr;
            int rc = scan_fn(dv, tiled_symbol(s, ctx->csum), &fn);
            if (rc) return rc;
            const int grid = plan_launch(ctx, dv, fn->blocks_per_cu, nunits, &ta.ntasks, &ta.nbig);
            ta.ntasks += unit0;  // see enqueue_chained
            ta.nbig += unit0;
            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)dv.counter[si], (int)unit0, 1, st));
            Launch L;
            rc = next_event(dv, &L.start);
            if (rc) return rc;
            rc = next_event(dv, &L.stop);
            if (rc) return rc;
            L.nonces = tile_span_nonces(s, t, nt);
            L.kind = HM_KIND_TILED;
            name_tiled(L.kernel, s, ctx->csum);
            L.grid = grid;
            L.compressions = count_compressions(s);
            L.comp_eff = executed_compressions(s);
            HIPCHK(hipEventRecord(L.start, st));
            rc = launch_scan(*fn, ta, grid, st);
            if (rc) return rc;
            HIPCHK(hipEventRecord(L.stop, st));
            HIPCHK(launch_fold(dv.cand[si], (uint32_t)grid * (kBlock / kWaveSize),
                               best + 2 * si, st));
            if (ctx->csum)
                HIPCHK(launch_sum_fold(dv.sums[si], (uint32_t)grid * (kBlock / kWaveSize),
                                       dv.acc + 2 * si, st));
            dv.launches.push_back(L);
            t += nt;
            if (t == 0) break;  // tile index wrapped (cannot happen for d <= 20)
        }
        return HM_OK;
    }
    // generic
    GenericArgs ga;
    ga.cand = dv.cand[si];
    ga.sums = ctx->csum ? dv.sums[si] : nullptr;
    ga.seg_lo = s.lo;
    ga.count_m1 = s.hi - s.lo;
    ga.total_bits = s.total_bits;
    ga.d = s.d;
    ga.r = mp.r;
    ga.nb = s.nb;
    memcpy(ga.pw, mp.pw, sizeof ga.pw);
    memcpy(ga.mid, mp.mid, sizeof ga.mid);
    const uint64_t need = ga.count_m1 / kBlock + 1;
    const uint64_t cap = (uint64_t)(kMaxCandWaves / (kBlock / kWaveSize));
    const int grid = (int)std::min<uint64_t>(need, std::min<uint64_t>(cap, (uint64_t)dv.cus * 8));
    const Device::Fn* fn = nullptr;
    int rc = scan_fn(dv, generic_symbol(ctx->csum), &fn);
    if (rc) return rc;
    Launch L;
    rc = next_event(dv, &L.start);
    if (rc) return rc;
    rc = next_event(dv, &L.stop);
    if (rc) return rc;
    L.nonces = ga.count_m1 + 1;  // generic segments are far below 2^64
    L.kind = HM_KIND_GENERIC;
    snprintf(L.kernel, sizeof L.kernel, ctx->csum ? "hm_generic_csum_kernel" : "hm_generic_kernel");
    L.grid = grid;
    L.compressions = count_compressions(s);
    L.comp_eff = executed_compressions(s);
    HIPCHK(hipEventRecord(L.start, st));
    rc = launch_scan(*fn, ga, grid, st);
    if (rc) return rc;
    HIPCHK(hipEventRecord(L.stop, st));
    HIPCHK(launch_fold(dv.cand[si], (uint32_t)grid * (kBlock / kWaveSize), best + 2 * si, st));
    if (ctx->csum)
        HIPCHK(launch_sum_fold(dv.sums[si], (uint32_t)grid * (kBlock / kWaveSize),
                               dv.acc + 2 * si, st));
    dv.launches.push_back(L);
    return HM_OK;
}

// Fused launch (kernels.hpp, fused_kernels.hip): can all of a request's
// segments run in one launch?  Up to kFusedNonces nonces and 20 segments;
// tiled and generic segments always, chained ones with one table of f <= 4
// digits (no epochs) whose rows fit the stream's aux buffer.
bool fusible(const std::vector<SegPlan>& segs) {
    if (segs.empty() || segs.size() > (size_t)kMaxFusedSegs) return false;
    long double n = 0;
    uint64_t rows = 0, tiles = 0;
    for (const auto& g : segs) {
        n += (long double)(g.hi - g.lo) + 1;
        if (g.kind == HM_KIND_CHAINED) {
            if (g.f > kMaxChainedF || g.fe != g.f) return false;
            rows += pow10_u64(g.f);
        }
        if (g.kind != HM_KIND_GENERIC) tiles += g.tile_hi - g.tile_lo + 1;
    }
    return n <= (long double)kFusedNonces && rows <= kFusedKwRows && tiles <= kMaxTilesPerLaunch;
}

// Per-task cost rank of a segment's layout in the fused launch: the queue
// hands out the costly tasks first, so the launch ends on the cheapest ones.
int fused_rank(const SegPlan& g) {
    if (g.kind == HM_KIND_CHAINED) return 0;   // 64 lanes x up to 100 blocks
    if (g.kind == HM_KIND_GENERIC) return 1;   // 640 nonces, full tail compressions
    return g.trailer ? 2 : 3;                  // 640 nonces, 2 or 1 compressions
}

// Enqueue every segment of one request as ONE fused launch on stream si:
// hm_fused_plan_kernel (records, tables, counter; and, when `seed_best`, the
// (MaxUint64, 0) seed of *best and zeroed coverage sums) -> hm_fused_kernel
// -> hm_fold_kernel into *best.  Tasks are ordered costliest layout first,
// larger segments first.
int enqueue_fused(hm_ctx* ctx, Device& dv, const MsgPlan& mp, std::vector<SegPlan> segs, int si,
                  uint64_t* best, bool seed_best, uint64_t* host = nullptr) {
    hipStream_t st = dv.stream[si];
    std::stable_sort(segs.begin(), segs.end(), [](const SegPlan& a, const SegPlan& b) {
        if (fused_rank(a) != fused_rank(b)) return fused_rank(a) < fused_rank(b);
        return a.hi - a.lo > b.hi - b.lo;
    });
    FusedPlanArgs pa;
    memset(&pa, 0, sizeof pa);
    FusedArgs fa;
    memset(&fa, 0, sizeof fa);
    pa.rec = dv.rec[si];
    pa.aux = dv.aux[si];
    pa.counter = dv.counter[si];
    pa.result = seed_best ? best : nullptr;
    // a lone request (seed_best) also zeroes every stream's coverage sums,
    // which hm_scan_checked adds up; in a batch they were zeroed up front
    // and hold the other requests' sums
    pa.acc = ctx->csum && seed_best ? dv.acc : nullptr;
    pa.n_acc = 2 * kStreams;
    pa.r = mp.r;
    memcpy(pa.pw, mp.pw, sizeof pa.pw);
    memcpy(pa.mid, mp.mid, sizeof pa.mid);
    fa.rec = dv.rec[si];
    fa.aux = dv.aux[si];
    fa.counter = dv.counter[si];
    fa.cand = dv.cand[si];
    fa.sums = ctx->csum ? dv.sums[si] : nullptr;
    fa.r = mp.r;
    memcpy(fa.pw, mp.pw, sizeof fa.pw);
    memcpy(fa.mid, mp.mid, sizeof fa.mid);
    uint64_t tasks = 0, jobs = 0, nonces = 0;
    uint32_t rec_next = 0, aux_next = 0, comp_max = 1;
    std::vector<double> ce_base(segs.size()), seg_units(segs.size());  // chained C_eff inputs
    std::vector<uint64_t> seg_cnt(segs.size());
    for (size_t i = 0; i < segs.size(); ++i) {
        const SegPlan& g = segs[i];
        FusedSeg& S = fa.segs[i];
        FusedPlanSeg& P = pa.segs[i];
        const uint64_t cnt = g.hi - g.lo + 1;  // one digit count: far below 2^64
        S.seg_lo = g.lo;
        S.seg_hi = g.hi;
        S.total_bits = g.total_bits;
        S.d = g.d;
        S.nb = g.nb;
        P.total_bits = g.total_bits;
        P.d = g.d;
        P.nb = g.nb;
        P.T = g.T;
        P.V = g.V;
        P.straddle = g.straddle;
        P.loop_shift = g.loop_shift;
        P.f = g.f;
        uint64_t seg_tasks = 0, seg_jobs = 0;
        double ce = (double)g.nb;
        if (g.kind == HM_KIND_TILED || g.kind == HM_KIND_CHAINED) {
            const bool ch = g.kind == HM_KIND_CHAINED;
            const uint64_t nt = g.tile_hi - g.tile_lo + 1;
            uint32_t unit0;
            uint64_t nunits;
            launch_units(g, g.tile_lo, nt, ch ? g.ntc : 1, ch ? pow10_u64(g.f) : 100, &unit0, &nunits);
            S.tile0 = P.tile0 = g.tile_lo;
            S.pow10V = P.pow10V = g.pow10V;
            S.rec0 = P.rec0 = rec_next;
            S.aux0 = P.aux0 = aux_next;
            S.unit0 = unit0;
            S.tpt = g.tpt;
            S.vmax = (uint32_t)(pow10_u64(g.q) - 1);
            S.q = g.q;
            P.ntiles = (uint32_t)nt;
            rec_next += (uint32_t)nt;
            if (ch) {
                S.variant = P.variant = kVarChained;
                S.pow10f = pow10_u64(g.f);
                S.ntc = g.ntc;
                S.tch = g.tch;
                S.tpu = (g.tch + kFusedChainedPiece - 1) / kFusedChainedPiece;
                P.fb = 0;  // tail block 0 kept raw: its compression is per lane
                seg_tasks = nunits * S.tpu;
                seg_jobs = nt + pow10_u64(g.f);
                aux_next += (uint32_t)pow10_u64(g.f) * 64;
                // 1 + block-0 compressions per loop value: one per task (and
                // per guided-tail piece, added below)
                ce = 1.0;
                seg_units[i] = (double)nunits * (double)g.tch;
            } else {
                S.variant = P.variant = (uint32_t)(g.W1 * 4 + (g.straddle ? 2 : 0) + (g.trailer ? 1 : 0));
                S.lane_shift = g.lane_shift;
                S.loop_shift = g.loop_shift;
                S.tpu = ctx->fused_parts;
                P.fb = g.fb;
                seg_tasks = nunits * 10 * ctx->fused_parts;
                seg_jobs = nt + 100 + (g.trailer ? 1 : 0);
                aux_next += 100 + (g.trailer ? 64 : 0);
                ce = executed_compressions(g);
            }
        } else {
            S.variant = P.variant = kVarGeneric;
            seg_tasks = (cnt + 639) / 640;
        }
        tasks += seg_tasks;
        jobs += seg_jobs;
        S.task_end = (uint32_t)tasks;
        P.job_end = (uint32_t)jobs;
        nonces += cnt;
        comp_max = std::max(comp_max, g.nb);
        ce_base[i] = ce;
        seg_cnt[i] = cnt;
    }
    // guided tail: waves that start together on equal tasks finish their
    // rounds together, so the launch ends on a partial round of
    // tasks mod waves tasks, with most of the GPU idle for a whole task's
    // time.  Those last tasks (the cheapest layouts, queued last) run as
    // pieces instead: the most pieces each (<= fused_tail; 10, 5, 2) that
    // still fit one round of the grid.  Splitting more (a whole round) costs
    // more than it saves: every piece is one more atomic on the launch's one
    // queue counter, which saturates (profiles/r06/experiments/fused_tail/).
    const uint64_t cap_waves =
        (uint64_t)persistent_grid(ctx, dv, kFusedPerCu, 1ull << 40) * (kBlock / kWaveSize);
    const uint64_t nsplit = tasks % cap_waves;
    uint32_t nparts = 1;
    for (uint32_t p : {10u, 5u, 2u})
        if (p <= ctx->fused_tail && nsplit * p <= cap_waves) { nparts = p; break; }
    const uint64_t nbig = nparts > 1 ? tasks - nsplit : tasks;
    const uint64_t ids = nbig + (nparts > 1 ? nsplit * nparts : 0);
    if (ids >= (1ull << 31) || jobs >= (1ull << 31) || aux_next > kFusedAuxWords)
        return HM_ERR_INTERNAL;  // excluded by fusible()
    double comp_w = 0;  // executed compressions x nonces (hm_stats)
    for (size_t i = 0; i < segs.size(); ++i) {
        double ce = ce_base[i];
        if (seg_units[i] > 0) {  // chained: block 0 per task, and per piece of a split task
            const uint64_t a = i ? fa.segs[i - 1].task_end : 0, b = fa.segs[i].task_end;
            const uint64_t split =
                nparts > 1 && b > std::max(a, nbig) ? b - std::max(a, nbig) : 0;
            ce += (double)(b - a + split * (nparts - 1)) / seg_units[i];
        }
        comp_w += ce * (double)seg_cnt[i];
    }
    fa.ntasks = (uint32_t)ids;
    fa.nbig = (uint32_t)nbig;
    if (ctx->fused_trace) {
        if (!dv.trace)
            HIPCHK(hipMalloc(&dv.trace, (size_t)kMaxCandWaves * 4 * sizeof(uint64_t)));
        fa.trace = dv.trace;
    }
    fa.nparts = nparts > 1 ? nparts : 1;
    fa.nseg = pa.nseg = (uint32_t)segs.size();
    pa.njobs = (uint32_t)jobs;
    const Device::Fn* fn = nullptr;
    int rc = scan_fn(dv, fused_symbol(ctx->csum), &fn);
    if (rc) return rc;
    // small launches: few waves per SIMD keep a task short, so the launch's
    // tail is short (kFusedPerCu = 3 workgroups per CU, profiles/r05/fused/)
    const int grid = persistent_grid(ctx, dv, kFusedPerCu, ids);
    fa.flags = ctx->fused_flags;
    // with static first tasks the queue starts past every wave slot
    pa.counter0 = (fa.flags & kFusedStaticFirst) ? (uint32_t)grid * (kBlock / kWaveSize) : 0;
    HIPCHK(launch_fused_plan(pa, st));
    if (fa.trace) dv.trace_waves = grid * (kBlock / kWaveSize);
    Launch L;
    rc = next_event(dv, &L.start);
    if (rc) return rc;
    rc = next_event(dv, &L.stop);
    if (rc) return rc;
    L.nonces = nonces;
    L.kind = HM_KIND_FUSED;
    snprintf(L.kernel, sizeof L.kernel, ctx->csum ? "hm_fused_csum_kernel" : "hm_fused_kernel");
    L.grid = grid;
    L.compressions = comp_max;
    L.comp_eff = comp_w / (double)nonces;
    HIPCHK(hipEventRecord(L.start, st));
    rc = launch_scan(*fn, fa, grid, st);
    if (rc) return rc;
    HIPCHK(hipEventRecord(L.stop, st));
    HIPCHK(launch_fold(dv.cand[si], (uint32_t)grid * (kBlock / kWaveSize), best, st, 1, host));
    if (ctx->csum)
        HIPCHK(launch_sum_fold(dv.sums[si], (uint32_t)grid * (kBlock / kWaveSize), dv.acc + 2 * si,
                               st));
    dv.launches.push_back(L);
    return HM_OK;
}

struct DevReq {
    const MsgPlan* mp;
    uint64_t lo, hi;
    bool empty;
};

// Enqueue a batch of scans on one device; request r's result lands in
// dv.result + 2r, and with `to_host` also in the pinned readback slot
// dv.host_out[r] (stored by the last fold kernel).  All segments of all
// requests are queued before any sync.  `first`: the call's first chunk,
// which records the timing origin dv.t0 (every launch of an hm_scan_many
// call is timed against it).
int enqueue_device_batch(hm_ctx* ctx, Device& dv, const std::vector<DevReq>& reqs, bool first,
                         bool to_host) {
    HIPCHK(hipSetDevice(dv.ordinal));
    const int n = (int)reqs.size();
    hipStream_t s0 = dv.stream[0];
    if (first) HIPCHK(hipEventRecord(dv.t0, s0));
    // one small request (config 1, short server chunks): the fused launch on
    // stream 0 alone, its planner seeding the result slot -- nothing else
    // runs between the call's first launch and the 16-B readback
    if (n == 1 && !reqs[0].empty && ctx->fused && !ctx->test_mid_sync) {
        std::vector<SegPlan> segs = plan_range(*reqs[0].mp, reqs[0].lo, reqs[0].hi,
                                               ctx->force_generic, ctx->table_digits);
        if (fusible(segs))
            return enqueue_fused(ctx, dv, *reqs[0].mp, segs, 0, dv.result, true,
                                 to_host ? dv.host_dev : nullptr);
    }
    // streams == 1: every segment in order on stream 0, so kernels never
    // overlap and per-kernel timings match rocprofv3 exactly.  streams > 1:
    // the segments run by the request's dominant kernel instantiation (most
    // nonces) go first, in order, on stream 0 (high priority); the others
    // are queued on the low-priority streams 1.., gated on stream 0 reaching
    // its last dominant segment: they start together with that launch, get
    // workgroup slots only as its persistent waves retire, and so run in its
    // tail instead of after it.  Small requests (<= kConcurrentNonces) skip
    // that order: all their segments run at once on all streams.
    const int nstreams = std::max(1, std::min(ctx->streams, kStreams));
    // instantiation key per segment
    auto key = [](const SegPlan& g) {
        return g.kind * 1000 + g.W1 * 4 + (g.straddle ? 2 : 0) + (g.trailer ? 1 : 0);
    };
    struct ReqPlan {
        std::vector<SegPlan> segs;
        int dom = -1;            // the key with the most nonces
        long double total = 0;   // nonces
        bool fused = false;      // the whole request in one fused launch
        std::vector<SegPlan> tail;  // segments off the dominant key (large requests)
        bool tail_fused = false;    // ... run as one fused launch
    };
    // plan every request first: the streams the batch needs are made (once
    // per context, make_streams) before anything is queued on them
    std::vector<ReqPlan> plans(n);
    int used = 1, nfused = 0;
    for (int r = 0; r < n; ++r) {
        if (reqs[r].empty) continue;
        ReqPlan& P = plans[r];
        P.segs = plan_range(*reqs[r].mp, reqs[r].lo, reqs[r].hi, ctx->force_generic,
                            ctx->table_digits);
        std::vector<std::pair<int, long double>> load;
        for (const auto& g : P.segs) {
            const long double cnt = (long double)(g.hi - g.lo) + 1;
            auto it = std::find_if(load.begin(), load.end(),
                                   [&](const auto& p) { return p.first == key(g); });
            if (it == load.end()) load.push_back({key(g), cnt});
            else it->second += cnt;
        }
        long double most = -1;
        for (const auto& p : load) {
            P.total += p.second;
            if (p.second > most) { most = p.second; P.dom = p.first; }
        }
        P.fused = ctx->fused && fusible(P.segs);
        if (P.fused) {
            used = std::max(used, std::min(nstreams, ++nfused));
        } else if (P.total <= (long double)kConcurrentNonces) {
            used = std::max(used, std::min(nstreams, (int)P.segs.size()));
        } else {
            // segments off the dominant key run in its tail: as ONE fused
            // launch when they fit it (cfg2's d <= 8, cfg3's trailer
            // segments), else one launch each on the tail streams
            for (const auto& g : P.segs)
                if (key(g) != P.dom) P.tail.push_back(g);
            P.tail_fused = ctx->fused && ctx->tail_fused && fusible(P.tail);
            const int off = P.tail_fused ? 1 : (int)P.tail.size();
            used = std::max(used, std::min(nstreams, 1 + off));
        }
    }
    const int ns = used;  // streams this batch enqueues onto (<= nstreams)
    {
        int rc = make_streams(dv, ns);
        if (rc) return rc;
    }
    HIPCHK(launch_init_best(dv.best, (uint32_t)(n * kStreams), s0));
    HIPCHK(launch_init_best(dv.result, (uint32_t)n, s0));
    if (ctx->csum) HIPCHK(hipMemsetAsync(dv.acc, 0, kStreams * 2 * sizeof(uint64_t), s0));
    HIPCHK(hipEventRecord(dv.join[0], s0));
    for (int s = 1; s < ns; ++s) HIPCHK(hipStreamWaitEvent(dv.stream[s], dv.join[0], 0));
    if (ctx->test_mid_sync) {  // HM_OPT_TEST_MID_SYNC: a host wait mid-enqueue, counted
        int rc = host_wait(ctx, s0);
        if (rc) return rc;
    }
    int rr = 0;
    for (int r = 0; r < n; ++r) {
        if (reqs[r].empty) continue;
        const std::vector<SegPlan>& segs = plans[r].segs;
        const int dom = plans[r].dom;
        uint64_t* best = dv.best + (size_t)r * kStreams * 2;
        if (plans[r].fused) {
            // a small request of a batch: one fused launch on the next stream
            const int si = rr++ % ns;
            int rc = enqueue_fused(ctx, dv, *reqs[r].mp, segs, si, best + 2 * si, false);
            if (rc) return rc;
            continue;
        }
        if (ns > 1 && plans[r].total <= (long double)kConcurrentNonces) {
            // a small request (config 1's [0, 10^7+1], short server chunks):
            // its launches are latency-bound, so every segment goes onto the
            // streams round-robin, ungated, largest first: the host enqueues
            // a segment every ~25 us, and the largest one should not be the
            // last to start
            std::vector<size_t> order(segs.size());
            for (size_t i = 0; i < order.size(); ++i) order[i] = i;
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
                return segs[a].hi - segs[a].lo > segs[b].hi - segs[b].lo;
            });
            for (size_t i : order) {
                int rc = enqueue_segment(ctx, dv, *reqs[r].mp, segs[i], rr++ % ns, best);
                if (rc) return rc;
            }
            continue;
        }
        size_t last_dom = 0;
        for (size_t i = 0; i < segs.size(); ++i)
            if (key(segs[i]) == dom) last_dom = i;
        for (int pass = 0; pass < (ns > 1 ? 2 : 1); ++pass) {
            if (pass == 1)
                for (int q = 1; q < ns; ++q)
                    HIPCHK(hipStreamWaitEvent(dv.stream[q], dv.gate, 0));
            if (pass == 1 && plans[r].tail_fused) {
                // every tail segment in one fused launch on a tail stream
                const int si = 1 + (rr++ % (ns - 1));
                int rc = enqueue_fused(ctx, dv, *reqs[r].mp, plans[r].tail, si, best + 2 * si,
                                       false);
                if (rc) return rc;
                continue;
            }
            for (size_t i = 0; i < segs.size(); ++i) {
                int si = 0;
                if (ns > 1) {
                    const bool is_dom = key(segs[i]) == dom;
                    if (is_dom != (pass == 0)) continue;
                    if (!is_dom) si = 1 + (rr++ % (ns - 1));
                    if (is_dom && i == last_dom) HIPCHK(hipEventRecord(dv.gate, dv.stream[0]));
                }
                int rc = enqueue_segment(ctx, dv, *reqs[r].mp, segs[i], si, best);
                if (rc) return rc;
            }
        }
    }
    for (int s = 1; s < ns; ++s) {
        HIPCHK(hipEventRecord(dv.join[s], dv.stream[s]));
        HIPCHK(hipStreamWaitEvent(s0, dv.join[s], 0));
    }
    for (int r = 0; r < n; ++r)
        HIPCHK(launch_fold(dv.best + (size_t)r * kStreams * 2, kStreams, dv.result + 2 * r, s0, 1,
                           to_host ? dv.host_dev + 2 * r : nullptr));
    return HM_OK;
}

bool lex_less(uint64_t k1, uint64_t n1, uint64_t k2, uint64_t n2) {
    return k1 < k2 || (k1 == k2 && n1 < n2);
}

// All-gather every device's n 16-B results over RCCL; device 0 folds them.
// Runs for any device count, including one (a 1-rank communicator), so the
// path the 8-GPU context takes is exercised on a 1-GPU box.
bool distinct_ordinals(const hm_ctx* ctx) {
    const size_t n = ctx->devs.size();
    for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < i; ++j)
            if (ctx->devs[i].ordinal == ctx->devs[j].ordinal) return false;
    return true;
}

int rccl_merge(hm_ctx* ctx, int nreq) {
    const int n = (int)ctx->devs.size();
    if (!ctx->devs[0].comm) {
        std::vector<ncclComm_t> comms(n);
        std::vector<int> ords(n);
        for (int i = 0; i < n; ++i) ords[i] = ctx->devs[i].ordinal;
        if (ncclCommInitAll(comms.data(), n, ords.data()) != ncclSuccess) return HM_ERR_RCCL;
        for (int i = 0; i < n; ++i) {
            ctx->devs[i].comm = comms[i];
            HIPCHK(hipSetDevice(ctx->devs[i].ordinal));
            HIPCHK(hipMalloc(&ctx->devs[i].gathered, (size_t)n * kMaxBatch * 2 * sizeof(uint64_t)));
        }
    }
    if (ncclGroupStart() != ncclSuccess) return HM_ERR_RCCL;
    for (int i = 0; i < n; ++i) {
        Device& dv = ctx->devs[i];
        HIPCHK(hipSetDevice(dv.ordinal));
        if (ncclAllGather(dv.result, dv.gathered, (size_t)2 * nreq, ncclUint64, dv.comm,
                          dv.stream[0]) != ncclSuccess) {
            ncclGroupEnd();
            return HM_ERR_RCCL;
        }
    }
    if (ncclGroupEnd() != ncclSuccess) return HM_ERR_RCCL;
    // gathered[d][r][2]: request r's candidates are strided by nreq pairs
    Device& d0 = ctx->devs[0];
    HIPCHK(hipSetDevice(d0.ordinal));
    HIPCHK(launch_init_best(d0.result, (uint32_t)nreq, d0.stream[0]));
    for (int r = 0; r < nreq; ++r)
        HIPCHK(launch_fold(d0.gathered + 2 * r, (uint32_t)n, d0.result + 2 * r, d0.stream[0],
                           (uint32_t)nreq, ctx->host_result ? d0.host_dev + 2 * r : nullptr));
    return HM_OK;
}

// One chunk (<= kMaxBatch requests) of hm_scan_many.
int scan_chunk(hm_ctx* ctx, const hm_request* reqs, int nreq, hm_result* outs, bool first) {
    const int ndev = (int)ctx->devs.size();
    // one RCCL rank per device (hm_set_option refuses the option otherwise);
    // checked again here, before any work is enqueued
    if (ctx->merge_rccl && !distinct_ordinals(ctx)) return HM_ERR_INVALID;
    std::vector<MsgPlan> plans(nreq);
    std::vector<std::vector<DevReq>> per_dev(ndev, std::vector<DevReq>(nreq));
    static const uint8_t empty_msg = 0;
    for (int r = 0; r < nreq; ++r) {
        const hm_request& q = reqs[r];
        plans[r] = plan_message(q.msg ? q.msg : &empty_msg, q.msg ? q.len : 0);
        // contiguous shards of equal modelled cost
        const std::vector<Shard> sh =
            partition_range(plans[r], q.lo, q.hi, ndev, ctx->force_generic);
        for (int i = 0; i < ndev; ++i) {
            DevReq& dr = per_dev[i][r];
            dr.mp = &plans[r];
            dr.empty = sh[i].empty;
            dr.lo = sh[i].empty ? 0 : sh[i].lo;
            dr.hi = sh[i].empty ? 0 : sh[i].hi;
        }
    }
    // every device's work is enqueued before the host waits on any of it
    const auto te = std::chrono::steady_clock::now();
    ctx->enqueuing = true;
    for (int i = 0; i < ndev; ++i) {
        int rc = enqueue_device_batch(ctx, ctx->devs[i], per_dev[i], first,
                                      ctx->host_result && !ctx->merge_rccl);
        if (rc) { ctx->enqueuing = false; return rc; }
    }
    ctx->enqueuing = false;
    ctx->enqueue_ms +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - te).count();
    if (ctx->merge_rccl) {
        int rc = rccl_merge(ctx, nreq);
        if (rc) return rc;
        ctx->merge = HM_MERGE_RCCL;
        Device& d0 = ctx->devs[0];
        HIPCHK(hipSetDevice(d0.ordinal));
        if (!ctx->host_result)
            HIPCHK(hipMemcpyAsync(d0.host_out, d0.result, nreq * sizeof(hm_result),
                                  hipMemcpyDeviceToHost, d0.stream[0]));
        for (auto& dv : ctx->devs) {
            HIPCHK(hipSetDevice(dv.ordinal));
            int rc = host_wait(ctx, dv.stream[0]);
            if (rc) return rc;
        }
        for (int r = 0; r < nreq; ++r) outs[r] = d0.host_out[r];
        return HM_OK;
    }
    ctx->merge = ndev > 1 ? HM_MERGE_HOST : HM_MERGE_NONE;
    for (auto& dv : ctx->devs) {
        if (ctx->host_result) break;  // the last fold stored them in host_out
        HIPCHK(hipSetDevice(dv.ordinal));
        HIPCHK(hipMemcpyAsync(dv.host_out, dv.result, nreq * sizeof(hm_result),
                              hipMemcpyDeviceToHost, dv.stream[0]));
    }
    for (int r = 0; r < nreq; ++r) outs[r] = hm_result{~0ull, 0};
    for (auto& dv : ctx->devs) {
        HIPCHK(hipSetDevice(dv.ordinal));
        int rc = host_wait(ctx, dv.stream[0]);
        if (rc) return rc;
        for (int r = 0; r < nreq; ++r)
            if (lex_less(dv.host_out[r].hash, dv.host_out[r].nonce, outs[r].hash, outs[r].nonce))
                outs[r] = dv.host_out[r];
    }
    return HM_OK;
}

int open_devices(const int* devices, int ndev, hm_ctx** out);

}  // namespace

extern "C" {

uint64_t hm_hash(const uint8_t* msg, size_t len, uint64_t nonce) {
    static const uint8_t empty = 0;
    return host_hash(msg ? msg : &empty, msg ? len : 0, nonce);
}

// 1.1: hm_scan_many, hm_stats.dom_*; 1.2: hm_partition; 1.3: hm_scan_checked;
// 1.4: hm_stats.merge / dom_compressions_eff, HM_OPT_MERGE_RCCL at any device count;
// 1.5: hm_scan_stats_sized, HM_OPT_MERGE_RCCL refused up front for repeated ordinals;
// 1.6: hm_build_id, hm_stats.enqueue_ms / mid_call_syncs / table_grows, HM_OPT_TABLE_ROWS_CAP;
// 1.7: hm_scan_cpu, hm_scan_stats frozen at HM_STATS_SIZE_1_4 bytes;
// 1.8: HM_OPT_DEADLINE_MS / HM_ERR_TIMEOUT, hm_stats.deadline_ms, streams 1..
//      made on first use
int hm_version(void) { return (1 << 16) | 8; }

// The digest of the sources this library was built from (build_id.py), kept
// in the binary behind a tag so tools can read it without loading the library.
static const char kBuildTag[] = "hipminer-build-id:" HM_BUILD_ID;
const char* hm_build_id(void) { return kBuildTag + sizeof("hipminer-build-id:") - 1; }

int hm_partition(const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, int n,
                 uint64_t* bounds) {
    if (n <= 0 || !bounds || (len > 0 && !msg)) return HM_ERR_INVALID;
    return guarded([&] {
        static const uint8_t empty = 0;
        const MsgPlan mp = plan_message(msg ? msg : &empty, msg ? len : 0);
        const std::vector<Shard> sh = partition_range(mp, lo, hi, n, false);
        for (int i = 0; i < n; ++i) {
            bounds[2 * i] = sh[i].empty ? 1 : sh[i].lo;
            bounds[2 * i + 1] = sh[i].empty ? 0 : sh[i].hi;
        }
        return (int)HM_OK;
    });
}

const char* hm_strerror(int rc) {
    switch (rc) {
        case HM_OK: return "ok";
        case HM_ERR_INVALID: return "invalid argument";
        case HM_ERR_NO_DEVICE: return "no usable HIP device";
        case HM_ERR_HIP: return "HIP runtime error (set HM_DEBUG=1 for details)";
        case HM_ERR_NOMEM: return "out of memory";
        case HM_ERR_RCCL: return "RCCL error";
        case HM_ERR_INTERNAL: return "internal planner error";
        case HM_ERR_TIMEOUT:
            return "GPU scan missed its deadline (HM_OPT_DEADLINE_MS); the context is "
                   "abandoned: close it, open a new one or scan on the host";
        default: return "unknown error";
    }
}

int hm_open(const int* devices, int ndev, hm_ctx** out) {
    if (!out || ndev < 0 || (ndev > 0 && !devices)) return HM_ERR_INVALID;
    *out = nullptr;
    return guarded([&] { return open_devices(devices, ndev, out); });
}

}  // extern "C"

namespace {

int open_devices(const int* devices, int ndev, hm_ctx** out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return HM_ERR_NO_DEVICE;
    std::vector<int> ords;
    if (ndev == 0) {
        for (int i = 0; i < count; ++i) ords.push_back(i);
    } else {
        for (int i = 0; i < ndev; ++i) {
            if (devices[i] < 0 || devices[i] >= count) return HM_ERR_INVALID;
            ords.push_back(devices[i]);
        }
    }
    hm_ctx* ctx = new (std::nothrow) hm_ctx;
    if (!ctx) return HM_ERR_NOMEM;
    int rc = HM_OK;
    try {
        ctx->devs.resize(ords.size());
        for (size_t i = 0; i < ords.size() && rc == HM_OK; ++i) rc = device_init(ctx->devs[i], ords[i]);
    } catch (const std::bad_alloc&) {
        rc = HM_ERR_NOMEM;
    }
    if (rc) {
        for (auto& dv : ctx->devs) device_free(dv);
        delete ctx;
        return rc;
    }
    *out = ctx;
    return HM_OK;
}

}  // namespace

extern "C" {

void hm_close(hm_ctx* ctx) {
    if (!ctx) return;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        // an abandoned context (HM_ERR_TIMEOUT) may still have work running:
        // its streams, buffers and pinned readback slot are left to the
        // process exit rather than waited for
        if (!ctx->abandoned)
            for (auto& dv : ctx->devs) device_free(dv);
    }
    delete ctx;
}

int hm_set_option(hm_ctx* ctx, int opt, int64_t value) {
    if (!ctx) return HM_ERR_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (ctx->abandoned) return HM_ERR_TIMEOUT;
    switch (opt) {
        case HM_OPT_DEADLINE_MS:
            if (value < -1) return HM_ERR_INVALID;
            ctx->deadline_opt = value;
            return HM_OK;
        case HM_OPT_FORCE_GENERIC: ctx->force_generic = value != 0; return HM_OK;
        case HM_OPT_MERGE_RCCL:
            // RCCL needs one rank per device: a context naming a device twice
            // can never merge over RCCL, so the option is refused up front
            if (value != 0 && !distinct_ordinals(ctx)) return HM_ERR_INVALID;
            ctx->merge_rccl = value != 0;
            return HM_OK;
        case HM_OPT_STREAMS:
            if (value < 1 || value > kStreams) return HM_ERR_INVALID;
            ctx->streams = (int)value;
            return HM_OK;
        case HM_OPT_TABLE_DIGITS:
            if (value < -1 || value > (int64_t)kMaxTableDigits) return HM_ERR_INVALID;
            ctx->table_digits = (int)value;
            return HM_OK;
        case HM_OPT_TABLE_ROWS_CAP:
            if (value < 0) return HM_ERR_INVALID;
            ctx->table_rows_cap = (uint64_t)value;
            return HM_OK;
        case HM_OPT_TEST_MID_SYNC:
            ctx->test_mid_sync = value != 0;
            return HM_OK;
        case HM_OPT_FUSED:
            ctx->fused = value != 0;
            return HM_OK;
        case HM_OPT_FUSED_FLAGS:
            if (value < 0 || value > 31) return HM_ERR_INVALID;
            ctx->fused_flags = (uint32_t)value;
            return HM_OK;
        case HM_OPT_FUSED_PARTS:
            if (value != 1 && value != 2 && value != 5 && value != 10) return HM_ERR_INVALID;
            ctx->fused_parts = (uint32_t)value;
            return HM_OK;
        case HM_OPT_FUSED_TRACE:
            ctx->fused_trace = value != 0;
            return HM_OK;
        case HM_OPT_QUEUE_BATCH:
            if (value != 0 && value != 4 && value != 8 && value != 16 && value != 32)
                return HM_ERR_INVALID;
            ctx->queue_batch = (int)value;
            return HM_OK;
        case HM_OPT_HOST_RESULT:
            ctx->host_result = value != 0;
            return HM_OK;
        case HM_OPT_TAIL_FUSED:
            ctx->tail_fused = value != 0;
            return HM_OK;
        case HM_OPT_FUSED_TAIL:
            if (value != 1 && value != 2 && value != 5 && value != 10) return HM_ERR_INVALID;
            ctx->fused_tail = (uint32_t)value;
            return HM_OK;
        case HM_OPT_GRID_PER_CU:
            if (value < 0 || value > 32) return HM_ERR_INVALID;
            ctx->grid_per_cu = (int)value;
            return HM_OK;
        default: return HM_ERR_INVALID;
    }
}

}  // extern "C"

namespace {

// HM_OPT_DEADLINE_MS = -1 (auto): kDeadlineFloorMs plus kDeadlineSlack times
// the call's modelled kernel time -- every segment's nonces at its layout's
// measured SIMD cycles per 64 nonces (seg_cost, the model hm_partition
// balances shards with), over every SIMD of the context's distinct devices at
// the nominal 2.4 GHz.  The slack covers a GPU shared with other processes,
// a lowered clock and the fused launch's partial grid; hm_miner and the Go
// gpuminer use it so a hung or starved GPU scan is answered on the host
//  long before any healthy scan could finish that late.
constexpr double kDeadlineFloorMs = 2000.0;
constexpr double kDeadlineSlack = 8.0;

double modelled_deadline_ms(const hm_request* reqs, int n, bool force_generic, int table_digits,
                            double simds) {
    static const uint8_t empty_msg = 0;
    long double cycles = 0;
    for (int r = 0; r < n; ++r) {
        const hm_request& q = reqs[r];
        if (q.lo > q.hi) continue;
        const MsgPlan mp = plan_message(q.msg ? q.msg : &empty_msg, q.msg ? q.len : 0);
        for (const SegPlan& g : plan_range(mp, q.lo, q.hi, force_generic, table_digits))
            cycles += ((long double)(g.hi - g.lo) + 1) * seg_cost(g) / kWaveSize;
    }
    return kDeadlineFloorMs + kDeadlineSlack * (double)(cycles / (long double)simds / 2.4e6L);
}

double auto_deadline_ms(const hm_ctx* ctx, const hm_request* reqs, int n) {
    std::vector<int> ords;
    for (const auto& dv : ctx->devs)
        if (std::find(ords.begin(), ords.end(), dv.ordinal) == ords.end()) ords.push_back(dv.ordinal);
    return modelled_deadline_ms(reqs, n, ctx->force_generic, ctx->table_digits,
                                4.0 * ctx->devs[0].cus * (double)ords.size());
}

// hm_scan_many with ctx->mu held.
int scan_many_locked(hm_ctx* ctx, const hm_request* reqs, int n, hm_result* outs) {
    const auto t0 = std::chrono::steady_clock::now();
    // an abandoned context's devices may still run its timed-out work
    if (ctx->abandoned) return HM_ERR_TIMEOUT;
    ctx->has_deadline = ctx->deadline_opt != 0;
    ctx->deadline_ms = !ctx->has_deadline ? 0.0
                       : ctx->deadline_opt > 0 ? (double)ctx->deadline_opt
                                               : auto_deadline_ms(ctx, reqs, n);
    if (ctx->has_deadline)
        ctx->deadline_at = t0 + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                    std::chrono::duration<double, std::milli>(ctx->deadline_ms));
    std::vector<hm_result> res(n);
    for (auto& dv : ctx->devs) {
        dv.evnext = 0;
        dv.launches.clear();
    }
    ctx->mid_syncs = 0;
    ctx->table_grows = 0;
    ctx->enqueue_ms = 0;
    uint64_t total = 0;
    for (int r = 0; r < n; ++r)
        if (reqs[r].lo <= reqs[r].hi) total += reqs[r].hi - reqs[r].lo + 1;  // wraps for 2^64
    ctx->merge = HM_MERGE_NONE;
    for (int c = 0; c < n; c += kMaxBatch) {
        const int m = std::min(kMaxBatch, n - c);
        int rc = scan_chunk(ctx, reqs + c, m, res.data() + c, c == 0);
        if (rc) return rc;
    }
    const int ndev = (int)ctx->devs.size();
    // stats
    hm_stats st{};
    st.ndev = ndev;
    st.nonces = total;
    // aggregate per kernel instantiation; the dominant one has the most nonces
    struct Agg { std::string name; double ms = 0; uint64_t nonces = 0; int launches = 0;
                 int kind = 0, grid = 0; uint32_t comp = 0; double comp_eff = 0;
                 uint64_t big = 0; };
    std::vector<Agg> aggs;
    for (auto& dv : ctx->devs) {
        // kernel_ms: time during which some scan kernel ran on this device
        // (union of the launches' event intervals; launches on several
        // streams overlap)
        std::vector<std::pair<float, float>> iv;
        for (auto& L : dv.launches) {
            float a = 0.f, b = 0.f;
            HIPCHK(hipEventElapsedTime(&a, dv.t0, L.start));
            HIPCHK(hipEventElapsedTime(&b, dv.t0, L.stop));
            iv.push_back({a, b});
        }
        std::sort(iv.begin(), iv.end());
        float cur_a = 0.f, cur_b = -1.f;
        for (const auto& x : iv) {
            if (x.first > cur_b) {
                if (cur_b > cur_a) st.kernel_ms += cur_b - cur_a;
                cur_a = x.first;
                cur_b = x.second;
            } else if (x.second > cur_b) {
                cur_b = x.second;
            }
        }
        if (cur_b > cur_a) st.kernel_ms += cur_b - cur_a;
        for (auto& L : dv.launches) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, L.start, L.stop));
            st.launches += 1;
            Agg* a = nullptr;
            for (auto& x : aggs)
                if (x.name == L.kernel) a = &x;
            if (!a) { aggs.push_back(Agg{}); a = &aggs.back(); a->name = L.kernel; }
            a->ms += ms;
            a->nonces += L.nonces;
            a->launches += 1;
            a->kind = L.kind;
            a->comp = std::max(a->comp, L.compressions);
            a->comp_eff += L.comp_eff * (double)L.nonces;  // nonce-weighted mean below
            if (L.nonces > a->big) { a->big = L.nonces; a->grid = L.grid; }
        }
    }
    for (auto& a : aggs) {
        if (a.nonces > st.dom_nonces) {
            st.dom_nonces = a.nonces;
            st.dom_kernel_ms = a.ms;
            st.dom_compressions = a.comp;
            st.dom_compressions_eff = a.nonces ? a.comp_eff / (double)a.nonces : 0.0;
            st.dom_kind = a.kind;
            st.dom_grid = a.grid;
            st.dom_launches = a.launches;
            snprintf(st.dom_kernel, sizeof st.dom_kernel, "%s", a.name.c_str());
        }
    }
    st.merge = ctx->merge;
    st.enqueue_ms = ctx->enqueue_ms;
    st.mid_call_syncs = ctx->mid_syncs;
    st.table_grows = ctx->table_grows;
    st.deadline_ms = ctx->deadline_ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                     .count();
    ctx->last = st;
    ctx->have_stats = true;
    for (int r = 0; r < n; ++r) outs[r] = res[r];
    return HM_OK;
}

}  // namespace

extern "C" {

int hm_scan_many(hm_ctx* ctx, const hm_request* reqs, int n, hm_result* outs) {
    if (!ctx || n < 0 || (n > 0 && (!reqs || !outs))) return HM_ERR_INVALID;
    for (int r = 0; r < n; ++r)
        if (!reqs[r].msg && reqs[r].len) return HM_ERR_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    return guarded([&] { return scan_many_locked(ctx, reqs, n, outs); });
}

int hm_scan(hm_ctx* ctx, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi,
            hm_result* out) {
    if (!ctx || !out || (!msg && len)) return HM_ERR_INVALID;
    hm_request q{msg, len, lo, hi};
    return hm_scan_many(ctx, &q, 1, out);
}

int hm_scan_checked(hm_ctx* ctx, const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi,
                    hm_result* out, uint64_t* sum, uint64_t* count) {
    if (!ctx || !out || !sum || !count || (!msg && len)) return HM_ERR_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    hm_request q{msg, len, lo, hi};
    hm_result res;
    ctx->csum = true;
    int rc = guarded([&] { return scan_many_locked(ctx, &q, 1, &res); });
    ctx->csum = false;
    if (rc) return rc;
    uint64_t s = 0, c = 0;
    for (auto& dv : ctx->devs) {
        uint64_t a[kStreams * 2];
        HIPCHK(hipSetDevice(dv.ordinal));
        rc = host_read(ctx, a, dv.acc, sizeof a);
        if (rc) return rc;
        for (int i = 0; i < kStreams; ++i) { s += a[2 * i]; c += a[2 * i + 1]; }
    }
    *out = res;
    *sum = s;
    *count = c;
    return HM_OK;
}


int hm_scan_stats(const hm_ctx* ctx, hm_stats* out) {
    // frozen at the 1.4/1.5 size (include/hipminer.h): newer fields only
    // through hm_scan_stats_sized
    return hm_scan_stats_sized(ctx, out, HM_STATS_SIZE_1_4);
}

int hm_scan_stats_sized(const hm_ctx* ctx, hm_stats* out, size_t size) {
    // a caller built against an older header passes its smaller struct:
    // only its prefix is written (the layout only ever grows at the end)
    if (!ctx || !out || size < HM_STATS_SIZE_1_0) return HM_ERR_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);  // scans write ctx->last under the lock
    if (!ctx->have_stats) return HM_ERR_INVALID;
    memcpy(out, &ctx->last, std::min(size, sizeof(hm_stats)));
    return HM_OK;
}

// ---- debug exports for host-side tests (not part of include/hipminer.h) ----
// The embedded scan code object (scan_blob.S): bench.py hashes these bytes to
// match a PMC summary to the build that actually runs.
size_t hm_debug_code_object(const unsigned char** p) {
    if (p) *p = hm_scan_code_object;
    return (size_t)(hm_scan_code_object_end - hm_scan_code_object);
}

// The timeline of the last traced fused launch on device 0 (HM_OPT_FUSED_TRACE):
// up to `cap` wave slots x 4 u64 -- wall_clock64 at the wave's start, at its
// last task's start, at its end, and its task count.  Returns the launch's
// wave slots (0: none traced).  Diagnostics (tools/fused_trace.py).
int hm_debug_fused_trace(hm_ctx* ctx, uint64_t* out, int cap) {
    if (!ctx || !out || cap < 0) return HM_ERR_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (ctx->abandoned) return HM_ERR_TIMEOUT;
    Device& dv = ctx->devs[0];
    if (!dv.trace || !dv.trace_waves) return 0;
    HIPCHK(hipSetDevice(dv.ordinal));
    const int n = std::min(cap, dv.trace_waves);
    int rc = host_read(ctx, out, dv.trace, (size_t)n * 4 * sizeof(uint64_t));
    return rc ? rc : dv.trace_waves;
}

// HM_OPT_DEADLINE_MS = -1's deadline for one request on `cus` compute units
// (host-only; tests/test_abi.py checks the model without a GPU).
double hm_debug_auto_deadline_ms(const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi,
                                 int cus) {
    const hm_request q{msg, msg ? len : 0, lo, hi};
    try {
        return modelled_deadline_ms(&q, 1, false, 0, 4.0 * cus);
    } catch (...) {
        return -1.0;
    }
}

// Streams (hardware queues) made so far on device i of ctx (make_streams):
// 1 after hm_open, up to HM_OPT_STREAMS once calls used them; -1 if i is out
// of range.
int hm_debug_streams_made(const hm_ctx* ctx, int i) {
    if (!ctx || i < 0 || i >= (int)ctx->devs.size()) return -1;
    std::lock_guard<std::mutex> g(ctx->mu);
    return ctx->devs[i].nmade;
}

// Writes up to `cap` segment descriptors as 13 x int64:
//   d, lo, hi, kind, W1, V, trailer, straddle, seg_cost (SIMD cycles / 64 nonces), lane3,
//   f (chained: final-block digits), tch (chained: loop values per unit),
//   fe (chained: table digits; f - fe epoch digits)
int hm_debug_plan(const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, int force_generic,
                  int64_t* outv, int cap) {
    if (lo > hi) return 0;
    static const uint8_t empty = 0;
    const MsgPlan mp = plan_message(msg ? msg : &empty, msg ? len : 0);
    std::vector<SegPlan> segs;
    try {
        segs = plan_range(mp, lo, hi, force_generic != 0);
    } catch (...) {
        return HM_ERR_NOMEM;
    }
    int i = 0;
    for (; i < (int)segs.size() && i < cap; ++i) {
        const SegPlan& s = segs[i];
        int64_t* o = outv + 13 * i;
        o[0] = s.d; o[1] = (int64_t)s.lo; o[2] = (int64_t)s.hi; o[3] = s.kind;
        o[4] = s.W1; o[5] = s.V; o[6] = s.trailer; o[7] = s.straddle;
        o[8] = (int64_t)seg_cost(s);
        o[9] = s.lane3;
        o[10] = s.kind == HM_KIND_CHAINED ? s.f : 0;
        o[11] = s.kind == HM_KIND_CHAINED ? s.tch : 0;
        o[12] = s.kind == HM_KIND_CHAINED ? s.fe : 0;
    }
    return (int)segs.size();
}

}  // extern "C"
