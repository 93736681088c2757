// kernels.hpp -- argument blocks and launchers of the gfx950 scan kernels.
//
// Hot path replaced: the miner scan loop (cmu440/bitcoin/miner/miner.go:46-59)
// calling bitcoin.Hash (cmu440/bitcoin/hash.go:13-17) once per nonce.
//
// Work decomposition:
//   segment  = nonces with the same decimal digit count d (message layout fixed)
//   tile     = 10^V consecutive nonces sharing the high d-V digits; its
//              record (chaining state + final-block words) is built once on
//              the GPU by hm_tile_plan_kernel
//   task     = one wave: 64 lanes x 100 loop steps; lane digits (q = V-2)
//              vary per lane, the last two digits are the uniform loop index
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hm {

constexpr int kWaveSize = 64;
constexpr int kBlock = 256;            // 4 waves per workgroup
constexpr int kRecWords = 32;          // tile record stride: state[8], W[16], pad
constexpr uint32_t kMaxTilesPerLaunch = 1u << 20;
constexpr uint32_t kMaxCandWaves = 32768;  // per-launch candidate slots (waves)
constexpr int kMaxBatch = 64;              // requests per hm_scan_many chunk
// Guided task sizes: a launch's first `nbig` work units are dequeued whole,
// the last ones (about one per wave of the grid) as kSplit tasks of a tenth
// of the loop each, so waves that finish early pick up small pieces and the
// launch's tail shrinks ~10x.
constexpr uint32_t kSplit = 10;

// Tile planner: one thread per tile.
struct PlanArgs {
    uint32_t* rec;       // out: ntiles * kRecWords
    uint64_t tile0;      // absolute tile index of record 0 (tile h = [h*10^V, (h+1)*10^V))
    uint64_t pow10V;
    uint64_t total_bits; // message bit length (len(msg) + 1 + d) * 8
    uint32_t ntiles;
    uint32_t V;          // varying low digits (left zero in the record)
    uint32_t d;          // digit count of the segment
    uint32_t r;          // prefix-remainder bytes in front of the digits
    uint32_t fb;         // tail block holding the last digit (0/1)
    uint32_t nb;         // tail blocks incl. a constant trailer (1/2)
    uint32_t pw[16];     // prefix remainder, big-endian words, zero padded
    uint32_t mid[8];     // midstate after the floor((len+1)/64) constant blocks
};

// Tiled scan: persistent waves pull tasks from a counter.
struct TiledArgs {
    const uint32_t* rec;
    unsigned int* counter;
    uint64_t* cand;      // 2 x u64 per wave slot: (key, nonce)
    uint64_t* sums;      // checked scans only: 2 x u64 per wave slot (sum of keys, count)
    uint64_t tile0;
    uint64_t pow10V;
    uint64_t seg_lo, seg_hi;
    uint32_t ntasks;     // task ids: nbig whole units, then kSplit per remaining unit
    uint32_t nbig;       // units dequeued whole (all 100 loop steps)
    uint32_t tpt;        // units (64-lane chunks) per tile = ceil(10^q / 64)
    uint32_t vmax;       // 10^q - 1
    uint32_t q;          // lane digits
    uint32_t lane_shift; // bit offset of the lowest lane digit in the (W[W1-1]:W[W1]) pair
    uint32_t loop_shift; // bit offset of the units loop digit (tens digit at +8)
    uint32_t lds_shift;  // log2 of the tasks one queue atomic fetches (scan_tasks.hpp lds_dequeue)
    uint32_t trailer_kw[64];  // K[i]+W[i] of the constant trailer block (TRAILER only)
    uint32_t s0_loop[100];    // sigma0 of the loop-digit part of W[W1], index t1*10+t0
};

// Chained scan (two-block tails): lanes vary the last q <= 5 digits of tail
// block 0 (W15, W14's last byte), the final block's digits are the loop index
// t and its schedule comes from a table of K[i]+W[i] per loop value.  A final
// block of f <= kMaxChainedF digits has one table of 10^f rows.  With more
// final-block digits (f >= 5) the table covers the low fe = min(f,
// kMaxTableDigits) of them and the high f - fe digits form an *epoch*: one
// table and one set of launches per epoch (ChainedArgs::ebase).
constexpr uint32_t kMaxChainedF = 4;
constexpr uint32_t kMaxTableDigits = 7;      // table rows <= 10^7 (2.56 GB)
constexpr uint32_t kMaxChainedTable = 10000; // rows allocated at hm_open (grown on demand)
struct ChainedArgs {
    const uint32_t* rec;     // tile records (state = midstate, W = tail block 0)
    const uint32_t* kwt;     // [nloop][64] K+W of the final block per loop value
    unsigned int* counter;
    uint64_t* cand;
    uint64_t* sums;          // checked scans only (see TiledArgs)
    uint64_t tile0;
    uint64_t pow10qf;        // nonces per tile = 10^(q+f)
    uint64_t pow10f;         // nonces per lane value = 10^f (f final-block digits)
    uint64_t ebase;          // epoch e * nloop: the final block's high f - fe digits
    uint64_t seg_lo, seg_hi;
    uint32_t ntasks;         // task ids: nbig whole units, then kSplit per remaining unit
    uint32_t nbig;           // units (lane chunk x loop chunk) dequeued whole
    uint32_t tpt;            // lane chunks per tile = ceil(10^q / 64)
    uint32_t ntc;            // loop chunks per lane chunk
    uint32_t tch;            // loop values per loop chunk
    uint32_t vmax;           // 10^q - 1
    uint32_t q;              // lane digits (<= 5: W15 and the last byte of W14)
    uint32_t nloop;          // loop values per lane value and epoch = table rows = 10^fe
    uint32_t lds_shift;      // log2 of the tasks one queue atomic fetches
};

// Generic scan: one nonce per lane (small / irregular segments, cross-checks).
struct GenericArgs {
    uint64_t* cand;
    uint64_t* sums;      // checked scans only (see TiledArgs)
    uint64_t seg_lo;
    uint64_t count_m1;   // nonces - 1
    uint64_t total_bits;
    uint32_t d, r, nb;
    uint32_t pw[16];
    uint32_t mid[8];
};

// ---------------------------------------------------------------------------
// Fused small requests (DESIGN.md §3 "Fused launch"): every digit segment of
// one request of <= kFusedNonces nonces in ONE persistent launch.  A task
// names its segment by its id (task_end is cumulative); each segment runs
// its own layout's task body (scan_tasks.hpp), selected per task by a
// wave-uniform switch on `variant`.  One planner launch first writes every
// segment's tile records and tables (s0_loop, trailer K+W, chained K+W rows)
// and resets the queue counter and the result slot.
// ---------------------------------------------------------------------------
constexpr int kMaxFusedSegs = 20;          // digit counts of a u64 nonce
constexpr uint64_t kFusedNonces = 1ull << 27;  // requests up to this size are fused
constexpr uint32_t kFusedKwRows = 12288;   // chained K+W rows per stream (f <= 4: <= 11110)
constexpr uint32_t kFusedAuxWords = kFusedKwRows * 64 + kMaxFusedSegs * 164;
// loop values per chained task: block 0 once per 100 values (C_eff 1.01).
// 1000 would amortise it 10x better, but a fused request (<= 2^27 nonces)
// then has fewer than 2^27 / 64000 = 2097 chained tasks, not one per wave of
// the grid (3072): the launch would run part-empty.
constexpr uint32_t kFusedChainedPiece = 100;
// variant ids: tiled W1 * 4 + 2 * straddle + trailer (4..63), then:
constexpr uint32_t kVarChained = 64;
constexpr uint32_t kVarGeneric = 65;

struct FusedSeg {
    uint64_t tile0;       // absolute index of the segment's first tile (tiled, chained)
    uint64_t pow10V;      // nonces per tile
    uint64_t pow10f;      // chained: nonces per lane value (10^f)
    uint64_t seg_lo, seg_hi;
    uint64_t total_bits;  // generic: message bit length
    uint32_t task_end;    // one past the segment's last task id (cumulative)
    uint32_t variant;
    uint32_t rec0;        // the segment's first record in FusedArgs::rec
    uint32_t aux0;        // word offset of its tables in FusedArgs::aux
    uint32_t unit0;       // first unit kept (edge trimming, launch_units)
    uint32_t tpt;         // lane chunks per tile
    uint32_t vmax, q;
    uint32_t lane_shift, loop_shift;  // tiled
    uint32_t ntc, tch;    // chained: loop chunks per lane chunk, values per chunk
    uint32_t tpu;         // chained: tasks per unit; tiled: parts per tens digit (1, 2, 5, 10)
    uint32_t d, nb;       // generic: digits, tail blocks
};

// FusedArgs::flags (HM_OPT_FUSED_FLAGS): how waves get their tasks
constexpr uint32_t kFusedStaticFirst = 1;  // first task = the wave's slot; the counter starts past them
constexpr uint32_t kFusedPrefetch = 2;     // dequeue the next task id while running the current one
constexpr uint32_t kFusedStatic = 4;       // no queue: wave w runs tasks w, w + nwaves, w + 2 nwaves, ...
constexpr uint32_t kFusedLds = 8;          // dequeue through the workgroup's LDS dispenser (scan_tasks.hpp)
// the SIMD's arbiter issues from the oldest wave first, so the youngest waves
// of a SIMD hold their first task for most of a small launch and finish it
// alone at the end (tools/fused_trace.py): with kFusedPrioEq a wave's
// priority (s_setprio) falls with the tasks it has run, 3, 2, 1, 0, so the
// waves of a SIMD progress together
constexpr uint32_t kFusedPrioEq = 16;

// Guided tail of the fused launch (round 6): task ids below `nbig` run one
// whole task each; the tasks of the last, partial wave-round (the cheapest
// layouts, queued last) are split into `nparts` pieces each, ids nbig +
// i*nparts + p, so that round fills the grid and lasts a piece, not a task
// (HM_OPT_FUSED_TAIL).
struct FusedArgs {
    const uint32_t* rec;
    const uint32_t* aux;
    unsigned int* counter;
    uint64_t* cand;
    uint64_t* sums;       // checked scans only
    uint32_t ntasks, nseg;
    uint32_t nbig;        // ids below run whole tasks
    uint32_t nparts;      // pieces per split task (1, 2, 5, 10)
    uint32_t flags;       // kFused*
    uint32_t r;           // prefix-remainder bytes (generic)
    uint32_t pw[16];      // prefix remainder words (generic)
    uint32_t mid[8];      // midstate (generic)
    // diagnostics (HM_OPT_FUSED_TRACE): per wave slot w, [4w..4w+3] = the
    // constant-rate wall clock (wall_clock64) at the wave's start, when it
    // takes its last task, at its end, and the tasks it ran; null = off
    uint64_t* trace;
    FusedSeg segs[kMaxFusedSegs];
};

struct FusedPlanSeg {
    uint64_t tile0, pow10V, total_bits;
    uint32_t job_end;     // one past the segment's last planner job (cumulative)
    uint32_t ntiles, rec0, aux0;
    uint32_t V, d, fb, nb, T;
    uint32_t variant, straddle, loop_shift, f;
};

struct FusedPlanArgs {
    uint32_t* rec;
    uint32_t* aux;
    unsigned int* counter;  // reset to counter0
    uint32_t counter0;
    uint64_t* result;       // if set: seeded (MaxUint64, 0)
    uint64_t* acc;          // if set (checked scans): [n_acc] zeroed
    uint32_t n_acc;
    uint32_t njobs, nseg, r;
    uint32_t pw[16];
    uint32_t mid[8];
    FusedPlanSeg segs[kMaxFusedSegs];
};

// Launchers of the auxiliary kernels (kernels.hip; return hipError_t of the
// launch).  The scan kernels (scan_kernels.hip: hm_tiled_kernel<W1,
// STRADDLE, TRAILER>, hm_chained_kernel, hm_generic_kernel and their
// hm_*_csum_kernel checked variants) live in their own code object and are
// launched by api.cpp through hipModuleLaunchKernel.
hipError_t launch_tile_plan(const PlanArgs& a, hipStream_t s);
// acc[0] += sum of sums[2i], acc[1] += sum of sums[2i+1] for i < n (wrapping).
hipError_t launch_sum_fold(const uint64_t* sums, uint32_t n, uint64_t* acc, hipStream_t s);
// K+W table of the final block for loop values t in [0, 10^f).
// rows t < 10^fe of the final block holding the f digits of base + t
hipError_t launch_kw_table(uint32_t* out, uint32_t f, uint32_t fe, uint64_t base,
                           uint64_t total_bits, hipStream_t s);
// Fold n (key, nonce) pairs (pair i at cand + 2*i*stride) plus *best into
// *best (lexicographic min); with `host` (pinned fine-grained host memory)
// the result is also written there, system-scope.
hipError_t launch_fold(const uint64_t* cand, uint32_t n, uint64_t* best, hipStream_t s,
                       uint32_t stride = 1, uint64_t* host = nullptr);
hipError_t launch_init_best(uint64_t* best, uint32_t n, hipStream_t s);
// The fused launch's planner: tile records, tables, counter/result/acc reset.
hipError_t launch_fused_plan(const FusedPlanArgs& a, hipStream_t s);

}  // namespace hm
