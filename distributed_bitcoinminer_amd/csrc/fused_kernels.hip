// fused_kernels.hip -- the fused small-request scan kernel (gfx950).
//
// A Request of the reference's size (config 1: the client's [0, 10^7] plus
// the server's +1, cmu440/bitcoin/server/server.go:169, scanned by
// cmu440/bitcoin/miner/miner.go:46-59) spans up to 20 decimal digit counts,
// each with its own tail layout.  Run as one launch per segment, such a
// request pays every launch's ramp and tail and queues its small segments
// behind its large one.  hm_fused_kernel instead runs every segment of the
// request in ONE persistent launch: waves dequeue task ids from one counter,
// a task id names its segment (FusedSeg::task_end is cumulative), and the
// task runs that segment's layout -- the same task bodies as the
// per-segment kernels (scan_tasks.hpp), chosen by a wave-uniform switch:
//   tiled  (any W1 / straddle / trailer): one unit's lane chunk x one tens
//          digit (64 lanes x 10 nonces), as the per-segment kernel's tail,
//          or a part of it (FusedSeg::tpu parts, HM_OPT_FUSED_PARTS);
//   chained (f <= 4 final-block digits, one K+W table): 64 lanes x up to
//          100 table-driven blocks, block 0 per lane per task;
//   generic: 64 lanes x 10 nonces, the byte-level tail builder.
// The last ~one wave-round of tasks is split into FusedArgs::nparts pieces
// (a guided tail), so the launch ends on pieces of a task, not whole tasks.
// The wave keeps one running (hash, nonce) minimum across all its tasks
// (one request), written to its candidate slot at exit; hm_fold_kernel then
// reduces the slots.  Tables (tile records, sigma0 of the loop digits, the
// trailer and chained K+W rows) come from hm_fused_plan_kernel.
//
// Compiled like scan_kernels.hip (device-only assembly -> align_loops.py,
// which places every hot loop of this kernel -> the same code object).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "scan_tasks.hpp"
#include "sha256_defs.hpp"
#include "sha_device.hpp"

namespace hm {

// The launch's FusedArgs read in place from the kernarg segment: with a
// runtime segment index, a by-value parameter would be copied to scratch.
typedef const __attribute__((address_space(4))) FusedArgs FusedArgsK;

// Piece `pp` of `np` of the run [b, e): [*b2, *e2) (empty when past e).
DEV void piece_of(uint32_t b, uint32_t e, uint32_t pp, uint32_t np, uint32_t* b2, uint32_t* e2) {
    const uint32_t len = (e - b + np - 1) / np;
    uint32_t x = b + pp * len, y = x + len;
    if (x > e) x = e;
    if (y > e) y = e;
    *b2 = x;
    *e2 = y;
}

template <int W1, bool STRADDLE, bool TRAILER, bool CSUM>
DEV void fused_tiled(FusedArgsK* A, const FusedSeg& S, uint32_t k, uint32_t pp, uint32_t np,
                     WaveBest& best, WaveSums& sums) {
    // task k: unit, tens digit t1 and part of the units loop (S.tpu parts
    // of 10 / S.tpu steps each); a guided-tail piece pp of np runs a share
    // of that part's steps
    const uint32_t per_unit = 10u * S.tpu;
    const uint32_t unit = S.unit0 + k / per_unit;
    const uint32_t rem = k - (k / per_unit) * per_unit;
    const uint32_t t1 = rem / S.tpu;
    const uint32_t part = rem - t1 * S.tpu;
    const uint32_t steps = 10u / S.tpu;
    uint32_t t0b, t0e;
    piece_of(part * steps, part * steps + steps, pp, np, &t0b, &t0e);
    const uint32_t tile = unit / S.tpt;
    const uint32_t chunk = unit - tile * S.tpt;
    const_u32* tab = (const_u32*)(A->aux + S.aux0);
    tiled_task<W1, STRADDLE, TRAILER, CSUM>(A->rec + (size_t)(S.rec0 + tile) * kRecWords, chunk, t1,
                                            t1 + 1, (S.tile0 + tile) * S.pow10V, S.seg_lo, S.seg_hi,
                                            S.vmax, S.q, S.lane_shift, S.loop_shift, tab, tab + 100,
                                            best, sums, t0b, t0e);
}

template <bool CSUM>
DEV void fused_chained(FusedArgsK* A, const FusedSeg& S, uint32_t k, uint32_t pp, uint32_t np,
                       WaveBest& best, WaveSums& sums) {
    const uint32_t unit = S.unit0 + k / S.tpu;
    const uint32_t part = k - (k / S.tpu) * S.tpu;
    const uint32_t per_tile = S.tpt * S.ntc;
    const uint32_t tile = unit / per_tile;
    const uint32_t rem = unit - tile * per_tile;
    const uint32_t chunk = rem / S.ntc;
    const uint32_t tc = rem - chunk * S.ntc;
    const uint32_t piece = (S.tch + S.tpu - 1) / S.tpu;
    const uint32_t t_begin = tc * S.tch + part * piece;
    uint32_t t_end = tc * S.tch + S.tch;
    if (t_end > t_begin + piece) t_end = t_begin + piece;
    uint32_t tb, te;
    piece_of(t_begin, t_end, pp, np, &tb, &te);
    if (tb >= te) return;  // uniform
    chained_task<CSUM>(A->rec + (size_t)(S.rec0 + tile) * kRecWords, chunk, tb, te,
                       (S.tile0 + tile) * S.pow10V, S.pow10f, S.seg_lo, S.seg_hi, S.vmax, S.q,
                       A->aux + S.aux0, best, sums);
}

// Generic task k: nonces seg_lo + 640k + lane + 64j, j < 10 (a guided-tail
// piece: its share of the j), one per lane and step, every tail block
// compressed per lane.
template <bool CSUM>
DEV void fused_generic(FusedArgsK* A, const FusedSeg& S, uint32_t k, uint32_t pp, uint32_t np,
                       WaveBest& best, WaveSums& sums) {
    const uint32_t lane = __lane_id();
    uint32_t pw[16], mid[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) pw[i] = A->pw[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) mid[i] = A->mid[i];
    const uint64_t base = S.seg_lo + (uint64_t)k * 640u;
    uint32_t jb, je;
    piece_of(0, 10, pp, np, &jb, &je);
    for (uint32_t j = jb; j < je; ++j) {
        const uint64_t nb0 = base + 64u * j;  // wave-uniform
        if (nb0 > S.seg_hi || nb0 < S.seg_lo) break;  // past the end (or wrapped)
        const uint64_t n = nb0 + lane;
        const bool in = n >= nb0 && n <= S.seg_hi;  // no wrap past 2^64-1
        uint32_t w[32];
        build_tail(w, pw, A->r, S.d, 0, in ? n : nb0, S.nb, S.total_bits);
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = mid[i];
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = w[i];
        d_compress(st, m);
        if (S.nb == 2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = w[16 + i];
            d_compress(st, m);
        }
        if constexpr (CSUM) {
            if (in) {
                sums.sum += ((uint64_t)st[0] << 32) | st[1];
                ++sums.cnt;
            }
        }
        take_step(best, in && st[0] <= best.hi, st[0], st[1], nb0, lane, S.seg_lo, S.seg_hi);
    }
}

#define HM_FUSED_CASE(W, S, T) \
    case (W) * 4 + (S) * 2 + (T): fused_tiled<W, S, T, CSUM>(A, S_, k, pp, np, best, sums); break;
#define HM_FUSED_CASE_S(W, T) HM_FUSED_CASE(W, false, T) HM_FUSED_CASE(W, true, T)

template <bool CSUM>
DEV void fused_body(FusedArgsK* A) {
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + uni(threadIdx.x / kWaveSize);
    WaveBest best;
    WaveSums sums;  // CSUM only
    const uint32_t flags = A->flags;
    const uint32_t nwaves = gridDim.x * (kBlock / kWaveSize);
    __shared__ LdsQueue queue;  // kFusedLds
    if (flags & kFusedLds) lds_queue_init(&queue);
    // task ids: with kFusedStaticFirst the first is the wave's slot (the
    // planner started the counter past every slot), so the launch opens
    // without a burst of queue atomics; with kFusedPrefetch the next id is
    // dequeued before the current task runs, hiding the atomic's latency;
    // kFusedLds dequeues through the workgroup's LDS dispenser (one queue
    // atomic per 4 tasks); kFusedStatic strides the wave slots over the task
    // ids (wslot, wslot + nwaves, ...) with no queue at all
    auto dequeue = [&]() -> uint32_t {
        if (flags & kFusedLds) return lds_dequeue(&queue, A->counter);
        uint32_t t = 0;
        if (__lane_id() == 0) t = atomicAdd(A->counter, 1u);
        return t;
    };
    uint64_t* const trace = A->trace;  // diagnostics, normally null
    uint64_t t_start = 0, t_last = 0;
    uint32_t ntask = 0;
    if (trace) t_start = wall_clock64();
    uint32_t next = (flags & (kFusedStaticFirst | kFusedStatic)) ? wslot : dequeue();
    const uint32_t nbig = A->nbig, nparts = A->nparts;
    for (;;) {
        const uint32_t id = uni(next);
        if (id >= A->ntasks) break;
        if (trace) t_last = wall_clock64();
        if (flags & kFusedPrioEq) {
            // s_setprio takes an immediate
            if (ntask == 0) __builtin_amdgcn_s_setprio(3);
            else if (ntask == 1) __builtin_amdgcn_s_setprio(2);
            else if (ntask == 2) __builtin_amdgcn_s_setprio(1);
            else if (ntask == 3) __builtin_amdgcn_s_setprio(0);
        }
        ++ntask;
        next = 0;
        if (flags & kFusedStatic) next = id + nwaves;
        else if (flags & kFusedPrefetch) next = dequeue();
        // guided tail: ids from nbig on are pieces pp of np of their task
        uint32_t task = id, pp = 0, np = 1;
        if (id >= nbig) {
            const uint32_t q = (id - nbig) / nparts;
            pp = id - nbig - q * nparts;
            np = nparts;
            task = nbig + q;
        }
        uint32_t i = 0;
        while (i + 1 < A->nseg && task >= A->segs[i].task_end) ++i;
        const FusedSeg S_ = A->segs[i];  // scalar loads of one descriptor
        const uint32_t k = task - (i ? A->segs[i - 1].task_end : 0u);
        switch (S_.variant) {
            HM_FUSED_CASE_S(1, false)
            HM_FUSED_CASE_S(2, false)
            HM_FUSED_CASE_S(3, false)
            HM_FUSED_CASE_S(4, false)
            HM_FUSED_CASE_S(5, false)
            HM_FUSED_CASE_S(6, false)
            HM_FUSED_CASE_S(7, false)
            HM_FUSED_CASE_S(8, false)
            HM_FUSED_CASE_S(9, false)
            HM_FUSED_CASE_S(10, false)
            HM_FUSED_CASE_S(11, false)
            HM_FUSED_CASE_S(12, false)
            HM_FUSED_CASE_S(13, false)
            HM_FUSED_CASE_S(13, true)
            HM_FUSED_CASE_S(14, true)
            HM_FUSED_CASE_S(15, true)
            case kVarChained: fused_chained<CSUM>(A, S_, k, pp, np, best, sums); break;
            default: fused_generic<CSUM>(A, S_, k, pp, np, best, sums); break;
        }
        if (!(flags & (kFusedPrefetch | kFusedStatic))) next = dequeue();
    }
    wave_store<CSUM>(A->cand, A->sums, wslot, best, sums);
    if (trace && __lane_id() == 0) {
        trace[4 * (size_t)wslot] = t_start;
        trace[4 * (size_t)wslot + 1] = t_last;
        trace[4 * (size_t)wslot + 2] = wall_clock64();
        trace[4 * (size_t)wslot + 3] = ntask;
    }
}

#undef HM_FUSED_CASE_S
#undef HM_FUSED_CASE

// The argument block is the kernel's only (explicit) parameter, so it starts
// the kernarg segment.
__global__ void __launch_bounds__(kBlock) hm_fused_kernel(const FusedArgs) {
    fused_body<false>((FusedArgsK*)__builtin_amdgcn_kernarg_segment_ptr());
}

__global__ void __launch_bounds__(kBlock) hm_fused_csum_kernel(const FusedArgs) {
    fused_body<true>((FusedArgsK*)__builtin_amdgcn_kernarg_segment_ptr());
}

}  // namespace hm
