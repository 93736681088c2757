// scan_kernels.hip -- the gfx950 scan kernels of the min-hash nonce search.
//
// Replaces the miner's sequential loop (cmu440/bitcoin/miner/miner.go:46-59)
// over bitcoin.Hash (cmu440/bitcoin/hash.go:13-17).  Integer-VALU bound: no
// MFMA, no LDS on the hot path, ~zero HBM traffic.
//
//   hm_tiled_kernel      persistent waves (tasks from a workgroup-level
//                        LDS dispenser); per task 64 lanes x 100 loop
//                        steps; one SHA-256 compression per nonce from the
//                        tile state (+ a constant trailer block when the
//                        padding spills); wave-uniform running min in SGPRs,
//                        refreshed by a 64-lane shuffle reduce only when some
//                        lane's H0 <= the wave's best H0.
//   hm_chained_kernel    two-block tails whose final block is wave-uniform:
//                        per lane block 0 once, then a table-driven block.
//   hm_generic_kernel    one nonce per lane with a byte-level tail builder;
//                        small or irregular segments and cross-checks.
//   hm_*_csum_kernel     checked variants (CSUM=true): also the wrapping sum
//                        of the keys and the count of nonces hashed, per wave
//                        (hm_scan_checked).
//
// This file is compiled for the device only (`--cuda-device-only -S`); the
// Makefile passes the assembly through align_loops.py (instruction placement
// of the hot loops) and links it into the code object that
// api.cpp embeds and loads with hipModuleLoadData.  Kernels are therefore
// looked up by their mangled names (scan_symbol() in api.cpp).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "scan_tasks.hpp"
#include "sha256_defs.hpp"
#include "sha_device.hpp"

namespace hm {

// ---------------------------------------------------------------------------
// Tiled scan (the hot kernel)
// ---------------------------------------------------------------------------
#ifndef HM_TILED_WAVES_PER_EU
#define HM_TILED_WAVES_PER_EU 0
#endif
#if HM_TILED_WAVES_PER_EU > 0
#define HM_TILED_BOUNDS __launch_bounds__(kBlock, HM_TILED_WAVES_PER_EU)
#else
#define HM_TILED_BOUNDS __launch_bounds__(kBlock)
#endif

// CSUM: checked variant (coverage sum and count of the hashed keys).
template <int W1, bool STRADDLE, bool TRAILER, bool CSUM>
DEV void tiled_body(const TiledArgs& A) {
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + uni(threadIdx.x / kWaveSize);
    WaveBest best;   // wave-uniform (SGPR)
    WaveSums sums;   // CSUM only
    __shared__ LdsQueue queue;
    lds_queue_init(&queue);

    for (;;) {
        const uint32_t task = lds_dequeue(&queue, A.counter, A.lds_shift);
        if (task >= A.ntasks) break;
        // guided sizes: whole units first, then tenths (one tens digit each)
        uint32_t unit = task, t1_begin = 0, t1_end = 10;
        if (task >= A.nbig) {
            const uint32_t k = task - A.nbig;
            const uint32_t u = k / kSplit;
            unit = A.nbig + u;
            t1_begin = k - u * kSplit;
            t1_end = t1_begin + 1;
        }
        const uint32_t tile = unit / A.tpt;
        const uint32_t chunk = unit - tile * A.tpt;
        tiled_task<W1, STRADDLE, TRAILER, CSUM>(
            A.rec + (size_t)tile * kRecWords, chunk, t1_begin, t1_end, (A.tile0 + tile) * A.pow10V,
            A.seg_lo, A.seg_hi, A.vmax, A.q, A.lane_shift, A.loop_shift, A.s0_loop, A.trailer_kw,
            best, sums);
    }
    wave_store<CSUM>(A.cand, A.sums, wslot, best, sums);
}

template <int W1, bool STRADDLE, bool TRAILER>
__global__ void HM_TILED_BOUNDS hm_tiled_kernel(const TiledArgs A) {
    tiled_body<W1, STRADDLE, TRAILER, false>(A);
}

template <int W1, bool STRADDLE, bool TRAILER>
__global__ void HM_TILED_BOUNDS hm_tiled_csum_kernel(const TiledArgs A) {
    tiled_body<W1, STRADDLE, TRAILER, true>(A);
}

// ---------------------------------------------------------------------------
// Chained scan: per lane one compression of tail block 0 per task, then one
// table-driven compression per loop value (the final block is wave-uniform).
// With an epoch (f > fe final-block digits) the loop covers the low fe digits
// and A.ebase supplies the high ones.
// ---------------------------------------------------------------------------
template <bool CSUM>
DEV void chained_body(const ChainedArgs& A) {
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + uni(threadIdx.x / kWaveSize);
    WaveBest best;
    WaveSums sums;  // CSUM only
    const uint32_t per_tile = A.tpt * A.ntc;
    __shared__ LdsQueue queue;
    lds_queue_init(&queue);

    for (;;) {
        const uint32_t task = lds_dequeue(&queue, A.counter, A.lds_shift);
        if (task >= A.ntasks) break;
        // guided sizes: whole loop chunks first, then kSplit pieces of each
        uint32_t unit = task, part = 0, nparts = 1;
        if (task >= A.nbig) {
            const uint32_t k = task - A.nbig;
            const uint32_t u = k / kSplit;
            unit = A.nbig + u;
            part = k - u * kSplit;
            nparts = kSplit;
        }
        const uint32_t tile = unit / per_tile;
        const uint32_t rem = unit - tile * per_tile;
        const uint32_t chunk = rem / A.ntc;
        const uint32_t tc = rem - chunk * A.ntc;
        const uint32_t piece = (A.tch + nparts - 1) / nparts;
        const uint32_t t_begin = tc * A.tch + part * piece;
        uint32_t t_end = tc * A.tch + A.tch;
        if (t_end > A.nloop) t_end = A.nloop;
        if (t_end > t_begin + piece) t_end = t_begin + piece;
        chained_task<CSUM>(A.rec + (size_t)tile * kRecWords, chunk, t_begin, t_end,
                           (A.tile0 + tile) * A.pow10qf + A.ebase, A.pow10f, A.seg_lo, A.seg_hi,
                           A.vmax, A.q, A.kwt, best, sums);
    }
    wave_store<CSUM>(A.cand, A.sums, wslot, best, sums);
}

__global__ void __launch_bounds__(kBlock) hm_chained_kernel(const ChainedArgs A) {
    chained_body<false>(A);
}

__global__ void __launch_bounds__(kBlock) hm_chained_csum_kernel(const ChainedArgs A) {
    chained_body<true>(A);
}

// ---------------------------------------------------------------------------
// Generic scan: one nonce per lane, any layout
// ---------------------------------------------------------------------------
template <bool CSUM>
DEV void generic_body(const GenericArgs& A) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t bk = ~0ull, bn = 0;
    uint64_t csum = 0, ccnt = 0;  // CSUM only
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= A.count_m1;) {
        const uint64_t n = A.seg_lo + k;
        uint32_t w[32];
        build_tail(w, A.pw, A.r, A.d, 0, n, A.nb, A.total_bits);
        uint32_t st[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) st[j] = A.mid[j];
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) m[j] = w[j];
        d_compress(st, m);
        if (A.nb == 2) {
#pragma unroll
            for (int j = 0; j < 16; ++j) m[j] = w[16 + j];
            d_compress(st, m);
        }
        const uint64_t key = ((uint64_t)st[0] << 32) | st[1];
        if constexpr (CSUM) { csum += key; ++ccnt; }
        if (key < bk || (key == bk && n < bn)) { bk = key; bn = n; }
        if (A.count_m1 - k < stride) break;
        k += stride;
    }
    wave_min(bk, bn);
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + threadIdx.x / kWaveSize;
    if (__lane_id() == 0) {
        A.cand[2 * wslot] = bk;
        A.cand[2 * wslot + 1] = bn;
    }
    if constexpr (CSUM) store_sums(A.sums, wslot, csum, ccnt);
}

__global__ void __launch_bounds__(kBlock) hm_generic_kernel(const GenericArgs A) {
    generic_body<false>(A);
}

__global__ void __launch_bounds__(kBlock) hm_generic_csum_kernel(const GenericArgs A) {
    generic_body<true>(A);
}

// Every tiled layout the planner can pick (plan.cpp layout): one tail block
// with W1 = 1..13, or W1 = 13..15 followed by a constant trailer block.
#define HM_TILED_INST(W, S, T)                                                 \
    template __global__ void hm_tiled_kernel<W, S, T>(const TiledArgs);        \
    template __global__ void hm_tiled_csum_kernel<W, S, T>(const TiledArgs);
#define HM_TILED_INST_S(W, T) HM_TILED_INST(W, false, T) HM_TILED_INST(W, true, T)
HM_TILED_INST_S(1, false)
HM_TILED_INST_S(2, false)
HM_TILED_INST_S(3, false)
HM_TILED_INST_S(4, false)
HM_TILED_INST_S(5, false)
HM_TILED_INST_S(6, false)
HM_TILED_INST_S(7, false)
HM_TILED_INST_S(8, false)
HM_TILED_INST_S(9, false)
HM_TILED_INST_S(10, false)
HM_TILED_INST_S(11, false)
HM_TILED_INST_S(12, false)
HM_TILED_INST_S(13, false)
HM_TILED_INST_S(13, true)
HM_TILED_INST_S(14, true)
HM_TILED_INST_S(15, true)
#undef HM_TILED_INST_S
#undef HM_TILED_INST

}  // namespace hm
