// scan_kernels.hip -- the gfx950 scan kernels of the min-hash nonce search.
//
// Replaces the miner's sequential loop (cmu440/bitcoin/miner/miner.go:46-59)
// over bitcoin.Hash (cmu440/bitcoin/hash.go:13-17).  Integer-VALU bound: no
// MFMA, no LDS on the hot path, ~zero HBM traffic.
//
//   hm_tiled_kernel      persistent waves; per task 64 lanes x 100 loop
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
    static_assert(W1 >= 1 && W1 <= 15, "varying words are W[W1-1], W[W1]");
    // Lane digits may reach back into W[W1-2] (the planner does so when the
    // last two words leave room for fewer than 5 lane digits: 10^3 or 10^4
    // lane values fill 64-lane chunks only to 97.7 / 99.5 %).  W[W1-2] is
    // loop-invariant, so this changes per-task work only: the hot loop's
    // instructions are the same (profiles/r02/isa_audit.txt).
    constexpr bool L3 = W1 >= 2;
    const uint32_t lane = __lane_id();
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + uni(threadIdx.x / kWaveSize);
    uint32_t best_hi = 0xffffffffu, best_lo = 0xffffffffu;  // wave-uniform (SGPR)
    uint64_t best_nonce = 0;
    uint64_t csum = 0, ccnt = 0;  // CSUM only

    for (;;) {
        uint32_t task = 0;
        if (lane == 0) task = atomicAdd(A.counter, 1u);
        task = uni(task);
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
        const uint32_t* __restrict__ R = A.rec + (size_t)tile * kRecWords;
        uint32_t st[8], W[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) st[k] = R[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) W[k] = R[8 + k];

        uint32_t v = chunk * kWaveSize + lane;
        const bool lane_ok = v <= A.vmax;  // CSUM: surplus lanes are not counted
        v = v > A.vmax ? A.vmax : v;  // surplus lanes repeat a valid nonce
        uint64_t packed = 0;
        uint32_t x = v;
        for (uint32_t k = 0; k < A.q; ++k) {
            const uint32_t y = x / 10u;
            packed |= (uint64_t)(0x30u + x - y * 10u) << (8u * k);
            x = y;
        }
        // the lane digits as a 96-bit big-endian window W[W1-2]:W[W1-1]:W[W1]
        uint32_t Xm2 = 0, X0, X1;
        if constexpr (L3) {
            const unsigned __int128 p = (unsigned __int128)packed << A.lane_shift;
            Xm2 = W[W1 - 2] | (uint32_t)(p >> 64);
            X0 = W[W1 - 1] | (uint32_t)(p >> 32);
            X1 = W[W1] | (uint32_t)p;
        } else {
            packed <<= A.lane_shift;  // fits: q + lane_shift/8 <= 8 bytes
            X0 = W[W1 - 1] | (uint32_t)(packed >> 32);
            X1 = W[W1] | (uint32_t)packed;
        }
        const uint64_t nbase = (A.tile0 + tile) * A.pow10V + (uint64_t)v * 100u;
        const uint32_t s0X1 = ssig0<false>(X1);  // lane part of sigma0(W[W1])

        // only W[W1] changes from one t0 step to the next
        constexpr uint32_t VM = 1u << W1;
        for (uint32_t t1 = t1_begin; t1 < t1_end; ++t1) {
            uint32_t mw[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) mw[k] = W[k];
            if constexpr (L3) mw[W1 - 2] = Xm2;
            // loop digits: wave-uniform, in bytes that are zero in X1
            uint32_t Lt1;
            if constexpr (STRADDLE) {
                // last digit opens W[W1], the tens digit closes W[W1-1]
                mw[W1 - 1] = X0 + (0x30u + t1);
                Lt1 = 0;
            } else {
                mw[W1 - 1] = X0;
                Lt1 = (0x30u + t1) << 8;
            }
            // rounds before W[W1] and round W1 without its loop digits: per
            // t1.  Round W1 in closed form: T1 = P + L with P invariant in the
            // t0 loop, so e and a each cost one add of the uniform L there
            // (the empty asm keeps d + P and P + T2 as the two hoisted sums;
            // else P + L is shared and costs a third add per nonce).
            State s1{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
            sha_rounds_range<VM, W1, 0, W1>(s1, mw, 0);
            const uint32_t P = s1.h + bsig1<false>(s1.e) + ch(s1.e, s1.f, s1.g) + (kK[W1] + X1);
            const uint32_t T2 = bsig0<false>(s1.a) + maj(s1.a, s1.b, s1.c);
            uint32_t dP = s1.d + P, PT = P + T2;
            asm volatile("" : "+v"(dP), "+v"(PT));
            for (uint32_t t0 = 0; t0 < 10; ++t0) {
                uint32_t m[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) m[k] = mw[k];
                const uint32_t L = STRADDLE ? (0x30u + t0) << 24 : (Lt1 | (0x30u + t0)) << A.loop_shift;
                // X1 and L are bit-disjoint: | is +
                m[W1] = X1 + L;
                const uint32_t s0w = s0X1 ^ A.s0_loop[t1 * 10u + t0];  // scalar load
                // the state after round W1: a = T1 + T2, e = d + T1
                State s{PT + L, s1.a, s1.b, s1.c, dP + L, s1.e, s1.f, s1.g};
                sha_rounds_range<VM, W1, W1 + 1, 64>(s, m, s0w);
                uint32_t h0, h1;
                if constexpr (TRAILER) {
                    State o{s.a + st[0], s.b + st[1], s.c + st[2], s.d + st[3],
                            s.e + st[4], s.f + st[5], s.g + st[6], s.h + st[7]};
                    State t = o;
                    sha_rounds_kw(t, A.trailer_kw);
                    h0 = t.a + o.a;
                    h1 = t.b + o.b;
                } else {
                    h0 = s.a + st[0];
                    h1 = s.b + st[1];
                }
                if constexpr (CSUM) {
                    const uint64_t n = nbase + t1 * 10u + t0;
                    if (lane_ok && n >= A.seg_lo && n <= A.seg_hi) {
                        csum += ((uint64_t)h0 << 32) | h1;
                        ++ccnt;
                    }
                }
                const bool cand = h0 <= best_hi;
                if (__builtin_amdgcn_ballot_w64(cand)) {
                    // rare: some lane may beat the wave's best
                    uint64_t key = ((uint64_t)h0 << 32) | h1;
                    uint64_t n = nbase + t1 * 10u + t0;
                    const bool ok = cand && n >= A.seg_lo && n <= A.seg_hi;
                    if (!ok) { key = ~0ull; n = ~0ull; }
                    wave_min(key, n);
                    key = uni64(key);
                    n = uni64(n);
                    const uint64_t bk = ((uint64_t)best_hi << 32) | best_lo;
                    if (key < bk || (key == bk && n < best_nonce)) {
                        best_hi = (uint32_t)(key >> 32);
                        best_lo = (uint32_t)key;
                        best_nonce = n;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        A.cand[2 * wslot] = ((uint64_t)best_hi << 32) | best_lo;
        A.cand[2 * wslot + 1] = best_nonce;
    }
    if constexpr (CSUM) store_sums(A.sums, wslot, csum, ccnt);
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
    const uint32_t lane = __lane_id();
    const uint32_t wslot = blockIdx.x * (kBlock / kWaveSize) + uni(threadIdx.x / kWaveSize);
    uint32_t best_hi = 0xffffffffu, best_lo = 0xffffffffu;
    uint64_t best_nonce = 0;
    uint64_t csum = 0, ccnt = 0;  // CSUM only
    const uint32_t per_tile = A.tpt * A.ntc;

    for (;;) {
        uint32_t task = 0;
        if (lane == 0) task = atomicAdd(A.counter, 1u);
        task = uni(task);
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
        const uint32_t* __restrict__ R = A.rec + (size_t)tile * kRecWords;
        uint32_t st[8], W[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) st[k] = R[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) W[k] = R[8 + k];

        uint32_t v = chunk * kWaveSize + lane;
        const bool lane_ok = v <= A.vmax;
        v = v > A.vmax ? A.vmax : v;
        // lane digits: the last q (<= 5) bytes of tail block 0, in W15 and
        // (q = 5) the last byte of W14
        uint64_t packed = 0;
        uint32_t x = v;
        for (uint32_t k = 0; k < A.q; ++k) {
            const uint32_t y = x / 10u;
            packed |= (uint64_t)(0x30u + x - y * 10u) << (8u * k);
            x = y;
        }
        uint32_t m[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) m[k] = W[k];
        m[14] = W[14] | (uint32_t)(packed >> 32);
        m[15] = W[15] | (uint32_t)packed;
        State s{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
        sha_rounds<3u << 14>(s, m);  // once per task: W14, W15 vary across lanes
        // chaining value into the final block (per lane)
        const State cs{s.a + st[0], s.b + st[1], s.c + st[2], s.d + st[3],
                       s.e + st[4], s.f + st[5], s.g + st[6], s.h + st[7]};
        const uint64_t nbase = (A.tile0 + tile) * A.pow10qf + (uint64_t)v * A.pow10f + A.ebase;
        const uint32_t piece = (A.tch + nparts - 1) / nparts;
        const uint32_t t_begin = tc * A.tch + part * piece;
        uint32_t t_end = tc * A.tch + A.tch;
        if (t_end > A.nloop) t_end = A.nloop;
        if (t_end > t_begin + piece) t_end = t_begin + piece;
        const_u32* kw = (const_u32*)(A.kwt + (size_t)t_begin * 64);
        for (uint32_t t = t_begin; t < t_end; ++t, kw += 64) {
            State u = cs;
            sha_rounds_kw<true>(u, kw);
            const uint32_t h0 = u.a + cs.a;
            if constexpr (CSUM) {
                const uint64_t n = nbase + t;
                if (lane_ok && n >= A.seg_lo && n <= A.seg_hi) {
                    csum += ((uint64_t)h0 << 32) | (u.b + cs.b);
                    ++ccnt;
                }
            }
            const bool cand = h0 <= best_hi;
            if (__builtin_amdgcn_ballot_w64(cand)) {
                uint64_t key = ((uint64_t)h0 << 32) | (u.b + cs.b);
                uint64_t n = nbase + t;
                const bool ok = cand && n >= A.seg_lo && n <= A.seg_hi;
                if (!ok) { key = ~0ull; n = ~0ull; }
                wave_min(key, n);
                key = uni64(key);
                n = uni64(n);
                const uint64_t bk = ((uint64_t)best_hi << 32) | best_lo;
                if (key < bk || (key == bk && n < best_nonce)) {
                    best_hi = (uint32_t)(key >> 32);
                    best_lo = (uint32_t)key;
                    best_nonce = n;
                }
            }
        }
    }
    if (lane == 0) {
        A.cand[2 * wslot] = ((uint64_t)best_hi << 32) | best_lo;
        A.cand[2 * wslot + 1] = best_nonce;
    }
    if constexpr (CSUM) store_sums(A.sums, wslot, csum, ccnt);
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
