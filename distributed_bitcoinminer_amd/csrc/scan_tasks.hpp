// scan_tasks.hpp -- one task of each scan kernel kind, shared by the
// per-segment kernels (scan_kernels.hip) and the fused small-request kernel
// (fused_kernels.hip).
//
// Replaces the miner's sequential loop (cmu440/bitcoin/miner/miner.go:46-59)
// over bitcoin.Hash (cmu440/bitcoin/hash.go:13-17) for one wave's share of
// it: 64 lanes x a run of loop values.  Each task folds its nonces into the
// wave's running (hash, nonce) minimum, which lives in SGPRs (wave-uniform)
// and is refreshed by a 64-lane reduce only when some lane may beat it
// (strict lexicographic order: ties to the lowest nonce, miner.go:56-58).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "sha256_defs.hpp"
#include "sha_device.hpp"

namespace hm {

// A wave's running minimum (uniform) and, for checked scans, its coverage
// sum and count (per lane until the final wave_sum).
struct WaveBest {
    uint32_t hi = 0xffffffffu, lo = 0xffffffffu;  // (MaxUint64, 0): miner.go:48-49
    uint64_t nonce = 0;
};
struct WaveSums {
    uint64_t sum = 0, cnt = 0;
};

// Fold one loop step's per-lane keys (h0, h1) of nonces nbase + off into
// the wave's best.  `cand` is h0 <= best.hi (the caller's one compare per
// nonce); only when some lane holds one does the 64-lane reduce run, and
// only then are the nonce and its range check formed.  Lanes outside
// [seg_lo, seg_hi] never win.
DEV void take_step(WaveBest& best, bool cand, uint32_t h0, uint32_t h1, uint64_t nbase,
                   uint32_t off, uint64_t seg_lo, uint64_t seg_hi) {
    if (__builtin_amdgcn_ballot_w64(cand)) {
        uint64_t key = ((uint64_t)h0 << 32) | h1;
        uint64_t nn = nbase + off;
        const bool ok = cand && nn >= seg_lo && nn <= seg_hi;
        if (!ok) { key = ~0ull; nn = ~0ull; }
        wave_min(key, nn);
        key = uni64(key);
        nn = uni64(nn);
        const uint64_t bk = ((uint64_t)best.hi << 32) | best.lo;
        if (key < bk || (key == bk && nn < best.nonce)) {
            best.hi = (uint32_t)(key >> 32);
            best.lo = (uint32_t)key;
            best.nonce = nn;
        }
    }
}

// Workgroup-level task dispenser (round 5; the per-segment kernels and,
// with kFusedLds, the fused one).  A wave draws a ticket from an
// LDS counter; the first ticket of each batch of kLdsBatch fetches the
// batch's task ids from the launch's queue with ONE device-scope atomic and
// publishes the base in a 4-entry LDS ring; the batch's other tickets wait
// for it there (at most one atomic's round trip, the waves of a workgroup
// rarely finish a task together).  The per-wave task granularity and the
// guided tail are unchanged; the queue sees a quarter of the atomics, which
// execute memory-side (PMC WRITE_SIZE per cfg2 launch 18.1 -> 4.6 MB; cfg2
// +0.1 %, cfg3 +1.0 %, d = 12 +0.04 % in an interleaved A/B,
// profiles/r05/experiments/lds_dispenser/).  The ring cannot be lapped: a
// batch's slot is rewritten only 4 batches (>= 16 tickets) later, and each
// of the 4 waves holds one ticket at a time.  The batch is 2^shift tasks:
// kLdsBatch by default; launches of >= 10^11 nonces (configs[3]'s d = 12
// segment) take 16 (round 6, HM_OPT_QUEUE_BATCH), since a tail imbalance of
// 16 tenth-units is nothing against their seconds of work.
constexpr uint32_t kLdsBatch = 4;
constexpr uint32_t kLdsShift = 2;  // log2(kLdsBatch)
struct LdsQueue {
    uint32_t ticket;
    uint32_t base[4];
    uint32_t ready[4];  // batch + 1 once base[batch & 3] is set
};
DEV void lds_queue_init(LdsQueue* q) {
    if (threadIdx.x == 0) {
        q->ticket = 0;
        for (int i = 0; i < 4; ++i) q->ready[i] = 0;
    }
    __syncthreads();
}
DEV uint32_t lds_dequeue(LdsQueue* q, unsigned int* counter, uint32_t shift = kLdsShift) {
    uint32_t task = 0;
    if (__lane_id() == 0) {
        const uint32_t t = atomicAdd(&q->ticket, 1u);
        const uint32_t batch = t >> shift, slot = batch & 3u;
        if (t - (batch << shift) == 0) {
            q->base[slot] = atomicAdd(counter, 1u << shift);
            __hip_atomic_store(&q->ready[slot], batch + 1, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            while (__hip_atomic_load(&q->ready[slot], __ATOMIC_ACQUIRE,
                                     __HIP_MEMORY_SCOPE_WORKGROUP) != batch + 1)
                __builtin_amdgcn_s_sleep(2);
        }
        task = q->base[slot] + (t - (batch << shift));
    }
    return uni(task);
}

// Lane digits: the q low decimal digits of v as ASCII bytes, least
// significant in the lowest byte.
DEV uint64_t lane_digits(uint32_t v, uint32_t q) {
    uint64_t packed = 0;
    uint32_t x = v;
    for (uint32_t k = 0; k < q; ++k) {
        const uint32_t y = x / 10u;
        packed |= (uint64_t)(0x30u + x - y * 10u) << (8u * k);
        x = y;
    }
    return packed;
}

// ---------------------------------------------------------------------------
// Tiled task: lane chunk `chunk` of the tile whose record is R (chaining
// state + final-block words, varying digits zeroed) and whose first nonce is
// tile_base; loop steps t1 in [t1_begin, t1_end) x t0 in [0, 10): one
// SHA-256 compression per nonce from the tile state (+ a constant trailer
// block, table kw, when the padding spills).  s0_loop[t1*10 + t0] = sigma0
// of the loop-digit bits of W[W1] (wave-uniform, read by scalar loads).
// t0 runs over [t0_begin, t0_end) (the fused launch's split tasks; the
// per-segment kernels take the constant defaults, so their loop is the full
// one).
// ---------------------------------------------------------------------------
template <int W1, bool STRADDLE, bool TRAILER, bool CSUM, typename S0, typename KW>
DEV void tiled_task(const uint32_t* __restrict__ R, uint32_t chunk, uint32_t t1_begin,
                    uint32_t t1_end, uint64_t tile_base, uint64_t seg_lo, uint64_t seg_hi,
                    uint32_t vmax, uint32_t q, uint32_t lane_shift, uint32_t loop_shift,
                    S0 s0_loop, KW trailer_kw, WaveBest& best, WaveSums& sums,
                    uint32_t t0_begin = 0, uint32_t t0_end = 10) {
    static_assert(W1 >= 1 && W1 <= 15, "varying words are W[W1-1], W[W1]");
    // Lane digits may reach back into W[W1-2] (the planner does so when the
    // last two words leave room for fewer than 5 lane digits: 10^3 or 10^4
    // lane values fill 64-lane chunks only to 97.7 / 99.5 %).  W[W1-2] is
    // loop-invariant, so this changes per-task work only: the hot loop's
    // instructions are the same (profiles/r02/isa_audit.txt).
    constexpr bool L3 = W1 >= 2;
    const uint32_t lane = __lane_id();
    uint32_t st[8], W[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = R[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) W[k] = R[8 + k];

    uint32_t v = chunk * kWaveSize + lane;
    const bool lane_ok = v <= vmax;  // CSUM: surplus lanes are not counted
    v = v > vmax ? vmax : v;  // surplus lanes repeat a valid nonce
    uint64_t packed = lane_digits(v, q);
    // the lane digits as a 96-bit big-endian window W[W1-2]:W[W1-1]:W[W1]
    uint32_t Xm2 = 0, X0, X1;
    if constexpr (L3) {
        const unsigned __int128 p = (unsigned __int128)packed << lane_shift;
        Xm2 = W[W1 - 2] | (uint32_t)(p >> 64);
        X0 = W[W1 - 1] | (uint32_t)(p >> 32);
        X1 = W[W1] | (uint32_t)p;
    } else {
        packed <<= lane_shift;  // fits: q + lane_shift/8 <= 8 bytes
        X0 = W[W1 - 1] | (uint32_t)(packed >> 32);
        X1 = W[W1] | (uint32_t)packed;
    }
    const uint64_t nbase = tile_base + (uint64_t)v * 100u;
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
        for (uint32_t t0 = t0_begin; t0 < t0_end; ++t0) {
            uint32_t m[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) m[k] = mw[k];
            const uint32_t L = STRADDLE ? (0x30u + t0) << 24 : (Lt1 | (0x30u + t0)) << loop_shift;
            // X1 and L are bit-disjoint: | is +
            m[W1] = X1 + L;
            const uint32_t s0w = s0X1 ^ s0_loop[t1 * 10u + t0];  // scalar load
            // the state after round W1: a = T1 + T2, e = d + T1
            State s{PT + L, s1.a, s1.b, s1.c, dP + L, s1.e, s1.f, s1.g};
            sha_rounds_range<VM, W1, W1 + 1, 64>(s, m, s0w);
            uint32_t h0, h1;
            if constexpr (TRAILER) {
                State o{s.a + st[0], s.b + st[1], s.c + st[2], s.d + st[3],
                        s.e + st[4], s.f + st[5], s.g + st[6], s.h + st[7]};
                State t = o;
                sha_rounds_kw(t, trailer_kw);
                h0 = t.a + o.a;
                h1 = t.b + o.b;
            } else {
                h0 = s.a + st[0];
                h1 = s.b + st[1];
            }
            if constexpr (CSUM) {
                const uint64_t n = nbase + t1 * 10u + t0;
                if (lane_ok && n >= seg_lo && n <= seg_hi) {
                    sums.sum += ((uint64_t)h0 << 32) | h1;
                    ++sums.cnt;
                }
            }
            take_step(best, h0 <= best.hi, h0, h1, nbase, t1 * 10u + t0, seg_lo, seg_hi);
        }
    }
}

// ---------------------------------------------------------------------------
// Chained task: per lane one compression of tail block 0 (lane digits in
// W15 and the last byte of W14) from the tile record R, then one
// table-driven compression per loop value t in [t_begin, t_end): the final
// block is wave-uniform, its K[i]+W[i] schedule row t comes from kwt (scalar
// loads).  nbase = the first nonce of the lane value (epoch included).
// ---------------------------------------------------------------------------
template <bool CSUM>
DEV void chained_task(const uint32_t* __restrict__ R, uint32_t chunk, uint32_t t_begin,
                      uint32_t t_end, uint64_t tile_base, uint64_t pow10f, uint64_t seg_lo,
                      uint64_t seg_hi, uint32_t vmax, uint32_t q, const uint32_t* kwt,
                      WaveBest& best, WaveSums& sums) {
    const uint32_t lane = __lane_id();
    uint32_t st[8], W[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = R[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) W[k] = R[8 + k];

    uint32_t v = chunk * kWaveSize + lane;
    const bool lane_ok = v <= vmax;
    v = v > vmax ? vmax : v;
    // lane digits: the last q (<= 5) bytes of tail block 0, in W15 and
    // (q = 5) the last byte of W14
    const uint64_t packed = lane_digits(v, q);
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
    const uint64_t nbase = tile_base + (uint64_t)v * pow10f;
    const_u32* kw = (const_u32*)(kwt + (size_t)t_begin * 64);
    for (uint32_t t = t_begin; t < t_end; ++t, kw += 64) {
        State u = cs;
        sha_rounds_kw<true>(u, kw);
        const uint32_t h0 = u.a + cs.a;
        if constexpr (CSUM) {
            const uint64_t n = nbase + t;
            if (lane_ok && n >= seg_lo && n <= seg_hi) {
                sums.sum += ((uint64_t)h0 << 32) | (u.b + cs.b);
                ++sums.cnt;
            }
        }
        take_step(best, h0 <= best.hi, h0, u.b + cs.b, nbase, t, seg_lo, seg_hi);
    }
}

// Write the wave's best (and, checked, its coverage pair) to its slot.
template <bool CSUM>
DEV void wave_store(uint64_t* cand, uint64_t* sums_out, uint32_t wslot, const WaveBest& best,
                    const WaveSums& sums) {
    if (__lane_id() == 0) {
        cand[2 * wslot] = ((uint64_t)best.hi << 32) | best.lo;
        cand[2 * wslot + 1] = best.nonce;
    }
    if constexpr (CSUM) store_sums(sums_out, wslot, sums.sum, sums.cnt);
}

}  // namespace hm
