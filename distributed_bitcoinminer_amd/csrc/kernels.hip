// kernels.hip -- gfx950 kernels of the min-hash nonce scan.
//
// Replaces the miner's sequential loop (cmu440/bitcoin/miner/miner.go:63-76)
// over bitcoin.Hash (cmu440/bitcoin/hash.go:13-17).  Integer-VALU bound: no
// MFMA, no LDS on the hot path, ~zero HBM traffic.
//
//   hm_tile_plan_kernel  one thread per tile: ASCII high digits, padding,
//                        length, and (two-block tails) the chaining state
//                        after the tail block that holds no varying digit.
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
//   hm_fold_kernel       second reduce pass (candidates -> 16-B best).
//   hm_*_csum_kernel     checked variants of the three scan kernels (same
//                        body, CSUM=true): also the wrapping sum of the keys
//                        and the count of nonces hashed, per wave, folded by
//                        hm_sum_fold_kernel (hm_scan_checked).
#include <hip/hip_runtime.h>

#include <array>
#include <utility>

#include "kernels.hpp"
#include "sha256_defs.hpp"

namespace hm {

#define DEV __device__ __forceinline__

DEV uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_rotateright32(x, n); }
// gfx950 v_bitop3_b32: any 3-input bitwise function in one VALU op (LUT
// index 4*src0 + 2*src1 + src2; 0x96 = three-way XOR).  hipcc forms bitop3
// for Ch/Maj but not for XOR chains, so the Sigma functions use it directly.
// Non-volatile asm: the compiler may still hoist/CSE it.
DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// V = the value varies across lanes (VGPR): use bitop3; otherwise plain C so
// the compiler folds wave-uniform work onto the scalar unit / hoists it.
template <bool V> DEV uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    if constexpr (V) return xor3(a, b, c);
    else return a ^ b ^ c;
}
template <bool V = true> DEV uint32_t bsig0(uint32_t x) { return x3<V>(rotr(x, 2), rotr(x, 13), rotr(x, 22)); }
template <bool V = true> DEV uint32_t bsig1(uint32_t x) { return x3<V>(rotr(x, 6), rotr(x, 11), rotr(x, 25)); }
template <bool V = true> DEV uint32_t ssig0(uint32_t x) { return x3<V>(rotr(x, 7), rotr(x, 18), x >> 3); }
template <bool V = true> DEV uint32_t ssig1(uint32_t x) { return x3<V>(rotr(x, 17), rotr(x, 19), x >> 10); }
// Ch = bfi(e, f, g); Maj = bfi(a ^ b, c, b) -- hipcc emits v_bitop3 for both
DEV uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return ((f ^ g) & e) ^ g; }
DEV uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return ((b ^ c) & (a ^ b)) ^ b; }

DEV uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
DEV uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

// Compile-time variability of the 64 schedule words given the mask VM of
// message words that vary across lanes (bit i = W[i]).
constexpr uint64_t sched_vary(uint32_t vm) {
    uint64_t m = vm;
    for (int t = 16; t < 64; ++t) {
        const uint64_t dep = (m >> (t - 2)) | (m >> (t - 7)) | (m >> (t - 15)) | (m >> (t - 16));
        if (dep & 1) m |= 1ull << t;
    }
    return m;
}
constexpr int first_vary(uint32_t vm) {
    int i = 0;
    while (i < 16 && !((vm >> i) & 1)) ++i;
    return i;
}

struct State { uint32_t a, b, c, d, e, f, g, h; };

// One round I of a message block.  VM marks the message words that vary
// from one evaluation to the next: across lanes for a one-shot compression,
// across iterations of the enclosing nonce loop for the tiled kernel (words
// that vary across lanes but not across the loop are loop-invariant and, as
// plain C, hoisted out of it).  SW >= 0 names a word whose sigma0 the caller
// supplies as s0w: sigma0 is XOR-linear, so for a word built from bit-disjoint
// lane and loop parts, sigma0(lane | loop) = sigma0(lane) ^ sigma0(loop) costs
// one XOR per iteration instead of four instructions.
template <uint32_t VM, int SW, int I>
DEV void round_step(State& s, uint32_t m[16], uint32_t s0w) {
    constexpr uint64_t WV = sched_vary(VM);
    constexpr int F = first_vary(VM);
    uint32_t w;
    if constexpr (I < 16) {
        w = m[I];
    } else {
        constexpr bool v2 = (WV >> (I - 2)) & 1, v7 = (WV >> (I - 7)) & 1;
        constexpr bool v15 = (WV >> (I - 15)) & 1, v16 = (WV >> (I - 16)) & 1;
        // uniform terms summed first (scalar), lane-varying terms after
        uint32_t u = 0, v = 0;
        const uint32_t t2 = ssig1<v2>(m[(I - 2) & 15]);
        uint32_t t15;
        if constexpr (I - 15 == SW) t15 = s0w;
        else t15 = ssig0<v15>(m[(I - 15) & 15]);
        if constexpr (v2) v += t2; else u += t2;
        if constexpr (v7) v += m[(I - 7) & 15]; else u += m[(I - 7) & 15];
        if constexpr (v15) v += t15; else u += t15;
        if constexpr (v16) v += m[I & 15]; else u += m[I & 15];
        w = v + u;
        m[I & 15] = w;
    }
    // a and e vary from the round after the first varying word enters
    constexpr bool ev = I > F;
    const uint32_t t1 = s.h + bsig1<ev>(s.e) + ch(s.e, s.f, s.g) + (kK[I] + w);
    const uint32_t t2 = bsig0<ev>(s.a) + maj(s.a, s.b, s.c);
    s.h = s.g; s.g = s.f; s.f = s.e; s.e = s.d + t1;
    s.d = s.c; s.c = s.b; s.b = s.a; s.a = t1 + t2;
}

template <uint32_t VM, int SW, int... I>
DEV void rounds_seq(State& s, uint32_t m[16], uint32_t s0w, std::integer_sequence<int, I...>) {
    (round_step<VM, SW, I>(s, m, s0w), ...);
}

// 64 rounds from state s over message m (m is clobbered into the schedule
// window).  VM marks the varying words (see round_step), SW/s0w an optional
// caller-supplied sigma0(m[SW]).  On return s.a = a64, s.b = a63 (= b64),
// the rest as well.
template <uint32_t VM, int SW = -1>
DEV void sha_rounds(State& s, uint32_t m[16], uint32_t s0w = 0) {
    rounds_seq<VM, SW>(s, m, s0w, std::make_integer_sequence<int, 64>{});
}

template <int I>
DEV void round_kw(State& s, uint32_t kw) {
    // INV_STATE: round 0 of a block whose start state is invariant in the
    // caller's loop -- plain C lets the compiler hoist its Sigma functions
    constexpr bool v = I > 0;
    const uint32_t t1 = s.h + bsig1<v>(s.e) + ch(s.e, s.f, s.g) + kw;
    const uint32_t t2 = bsig0<v>(s.a) + maj(s.a, s.b, s.c);
    s.h = s.g; s.g = s.f; s.f = s.e; s.e = s.d + t1;
    s.d = s.c; s.c = s.b; s.b = s.a; s.a = t1 + t2;
}

template <bool INV_STATE, int... I>
DEV void rounds_kw_seq(State& s, const uint32_t* __restrict__ kw,
                       std::integer_sequence<int, I...>) {
    (round_kw<INV_STATE ? I : I + 1>(s, kw[I]), ...);
}

// 64 rounds over a constant block given as K[i]+W[i] (wave-uniform).
// INV_STATE: the start state s does not change across the caller's loop.
template <bool INV_STATE = false>
DEV void sha_rounds_kw(State& s, const uint32_t* __restrict__ kw) {
    rounds_kw_seq<INV_STATE>(s, kw, std::make_integer_sequence<int, 64>{});
}

// Lexicographic (key, nonce) min across the 64 lanes; every lane gets it.
DEV void wave_min(uint64_t& k, uint64_t& n) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t k2 = __shfl_xor(k, off, kWaveSize);
        const uint64_t n2 = __shfl_xor(n, off, kWaveSize);
        const bool take = (k2 < k) || (k2 == k && n2 < n);
        k = take ? k2 : k;
        n = take ? n2 : n;
    }
}

// Wrapping sum across the 64 lanes; every lane gets it.
DEV uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, kWaveSize);
    return x;
}

// Checked scans: lane 0 stores the wave's (sum of keys, count) coverage pair.
DEV void store_sums(uint64_t* sums, uint32_t wslot, uint64_t sum, uint64_t cnt) {
    sum = wave_sum(sum);
    cnt = wave_sum(cnt);
    if (__lane_id() == 0) {
        sums[2 * wslot] = sum;
        sums[2 * wslot + 1] = cnt;
    }
}

DEV void put_byte(uint32_t* w, uint32_t pos, uint32_t byte) {
    w[pos >> 2] |= byte << (24u - 8u * (pos & 3u));
}

// ---------------------------------------------------------------------------
// Tile planner
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) hm_tile_plan_kernel(const PlanArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.ntiles) return;
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) w[k] = k < 16 ? A.pw[k] : 0u;
    uint64_t x = (A.tile0 + i) * A.pow10V;  // tile base: low V digits are zero
    for (int j = (int)A.d - 1; j >= 0; --j) {
        const uint64_t y = x / 10u;
        const uint32_t dig = (uint32_t)(x - y * 10u);
        x = y;
        if ((uint32_t)j < A.d - A.V) put_byte(w, A.r + (uint32_t)j, 0x30u + dig);
    }
    put_byte(w, A.r + A.d, 0x80u);
    w[16 * A.nb - 2] = (uint32_t)(A.total_bits >> 32);
    w[16 * A.nb - 1] = (uint32_t)A.total_bits;
    uint32_t st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = A.mid[k];
    uint32_t* out = A.rec + (size_t)i * kRecWords;
    if (A.fb == 1) {
        h_compress(st, w);
#pragma unroll
        for (int k = 0; k < 16; ++k) out[8 + k] = w[16 + k];
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) out[8 + k] = w[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
}

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
        packed <<= A.lane_shift;
        const uint32_t X0 = W[W1 - 1] | (uint32_t)(packed >> 32);
        const uint32_t X1 = W[W1] | (uint32_t)packed;
        const uint64_t nbase = (A.tile0 + tile) * A.pow10V + (uint64_t)v * 100u;
        const uint32_t s0X1 = ssig0<false>(X1);  // lane part of sigma0(W[W1])

        for (uint32_t t1 = t1_begin; t1 < t1_end; ++t1) {
            for (uint32_t t0 = 0; t0 < 10; ++t0) {
                uint32_t m[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) m[k] = W[k];
                // loop digits: wave-uniform, in bytes that are zero in X1
                uint32_t L;
                if constexpr (STRADDLE) {
                    // last digit opens W[W1], the tens digit closes W[W1-1]:
                    // work on W[W1-1] depends on t1 only and is hoisted out
                    // of the t0 loop
                    m[W1 - 1] = X0 + (0x30u + t1);
                    L = (0x30u + t0) << 24;
                } else {
                    m[W1 - 1] = X0;
                    L = (((0x30u + t1) << 8) | (0x30u + t0)) << A.loop_shift;
                }
                m[W1] = X1 | L;
                // only W[W1] changes from one t0 step to the next
                constexpr uint32_t VM = 1u << W1;
                const uint32_t s0w = s0X1 ^ A.s0_loop[t1 * 10u + t0];  // scalar load
                State s{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
                sha_rounds<VM, W1>(s, m, s0w);
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
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) hm_kw_table_kernel(uint32_t* __restrict__ out,
                                                             uint32_t f, uint32_t n,
                                                             uint64_t total_bits) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t w[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) w[k] = 0;
    uint32_t x = t;
    for (int j = (int)f - 1; j >= 0; --j) {  // f digits with leading zeros
        const uint32_t y = x / 10u;
        put_byte(w, (uint32_t)j, 0x30u + x - y * 10u);
        x = y;
    }
    put_byte(w, f, 0x80u);
    w[14] = (uint32_t)(total_bits >> 32);
    w[15] = (uint32_t)total_bits;
    h_schedule(w);
    uint32_t* o = out + (size_t)t * 64;
#pragma unroll
    for (int k = 0; k < 64; ++k) o[k] = kK[k] + w[k];
}

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
        uint32_t packed = 0, x = v;
        for (uint32_t k = 0; k < A.q; ++k) {
            const uint32_t y = x / 10u;
            packed |= (0x30u + x - y * 10u) << (8u * k);
            x = y;
        }
        uint32_t m[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) m[k] = W[k];
        m[15] = W[15] | packed;
        State s{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
        sha_rounds<1u << 15>(s, m);
        // chaining value into the final block (per lane)
        const State cs{s.a + st[0], s.b + st[1], s.c + st[2], s.d + st[3],
                       s.e + st[4], s.f + st[5], s.g + st[6], s.h + st[7]};
        const uint64_t nbase = (A.tile0 + tile) * A.pow10qf + (uint64_t)v * A.pow10f;
        const uint32_t piece = (A.tch + nparts - 1) / nparts;
        const uint32_t t_begin = tc * A.tch + part * piece;
        uint32_t t_end = tc * A.tch + A.tch;
        if (t_end > (uint32_t)A.pow10f) t_end = (uint32_t)A.pow10f;
        if (t_end > t_begin + piece) t_end = t_begin + piece;
        const uint32_t* __restrict__ kw = A.kwt + (size_t)t_begin * 64;
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
#pragma unroll
        for (int j = 0; j < 32; ++j) w[j] = j < 16 ? A.pw[j] : 0u;
        uint64_t x = n;
        for (int j = (int)A.d - 1; j >= 0; --j) {
            const uint64_t y = x / 10u;
            put_byte(w, A.r + (uint32_t)j, 0x30u + (uint32_t)(x - y * 10u));
            x = y;
        }
        put_byte(w, A.r + A.d, 0x80u);
        w[16 * A.nb - 2] = (uint32_t)(A.total_bits >> 32);
        w[16 * A.nb - 1] = (uint32_t)A.total_bits;
        uint32_t st[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) st[j] = A.mid[j];
        h_compress(st, w);
        if (A.nb == 2) h_compress(st, w + 16);
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

// ---------------------------------------------------------------------------
// Second reduce pass and init
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) hm_fold_kernel(const uint64_t* __restrict__ cand,
                                                         uint32_t n, uint32_t stride,
                                                         uint64_t* best) {
    __shared__ uint64_t sk[kBlock / kWaveSize], sn[kBlock / kWaveSize];
    uint64_t k = ~0ull, nn = ~0ull;
    if (threadIdx.x == 0) { k = best[0]; nn = best[1]; }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t k2 = cand[2 * (size_t)i * stride], n2 = cand[2 * (size_t)i * stride + 1];
        if (k2 < k || (k2 == k && n2 < nn)) { k = k2; nn = n2; }
    }
    wave_min(k, nn);
    if (__lane_id() == 0) { sk[threadIdx.x / kWaveSize] = k; sn[threadIdx.x / kWaveSize] = nn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWaveSize; ++w)
            if (sk[w] < k || (sk[w] == k && sn[w] < nn)) { k = sk[w]; nn = sn[w]; }
        best[0] = k;
        best[1] = nn;
    }
}

__global__ void __launch_bounds__(kBlock) hm_sum_fold_kernel(const uint64_t* __restrict__ sums,
                                                             uint32_t n, uint64_t* acc) {
    __shared__ uint64_t ss[kBlock / kWaveSize], sc[kBlock / kWaveSize];
    uint64_t a = 0, c = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        a += sums[2 * (size_t)i];
        c += sums[2 * (size_t)i + 1];
    }
    a = wave_sum(a);
    c = wave_sum(c);
    if (__lane_id() == 0) { ss[threadIdx.x / kWaveSize] = a; sc[threadIdx.x / kWaveSize] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWaveSize; ++w) { a += ss[w]; c += sc[w]; }
        acc[0] += a;
        acc[1] += c;
    }
}

__global__ void hm_init_best_kernel(uint64_t* best, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { best[2 * i] = ~0ull; best[2 * i + 1] = 0; }  // (MaxUint64, 0): miner.go:65-66
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
hipError_t launch_tile_plan(const PlanArgs& a, hipStream_t s) {
    const uint32_t grid = (a.ntiles + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(hm_tile_plan_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

using TiledFn = void (*)(const TiledArgs);

// Instantiated layouts: one tail block W1 1..13, or W1 13..15 with a constant
// trailer block; nullptr = a layout that cannot occur.
template <int W, bool S, bool T, bool C>
constexpr TiledFn tiled_ptr() {
    if constexpr (W >= 1 && W <= 15 && (T ? W >= 13 : W <= 13)) {
        if constexpr (C) return &hm_tiled_csum_kernel<W, S, T>;
        else return &hm_tiled_kernel<W, S, T>;
    } else {
        return nullptr;
    }
}

template <bool S, bool T, bool C, int... W>
constexpr std::array<TiledFn, 16> tiled_row(std::integer_sequence<int, W...>) {
    return {{tiled_ptr<W, S, T, C>()...}};
}

template <bool S, bool T, bool C>
constexpr std::array<TiledFn, 16> tiled_row() {
    return tiled_row<S, T, C>(std::make_integer_sequence<int, 16>{});
}

// [csum][trailer][straddle][W1]
static const std::array<TiledFn, 16> kTiled[2][2][2] = {
    {{tiled_row<false, false, false>(), tiled_row<true, false, false>()},
     {tiled_row<false, true, false>(), tiled_row<true, true, false>()}},
    {{tiled_row<false, false, true>(), tiled_row<true, false, true>()},
     {tiled_row<false, true, true>(), tiled_row<true, true, true>()}}};

static TiledFn tiled_fn(int W1, bool straddle, bool trailer, bool csum = false) {
    if (W1 < 1 || W1 > 15) return nullptr;
    return kTiled[csum ? 1 : 0][trailer ? 1 : 0][straddle ? 1 : 0][W1];
}

hipError_t launch_tiled(const TiledArgs& a, int W1, bool straddle, bool trailer, int grid,
                        hipStream_t s, bool csum) {
    TiledFn fn = tiled_fn(W1, straddle, trailer, csum);
    if (!fn || (csum && !a.sums)) return hipErrorInvalidValue;
    if (grid < 1 || (uint32_t)grid * (kBlock / kWaveSize) > kMaxCandWaves)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

int tiled_blocks_per_cu(int W1, bool straddle, bool trailer) {
    TiledFn fn = tiled_fn(W1, straddle, trailer);
    if (!fn) return 0;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(fn),
                                                     kBlock, 0) != hipSuccess)
        return 0;
    return nb;
}

hipError_t launch_generic(const GenericArgs& a, int grid, hipStream_t s, bool csum) {
    if (grid < 1 || (uint32_t)grid * (kBlock / kWaveSize) > kMaxCandWaves ||
        (csum && !a.sums))
        return hipErrorInvalidValue;
    if (csum) hipLaunchKernelGGL(hm_generic_csum_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL(hm_generic_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_chained(const ChainedArgs& a, int grid, hipStream_t s, bool csum) {
    if (grid < 1 || (uint32_t)grid * (kBlock / kWaveSize) > kMaxCandWaves ||
        (csum && !a.sums))
        return hipErrorInvalidValue;
    if (csum) hipLaunchKernelGGL(hm_chained_csum_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL(hm_chained_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sum_fold(const uint64_t* sums, uint32_t n, uint64_t* acc, hipStream_t s) {
    hipLaunchKernelGGL(hm_sum_fold_kernel, dim3(1), dim3(kBlock), 0, s, sums, n, acc);
    return hipGetLastError();
}

int chained_blocks_per_cu() {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, reinterpret_cast<const void*>(&hm_chained_kernel), kBlock, 0) != hipSuccess)
        return 0;
    return nb;
}

hipError_t launch_kw_table(uint32_t* out, uint32_t f, uint64_t total_bits, hipStream_t s) {
    if (f < 1 || f > kMaxChainedF) return hipErrorInvalidValue;
    uint32_t n = 1;
    for (uint32_t i = 0; i < f; ++i) n *= 10u;
    hipLaunchKernelGGL(hm_kw_table_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                       out, f, n, total_bits);
    return hipGetLastError();
}

hipError_t launch_fold(const uint64_t* cand, uint32_t n, uint64_t* best, hipStream_t s,
                       uint32_t stride) {
    hipLaunchKernelGGL(hm_fold_kernel, dim3(1), dim3(kBlock), 0, s, cand, n, stride, best);
    return hipGetLastError();
}

hipError_t launch_init_best(uint64_t* best, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(hm_init_best_kernel, dim3((n + 63) / 64), dim3(64), 0, s, best, n);
    return hipGetLastError();
}

}  // namespace hm
