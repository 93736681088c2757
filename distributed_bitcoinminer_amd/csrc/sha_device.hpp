// sha_device.hpp -- device-side building blocks of the scan kernels (gfx950):
// SHA-256 rounds specialised by which message words vary, wave reductions.
//
// The reference computes SHA-256 through Go's crypto/sha256 inside
// bitcoin.Hash (cmu440/bitcoin/hash.go:14-16); the scan loop is
// cmu440/bitcoin/miner/miner.go:46-59.
#pragma once
#include <hip/hip_runtime.h>

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

template <uint32_t VM, int SW, int FROM = 0, int... I>
DEV void rounds_seq(State& s, uint32_t m[16], uint32_t s0w, std::integer_sequence<int, I...>) {
    (round_step<VM, SW, FROM + I>(s, m, s0w), ...);
}

// Rounds [FROM, TO) only (see sha_rounds).
template <uint32_t VM, int SW, int FROM, int TO>
DEV void sha_rounds_range(State& s, uint32_t m[16], uint32_t s0w = 0) {
    rounds_seq<VM, SW, FROM>(s, m, s0w, std::make_integer_sequence<int, TO - FROM>{});
}

// 64 rounds from state s over message m (m is clobbered into the schedule
// window).  VM marks the varying words (see round_step), SW/s0w an optional
// caller-supplied sigma0(m[SW]).  On return s.a = a64, s.b = a63 (= b64),
// the rest as well.
template <uint32_t VM, int SW = -1>
DEV void sha_rounds(State& s, uint32_t m[16], uint32_t s0w = 0) {
    rounds_seq<VM, SW>(s, m, s0w, std::make_integer_sequence<int, 64>{});
}

// One full compression of a lane-varying block (generic kernel): st += rounds(m).
DEV void d_compress(uint32_t st[8], uint32_t m[16]) {
    State s{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
    sha_rounds<0xFFFFu>(s, m);
    st[0] += s.a; st[1] += s.b; st[2] += s.c; st[3] += s.d;
    st[4] += s.e; st[5] += s.f; st[6] += s.g; st[7] += s.h;
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

template <bool INV_STATE, typename KW, int... I>
DEV void rounds_kw_seq(State& s, KW kw, std::integer_sequence<int, I...>) {
    (round_kw<INV_STATE ? I : I + 1>(s, kw[I]), ...);
}

// 64 rounds over a constant block given as K[i]+W[i] (wave-uniform).
// INV_STATE: the start state s does not change across the caller's loop.
template <bool INV_STATE = false, typename KW>
DEV void sha_rounds_kw(State& s, KW kw) {
    rounds_kw_seq<INV_STATE>(s, kw, std::make_integer_sequence<int, 64>{});
}

// A table pointer in the constant address space: with a wave-uniform index
// the compiler reads it with scalar loads (SGPR operands, no VMEM in the loop).
typedef const __attribute__((address_space(4))) uint32_t const_u32;

// Cross-lane exchange without LDS (gfx950).  Each step gives every lane a
// second value so that, after the six steps of a reduction, every lane has
// seen all 64: DPP within rows of 16 (quad_perm [1,0,3,2] and [2,3,0,1], then
// row_half_mirror and row_mirror, which reach the other quad / half-row once
// those hold equal values), v_permlane16_swap across row pairs and
// v_permlane32_swap across the wave halves.  A swap of x with itself returns
// (x from one side, x from the other) for a lane pair, i.e. both operands of
// the pair's combine, on both lanes.
template <int CTRL> DEV uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int CTRL> DEV uint64_t dpp64(uint64_t x) {
    return ((uint64_t)dpp32<CTRL>((uint32_t)(x >> 32)) << 32) | dpp32<CTRL>((uint32_t)x);
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror: lane i <-> 7-i within 8
constexpr int kDppMirror = 0x140;     // row_mirror: lane i <-> 15-i within 16

// permlane{16,32}_swap of a 64-bit value with itself: (side A, side B).
template <int W> DEV void swap64(uint64_t x, uint64_t& a, uint64_t& b) {
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    if constexpr (W == 16) {
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        a = ((uint64_t)h[0] << 32) | l[0];
        b = ((uint64_t)h[1] << 32) | l[1];
    } else {
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        a = ((uint64_t)h[0] << 32) | l[0];
        b = ((uint64_t)h[1] << 32) | l[1];
    }
}

DEV void lex_take(uint64_t& k, uint64_t& n, uint64_t k2, uint64_t n2) {
    const bool take = (k2 < k) || (k2 == k && n2 < n);
    k = take ? k2 : k;
    n = take ? n2 : n;
}

template <int CTRL> DEV void min_step_dpp(uint64_t& k, uint64_t& n) {
    lex_take(k, n, dpp64<CTRL>(k), dpp64<CTRL>(n));
}
template <int W> DEV void min_step_swap(uint64_t& k, uint64_t& n) {
    uint64_t ka, kb, na, nb;
    swap64<W>(k, ka, kb);
    swap64<W>(n, na, nb);
    k = ka;
    n = na;
    lex_take(k, n, kb, nb);
}

// Lexicographic (key, nonce) min across the 64 lanes; every lane gets it.
DEV void wave_min(uint64_t& k, uint64_t& n) {
    min_step_dpp<kDppXor1>(k, n);
    min_step_dpp<kDppXor2>(k, n);
    min_step_dpp<kDppHalfMirror>(k, n);
    min_step_dpp<kDppMirror>(k, n);
    min_step_swap<16>(k, n);
    min_step_swap<32>(k, n);
}

// Wrapping sum across the 64 lanes; every lane gets it.
DEV uint64_t wave_sum(uint64_t x) {
    x += dpp64<kDppXor1>(x);
    x += dpp64<kDppXor2>(x);
    x += dpp64<kDppHalfMirror>(x);
    x += dpp64<kDppMirror>(x);
    uint64_t a, b;
    swap64<16>(x, a, b);
    x = a + b;
    swap64<32>(x, a, b);
    return a + b;
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

// Tail block words of msg ‖ ' ' ‖ decimal(n) after the midstate (hash.go:15):
// r prefix bytes (pw, zero past r), the d digits of n, 0x80, zeros and the
// 64-bit bit length in the last two words of block nb-1.  The `skip` lowest
// digits are left as zero bytes (the tile planner's varying digits).
// Every array index is a compile-time constant after unrolling, so w and the
// digit words stay in registers (no scratch).  Digit positions are taken
// relative to E = r + d - 1 (wave-uniform): the k-th least significant digit
// lands in word kE - k/4 or the one below, so the digits and 0x80 fill a
// 7-word window (words kE - 5 .. kE + 1), which a 5-stage barrel shift by
// the uniform kE moves into place -- 5 uniform conditions instead of a
// compare per (word, window slot), which would all be loop-invariant SGPR
// masks.
DEV void build_tail(uint32_t w[32], const uint32_t* pw, uint32_t r, uint32_t d, uint32_t skip,
                    uint64_t n, uint32_t nb, uint64_t total_bits) {
    const uint32_t E = r + d - 1, kE = E >> 2, e = E & 3u;
    // before the shift v[i] holds word i - 5 + kE of the window (i in [0, 6]:
    // words kE - 5 .. kE + 1); after it v[5 + k] holds word k
    uint32_t v[37];
#pragma unroll
    for (int i = 0; i < 37; ++i) v[i] = 0u;
    uint64_t x = n;
#pragma unroll
    for (uint32_t k = 0; k < 20; ++k) {
        if (k < d) {
            const uint64_t y = x / 10u;
            const uint32_t b = k < skip ? 0u : (0x30u + (uint32_t)(x - y * 10u))
                                                   << (24u - 8u * ((e - k) & 3u));
            x = y;
            const bool below = (k & 3u) > e;  // crosses into the next lower word
            v[5 - (k >> 2)] |= below ? 0u : b;
            v[4 - (k >> 2)] |= below ? b : 0u;
        }
    }
    if (e == 3u) v[6] = 0x80u << 24;
    else v[5] |= 0x80u << (16u - 8u * e);
    // shift left by kE words: afterwards v[5 + k] = word k (k in [0, 31])
#pragma unroll
    for (int b = 1; b <= 16; b <<= 1) {
        const bool on = (kE & (uint32_t)b) != 0;
#pragma unroll
        for (int i = 36; i >= 0; --i) v[i] = on ? (i >= b ? v[i - b] : 0u) : v[i];
    }
    const bool two = nb == 2;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        uint32_t o = (k < 16 ? pw[k] : 0u) | v[5 + k];
        if (k == 14) o = two ? o : (uint32_t)(total_bits >> 32);
        if (k == 15) o = two ? o : (uint32_t)total_bits;
        if (k == 30) o = two ? (uint32_t)(total_bits >> 32) : o;
        if (k == 31) o = two ? (uint32_t)total_bits : o;
        w[k] = o;
    }
}

}  // namespace hm
