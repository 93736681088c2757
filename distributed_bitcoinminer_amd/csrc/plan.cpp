// plan.cpp -- host planner (see plan.hpp and DESIGN.md §3).
#include "plan.hpp"

#include <math.h>
#include <string.h>

#include <algorithm>

#include "../../include/hipminer.h"
#include "sha256_defs.hpp"

namespace hm {

uint32_t digits_u64(uint64_t n) {
    uint32_t d = 1;
    while (n >= 10) { n /= 10; ++d; }
    return d;
}

uint64_t pow10_u64(uint32_t k) {
    uint64_t p = 1;
    for (uint32_t i = 0; i < k; ++i) p *= 10u;
    return p;
}

MsgPlan plan_message(const uint8_t* msg, uint64_t len) {
    MsgPlan mp;
    memcpy(mp.mid, kIV, sizeof mp.mid);
    mp.len = len;
    const uint64_t plen = len + 1;  // msg ‖ ' '
    const uint64_t nconst = plen / 64;
    uint8_t blk[64];
    for (uint64_t b = 0; b < nconst; ++b) {
        for (int i = 0; i < 64; ++i) {
            const uint64_t p = 64 * b + i;
            blk[i] = p < len ? msg[p] : 0x20;
        }
        uint32_t m[16];
        h_load_block(m, blk);
        h_compress(mp.mid, m);
    }
    mp.r = (uint32_t)(plen - 64 * nconst);
    memset(blk, 0, sizeof blk);
    for (uint32_t i = 0; i < mp.r; ++i) {
        const uint64_t p = 64 * nconst + i;
        blk[i] = p < len ? msg[p] : 0x20;
    }
    h_load_block(mp.pw, blk);
    return mp;
}

static void tiled_layout(const MsgPlan& mp, SegPlan& s);

// Final-block digits a chained K+W table covers (10^7 rows, 2.56 GB: with 3
// lane digits a launch then covers 10^10 nonces, ~0.2 s, so its tail is
// small); more final-block digits run as epochs (kernels.hpp kMaxTableDigits).
constexpr uint32_t kTableDigits = 7;
// Loop values per unit of a chained layout with >= 5 final-block digits:
// 64 lanes x 100 table-driven blocks, a wave's task ~1 ms (block 0 adds 1 %).
constexpr uint32_t kEpochTch = 100;

double chained_lane_eff(const SegPlan& s) {
    const uint64_t P = s.pow10V, S = pow10_u64(s.f);
    const uint64_t tlo = s.lo / P, thi = s.hi / P;
    const uint64_t cf = (s.lo - tlo * P) / S / 64, cl = (s.hi - thi * P) / S / 64;
    const long double chunks = (long double)(thi - tlo) * s.tpt + (long double)cl - (long double)cf + 1;
    return (double)(((long double)(s.hi - s.lo) + 1) / (chunks * 64.0L * (long double)S));
}

// Two-block tails with f >= 5 final-block digits whose tail block 0 holds
// >= 3 digits: the chained layout (lanes in block 0, the final block from a
// K+W table, epochs beyond 10^7 rows) replaces the tiled one when its
// modelled cost, with the out-of-range lanes of its edge chunks, is lower.
static void consider_chained_epochs(const MsgPlan& mp, SegPlan& s, int table_digits) {
    const uint32_t f = s.T - 64;
    if (table_digits < 0) return;
    const uint32_t q = std::min<uint32_t>(5u, 64u - mp.r);  // 64 - r digits in block 0
    if (f < 5 || q < 3 || q + f > 19) return;  // 10^(q+f) nonces per tile fit in u64
    SegPlan c = s;  // W1 / straddle keep the tail's geometry, as for f <= 4
    c.kind = HM_KIND_CHAINED;
    c.trailer = false;
    c.lane3 = false;
    c.lane_shift = c.loop_shift = 0;
    c.f = f;
    c.fe = std::min(f, table_digits >= 1 && table_digits <= (int)kTableDigits ? (uint32_t)table_digits
                                                                                 : kTableDigits);
    c.q = q;
    c.V = q + f;
    c.pow10V = pow10_u64(c.V);
    c.tpt = (uint32_t)((pow10_u64(q) + 63) / 64);
    c.tch = (uint32_t)std::min<uint64_t>(kEpochTch, pow10_u64(c.fe));
    c.ntc = (uint32_t)(pow10_u64(c.fe) / c.tch);
    c.tile_lo = c.lo / c.pow10V;
    c.tile_hi = c.hi / c.pow10V;
    if (seg_cost(c) < seg_cost(s)) s = c;
}

static void layout(const MsgPlan& mp, SegPlan& s, bool force_generic, int table_digits) {
    s.T = mp.r + s.d;
    s.nb = (s.T + 9 <= 64) ? 1 : 2;
    s.fb = (s.T - 1) / 64;
    s.p_end = (s.T - 1) % 64;
    s.total_bits = (mp.len + 1 + s.d) * 8;
    s.kind = HM_KIND_GENERIC;
    s.W1 = (int)(s.p_end / 4);
    const uint32_t k = s.p_end % 4;
    s.straddle = (k == 0);
    s.trailer = (s.nb - 1 > s.fb);
    s.V = s.q = s.lane_shift = s.loop_shift = s.tpt = 0;
    s.lane3 = false;
    s.f = s.fe = s.tch = s.ntc = 0;
    s.pow10V = 1;
    s.tile_lo = s.tile_hi = 0;
    if (force_generic) return;
    if (s.fb == 1 && s.T - 64 <= 4) {
        // Chained: the final block holds only f <= 4 digits (uniform loop
        // index, schedule from a K+W table); lanes vary the last q <= 5
        // digits of tail block 0 (W15 and the last byte of W14): 10^5 lane
        // values fill 64-lane chunks to 99.97 % (10^4: 99.5 %).
        const uint32_t f = s.T - 64;
        const uint32_t q = std::min<uint32_t>(5u, 64u - mp.r);
        if (q >= 2) {
            s.kind = HM_KIND_CHAINED;
            s.f = f;
            s.fe = f;
            s.q = q;
            s.V = q + f;
            s.pow10V = pow10_u64(s.V);
            s.tpt = (uint32_t)((pow10_u64(q) + 63) / 64);
            const uint32_t nloop = (uint32_t)pow10_u64(f);
            s.tch = std::min<uint32_t>(nloop, 1000u);
            s.ntc = (nloop + s.tch - 1) / s.tch;
            s.tile_lo = s.lo / s.pow10V;
            s.tile_hi = s.hi / s.pow10V;
            return;
        }
    }
    tiled_layout(mp, s);
    if (s.fb == 1) consider_chained_epochs(mp, s, table_digits);
}

// The tiled layout of segment s, if any (else s stays generic).
static void tiled_layout(const MsgPlan& mp, SegPlan& s) {
    const uint32_t k = s.p_end % 4;
    if (s.W1 < 1) return;
    const uint32_t ds = (s.fb == 0) ? mp.r : 0;  // first digit byte within block fb
    const uint32_t vs = std::max<uint32_t>(4u * (uint32_t)(s.W1 - 1), ds);
    if (vs > s.p_end) return;
    s.V = s.p_end - vs + 1;
    // 10^q lane values fill ceil(10^q / 64) chunks of 64 lanes: q = 3 wastes
    // 2.3 % of the lanes, q = 4 0.5 %, q = 5 0.03 %.  When the last two words
    // hold fewer than 5 lane digits (the last digit in byte 0 or 1 of W[W1]),
    // the lanes reach back into W[W1-2] for q = 5.
    if (s.V < 7 && s.W1 >= 2) {
        const uint32_t vs3 = std::max<uint32_t>(4u * (uint32_t)(s.W1 - 2), ds);
        const uint32_t V3 = std::min<uint32_t>(s.p_end - vs3 + 1, 7u);
        if (vs3 <= s.p_end && V3 > s.V) {
            s.V = V3;
            s.lane3 = true;
        }
    }
    if (s.V < 5) return;  // q >= 3 lane digits keeps surplus lanes under 3 %
    s.q = s.V - 2;
    s.lane_shift = 8u * (5u - k);
    s.loop_shift = 8u * (3u - k);
    s.pow10V = pow10_u64(s.V);
    const uint64_t lanes = pow10_u64(s.q);
    s.tpt = (uint32_t)((lanes + 63) / 64);
    s.tile_lo = s.lo / s.pow10V;
    s.tile_hi = s.hi / s.pow10V;
    s.kind = HM_KIND_TILED;
}

std::vector<SegPlan> plan_range(const MsgPlan& mp, uint64_t lo, uint64_t hi, bool force_generic,
                                int table_digits) {
    std::vector<SegPlan> out;
    const uint32_t d0 = digits_u64(lo), d1 = digits_u64(hi);
    for (uint32_t d = d0; d <= d1; ++d) {
        SegPlan s;
        s.d = d;
        const uint64_t dlo = d == 1 ? 0 : pow10_u64(d - 1);
        const uint64_t dhi = d == 20 ? ~0ull : pow10_u64(d) - 1;
        s.lo = std::max(lo, dlo);
        s.hi = std::min(hi, dhi);
        if (s.lo > s.hi) continue;
        layout(mp, s, force_generic, table_digits);
        out.push_back(s);
    }
    return out;
}

double seg_cost(const SegPlan& s) {
    // Measured SIMD cycles per 64 nonces of the kernel instantiation that
    // runs the segment: 64 * 1024 SIMDs * 2.38 GHz / kernel GH/s from the
    // layout sweep (tools/layout_perf.py, profiles/r01/session2/layout_perf.txt).
    // tiled, one block, by W1 (straddle variants differ by < 0.3 %)
    static const double kTiled[14] = {0,    4481, 4404, 4311, 4232, 4149, 4074,
                                      3987, 3913, 4007, 3927, 3837, 3751, 3673};
    switch (s.kind) {
        case HM_KIND_TILED:
            if (s.trailer) return 6980.0;  // digit block + constant trailer block (W1 13..15)
            return kTiled[std::min(std::max(s.W1, 1), 13)];
        case HM_KIND_CHAINED:
            // per-lane block 0 amortised over 10^f table-driven final blocks;
            // f >= 5: block 0 once per 100 loop values (+1 %), and the edge
            // chunks' out-of-range lanes
            if (s.f >= 5) return 3275.0 / chained_lane_eff(s);
            return s.f == 1 ? 3777.0 : 3240.0;
        default:
            // generic: every tail block per lane, no hoisting (estimate)
            return 6000.0 * s.nb;
    }
}

std::vector<Shard> partition_range(const MsgPlan& mp, uint64_t lo, uint64_t hi, int n,
                                   bool force_generic) {
    std::vector<Shard> out(n > 0 ? n : 0, Shard{0, 0, true});
    if (n <= 0 || lo > hi) return out;
    typedef unsigned __int128 u128;
    const std::vector<SegPlan> segs = plan_range(mp, lo, hi, force_generic);
    std::vector<long double> cost(segs.size());
    long double total = 0;
    for (size_t i = 0; i < segs.size(); ++i) {
        cost[i] = (long double)(segs[i].hi - segs[i].lo + 1) * seg_cost(segs[i]);
        total += cost[i];
    }
    // start[i] = offset of shard i's first nonce from lo; start[n] = count
    const u128 count = (u128)(hi - lo) + 1;
    std::vector<u128> start(n + 1);
    start[0] = 0;
    start[n] = count;
    size_t si = 0;
    long double before = 0;  // cost of the segments ahead of segs[si]
    for (int i = 1; i < n; ++i) {
        const long double target = total * i / n;
        while (si < segs.size() && before + cost[si] <= target) before += cost[si++];
        u128 b = count;
        if (si < segs.size()) {
            const uint64_t cnt_m1 = segs[si].hi - segs[si].lo;
            long double k = floorl((target - before) / seg_cost(segs[si]));
            if (k < 0) k = 0;
            const u128 kk = k > (long double)cnt_m1 ? (u128)cnt_m1 + 1 : (u128)(uint64_t)k;
            b = (u128)(segs[si].lo - lo) + kk;
            const SegPlan& g = segs[si];
            if (g.kind == HM_KIND_CHAINED && g.f >= 5 && kk > 0 && kk <= cnt_m1) {
                // A chained f >= 5 lane chunk spans 64 * 10^f nonces (lanes
                // stride 10^f) and is hashed whole by every shard that touches
                // it: a cut inside one would hash it twice.  Cut at the nearest
                // lane-chunk boundary of the tile instead (at most half a
                // chunk away from the cost target).
                const u128 x = (u128)lo + b;  // the next shard's first nonce
                const u128 P = g.pow10V, C = (u128)64 * pow10_u64(g.f);
                const u128 t0 = x / P * P;
                const u128 c = (x - t0 + C / 2) / C;
                const u128 snapped = t0 + std::min(c * C, P);
                if (snapped > (u128)g.lo && snapped <= (u128)g.hi) b = snapped - lo;
            }
        }
        start[i] = std::min(count, std::max(b, start[i - 1]));
    }
    for (int i = 0; i < n; ++i) {
        if (start[i + 1] > start[i]) {
            out[i].empty = false;
            out[i].lo = lo + (uint64_t)start[i];
            out[i].hi = lo + (uint64_t)(start[i + 1] - 1);
        }
    }
    return out;
}

uint64_t host_hash(const uint8_t* msg, uint64_t len, uint64_t nonce) {
    char dig[24];
    int nd = 0;
    do { dig[nd++] = (char)('0' + nonce % 10); nonce /= 10; } while (nonce);
    const uint64_t total = len + 1 + (uint64_t)nd;
    uint32_t st[8];
    memcpy(st, kIV, sizeof st);
    uint8_t blk[64];
    uint64_t pos = 0;
    auto byte_at = [&](uint64_t p) -> uint8_t {
        if (p < len) return msg[p];
        if (p == len) return 0x20;
        return (uint8_t)dig[nd - 1 - (int)(p - len - 1)];
    };
    while (total - pos >= 64) {
        for (int i = 0; i < 64; ++i) blk[i] = byte_at(pos + i);
        uint32_t m[16];
        h_load_block(m, blk);
        h_compress(st, m);
        pos += 64;
    }
    uint8_t tail[128];
    memset(tail, 0, sizeof tail);
    const uint32_t rem = (uint32_t)(total - pos);
    for (uint32_t i = 0; i < rem; ++i) tail[i] = byte_at(pos + i);
    tail[rem] = 0x80;
    const uint32_t tl = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = total * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    for (uint32_t b = 0; b < tl; b += 64) {
        uint32_t m[16];
        h_load_block(m, tail + b);
        h_compress(st, m);
    }
    return ((uint64_t)st[0] << 32) | st[1];
}

void tiled_loop_sigma0(const SegPlan& s, uint32_t out[100]) {
    for (uint32_t t1 = 0; t1 < 10; ++t1)
        for (uint32_t t0 = 0; t0 < 10; ++t0) {
            // the loop digits' bits of W[W1] (hm_tiled_kernel): the units digit
            // opens the word when the tens digit straddles into W[W1-1]
            const uint32_t L = s.straddle ? (0x30u + t0) << 24
                                          : (((0x30u + t1) << 8) | (0x30u + t0)) << s.loop_shift;
            out[t1 * 10 + t0] = h_rotr(L, 7) ^ h_rotr(L, 18) ^ (L >> 3);
        }
}

void trailer_kw(const SegPlan& s, uint32_t kw[64]) {
    uint32_t w[64];
    memset(w, 0, sizeof w);
    if (s.T == 64) w[0] = 0x80000000u;  // 0x80 opens the trailer block
    w[14] = (uint32_t)(s.total_bits >> 32);
    w[15] = (uint32_t)s.total_bits;
    h_schedule(w);
    for (int i = 0; i < 64; ++i) kw[i] = kK[i] + w[i];
}

}  // namespace hm
