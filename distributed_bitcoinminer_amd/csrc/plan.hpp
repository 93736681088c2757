// plan.hpp -- host planner: splits [lo, hi] into digit-count segments and
// picks each segment's kernel layout.  Pure host code (no HIP calls), so the
// CPU test suite can exercise it through hm_plan_* debug exports.
//
// Bytes hashed per nonce (cmu440/bitcoin/hash.go:15):
//     msg ‖ 0x20 ‖ decimal(nonce)
// The first floor((len+1)/64) 64-byte blocks are nonce-independent and are
// folded into a host midstate.  The remaining "tail" holds r = (len+1) % 64
// prefix bytes, the d digits, 0x80 and the bit length, in nb (1 or 2) blocks.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace hm {

struct MsgPlan {
    uint32_t mid[8];    // midstate after the constant prefix blocks
    uint32_t pw[16];    // prefix remainder as big-endian words (zero padded)
    uint32_t r;         // prefix remainder length (0..63)
    uint64_t len;       // message length in bytes
};

struct SegPlan {
    uint32_t d;                 // digits of every nonce in [lo, hi]
    uint64_t lo, hi;            // inclusive
    uint32_t T, nb, fb;         // tail bytes before 0x80; tail blocks; block of last digit
    uint32_t p_end;             // in-block byte index of the last digit
    int kind;                   // HM_KIND_TILED or HM_KIND_GENERIC
    // tiled layout
    int W1;                     // word holding the last digit (varying words W1-1, W1)
    bool straddle, trailer;
    bool lane3;                 // lane digits reach back into W[W1-2] (q = 5 where two words give 3-4)
    uint32_t V, q;              // varying digits; lane digits (V = q + 2 loop digits)
    uint32_t lane_shift, loop_shift;
    uint64_t pow10V;
    uint32_t tpt;               // lane chunks (waves) per tile
    // chained layout (kind HM_KIND_CHAINED): f digits in the final block, the
    // low fe of them from a K+W table of 10^fe rows, the high f - fe as epochs
    uint32_t f, fe, tch, ntc;   // final-block digits; table digits; loop values per unit; loop chunks
    uint64_t tile_lo, tile_hi;  // inclusive tile range
    uint64_t total_bits;
};

uint32_t digits_u64(uint64_t n);
uint64_t pow10_u64(uint32_t k);  // k <= 19
MsgPlan plan_message(const uint8_t* msg, uint64_t len);
// Segment list for inclusive [lo, hi] (lo <= hi).  table_digits (1..7, 0 =
// default 7 = kTableDigits in plan.cpp) caps the final-block digits a chained
// K+W table covers; -1 turns the chained layout of >= 5 final-block digits
// off (HM_OPT_TABLE_DIGITS, a test hook: small tables make epochs on small
// ranges).
std::vector<SegPlan> plan_range(const MsgPlan& mp, uint64_t lo, uint64_t hi, bool force_generic,
                                int table_digits = 0);
// Fraction of the nonces a chained layout hashes that lie in [s.lo, s.hi]: its
// lanes vary block-0 digits (nonce stride 10^f), so the 64-lane chunks at the
// range's two ends carry out-of-range lane values.
double chained_lane_eff(const SegPlan& s);
// Modelled GPU cost of one nonce of segment s: SIMD cycles per 64 nonces of
// the kernel instantiation that runs it, as measured per layout on MI355X
// (DESIGN.md §4 "Every layout").  Only shard balancing uses it.
double seg_cost(const SegPlan& s);

struct Shard {
    uint64_t lo, hi;  // inclusive; meaningful only when !empty
    bool empty;
};
// Split inclusive [lo, hi] into n contiguous, ascending shards of near-equal
// modelled cost (sum over nonces of seg_cost), SURVEY §8(e).  Shards cover
// [lo, hi] exactly; a shard is empty when the range has too few nonces.
// lo > hi gives n empty shards.
std::vector<Shard> partition_range(const MsgPlan& mp, uint64_t lo, uint64_t hi, int n,
                                   bool force_generic);
// Host SHA-256 of msg ‖ ' ' ‖ decimal(nonce), first 8 bytes big-endian.
uint64_t host_hash(const uint8_t* msg, uint64_t len, uint64_t nonce);
// sigma0 of the wave-uniform loop-digit bits of W[W1] for each loop value
// t1*10+t0 of hm_tiled_kernel (sigma0 is XOR-linear, the lane bits are disjoint).
void tiled_loop_sigma0(const SegPlan& s, uint32_t out[100]);
// K[i] + W[i] of the constant trailer block of a trailer segment.
void trailer_kw(const SegPlan& s, uint32_t kw[64]);

}  // namespace hm
