// host_scan.cpp -- hm_scan_cpu: the min-hash scan on the host's cores.
//
// SURVEY §8(b)'s liveness path.  The reference miner always answers a
// Request with a Result (cmu440/bitcoin/miner/miner.go:60-62); a GPU miner
// whose device is missing or failed keeps that contract by scanning here,
// bit-identically to hm_scan: the lexicographic min of (Hash(msg, n), n) over
// the INCLUSIVE [lo, hi] (miner.go:46-59 over bitcoin.Hash, hash.go:13-17),
// seeded (2^64-1, 0).
//
// Work split: `threads` contiguous, near-equal chunks of [lo, hi], one
// std::thread each, merged lexicographically (the merge is associative and
// ties go to the lowest nonce, so the split does not change the answer).
// Per chunk and digit segment: the planner's midstate over the constant
// message blocks (plan_message), the tail bytes built once, the decimal
// digits incremented in place, and a two-block tail's first block
// recompressed only when a carry reaches it.  The compression uses the x86
// SHA extensions when the CPU has them (HM_CPU_NO_SHA=1 forces the portable
// C compression, for tests), else the planner's h_compress.
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../../include/hipminer.h"
#include "plan.hpp"
#include "sha256_defs.hpp"

namespace hm {
namespace {

struct Best {
    uint64_t key = ~0ull, nonce = 0;  // miner.go:48-49
    void take(uint64_t k, uint64_t n) {
        if (k < key || (k == key && n < nonce)) { key = k; nonce = n; }
    }
};

inline uint32_t load_be32(const uint8_t* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return __builtin_bswap32(v);
}

// Portable compression of one 64-byte block from `st` into `out`.
void compress_c(const uint32_t st[8], const uint8_t* blk, uint32_t out[8]) {
    uint32_t m[16];
    for (int i = 0; i < 16; ++i) m[i] = load_be32(blk + 4 * i);
    for (int i = 0; i < 8; ++i) out[i] = st[i];
    h_compress(out, m);
}

#if defined(__x86_64__)
// The same compression with the SHA extensions.  The state lives in two
// registers as (A, B, E, F) and (C, D, G, H), the order sha256rnds2 takes;
// each sha256rnds2 runs two rounds on the two low dwords of its message
// operand (W[i] + K[i] already added), so four rounds take two of them with
// the message shifted by 8 bytes in between.  Schedule: W[t..t+3] =
// msg2(msg1(W[t-16..], W[t-12..]) + W[t-7..t-4], W[t-4..]).
__attribute__((target("sha,sse4.1,ssse3"))) void compress_ni(const uint32_t st[8],
                                                             const uint8_t* blk,
                                                             uint32_t out[8]) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i dcba = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st));      // lanes a b c d
    __m128i hgfe = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4));  // lanes e f g h
    const __m128i cdab = _mm_shuffle_epi32(dcba, 0xB1);                       // b a d c
    const __m128i efgh = _mm_shuffle_epi32(hgfe, 0x1B);                       // h g f e
    __m128i abef = _mm_alignr_epi8(cdab, efgh, 8);                            // f e b a
    __m128i cdgh = _mm_blend_epi16(efgh, cdab, 0xF0);                         // h g d c
    const __m128i abef0 = abef, cdgh0 = cdgh;
    __m128i w[4];
    for (int i = 0; i < 4; ++i)
        w[i] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(blk + 16 * i)),
                                bswap);
    for (int q = 0; q < 16; ++q) {
        __m128i cur;
        if (q < 4) {
            cur = w[q];
        } else {
            // w[q & 3] holds W[4q-16 ..]; the others the three groups after it
            const __m128i a = w[q & 3], b = w[(q + 1) & 3], c = w[(q + 2) & 3], d = w[(q + 3) & 3];
            const __m128i t = _mm_add_epi32(_mm_sha256msg1_epu32(a, b), _mm_alignr_epi8(d, c, 4));
            cur = _mm_sha256msg2_epu32(t, d);
            w[q & 3] = cur;
        }
        __m128i kw = _mm_add_epi32(cur, _mm_loadu_si128(reinterpret_cast<const __m128i*>(kK + 4 * q)));
        cdgh = _mm_sha256rnds2_epu32(cdgh, abef, kw);
        kw = _mm_shuffle_epi32(kw, 0x0E);
        abef = _mm_sha256rnds2_epu32(abef, cdgh, kw);
    }
    abef = _mm_add_epi32(abef, abef0);
    cdgh = _mm_add_epi32(cdgh, cdgh0);
    const __m128i feba = _mm_shuffle_epi32(abef, 0x1B);                 // a b e f
    const __m128i dchg = _mm_shuffle_epi32(cdgh, 0xB1);                 // g h c d
    dcba = _mm_blend_epi16(feba, dchg, 0xF0);                           // a b c d
    hgfe = _mm_alignr_epi8(dchg, feba, 8);                              // e f g h
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out), dcba);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 4), hgfe);
}
#endif

typedef void (*CompressFn)(const uint32_t[8], const uint8_t*, uint32_t[8]);

CompressFn pick_compress() {
    const char* off = getenv("HM_CPU_NO_SHA");
    if (off && *off && strcmp(off, "0") != 0) return compress_c;
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1")) return compress_ni;
#endif
    return compress_c;
}

// Scan [a, b] (a <= b, one thread): every digit segment of it in turn.
void scan_chunk(const MsgPlan& mp, uint64_t a, uint64_t b, CompressFn compress, Best* out) {
    Best best;
    const uint32_t r = mp.r;
    for (uint32_t d = digits_u64(a); d <= digits_u64(b); ++d) {
        const uint64_t dlo = d == 1 ? 0 : pow10_u64(d - 1);
        const uint64_t dhi = d == 20 ? ~0ull : pow10_u64(d) - 1;
        const uint64_t slo = std::max(a, dlo), shi = std::min(b, dhi);
        if (slo > shi) continue;
        // tail: r prefix bytes, d digits, 0x80, zeros, 64-bit bit length
        uint8_t tail[128];
        memset(tail, 0, sizeof tail);
        for (uint32_t i = 0; i < r; ++i) tail[i] = (uint8_t)(mp.pw[i / 4] >> (24 - 8 * (i % 4)));
        uint64_t x = slo;
        for (uint32_t k = 0; k < d; ++k) {
            tail[r + d - 1 - k] = (uint8_t)('0' + x % 10);
            x /= 10;
        }
        const uint32_t T = r + d;
        tail[T] = 0x80;
        const uint32_t nb = T + 9 <= 64 ? 1 : 2;
        const uint64_t bits = (mp.len + 1 + d) * 8;
        for (int i = 0; i < 8; ++i) tail[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
        const uint8_t* last = tail + 64 * (nb - 1);
        uint32_t s0[8];  // state entering the last tail block
        if (nb == 2) compress(mp.mid, tail, s0);
        else memcpy(s0, mp.mid, sizeof s0);
        const uint64_t count_m1 = shi - slo;
        for (uint64_t i = 0;; ++i) {
            uint32_t o[8];
            compress(s0, last, o);
            best.take(((uint64_t)o[0] << 32) | o[1], slo + i);
            if (i == count_m1) break;
            // next nonce: increment the ASCII digits in place (no carry out:
            // every nonce of the segment has d digits)
            uint32_t p = T - 1;
            while (tail[p] == '9') tail[p--] = '0';
            ++tail[p];
            if (nb == 2 && p < 64) compress(mp.mid, tail, s0);
        }
    }
    *out = best;
}

// Default thread count: the CPUs this process may run on.  A GPU box's
// per-GPU share is an affinity set inside a machine whose
// hardware_concurrency() counts every CPU, many times more.
unsigned default_threads() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) {
        const int c = CPU_COUNT(&set);
        if (c > 0) return (unsigned)c;
    }
    return std::max(1u, std::thread::hardware_concurrency());
}

}  // namespace
}  // namespace hm

extern "C" int hm_scan_cpu(const uint8_t* msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                           hm_result* out) {
    using namespace hm;
    if (!out || (!msg && len)) return HM_ERR_INVALID;
    try {
        if (lo > hi) {
            *out = hm_result{~0ull, 0};
            return HM_OK;
        }
        static const uint8_t empty = 0;
        const MsgPlan mp = plan_message(msg ? msg : &empty, msg ? len : 0);
        const CompressFn compress = pick_compress();
        typedef unsigned __int128 u128;
        const u128 count = (u128)(hi - lo) + 1;
        unsigned n = threads > 0 ? (unsigned)threads : default_threads();
        n = std::min(n, 1024u);
        if (count < (u128)n * 4096) n = (unsigned)std::max<u128>(1, count / 4096);
        std::vector<Best> part(n);
        std::vector<std::thread> pool;
        pool.reserve(n);
        const u128 per = count / n, extra = count % n;
        u128 start = 0;
        int rc = HM_OK;
        for (unsigned t = 0; t < n; ++t) {
            const u128 len_t = per + (t < extra ? 1 : 0);
            const uint64_t a = lo + (uint64_t)start, b = lo + (uint64_t)(start + len_t - 1);
            start += len_t;
            if (t + 1 == n) {
                scan_chunk(mp, a, b, compress, &part[t]);  // the calling thread
                break;
            }
            try {
                pool.emplace_back(scan_chunk, std::cref(mp), a, b, compress, &part[t]);
            } catch (...) {  // no thread: join the started ones before failing
                rc = HM_ERR_INTERNAL;
                break;
            }
        }
        for (auto& th : pool) th.join();
        if (rc) return rc;
        Best best;
        for (const Best& p : part) best.take(p.key, p.nonce);
        *out = hm_result{best.key, best.nonce};
        return HM_OK;
    } catch (const std::bad_alloc&) {
        return HM_ERR_NOMEM;
    } catch (...) {
        return HM_ERR_INTERNAL;
    }
}
