/*
 * hm_oracle_fast.c -- a second, fast CPU restatement of the reference scan,
 * for fixtures at sizes the plain oracle cannot reach in a session.
 *
 * TEST INFRASTRUCTURE ONLY (like hm_oracle.c): it generates the full-size
 * golden fixtures of tests/golden/ (gen_large.py) in the build container and
 * is checked against hm_oracle.c by tests/test_oracle_fast.py.  The product
 * library never links, calls or falls back to it, and it never runs on the
 * GPU box.
 *
 * Same semantics as oracle_scan_sum (hm_oracle.c), i.e. the reference's
 * cmu440/bitcoin/hash.go:13-17 per nonce and cmu440/bitcoin/miner/miner.go:46-59
 * over the inclusive range (strict <, ascending, seed (MaxUint64, 0)), plus the
 * coverage checksum (wrapping sum of keys, count).  It differs from hm_oracle.c
 * only in HOW the same bytes are hashed:
 *   - the bytes msg ‖ 0x20 ‖ decimal(n) are kept in a buffer whose ASCII
 *     digits are incremented in place (no snprintf per nonce);
 *   - the nonce-independent 64-B blocks are compressed once per digit segment
 *     (midstate), the remaining 1-2 tail blocks per nonce;
 *   - the compression uses the x86 SHA extensions (sha256rnds2/msg1/msg2),
 *     four nonces interleaved to cover the instruction latency.
 * The digit bookkeeping, padding and BE truncation are written independently
 * of hm_oracle.c so that agreement of the two is evidence for both.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXU64 0xFFFFFFFFFFFFFFFFull
#define LANES 4

static const uint32_t FK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u,
    0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u,
    0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u,
    0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
    0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u,
    0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au,
    0x5b9cca4fu, 0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
    0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
static const uint32_t FIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

/* State in the SHA-NI register form: s[0] = ABEF, s[1] = CDGH. */
typedef struct { __m128i abef, cdgh; } nstate;

__attribute__((target("sha,sse4.1"))) static nstate to_ni(const uint32_t st[8]) {
    __m128i t = _mm_loadu_si128((const __m128i *)&st[0]);  /* DCBA */
    __m128i u = _mm_loadu_si128((const __m128i *)&st[4]);  /* HGFE */
    t = _mm_shuffle_epi32(t, 0xB1);                        /* CDAB */
    u = _mm_shuffle_epi32(u, 0x1B);                        /* EFGH */
    nstate s;
    s.abef = _mm_alignr_epi8(t, u, 8);                     /* ABEF */
    s.cdgh = _mm_blend_epi16(u, t, 0xF0);                  /* CDGH */
    return s;
}

__attribute__((target("sha,sse4.1"))) static void from_ni(nstate s, uint32_t st[8]) {
    __m128i t = _mm_shuffle_epi32(s.abef, 0x1B);           /* FEBA */
    __m128i u = _mm_shuffle_epi32(s.cdgh, 0xB1);           /* DCHG */
    _mm_storeu_si128((__m128i *)&st[0], _mm_blend_epi16(t, u, 0xF0)); /* DCBA */
    _mm_storeu_si128((__m128i *)&st[4], _mm_alignr_epi8(u, t, 8));    /* HGFE */
}

/* LANES independent compressions of 64-B big-endian blocks blk[j] from s[j]. */
__attribute__((target("sha,ssse3,sse4.1"))) static void compress_n(nstate s[LANES],
                                                                 const uint8_t *blk[LANES]) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i m[LANES][4], a[LANES], c[LANES];
    for (int j = 0; j < LANES; ++j) {
        for (int q = 0; q < 4; ++q)
            m[j][q] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blk[j] + 16 * q)), bswap);
        a[j] = s[j].abef;
        c[j] = s[j].cdgh;
    }
    for (int g = 0; g < 16; ++g) {
        const __m128i k = _mm_loadu_si128((const __m128i *)&FK[4 * g]);
        __m128i w[LANES];
        for (int j = 0; j < LANES; ++j) {
            w[j] = _mm_add_epi32(m[j][g & 3], k);
            c[j] = _mm_sha256rnds2_epu32(c[j], a[j], w[j]);
        }
        if (g >= 3 && g < 15)  /* W of group g+1: msg2(W_{g+1} + alignr(W_g, W_{g-1}), W_g) */
            for (int j = 0; j < LANES; ++j) {
                const __m128i t = _mm_alignr_epi8(m[j][g & 3], m[j][(g - 1) & 3], 4);
                m[j][(g + 1) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(m[j][(g + 1) & 3], t),
                                                        m[j][g & 3]);
            }
        for (int j = 0; j < LANES; ++j)
            a[j] = _mm_sha256rnds2_epu32(a[j], c[j], _mm_shuffle_epi32(w[j], 0x0E));
        if (g >= 1 && g < 13)
            for (int j = 0; j < LANES; ++j)
                m[j][(g - 1) & 3] = _mm_sha256msg1_epu32(m[j][(g - 1) & 3], m[j][g & 3]);
    }
    for (int j = 0; j < LANES; ++j) {
        s[j].abef = _mm_add_epi32(a[j], s[j].abef);
        s[j].cdgh = _mm_add_epi32(c[j], s[j].cdgh);
    }
}

/* Key of a final state: (H0 << 32) | H1, hash.go:16 (A is ABEF's lane 3, B lane 2). */
__attribute__((target("sse4.1"))) static inline uint64_t key_of(nstate s) {
    return ((uint64_t)(uint32_t)_mm_extract_epi32(s.abef, 3) << 32) |
           (uint32_t)_mm_extract_epi32(s.abef, 2);
}

static int ndigits(uint64_t n) {
    int d = 1;
    while (n >= 10u) { n /= 10u; ++d; }
    return d;
}

static uint64_t pow10u(int k) {
    uint64_t p = 1;
    while (k-- > 0) p *= 10u;
    return p;
}

/* Per digit count d: midstate over the constant blocks and the tail template.
 * `lanes[j]` holds LANES copies of the tail (one per interleaved nonce). */
typedef struct {
    uint32_t mid[8];
    uint8_t tail[LANES][128];
    int r;   /* prefix bytes in the tail */
    int nb;  /* tail blocks */
    int d;
} seg_t;

static void seg_init(seg_t *S, const uint8_t *msg, size_t len, int d, uint64_t first) {
    /* constant part: msg ‖ ' ' */
    const size_t pre = len + 1;
    const size_t cb = pre / 64;          /* constant blocks, hashed once */
    uint32_t st[8];
    memcpy(st, FIV, sizeof st);
    uint8_t blk[64];
    for (size_t b = 0; b < cb; ++b) {
        for (int i = 0; i < 64; ++i) {
            const size_t p = 64 * b + (size_t)i;
            blk[i] = p < len ? msg[p] : 0x20;
        }
        nstate ns = to_ni(st);
        nstate v[LANES];
        const uint8_t *bp[LANES];
        for (int j = 0; j < LANES; ++j) { v[j] = ns; bp[j] = blk; }
        compress_n(v, bp);
        from_ni(v[0], st);
    }
    memcpy(S->mid, st, sizeof st);
    S->r = (int)(pre - 64 * cb);
    S->d = d;
    const int tl = S->r + d + 1 + 8;
    S->nb = tl <= 64 ? 1 : 2;
    const uint64_t bits = (uint64_t)(len + 1 + (size_t)d) * 8u;
    for (int j = 0; j < LANES; ++j) {
        uint8_t *t = S->tail[j];
        memset(t, 0, 128);
        for (int i = 0; i < S->r; ++i) {
            const size_t p = 64 * cb + (size_t)i;
            t[i] = p < len ? msg[p] : 0x20;
        }
        uint64_t x = first;
        for (int i = d - 1; i >= 0; --i) { t[S->r + i] = (uint8_t)('0' + x % 10u); x /= 10u; }
        t[S->r + d] = 0x80;
        for (int i = 0; i < 8; ++i) t[64 * S->nb - 1 - i] = (uint8_t)(bits >> (8 * i));
    }
}

/* ASCII decimal increment of the digits at t[r .. r+d) (no carry out). */
static inline void inc_digits(uint8_t *t, int r, int d) {
    int i = r + d - 1;
    while (t[i] == '9') { t[i] = '0'; --i; }
    t[i]++;
    (void)r;
}

typedef struct { uint64_t hash, nonce, sum, count; } res_t;

/* Scan the nonces [lo, hi] (same digit count d, hi - lo < 2^63). */
__attribute__((target("sha,ssse3,sse4.1"))) static void scan_seg(const uint8_t *msg, size_t len,
                                                               uint64_t lo, uint64_t hi, res_t *R) {
    const int d = ndigits(lo);
    seg_t S;
    /* lane j starts at lo + j and steps by LANES */
    seg_init(&S, msg, len, d, lo);
    /* lane j holds nonce min(n + j, hi): lanes past hi (last group only)
     * repeat hi and are not counted, and no digit string ever carries out */
    uint64_t ln[LANES];
    for (int j = 0; j < LANES; ++j) {
        ln[j] = lo;
        while (ln[j] < hi && ln[j] - lo < (uint64_t)j) { inc_digits(S.tail[j], S.r, d); ++ln[j]; }
    }
    const nstate mid = to_ni(S.mid);
    uint64_t n = lo;
    const uint64_t count = hi - lo + 1;
    uint64_t done = 0;
    uint64_t bh = R->hash, bn = R->nonce, sum = R->sum;
    while (done < count) {
        nstate v[LANES];
        const uint8_t *bp[LANES];
        for (int j = 0; j < LANES; ++j) { v[j] = mid; bp[j] = S.tail[j]; }
        compress_n(v, bp);
        if (S.nb == 2) {
            for (int j = 0; j < LANES; ++j) bp[j] = S.tail[j] + 64;
            compress_n(v, bp);
        }
        const uint64_t take = count - done < LANES ? count - done : LANES;
        for (uint64_t j = 0; j < take; ++j) {
            const uint64_t k = key_of(v[j]);
            sum += k;
            if (k < bh) { bh = k; bn = n + j; }  /* ascending, strict < */
        }
        done += take;
        n += take;
        if (done < count)
            for (int j = 0; j < LANES; ++j) {
                const uint64_t target = hi - n < (uint64_t)j ? hi : n + (uint64_t)j;
                while (ln[j] < target) { inc_digits(S.tail[j], S.r, d); ++ln[j]; }
            }
    }
    R->hash = bh;
    R->nonce = bn;
    R->sum = sum;
    R->count += count;
}

/* Scan [lo, hi] that may cross digit boundaries (in order, ascending). */
static void scan_range(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, res_t *R) {
    uint64_t a = lo;
    for (;;) {
        const int d = ndigits(a);
        const uint64_t seg_hi = d >= 20 ? MAXU64 : pow10u(d) - 1;
        const uint64_t b = seg_hi < hi ? seg_hi : hi;
        scan_seg(msg, len, a, b, R);
        if (b == hi) break;
        a = b + 1;
    }
}

typedef struct {
    const uint8_t *msg;
    size_t len;
    uint64_t lo, hi;
    uint64_t chunk, nchunks;
    _Atomic uint64_t next;
    res_t *parts;
} job_t;

static void *worker(void *arg) {
    job_t *J = (job_t *)arg;
    for (;;) {
        const uint64_t c = atomic_fetch_add(&J->next, 1);
        if (c >= J->nchunks) break;
        const uint64_t a = J->lo + c * J->chunk;
        const uint64_t b = (c + 1 == J->nchunks) ? J->hi : a + J->chunk - 1;
        res_t r = {MAXU64, 0, 0, 0};
        scan_range(J->msg, J->len, a, b, &r);
        J->parts[c] = r;
    }
    return NULL;
}

/* 1 when this CPU has the SHA extensions (the only requirement). */
int oracle_fast_available(void) {
    unsigned a, b, c, d;
    __asm__("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    return (b >> 29) & 1;
}

/* Same contract as oracle_scan_sum (hm_oracle.c). */
void oracle_fast_scan_sum(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                          uint64_t *out_hash, uint64_t *out_nonce, uint64_t *out_sum,
                          uint64_t *out_count) {
    *out_hash = MAXU64;
    *out_nonce = 0;
    *out_sum = 0;
    *out_count = 0;
    if (lo > hi) return;
    if (threads < 1) threads = 1;
    const uint64_t span_m1 = hi - lo;
    uint64_t chunk = 1ull << 22;
    uint64_t nchunks = span_m1 / chunk + 1;  /* the last one takes the remainder */
    if (nchunks > (1ull << 20)) { chunk = span_m1 / (1ull << 20) + 1; nchunks = span_m1 / chunk + 1; }
    job_t J;
    J.msg = msg; J.len = len; J.lo = lo; J.hi = hi; J.chunk = chunk; J.nchunks = nchunks;
    atomic_init(&J.next, 0);
    J.parts = (res_t *)calloc(nchunks, sizeof(res_t));
    if (!J.parts) return;
    if ((uint64_t)threads > nchunks) threads = (int)nchunks;
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 1; t < threads; ++t) pthread_create(&tids[t], NULL, worker, &J);
    worker(&J);
    for (int t = 1; t < threads; ++t) pthread_join(tids[t], NULL);
    uint64_t bh = MAXU64, bn = 0, s = 0, c = 0;
    for (uint64_t i = 0; i < nchunks; ++i) {  /* chunks ascend: strict < keeps the lowest nonce */
        if (J.parts[i].hash < bh) { bh = J.parts[i].hash; bn = J.parts[i].nonce; }
        s += J.parts[i].sum;
        c += J.parts[i].count;
    }
    *out_hash = bh; *out_nonce = bn; *out_sum = s; *out_count = c;
    free(J.parts);
    free(tids);
}
