/*
 * hm_oracle.c -- CPU restatement of the reference miner's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the CPU
 * baseline ("port") for bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library
 * (libhipminer.so) never links, calls or falls back to it.
 *
 * What it restates (paths relative to /root/reference,
 * cmu440/ = p1/src/github.com/cmu440/):
 *
 *   oracle_hash   <- cmu440/bitcoin/hash.go:13-17
 *       hasher.Write([]byte(fmt.Sprintf("%s %d", msg, nonce)))   (:15)
 *       binary.BigEndian.Uint64(hasher.Sum(nil))                 (:16)
 *     The bytes hashed are msg verbatim, one 0x20, then the decimal nonce with
 *     no sign, padding or leading zeros ("0" for 0).  SHA-256 runs from the IV
 *     for every nonce (no midstate), exactly like the Go loop.  SHA-256 is
 *     Go's crypto/sha256 (stdlib, unpinned version; the staff binaries were
 *     built with go1.10.3); it is restated here from FIPS 180-4.
 *
 *   oracle_scan   <- cmu440/bitcoin/miner/miner.go:46-59
 *       result = maxUint; index = 0                               (:48-49)
 *       for i := lower; i < upper; i++ { if hash < result {...} } (:53-59)
 *     over the truly inclusive range [lo, hi] (hi may be 2^64-1).  Ties keep
 *     the lowest nonce (strict <, ascending).  Multi-threaded runs split the
 *     range into contiguous chunks and merge lexicographically on
 *     (hash, nonce), which is equivalent to one ascending strict-< scan.
 *
 *   oracle_miner_eval <- miner.go:50-59 including the `upper := Upper+1`
 *     wrap (:52): Upper == 2^64-1 scans nothing and returns (MaxUint64, 0).
 *
 * Parity status: the reference ships no golden vectors for this path and its
 * Go toolchain is absent, so this restatement is pinned to FIPS 180-4 KATs
 * and to fixtures produced by an independent Python hashlib restatement
 * (tests/golden/gen_golden.py); see DESIGN.md "Oracle".
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXU64 0xFFFFFFFFFFFFFFFFull

static const uint32_t OK[64] = {
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

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void o_block(uint32_t st[8], const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
               ((uint32_t)p[4 * i + 2] << 8) | (uint32_t)p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROTR(w[i - 15], 7) ^ ROTR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROTR(w[i - 2], 17) ^ ROTR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + OK[i] + w[i];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* Plain FIPS 180-4 SHA-256 of an arbitrary byte string. */
void oracle_sha256(const uint8_t *data, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    size_t full = len / 64;
    for (size_t i = 0; i < full; i++) o_block(st, data + 64 * i);
    uint8_t tail[128];
    size_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    memcpy(tail, data + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    o_block(st, tail);
    if (tl == 128) o_block(st, tail + 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* hash.go:13-17: Sprintf("%s %d") -> SHA-256 -> BigEndian.Uint64(sum[:8]).
 * `buf` must hold len + 22 bytes. */
static uint64_t o_hash_buf(const uint8_t *msg, size_t len, uint64_t nonce, uint8_t *buf) {
    memcpy(buf, msg, len);
    int n = snprintf((char *)buf + len, 24, " %llu", (unsigned long long)nonce);
    uint8_t dg[32];
    oracle_sha256(buf, len + (size_t)n, dg);
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | dg[i];
    return v;
}

uint64_t oracle_hash(const uint8_t *msg, size_t len, uint64_t nonce) {
    uint8_t *buf = (uint8_t *)malloc(len + 32);
    if (!buf) return 0;
    uint64_t v = o_hash_buf(msg, len, nonce, buf);
    free(buf);
    return v;
}

typedef struct {
    const uint8_t *msg;
    size_t len;
    uint64_t lo, hi; /* inclusive */
    int empty;
    uint64_t hash, nonce;
    uint64_t sum, count; /* coverage checksum: wrapping sum of keys, nonces hashed */
} o_job;

/* miner.go:48-59 over inclusive [lo, hi], strict <, ascending. */
static void *o_scan_job(void *arg) {
    o_job *j = (o_job *)arg;
    uint64_t result = MAXU64, index = 0, sum = 0, count = 0;
    if (!j->empty) {
        uint8_t *buf = (uint8_t *)malloc(j->len + 32);
        uint64_t i = j->lo;
        for (;;) {
            uint64_t h = o_hash_buf(j->msg, j->len, i, buf);
            sum += h;
            count++;
            if (h < result) { result = h; index = i; }
            if (i == j->hi) break;
            i++;
        }
        free(buf);
    }
    j->hash = result;
    j->nonce = index;
    j->sum = sum;
    j->count = count;
    return NULL;
}

/* Inclusive scan [lo, hi] (hi may be 2^64-1).  lo > hi is an empty range and
 * returns (MaxUint64, 0), the miner's initial value (miner.go:48-49).
 * Also returns the coverage checksum that hm_scan_checked computes on the
 * GPU: the wrapping (mod 2^64) sum of every key and the number of nonces. */
void oracle_scan_sum(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                     uint64_t *out_hash, uint64_t *out_nonce, uint64_t *out_sum,
                     uint64_t *out_count) {
    *out_sum = 0;
    *out_count = 0;
    if (lo > hi) { *out_hash = MAXU64; *out_nonce = 0; return; }
    if (threads < 1) threads = 1;
    uint64_t span_m1 = hi - lo; /* count - 1, never overflows */
    if ((uint64_t)threads - 1 > span_m1) threads = (int)(span_m1 + 1);
    o_job *jobs = (o_job *)calloc((size_t)threads, sizeof(o_job));
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    /* count = span_m1 + 1 = threads*q + (rr + 1): chunks 0..rr get q + 1
     * nonces, the rest q (q == 0 only when threads == count == rr + 1). */
    uint64_t q = span_m1 / (uint64_t)threads, rr = span_m1 % (uint64_t)threads;
    uint64_t start = lo;
    for (int c = 0; c < threads; c++) {
        uint64_t cnt_m1 = q - 1u + ((uint64_t)c <= rr ? 1u : 0u); /* modular */
        jobs[c].msg = msg; jobs[c].len = len;
        jobs[c].lo = start; jobs[c].hi = start + cnt_m1; jobs[c].empty = 0;
        start = start + cnt_m1 + 1;
    }
    if (threads == 1) {
        o_scan_job(&jobs[0]);
    } else {
        for (int c = 0; c < threads; c++) pthread_create(&tids[c], NULL, o_scan_job, &jobs[c]);
        for (int c = 0; c < threads; c++) pthread_join(tids[c], NULL);
    }
    uint64_t bh = MAXU64, bn = 0, bs = 0, bc = 0;
    for (int c = 0; c < threads; c++) { /* chunks ascend: strict < keeps lowest nonce */
        if (jobs[c].hash < bh) { bh = jobs[c].hash; bn = jobs[c].nonce; }
        bs += jobs[c].sum;
        bc += jobs[c].count;
    }
    *out_hash = bh; *out_nonce = bn;
    *out_sum = bs; *out_count = bc;
    free(jobs); free(tids);
}

void oracle_scan(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                 uint64_t *out_hash, uint64_t *out_nonce) {
    uint64_t s, c;
    oracle_scan_sum(msg, len, lo, hi, threads, out_hash, out_nonce, &s, &c);
}

/* miner.go:50-59 verbatim semantics, including `upper := Upper + 1` wrapping
 * to 0 when Upper == MaxUint64 (then the loop runs zero times). */
void oracle_miner_eval(const uint8_t *msg, size_t len, uint64_t lower, uint64_t upper_incl,
                       int threads, uint64_t *out_hash, uint64_t *out_nonce) {
    uint64_t upper = upper_incl + 1u; /* wraps like Go uint64 */
    if (!(lower < upper)) { *out_hash = MAXU64; *out_nonce = 0; return; }
    oracle_scan(msg, len, lower, upper - 1u, threads, out_hash, out_nonce);
}
