// sha256_defs.hpp -- SHA-256 constants and the host-side compression used by
// the planner (midstates over constant message blocks, constant trailer-block
// schedules, and hm_hash).  FIPS 180-4.  Shared by host code and kernels.
//
// The reference computes SHA-256 through Go's crypto/sha256 inside
// bitcoin.Hash (cmu440/bitcoin/hash.go:14-16).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define HM_HD __host__ __device__ __forceinline__
#else
#define HM_HD inline
#endif

namespace hm {

static constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

static constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

HM_HD uint32_t h_rotr(uint32_t x, uint32_t n) { return (x >> n) | (x << (32u - n)); }

// Message schedule of one block: w[0..15] in, w[0..63] out.
// (Loops are fully unrolled so that on the device w stays in registers.)
HM_HD void h_schedule(uint32_t w[64]) {
#pragma unroll
    for (int i = 16; i < 64; ++i) {
        uint32_t a = w[i - 15], b = w[i - 2];
        uint32_t s0 = h_rotr(a, 7) ^ h_rotr(a, 18) ^ (a >> 3);
        uint32_t s1 = h_rotr(b, 17) ^ h_rotr(b, 19) ^ (b >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
}

// One compression, state updated in place (with the feed-forward add).
HM_HD void h_compress(uint32_t st[8], const uint32_t m[16]) {
    uint32_t w[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = m[i];
    h_schedule(w);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (h_rotr(e, 6) ^ h_rotr(e, 11) ^ h_rotr(e, 25)) + (((f ^ g) & e) ^ g) +
                      kK[i] + w[i];
        uint32_t t2 = (h_rotr(a, 2) ^ h_rotr(a, 13) ^ h_rotr(a, 22)) + (((a ^ b) & (b ^ c)) ^ b);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Big-endian load of 64 bytes into 16 words.
HM_HD void h_load_block(uint32_t m[16], const uint8_t* p) {
    for (int i = 0; i < 16; ++i)
        m[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
               ((uint32_t)p[4 * i + 2] << 8) | (uint32_t)p[4 * i + 3];
}

}  // namespace hm
