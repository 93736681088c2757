// place_ubench.hip -- issue cost vs. instruction placement on gfx950 (dev tool).
//
// Each pattern is one inline-asm block over 8 independent accumulators.  The
// block opens with `.p2align 3` (the assembler pads with s_nop 0) and, for the
// "@4" variants, one extra `s_nop 0`, so every instruction's start address
// mod 8 is known.  Reports cycles per VALU instruction per SIMD.
// build: hipcc -O3 --offload-arch=gfx950 tools/place_ubench.hip -o build/place_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 1024;
#define A(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t"       /* 8 B, half rate */
#define B(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t" /* 8 B, full rate */
#define T(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"               /* 8 B, half rate */
#define E(i) "v_add_u32_e64 %" #i ", %" #i ", %8\n\t"                /* 8 B, full rate */
#define D(i) "v_add_u32_e32 %" #i ", %" #i ", %8\n\t"                /* 4 B, full rate */
#define S(i) "v_lshrrev_b32_e32 %" #i ", 3, %" #i "\n\t"             /* 4 B, full rate */
#define L(i) "v_lshrrev_b32_e64 %" #i ", 3, %" #i "\n\t"             /* 8 B */
#define F(i) "v_bfe_u32 %" #i ", %" #i ", 3, 29\n\t"                 /* 8 B */
#define N "s_nop 0\n\t"
#define Q(i) A(i) B(i)
#define R(i) B(i) A(i)
#define U(i) A(i) D(i) D(i)
#define V(i) A(i) E(i) E(i)
#define Y(i) A(i) B(i) B(i)
#define Z(i) A(i) A(i) B(i)
#define P0 ".p2align 3\n\t"
#define P4 ".p2align 3\n\t" N
#define OUTS "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
#define INS "v"(y), "v"(z)
#define X8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
// returns VALU instructions per block
template <int P>
__device__ __forceinline__ int pat(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                   uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t z) {
    if constexpr (P == 0) { asm volatile(P0 X8(A) X8(A) : OUTS : INS); return 16; }
    if constexpr (P == 1) { asm volatile(P4 X8(A) X8(A) : OUTS : INS); return 16; }
    if constexpr (P == 2) { asm volatile(P0 X8(B) X8(B) : OUTS : INS); return 16; }
    if constexpr (P == 3) { asm volatile(P4 X8(B) X8(B) : OUTS : INS); return 16; }
    if constexpr (P == 4) { asm volatile(P0 X8(E) X8(E) : OUTS : INS); return 16; }
    if constexpr (P == 5) { asm volatile(P4 X8(E) X8(E) : OUTS : INS); return 16; }
    if constexpr (P == 6) { asm volatile(P0 X8(D) X8(D) : OUTS : INS); return 16; }
    if constexpr (P == 7) { asm volatile(P4 X8(D) X8(D) : OUTS : INS); return 16; }
    // SHA-like: per accumulator pair A A S B (sigma) and T E: 8-byte ops keep
    // their phase, the lone 4-byte S is paired with a D to keep parity
    if constexpr (P == 8) { asm volatile(P0 A(0) A(1) S(2) D(3) B(4) T(5) E(6) A(7) A(0) T(1) B(2) A(3) S(4) D(5) E(6) T(7) : OUTS : INS); return 16; }
    if constexpr (P == 9) { asm volatile(P4 A(0) A(1) S(2) D(3) B(4) T(5) E(6) A(7) A(0) T(1) B(2) A(3) S(4) D(5) E(6) T(7) : OUTS : INS); return 16; }
    // alternating half/full 8-byte ops
    if constexpr (P == 10) { asm volatile(P0 A(0) B(1) A(2) B(3) A(4) B(5) A(6) B(7) A(0) B(1) A(2) B(3) A(4) B(5) A(6) B(7) : OUTS : INS); return 16; }
    if constexpr (P == 11) { asm volatile(P4 A(0) B(1) A(2) B(3) A(4) B(5) A(6) B(7) A(0) B(1) A(2) B(3) A(4) B(5) A(6) B(7) : OUTS : INS); return 16; }
    // 8-byte shift forms (candidates to replace a lone 4-byte lshrrev)
    if constexpr (P == 12) { asm volatile(P4 X8(L) X8(L) : OUTS : INS); return 16; }
    if constexpr (P == 13) { asm volatile(P4 X8(F) X8(F) : OUTS : INS); return 16; }
    if constexpr (P == 14) { asm volatile(P4 X8(S) X8(S) : OUTS : INS); return 16; }
    // nop cost: the SHA-like @4 block with 4 extra s_nop pairs (parity kept)
    if constexpr (P == 15) { asm volatile(P4 A(0) A(1) N N S(2) D(3) B(4) T(5) N N E(6) A(7) A(0) T(1) N N B(2) A(3) S(4) D(5) N N E(6) T(7) : OUTS : INS); return 16; }
    // finer phases of the alternating half/full pattern: start at 4 / 12 mod 16
    if constexpr (P == 16) { asm volatile(".p2align 4\n\t" N X8(Q) X8(Q) : OUTS : INS); return 32; }
    if constexpr (P == 17) { asm volatile(".p2align 4\n\t" N N N X8(Q) X8(Q) : OUTS : INS); return 32; }
    // start at 4 / 12 / 20 / 28 mod 32
    if constexpr (P == 18) { asm volatile(".p2align 5\n\t" N X8(Q) X8(Q) : OUTS : INS); return 32; }
    if constexpr (P == 19) { asm volatile(".p2align 5\n\t" N N N N N X8(Q) X8(Q) : OUTS : INS); return 32; }
    // full-rate 8-byte op then half-rate (B A order) at 4 mod 8
    if constexpr (P == 20) { asm volatile(P4 X8(R) X8(R) : OUTS : INS); return 32; }
    // half-rate + two 4-byte full-rate ops (A D D): A always @0 or @4
    if constexpr (P == 21) { asm volatile(P0 X8(U) : OUTS : INS); return 24; }
    if constexpr (P == 22) { asm volatile(P4 X8(U) : OUTS : INS); return 24; }
    // same with the full-rate ops as 8-byte e64 (A E E)
    if constexpr (P == 23) { asm volatile(P0 X8(V) : OUTS : INS); return 24; }
    if constexpr (P == 24) { asm volatile(P4 X8(V) : OUTS : INS); return 24; }
    // grouping of half-rate (A, T) and full-rate (B, E) 8-byte ops, all @4
    if constexpr (P == 25) { asm volatile(P4 A(0) A(1) B(2) B(3) A(4) A(5) B(6) B(7) A(0) A(1) B(2) B(3) A(4) A(5) B(6) B(7) : OUTS : INS); return 16; }
    if constexpr (P == 26) { asm volatile(P4 A(0) A(1) A(2) A(3) B(4) B(5) B(6) B(7) A(0) A(1) A(2) A(3) B(4) B(5) B(6) B(7) : OUTS : INS); return 16; }
    if constexpr (P == 27) { asm volatile(P4 X8(Y) : OUTS : INS); return 24; }
    if constexpr (P == 28) { asm volatile(P4 X8(Z) : OUTS : INS); return 24; }
    if constexpr (P == 29) { asm volatile(P4 T(0) E(1) T(2) E(3) T(4) E(5) T(6) E(7) T(0) E(1) T(2) E(3) T(4) E(5) T(6) E(7) : OUTS : INS); return 16; }
    if constexpr (P == 30) { asm volatile(P4 X8(A) X8(B) : OUTS : INS); return 16; }
    return 0;
}
template <int P>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t x0 = seed ^ threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 11, x5 = x0 * 13, x6 = x0 * 17, x7 = x0 * 19;
    uint32_t y = seed + 1, z = seed * 7;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int n = 0;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) n += pat<P>(x0, x1, x2, x3, x4, x5, x6, x7, y, z);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ n;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
template <int P>
constexpr int pat_count() {
    return (P == 16 || P == 17 || P == 18 || P == 19 || P == 20) ? 32
         : ((P >= 21 && P <= 24) || P == 27 || P == 28) ? 24 : 16;
}
template <int P>
int run(const char* name, int wpsimd, int cus, uint32_t* out, uint64_t* clk) {
    int grid = wpsimd * cus;
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern<P>, dim3(grid), dim3(256), 0, 0, out, clk, 1u);
    CHK(hipDeviceSynchronize()); CHK(hipEventRecord(a));
    for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(kern<P>, dim3(grid), dim3(256), 0, 0, out, clk, 2u + r);
    CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    static uint64_t h[2 * 8192]; CHK(hipMemcpy(h, clk, 2 * grid * 8, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0; for (int i = 0; i < grid; ++i) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
    double ghz = cyc / rt * 0.1;
    const int per_block = pat_count<P>();
    double inst_per_simd = (double)grid * 4 * 4 * ITERS * 8 * per_block / (cus * 4.0);
    printf("%-34s waves/SIMD=%d clk=%.3f cyc/VALU=%.3f\n", name, wpsimd, ghz, ms * 1e-3 * ghz * 1e9 / inst_per_simd);
    return 0;
}
int main() {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    uint32_t* out; uint64_t* clk; CHK(hipMalloc(&out, 8192 * 256 * 4)); CHK(hipMalloc(&clk, 8192 * 16));
    for (int w : {5}) {
        run<0>("alignbit (8B) @0", w, cus, out, clk);
        run<1>("alignbit (8B) @4", w, cus, out, clk);
        run<2>("bitop3 (8B) @0", w, cus, out, clk);
        run<3>("bitop3 (8B) @4", w, cus, out, clk);
        run<4>("add_e64 (8B) @0", w, cus, out, clk);
        run<5>("add_e64 (8B) @4", w, cus, out, clk);
        run<6>("add_e32 (4B) from @0", w, cus, out, clk);
        run<7>("add_e32 (4B) from @4", w, cus, out, clk);
        run<8>("SHA-like mix, 8B @0", w, cus, out, clk);
        run<9>("SHA-like mix, 8B @4", w, cus, out, clk);
        run<10>("alignbit/bitop3 alt @0", w, cus, out, clk);
        run<11>("alignbit/bitop3 alt @4", w, cus, out, clk);
        run<12>("lshrrev_e64 (8B) @4", w, cus, out, clk);
        run<13>("bfe_u32 (8B) @4", w, cus, out, clk);
        run<14>("lshrrev_e32 (4B)", w, cus, out, clk);
        run<15>("SHA-like @4 + 8 s_nop", w, cus, out, clk);
        run<16>("A/B alt, A @4 mod 16", w, cus, out, clk);
        run<17>("A/B alt, A @12 mod 16", w, cus, out, clk);
        run<18>("A/B alt, A @4,20 mod 32", w, cus, out, clk);
        run<19>("A/B alt, A @20,4 mod 32 (shift 16)", w, cus, out, clk);
        run<20>("B/A alt @4 mod 8", w, cus, out, clk);
        run<21>("A D4 D4, A @0", w, cus, out, clk);
        run<22>("A D4 D4, A @4", w, cus, out, clk);
        run<23>("A E8 E8 @0", w, cus, out, clk);
        run<24>("A E8 E8 @4", w, cus, out, clk);
        run<25>("AABB @4", w, cus, out, clk);
        run<26>("AAAABBBB @4", w, cus, out, clk);
        run<27>("ABB @4", w, cus, out, clk);
        run<28>("AAB @4", w, cus, out, clk);
        run<29>("add3/add_e64 alt @4", w, cus, out, clk);
        run<30>("8A then 8B @4", w, cus, out, clk);
    }
    return 0;
}
