// mix_ubench.hip -- issue cost of MIXED instruction streams on gfx950 (dev tool).
// Each statement is a fixed pattern over 8 independent accumulators.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 2048;
#define A(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t"
#define X(i) "v_xor_b32 %" #i ", %" #i ", %8\n\t"
#define B(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t"
#define D(i) "v_add_u32 %" #i ", %" #i ", %8\n\t"
#define T(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"
#define OUTS "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
#define INS "v"(y), "v"(z)
template <int P>
__device__ __forceinline__ int pat(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                   uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t z) {
    // returns instructions per statement
    if constexpr (P == 0) { asm volatile(A(0) A(1) A(2) A(3) A(4) A(5) A(6) A(7) : OUTS : INS); return 8; }
    if constexpr (P == 1) { asm volatile(D(0) D(1) D(2) D(3) D(4) D(5) D(6) D(7) : OUTS : INS); return 8; }
    if constexpr (P == 2) { asm volatile(A(0) D(1) A(2) D(3) A(4) D(5) A(6) D(7) : OUTS : INS); return 8; }   // 1:1 alternating
    if constexpr (P == 3) { asm volatile(A(0) A(2) A(4) A(6) D(1) D(3) D(5) D(7) : OUTS : INS); return 8; }   // 1:1 grouped
    if constexpr (P == 4) { asm volatile(A(0) A(1) A(2) B(3) A(4) A(5) A(6) B(7) : OUTS : INS); return 8; }   // sigma-like 3:1
    if constexpr (P == 5) { asm volatile(A(0) D(1) D(2) A(3) D(4) D(5) A(6) D(7) : OUTS : INS); return 8; }   // 3:5
    if constexpr (P == 6) { asm volatile(T(0) D(1) T(2) D(3) T(4) D(5) T(6) D(7) : OUTS : INS); return 8; }   // add3/add
    if constexpr (P == 7) { asm volatile(A(0) B(1) A(2) B(3) A(4) B(5) A(6) B(7) : OUTS : INS); return 8; }   // align/bitop3
    if constexpr (P == 8) { asm volatile(A(0) X(1) A(2) X(3) A(4) X(5) A(6) X(7) : OUTS : INS); return 8; }   // align/xor
    if constexpr (P == 9) { asm volatile(T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7) : OUTS : INS); return 8; }
    if constexpr (P == 10) { asm volatile(B(0) B(1) B(2) B(3) B(4) B(5) B(6) B(7) : OUTS : INS); return 8; }
    if constexpr (P == 11) { asm volatile(A(0) A(1) D(2) D(3) A(4) A(5) D(6) D(7) : OUTS : INS); return 8; }  // 2:2
    return 0;
}
template <int P>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t x0 = seed ^ threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 11, x5 = x0 * 13, x6 = x0 * 17, x7 = x0 * 19;
    uint32_t y = seed + 1, z = seed * 7;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) pat<P>(x0, x1, x2, x3, x4, x5, x6, x7, y, z);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
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
    double inst_per_simd = (double)grid * 4 * 4 * ITERS * 8 * 8 / (cus * 4.0);
    printf("%-22s waves/SIMD=%d clk=%.3f cyc/inst=%.3f\n", name, wpsimd, ghz, ms * 1e-3 * ghz * 1e9 / inst_per_simd);
    return 0;
}
int main() {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    uint32_t* out; uint64_t* clk; CHK(hipMalloc(&out, 8192 * 256 * 4)); CHK(hipMalloc(&clk, 8192 * 16));
    for (int w : {2, 4}) {
        run<0>("align only", w, cus, out, clk);
        run<1>("add only", w, cus, out, clk);
        run<10>("bitop3 only", w, cus, out, clk);
        run<9>("add3 only", w, cus, out, clk);
        run<2>("align/add alternate", w, cus, out, clk);
        run<3>("align4 then add4", w, cus, out, clk);
        run<11>("align2 add2", w, cus, out, clk);
        run<4>("3 align : 1 bitop3", w, cus, out, clk);
        run<5>("3 align : 5 add", w, cus, out, clk);
        run<6>("add3/add alternate", w, cus, out, clk);
        run<7>("align/bitop3 alt", w, cus, out, clk);
        run<8>("align/xor alt", w, cus, out, clk);
    }
    return 0;
}
