// bank_ubench.hip -- VGPR bank conflicts on gfx950 (dev tool): 3-source VALU ops
// whose sources sit in the same VGPR bank (register number mod 4) or in three
// different banks.  Explicit registers v40..v71, 8-byte ops placed at 4 mod 8.
// build: hipcc -O3 --offload-arch=gfx950 tools/bank_ubench.hip -o build/bank_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 1024;
#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"
#define P4 ".p2align 3\n\ts_nop 0\n\t"
// same bank: dst/src0 v40+i, src1 v48+i, src2 v56+i  (i, i+8, i+16: equal mod 4)
#define BS(i) "v_bitop3_b32 v" #i ", v" #i ", v" #i "+8, v" #i "+16 bitop3:0x96\n\t"
template <int P>
__device__ __forceinline__ void pat() {
    // bitop3: three sources in one bank / in three banks
    if constexpr (P == 0) asm volatile(P4
        "v_bitop3_b32 v40, v40, v48, v56 bitop3:0x96\n\t" "v_bitop3_b32 v41, v41, v49, v57 bitop3:0x96\n\t"
        "v_bitop3_b32 v42, v42, v50, v58 bitop3:0x96\n\t" "v_bitop3_b32 v43, v43, v51, v59 bitop3:0x96\n\t"
        "v_bitop3_b32 v44, v44, v52, v60 bitop3:0x96\n\t" "v_bitop3_b32 v45, v45, v53, v61 bitop3:0x96\n\t"
        "v_bitop3_b32 v46, v46, v54, v62 bitop3:0x96\n\t" "v_bitop3_b32 v47, v47, v55, v63 bitop3:0x96\n\t" ::: CLOB);
    if constexpr (P == 1) asm volatile(P4
        "v_bitop3_b32 v40, v40, v49, v58 bitop3:0x96\n\t" "v_bitop3_b32 v41, v41, v50, v59 bitop3:0x96\n\t"
        "v_bitop3_b32 v42, v42, v51, v56 bitop3:0x96\n\t" "v_bitop3_b32 v43, v43, v48, v57 bitop3:0x96\n\t"
        "v_bitop3_b32 v44, v44, v53, v62 bitop3:0x96\n\t" "v_bitop3_b32 v45, v45, v54, v63 bitop3:0x96\n\t"
        "v_bitop3_b32 v46, v46, v55, v60 bitop3:0x96\n\t" "v_bitop3_b32 v47, v47, v52, v61 bitop3:0x96\n\t" ::: CLOB);
    // add3 (half rate): same bank / three banks
    if constexpr (P == 2) asm volatile(P4
        "v_add3_u32 v40, v40, v48, v56\n\t" "v_add3_u32 v41, v41, v49, v57\n\t" "v_add3_u32 v42, v42, v50, v58\n\t" "v_add3_u32 v43, v43, v51, v59\n\t"
        "v_add3_u32 v44, v44, v52, v60\n\t" "v_add3_u32 v45, v45, v53, v61\n\t" "v_add3_u32 v46, v46, v54, v62\n\t" "v_add3_u32 v47, v47, v55, v63\n\t" ::: CLOB);
    if constexpr (P == 3) asm volatile(P4
        "v_add3_u32 v40, v40, v49, v58\n\t" "v_add3_u32 v41, v41, v50, v59\n\t" "v_add3_u32 v42, v42, v51, v56\n\t" "v_add3_u32 v43, v43, v48, v57\n\t"
        "v_add3_u32 v44, v44, v53, v62\n\t" "v_add3_u32 v45, v45, v54, v63\n\t" "v_add3_u32 v46, v46, v55, v60\n\t" "v_add3_u32 v47, v47, v52, v61\n\t" ::: CLOB);
    // two sources in one bank (the third elsewhere)
    if constexpr (P == 4) asm volatile(P4
        "v_bitop3_b32 v40, v40, v48, v57 bitop3:0x96\n\t" "v_bitop3_b32 v41, v41, v49, v58 bitop3:0x96\n\t"
        "v_bitop3_b32 v42, v42, v50, v59 bitop3:0x96\n\t" "v_bitop3_b32 v43, v43, v51, v56 bitop3:0x96\n\t"
        "v_bitop3_b32 v44, v44, v52, v61 bitop3:0x96\n\t" "v_bitop3_b32 v45, v45, v53, v62 bitop3:0x96\n\t"
        "v_bitop3_b32 v46, v46, v54, v63 bitop3:0x96\n\t" "v_bitop3_b32 v47, v47, v55, v60 bitop3:0x96\n\t" ::: CLOB);
    if constexpr (P == 5) asm volatile(P4
        "v_add3_u32 v40, v40, v48, v57\n\t" "v_add3_u32 v41, v41, v49, v58\n\t" "v_add3_u32 v42, v42, v50, v59\n\t" "v_add3_u32 v43, v43, v51, v56\n\t"
        "v_add3_u32 v44, v44, v52, v61\n\t" "v_add3_u32 v45, v45, v53, v62\n\t" "v_add3_u32 v46, v46, v54, v63\n\t" "v_add3_u32 v47, v47, v55, v60\n\t" ::: CLOB);
}
template <int P>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
    asm volatile("v_mov_b32 v40, %0\n\tv_mov_b32 v48, %0\n\tv_mov_b32 v56, %0" :: "v"(seed ^ threadIdx.x) : CLOB);
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) pat<P>();
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t r;
    asm volatile("v_mov_b32 %0, v40" : "=v"(r) :: CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
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
    printf("%-34s waves/SIMD=%d clk=%.3f cyc/VALU=%.3f\n", name, wpsimd, ghz, ms * 1e-3 * ghz * 1e9 / inst_per_simd);
    return 0;
}
int main() {
    hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    uint32_t* out; uint64_t* clk; CHK(hipMalloc(&out, 8192 * 256 * 4)); CHK(hipMalloc(&clk, 8192 * 16));
    for (int w : {2, 5}) {
        run<0>("bitop3, 3 sources one bank", w, cus, out, clk);
        run<1>("bitop3, 3 banks", w, cus, out, clk);
        run<4>("bitop3, 2 sources one bank", w, cus, out, clk);
        run<2>("add3, 3 sources one bank", w, cus, out, clk);
        run<3>("add3, 3 banks", w, cus, out, clk);
        run<5>("add3, 2 sources one bank", w, cus, out, clk);
    }
    return 0;
}
