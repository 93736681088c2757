// valu_ubench.hip -- measures gfx950 VALU issue rates of the integer ops the
// SHA-256 scan uses (dev tool; results in profiles/ and DESIGN.md §5).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_ubench.hip -o build/valu_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                          \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);     \
            return 1;                                                   \
        }                                                               \
    } while (0)

constexpr int ITERS = 4096;

template <int OP>
__device__ __forceinline__ void op(uint32_t& x, uint32_t y, uint32_t z) {
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(y));
    if constexpr (OP == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 4) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 5) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 6) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));
    if constexpr (OP == 7) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "s"(y));
    if constexpr (OP == 9) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
    if constexpr (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 11) asm volatile("v_lshl_add_u32 %0, %0, 7, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 12) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 13) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 14) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(x) : "v"(y));
    if constexpr (OP == 15) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(z));
    if constexpr (OP == 16) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 17) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(y) : "vcc");
    if constexpr (OP == 18) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 19) asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 20) asm volatile("v_add_lshl_u32 %0, %0, %1, 0" : "+v"(x) : "v"(y));
    if constexpr (OP == 21) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 22) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 23) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 24) asm volatile("v_lshlrev_b32_e64 %0, 7, %0" : "+v"(x));
    if constexpr (OP == 25) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 26) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "s"(y), "v"(z));
    if constexpr (OP == 27) asm volatile("v_bitop3_b16 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 28) asm volatile("v_alignbit_b32 %0, %0, %0, 7\n\tv_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 29) asm volatile("v_add_u32_dpp %0, %0, %1 row_shr:1 bound_ctrl:0" : "+v"(x) : "v"(y));
    if constexpr (OP == 30) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y));
    if constexpr (OP == 31) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(z));
    if constexpr (OP == 32) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(y));
    if constexpr (OP == 33) asm volatile("v_lshl_or_b32 %0, %1, 7, %0" : "+v"(x) : "v"(y));
    if constexpr (OP == 34) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (OP == 35) asm volatile("v_lshrrev_b32 %0, 3, %0\n\tv_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
}

// CHAINS independent accumulators per lane
template <int OP, int CHAINS>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = seed * (threadIdx.x + c + 1);
    uint32_t y = seed ^ threadIdx.x, z = seed + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) op<OP>(x[c], y, z);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int OP, int CHAINS>
int run(const char* name, int blocks_per_cu, int cus, uint32_t* out, uint64_t* clk) {
    int grid = blocks_per_cu * cus;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL((kern<OP, CHAINS>), dim3(grid), dim3(256), 0, 0, out, clk, 12345u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL((kern<OP, CHAINS>), dim3(grid), dim3(256), 0, 0, out, clk, 777u + r);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    static uint64_t h[2 * 8192];
    CHK(hipMemcpy(h, clk, 2 * grid * sizeof(uint64_t), hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < grid; ++i) {
        cyc += h[2 * i];
        rt += h[2 * i + 1];
    }
    double ghz = (cyc / rt) * 0.1;  // memrealtime = 100 MHz
    double waves = (double)grid * 4 * 5;
    double winst = waves * ITERS * 4 * CHAINS;
    double per_simd = winst / (cus * 4.0);
    double secs = ms * 1e-3;
    double cyc_per_inst_wall = secs * ghz * 1e9 / per_simd;
    double lane_ops = winst * 64 / secs;
    printf("%-16s chains=%d waves/SIMD=%d  clk=%.3f GHz  cycles/wave-asm-stmt=%.3f  lane-Tstmt/s=%.2f\n",
           name, CHAINS, blocks_per_cu, ghz, cyc_per_inst_wall, lane_ops * 1e-12);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    printf("device %s CUs=%d clockRate=%d kHz\n", p.gcnArchName, cus, p.clockRate);
    uint32_t* out;
    uint64_t* clk;
    CHK(hipMalloc(&out, 8192 * 256 * 4));
    CHK(hipMalloc(&clk, 8192 * 2 * 8));
#define R(OP, NAME) run<OP, 8>(NAME, 8, cus, out, clk)
    R(0, "v_add_u32"); R(3, "v_bitop3 xor3"); R(34, "v_bitop3 maj"); R(1, "v_alignbit xy");
    R(9, "v_alignbit xx"); R(10, "v_lshl_or"); R(33, "v_lshl_or y"); R(11, "v_lshl_add");
    R(12, "v_or3"); R(13, "v_perm"); R(14, "v_alignbyte"); R(2, "v_add3 vvv");
    R(15, "v_add3 vvs"); R(16, "v_sub_u32"); R(17, "v_add_co"); R(18, "v_pk_add_u16");
    R(19, "v_mov"); R(20, "v_add_lshl"); R(21, "v_and_or"); R(22, "v_add_e64");
    R(23, "v_xor_e64"); R(24, "v_lshl_e64"); R(25, "v_mul_lo_u32"); R(26, "v_bitop3 svv");
    R(27, "v_bitop3_b16"); R(28, "align+xor pair"); R(35, "lshr+align pair"); R(29, "v_add dpp");
    R(30, "v_add_f32"); R(31, "v_xad vvs"); R(32, "v_add sdwa"); R(7, "v_bfi"); R(4, "v_xad");
    R(5, "v_xor_b32"); R(6, "v_lshrrev"); R(8, "v_add sgpr");
    return 0;
}
