// rot_ubench.hip -- issue rates of gfx950 VALU forms that could build a
// rotate (or a left shift) at full rate, beside v_alignbit_b32, the half-rate
// rotate the scan kernels use (dev tool; same method as valu_ubench.hip:
// 8 waves/SIMD, 8 independent chains, cycles per wave64 instruction).
// Build: hipcc --offload-arch=gfx950 -O3 tools/rot_ubench.hip -o build/rot_ubench
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

// x: a 64-bit VGPR pair per chain; y, z: 32-bit operands
template <int OP>
__device__ __forceinline__ void op(uint64_t& x, uint32_t y, uint32_t z) {
    if constexpr (OP == 0) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 1) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(x));
    if constexpr (OP == 2) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(x));
    if constexpr (OP == 3) asm volatile("v_lshlrev_b32_e32 %0, 7, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 5) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 6) asm volatile("v_pk_lshrrev_b16 %0, 7, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 7) asm volatile("v_lshl_add_u64 %0, %0, 7, %0" : "+v"(x));
    if constexpr (OP == 8) asm volatile("v_bfe_u32 %0, %0, 7, 20" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 9) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(x));
    if constexpr (OP == 10) asm volatile("v_mov_b64 %0, %0" : "+v"(x));
    if constexpr (OP == 11) asm volatile("v_ashrrev_i64 %0, 7, %0" : "+v"(x));
    if constexpr (OP == 12) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 13) asm volatile("v_and_b32 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 14) asm volatile("v_or_b32 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 15) asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 16) asm volatile("v_lshlrev_b16 %0, 7, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 17) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 18) asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(x));
    if constexpr (OP == 19) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(*(uint32_t*)&x) : "v"(y));
    if constexpr (OP == 20) asm volatile("v_lshrrev_b32_e64 %0, 7, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 21) asm volatile("v_lshrrev_b16 %0, 7, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 22) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(*(uint32_t*)&x));
    if constexpr (OP == 23) asm volatile("v_add_u16 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"(y));
}

template <int OP, int CHAINS>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint64_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = (uint64_t)seed * (threadIdx.x + c + 1) * 0x9e3779b97f4a7c15ull;
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
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)acc ^ (uint32_t)(acc >> 32);
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
    printf("%-22s clk=%.3f GHz  cycles/wave-instr=%.3f\n", name, ghz, secs * ghz * 1e9 / per_simd);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    printf("device %s CUs=%d\n", p.gcnArchName, cus);
    uint32_t* out;
    uint64_t* clk;
    CHK(hipMalloc(&out, 8192 * 256 * 4));
    CHK(hipMalloc(&clk, 8192 * 2 * 8));
#define R(OP, NAME) run<OP, 8>(NAME, 8, cus, out, clk)
    R(0, "v_alignbit_b32"); R(1, "v_lshrrev_b64"); R(2, "v_lshlrev_b64");
    R(3, "v_lshlrev_b32_e32"); R(4, "v_mul_u32_u24"); R(5, "v_mul_hi_u32_u24");
    R(6, "v_pk_lshrrev_b16"); R(7, "v_lshl_add_u64"); R(8, "v_bfe_u32");
    R(9, "v_pk_mov_b32"); R(10, "v_mov_b64"); R(11, "v_ashrrev_i64");
    R(12, "v_cndmask_b32"); R(13, "v_and_b32"); R(14, "v_or_b32"); R(15, "v_mul_lo_u16");
    R(16, "v_lshlrev_b16"); R(17, "v_mul_f32"); R(18, "v_pk_add_f32"); R(19, "v_sub_u32 rev");
    R(20, "v_lshrrev_b32_e64"); R(21, "v_lshrrev_b16"); R(22, "v_cvt_u32_f32"); R(23, "v_add_u16");
    return 0;
}
