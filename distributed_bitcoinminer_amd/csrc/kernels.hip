// kernels.hip -- the auxiliary gfx950 kernels of the min-hash nonce scan.
//
//   hm_tile_plan_kernel  one thread per tile: ASCII high digits, padding,
//                        length, and (two-block tails) the chaining state
//                        after the tail block that holds no varying digit.
//   hm_kw_table_kernel   K[i]+W[i] of the chained kernel's wave-uniform final
//                        block for each loop value.
//   hm_fold_kernel       second reduce pass (candidates -> 16-B best).
//   hm_sum_fold_kernel   coverage sums of checked scans (per wave -> total).
//   hm_init_best_kernel  (MaxUint64, 0) seeds (miner.go:48-49).
//
// The scan kernels themselves are in scan_kernels.hip (own code object).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "sha256_defs.hpp"
#include "sha_device.hpp"

namespace hm {

// ---------------------------------------------------------------------------
// Tile planner
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) hm_tile_plan_kernel(const PlanArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.ntiles) return;
    uint32_t w[32];
    // tile base; its low V digits (varied by the scan kernels) stay zero bytes
    build_tail(w, A.pw, A.r, A.d, A.V, (A.tile0 + i) * A.pow10V, A.nb, A.total_bits);
    uint32_t st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = A.mid[k];
    uint32_t* out = A.rec + (size_t)i * kRecWords;
    if (A.fb == 1) {
        h_compress(st, w);
#pragma unroll
        for (int k = 0; k < 16; ++k) out[8 + k] = w[16 + k];
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) out[8 + k] = w[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
}

// One thread per table row computes the row's 64 words; the workgroup's 256
// rows (64 KB) are staged in LDS and written out as one contiguous block, so
// the stores coalesce (a row per thread written directly strides 256 B across
// the lanes of every store: 10^7 rows took 2.7 ms that way, round 3).
constexpr uint32_t kRowPad = 65;  // LDS row stride in words: conflict-free both ways
__global__ void __launch_bounds__(kBlock) hm_kw_table_kernel(uint32_t* __restrict__ out,
                                                             uint32_t f, uint32_t n,
                                                             uint64_t base,
                                                             uint64_t total_bits) {
    __shared__ uint32_t rows[kBlock * kRowPad];
    const uint32_t row0 = blockIdx.x * kBlock;
    const uint32_t t = row0 + threadIdx.x;
    if (t < n) {
        // f digits of base + t with leading zeros (< 10^f), then 0x80 and the length
        uint32_t b[32];
        const uint32_t zero[16] = {0};
        build_tail(b, zero, 0, f, 0, base + t, 1, total_bits);
        uint32_t w[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) w[k] = k < 16 ? b[k] : 0u;
        h_schedule(w);
#pragma unroll
        for (int k = 0; k < 64; ++k) rows[threadIdx.x * kRowPad + k] = kK[k] + w[k];
    }
    __syncthreads();
    const uint32_t nrows = n - row0 < kBlock ? n - row0 : kBlock;
    uint32_t* __restrict__ o = out + (size_t)row0 * 64;
    for (uint32_t i = threadIdx.x; i < nrows * 64; i += kBlock) o[i] = rows[(i >> 6) * kRowPad + (i & 63)];
}

// ---------------------------------------------------------------------------
// Fused launch planner: one thread per job.  Per segment (FusedPlanSeg, in
// job order): its tile records (as hm_tile_plan_kernel); then, tiled, the
// 100 sigma0 values of the loop-digit bits (tiled_loop_sigma0 in plan.cpp)
// and, with a trailer, the trailer block's 64 K+W words (one job); chained,
// its 10^f K+W rows (as hm_kw_table_kernel, without epochs).  Thread 0 also
// resets the queue counter, seeds the result slot and zeroes the checked
// scans' accumulators, so nothing else runs between this and the scan.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) hm_fused_plan_kernel(const FusedPlanArgs A) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) {
        *A.counter = A.counter0;
        if (A.result) { A.result[0] = ~0ull; A.result[1] = 0; }  // miner.go:48-49
        for (uint32_t i = 0; A.acc && i < A.n_acc; ++i) A.acc[i] = 0;
    }
    if (g >= A.njobs) return;
    uint32_t si = 0;
    while (g >= A.segs[si].job_end) ++si;
    const FusedPlanSeg& S = A.segs[si];
    uint32_t j = g - (si ? A.segs[si - 1].job_end : 0);
    if (j < S.ntiles) {
        uint32_t w[32];
        build_tail(w, A.pw, A.r, S.d, S.V, (S.tile0 + j) * S.pow10V, S.nb, S.total_bits);
        uint32_t st[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) st[k] = A.mid[k];
        uint32_t* out = A.rec + (size_t)(S.rec0 + j) * kRecWords;
        if (S.fb == 1) {
            h_compress(st, w);
#pragma unroll
            for (int k = 0; k < 16; ++k) out[8 + k] = w[16 + k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) out[8 + k] = w[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = st[k];
        return;
    }
    j -= S.ntiles;
    uint32_t* aux = A.aux + S.aux0;
    if (S.variant == kVarChained) {
        // K+W row j of the final block holding the f digits of j
        uint32_t b[32];
        const uint32_t zero[16] = {0};
        build_tail(b, zero, 0, S.f, 0, j, 1, S.total_bits);
        uint32_t w[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) w[k] = k < 16 ? b[k] : 0u;
        h_schedule(w);
        uint32_t* o = aux + (size_t)j * 64;
#pragma unroll
        for (int k = 0; k < 64; ++k) o[k] = kK[k] + w[k];
        return;
    }
    if (j < 100) {  // tiled: sigma0 of the loop digits' bits of W[W1], t1 * 10 + t0
        const uint32_t t1 = j / 10, t0 = j - t1 * 10;
        const uint32_t L = S.straddle ? (0x30u + t0) << 24
                                      : (((0x30u + t1) << 8) | (0x30u + t0)) << S.loop_shift;
        aux[j] = h_rotr(L, 7) ^ h_rotr(L, 18) ^ (L >> 3);
        return;
    }
    // tiled with a trailer: K+W of the constant padding block (trailer_kw)
    uint32_t w[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) w[k] = 0;
    if (S.T == 64) w[0] = 0x80000000u;  // 0x80 opens the trailer block
    w[14] = (uint32_t)(S.total_bits >> 32);
    w[15] = (uint32_t)S.total_bits;
    h_schedule(w);
#pragma unroll
    for (int k = 0; k < 64; ++k) aux[100 + k] = kK[k] + w[k];
}

// ---------------------------------------------------------------------------
// Second reduce pass and init
// ---------------------------------------------------------------------------
// `host`, when set, is pinned fine-grained host memory (the call's 16-B
// readback slot): the result is also stored there with system-scope vector
// stores, so the host reads it once the stream is done -- no device-to-host
// copy (a blit kernel and a launch gap) after the fold.
__global__ void __launch_bounds__(kBlock) hm_fold_kernel(const uint64_t* __restrict__ cand,
                                                         uint32_t n, uint32_t stride,
                                                         uint64_t* best, uint64_t* host) {
    __shared__ uint64_t sk[kBlock / kWaveSize], sn[kBlock / kWaveSize];
    uint64_t k = ~0ull, nn = ~0ull;
    if (threadIdx.x == 0) { k = best[0]; nn = best[1]; }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t k2 = cand[2 * (size_t)i * stride], n2 = cand[2 * (size_t)i * stride + 1];
        if (k2 < k || (k2 == k && n2 < nn)) { k = k2; nn = n2; }
    }
    wave_min(k, nn);
    if (__lane_id() == 0) { sk[threadIdx.x / kWaveSize] = k; sn[threadIdx.x / kWaveSize] = nn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWaveSize; ++w)
            if (sk[w] < k || (sk[w] == k && sn[w] < nn)) { k = sk[w]; nn = sn[w]; }
        best[0] = k;
        best[1] = nn;
        if (host) {
            __hip_atomic_store(&host[0], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&host[1], nn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
        }
    }
}

__global__ void __launch_bounds__(kBlock) hm_sum_fold_kernel(const uint64_t* __restrict__ sums,
                                                             uint32_t n, uint64_t* acc) {
    __shared__ uint64_t ss[kBlock / kWaveSize], sc[kBlock / kWaveSize];
    uint64_t a = 0, c = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        a += sums[2 * (size_t)i];
        c += sums[2 * (size_t)i + 1];
    }
    a = wave_sum(a);
    c = wave_sum(c);
    if (__lane_id() == 0) { ss[threadIdx.x / kWaveSize] = a; sc[threadIdx.x / kWaveSize] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWaveSize; ++w) { a += ss[w]; c += sc[w]; }
        acc[0] += a;
        acc[1] += c;
    }
}

__global__ void hm_init_best_kernel(uint64_t* best, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { best[2 * i] = ~0ull; best[2 * i + 1] = 0; }  // (MaxUint64, 0): miner.go:48-49
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
hipError_t launch_tile_plan(const PlanArgs& a, hipStream_t s) {
    const uint32_t grid = (a.ntiles + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(hm_tile_plan_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_sum_fold(const uint64_t* sums, uint32_t n, uint64_t* acc, hipStream_t s) {
    hipLaunchKernelGGL(hm_sum_fold_kernel, dim3(1), dim3(kBlock), 0, s, sums, n, acc);
    return hipGetLastError();
}

hipError_t launch_kw_table(uint32_t* out, uint32_t f, uint32_t fe, uint64_t base,
                           uint64_t total_bits, hipStream_t s) {
    // f final-block digits (a u64 has at most 20), fe of them from the table
    if (fe < 1 || fe > kMaxTableDigits || fe > f || f > 20) return hipErrorInvalidValue;
    uint32_t n = 1;
    for (uint32_t i = 0; i < fe; ++i) n *= 10u;
    hipLaunchKernelGGL(hm_kw_table_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                       out, f, n, base, total_bits);
    return hipGetLastError();
}

hipError_t launch_fold(const uint64_t* cand, uint32_t n, uint64_t* best, hipStream_t s,
                       uint32_t stride, uint64_t* host) {
    hipLaunchKernelGGL(hm_fold_kernel, dim3(1), dim3(kBlock), 0, s, cand, n, stride, best, host);
    return hipGetLastError();
}

hipError_t launch_fused_plan(const FusedPlanArgs& a, hipStream_t s) {
    const uint32_t grid = a.njobs ? (a.njobs + kBlock - 1) / kBlock : 1;
    hipLaunchKernelGGL(hm_fused_plan_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_init_best(uint64_t* best, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(hm_init_best_kernel, dim3((n + 63) / 64), dim3(64), 0, s, best, n);
    return hipGetLastError();
}

}  // namespace hm
