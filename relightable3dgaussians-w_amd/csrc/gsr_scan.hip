// gsr_scan.hip -- device-wide exclusive scan for the binning stage (replaces the
// reference's cub::DeviceScan::InclusiveSum, rasterizer_impl.cu:276-277).
//
// Reduce-then-scan over 4096-item tiles, each thread owning 16 consecutive items.
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

// ---------------- generic exclusive scan (u32) ---------------------------------------------
__device__ __forceinline__ uint32_t load_item(const uint32_t* in, const uint32_t* gather, long long i) {
    return gather ? in[gather[i]] : in[i];
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(long long n, const uint32_t* in,
                                                                const uint32_t* gather, uint32_t* block_tmp) {
    __shared__ uint32_t sh[4];
    const long long base = (long long)blockIdx.x * SCAN_TILE + (long long)threadIdx.x * SCAN_ITEMS;
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const long long i = base + k;
        if (i < n) sum += load_item(in, gather, i);
    }
    sum = wave_reduce_sum(sum);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) block_tmp[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_spine(int nb, uint32_t* block_tmp, uint32_t* total) {
    __shared__ uint32_t sh[4];
    uint32_t carry = 0;
    for (int c = 0; c < nb; c += SCAN_THREADS) {
        const int i = c + threadIdx.x;
        uint32_t v = i < nb ? block_tmp[i] : 0u;
        uint32_t tot;
        uint32_t ex = block256_exclusive_scan(v, sh, &tot);
        if (i < nb) block_tmp[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_down(long long n, const uint32_t* in, const uint32_t* gather,
                                                              uint32_t* out, const uint32_t* block_tmp) {
    __shared__ uint32_t sh[4];
    const long long base = (long long)blockIdx.x * SCAN_TILE + (long long)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const long long i = base + k;
        v[k] = i < n ? load_item(in, gather, i) : 0u;
        sum += v[k];
    }
    uint32_t run = block256_exclusive_scan(sum, sh, (uint32_t*)nullptr) + block_tmp[blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const long long i = base + k;
        if (i < n) out[i] = run;
        run += v[k];
    }
}

void launch_exclusive_scan_u32(long long n, const uint32_t* in, const uint32_t* gather, uint32_t* out,
                               uint32_t* block_tmp, uint32_t* total, hipStream_t s) {
    const int nb = scan_blocks(n);
    if (nb == 0) {
        if (total) (void)hipMemsetAsync(total, 0, sizeof(uint32_t), s);
        return;
    }
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SCAN_THREADS), 0, s, n, in, gather, block_tmp);
    hipLaunchKernelGGL(k_scan_spine, dim3(1), dim3(SCAN_THREADS), 0, s, nb, block_tmp, total);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SCAN_THREADS), 0, s, n, in, gather, out, block_tmp);
}

}  // namespace gsr
