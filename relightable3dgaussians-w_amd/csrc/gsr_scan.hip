// gsr_scan.hip -- device-wide scans for the binning stage (replaces the reference's
// cub::DeviceScan::InclusiveSum, rasterizer_impl.cu:276-277).
//
// Reduce-then-scan over 4096-item tiles, each thread owning 16 consecutive items
// (4 x 16-B loads), so compaction is stable (index order preserved) with one workgroup
// scan per tile.
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

// ---------------- visibility compaction ----------------------------------------------
__global__ void __launch_bounds__(SCAN_THREADS) k_vis_reduce(int P, const uint32_t* tiles, const uint32_t* stc,
                                                               unsigned long long* block_tmp) {
    __shared__ unsigned long long sh[3][4];
    const long long base = (long long)blockIdx.x * SCAN_TILE + (long long)threadIdx.x * SCAN_ITEMS;
    unsigned long long cnt = 0, sum = 0, ssum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const long long i = base + k;
        if (i < P) {
            const uint32_t t = tiles[i];
            cnt += t > 0;
            sum += t;
            ssum += stc[i];
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    cnt = wave_reduce_sum(cnt);
    sum = wave_reduce_sum(sum);
    ssum = wave_reduce_sum(ssum);
    if (lane == 0) {
        sh[0][wave] = cnt;
        sh[1][wave] = sum;
        sh[2][wave] = ssum;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        block_tmp[3 * blockIdx.x + k] = sh[k][0] + sh[k][1] + sh[k][2] + sh[k][3];
    }
}

__global__ void __launch_bounds__(SCAN_THREADS) k_vis_spine(int nb, unsigned long long* block_tmp,
                                                              unsigned long long* totals) {
    __shared__ unsigned long long sh[4];
    unsigned long long carry = 0, tsum = 0, ssum = 0;
    for (int c = 0; c < nb; c += SCAN_THREADS) {
        const int i = c + threadIdx.x;
        unsigned long long v = i < nb ? block_tmp[3 * i] : 0ull;
        unsigned long long t = i < nb ? block_tmp[3 * i + 1] : 0ull;
        unsigned long long u = i < nb ? block_tmp[3 * i + 2] : 0ull;
        unsigned long long tot, tt, uu;
        unsigned long long ex = block256_exclusive_scan(v, sh, &tot);
        block256_exclusive_scan(t, sh, &tt);
        block256_exclusive_scan(u, sh, &uu);
        if (i < nb) block_tmp[3 * i] = carry + ex;
        carry += tot;
        tsum += tt;
        ssum += uu;
    }
    if (threadIdx.x == 0) {
        totals[0] = carry;
        totals[1] = tsum;
        totals[2] = ssum;
    }
}

__global__ void __launch_bounds__(SCAN_THREADS) k_vis_scatter(int P, const uint32_t* tiles,
                                                                const uint32_t* depth_key, uint32_t* vis_key,
                                                                uint32_t* vis_val,
                                                                const unsigned long long* block_tmp) {
    __shared__ unsigned long long sh[4];
    const long long base = (long long)blockIdx.x * SCAN_TILE + (long long)threadIdx.x * SCAN_ITEMS;
    uint32_t t[SCAN_ITEMS];
    unsigned long long cnt = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        const long long i = base + k;
        t[k] = i < P ? tiles[i] : 0u;
        cnt += t[k] > 0;
    }
    unsigned long long pos = block256_exclusive_scan(cnt, sh, (unsigned long long*)nullptr) +
                             block_tmp[3 * blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        if (t[k] > 0) {
            const long long i = base + k;
            vis_key[pos] = depth_key[i];
            vis_val[pos] = (uint32_t)i;
            pos++;
        }
    }
}

void launch_compact_visible(int P, const uint32_t* tiles, const uint32_t* st_count, const uint32_t* depth_key,
                            uint32_t* vis_key, uint32_t* vis_val, unsigned long long* block_tmp,
                            unsigned long long* totals, hipStream_t s) {
    const int nb = scan_blocks(P);
    if (nb == 0) {
        (void)hipMemsetAsync(totals, 0, 3 * sizeof(unsigned long long), s);
        return;
    }
    hipLaunchKernelGGL(k_vis_reduce, dim3(nb), dim3(SCAN_THREADS), 0, s, P, tiles, st_count, block_tmp);
    hipLaunchKernelGGL(k_vis_spine, dim3(1), dim3(SCAN_THREADS), 0, s, nb, block_tmp, totals);
    hipLaunchKernelGGL(k_vis_scatter, dim3(nb), dim3(SCAN_THREADS), 0, s, P, tiles, depth_key, vis_key, vis_val,
                       block_tmp);
}

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
