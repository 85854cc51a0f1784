// gsr_binning.hip -- instance emission and tile ranges (rasterizer_impl.cu:70-138).
//
// Differences from the reference, with identical results:
//  * instances are emitted in DEPTH order (after sorting the visible Gaussians by their
//    depth key), carrying the tile id alone as the sort key; the stable tile-only sort
//    then reproduces the reference's (tile, depth, index) order exactly;
//  * ranges are produced for the T tiles only (the reference sizes its image buffer by
//    pixel count, :172-179, but only T entries are ever used).
#include "gsr_kernels.hpp"

namespace gsr {

// One wave emits the instances of 64 consecutive depth-sorted Gaussians as one flat,
// contiguous run: lane i writes instance i, i+64, ... (coalesced 4-B stores), finding its
// Gaussian by binary search over the wave's inclusive tile-count prefix in LDS.
__global__ void __launch_bounds__(256) k_duplicate(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets,
                                                    const uint2* rect, unsigned grid_x, uint32_t* tile_keys,
                                                    uint32_t* gauss_vals) {
    __shared__ uint32_t s_inc[4][64];
    __shared__ uint32_t s_id[4][64];
    __shared__ uint2 s_rect[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t idx = 0, cnt = 0;
    uint2 r = make_uint2(0, 0);
    if (s < Pv) {
        idx = sorted_ids[s];
        r = rect[idx];
        cnt = ((r.x >> 16) - (r.x & 0xffffu)) * ((r.y >> 16) - (r.y & 0xffffu));
    }
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    s_inc[wave][lane] = inc;
    s_id[wave][lane] = idx;
    s_rect[wave][lane] = r;
    const int s0 = blockIdx.x * blockDim.x + wave * 64;
    const uint32_t base = s0 < Pv ? offsets[s0] : 0u;
    const uint32_t total = __shfl(inc, 63, 64);
    __syncthreads();
    for (uint32_t i = lane; i < total; i += 64) {
        // first j with s_inc[j] > i
        int lo = 0, hi = 63;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_inc[wave][mid] > i) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t k = i - (lo ? s_inc[wave][lo - 1] : 0u);
        const uint2 rr = s_rect[wave][lo];
        const uint32_t x0 = rr.x & 0xffffu, w = (rr.x >> 16) - x0, y0 = rr.y & 0xffffu;
        const uint32_t yy = k / w, xx = k - yy * w;
        tile_keys[base + i] = (y0 + yy) * grid_x + (x0 + xx);
        gauss_vals[base + i] = s_id[wave][lo];
    }
}

__global__ void __launch_bounds__(256) k_ranges(long long R, const uint32_t* keys, uint2* ranges) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint32_t cur = keys[i];
    if (i == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys[i - 1];
        if (cur != prev) {
            ranges[prev].y = (uint32_t)i;
            ranges[cur].x = (uint32_t)i;
        }
    }
    if (i == R - 1) ranges[cur].y = (uint32_t)R;
}

void launch_duplicate(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets, const uint2* rect,
                      unsigned grid_x, uint32_t* tile_keys, uint32_t* gauss_vals, hipStream_t s) {
    if (Pv == 0) return;
    hipLaunchKernelGGL(k_duplicate, dim3((Pv + 255) / 256), dim3(256), 0, s, Pv, sorted_ids, offsets, rect, grid_x,
                       tile_keys, gauss_vals);
}

void launch_ranges(long long R, int T, const uint32_t* sorted_tile_keys, uint2* ranges, hipStream_t s) {
    hipMemsetAsync(ranges, 0, sizeof(uint2) * (size_t)T, s);
    if (R == 0) return;
    hipLaunchKernelGGL(k_ranges, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, R, sorted_tile_keys, ranges);
}

}  // namespace gsr
