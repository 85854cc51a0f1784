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

__global__ void __launch_bounds__(256) k_duplicate(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets,
                                                    const uint2* rect, unsigned grid_x, uint32_t* tile_keys,
                                                    uint32_t* gauss_vals) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= Pv) return;
    const uint32_t idx = sorted_ids[s];
    const uint2 r = rect[idx];
    const unsigned x0 = r.x & 0xffffu, x1 = r.x >> 16, y0 = r.y & 0xffffu, y1 = r.y >> 16;
    uint32_t o = offsets[s];
    for (unsigned y = y0; y < y1; y++)
        for (unsigned x = x0; x < x1; x++) {
            tile_keys[o] = y * grid_x + x;
            gauss_vals[o] = idx;
            o++;
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
