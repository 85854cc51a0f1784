// gsr_schedule.hip -- heaviest-first dispatch order of the tile passes.
//
// The tile passes run one wave per tile, and tiles differ in cost by an order of magnitude
// (list length, early saturation).  Each XCD band of the image (the bands of xcd_remap:
// neighbouring tiles share Gaussian records in that XCD's L2) is ordered heaviest-first by
// a log2 bucketing of a cost estimate; the passes dispatch block b on position b / 8 of band
// b mod 8, so the hardware dispatcher runs a longest-first schedule per XCD.  Tiles above a
// cost threshold (lists in the thousands: dense centres of real scenes) are split over the
// four waves of their workgroup, one 8x8 quadrant each; the rest run four to a workgroup,
// one wave each (TileUnit in gsr_tile.hpp).
// (A persistent variant pulling tiles from per-XCD atomic queues measured 2x slower: the
// returning atomics cost ~13 us per pull under load.)
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

// One workgroup per band: order[lo .. lo+len) = the band's tiles, cost buckets descending;
// nheavy[band] = how many lead the order with a cost >= 2^heavy_bits (split 4 ways).
// The cost of tile t: cost[t]; else with st_ranges its super-tile's entry count (the
// forward: gx tiles per row, gsx super-tiles per row); else its list length.  zero_a / zero_b
// (optional): zeroed per tile (the forward's atomicMax targets).
__device__ __forceinline__ uint32_t tile_cost(unsigned t, const uint2* ranges, const uint32_t* cost,
                                              const uint2* st_ranges, unsigned gx, unsigned gsx) {
    if (cost) return cost[t];
    if (st_ranges) {
        const uint2 r = st_ranges[(t / gx) / GSR_ST_H * gsx + (t % gx) / GSR_ST_W];
        return r.y - r.x;
    }
    return ranges[t].y - ranges[t].x;
}

__global__ void __launch_bounds__(1024) k_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost,
                                                      uint32_t* order, uint32_t* nheavy, int heavy_bits,
                                                      const uint2* st_ranges, unsigned gx, unsigned gsx,
                                                      uint32_t* zero_a, uint32_t* zero_b) {
    __shared__ uint32_t hist[33];
    __shared__ uint32_t cur[33];
    unsigned lo, len;
    band_of(blockIdx.x, ntile, lo, len);
    if (threadIdx.x < 33) hist[threadIdx.x] = 0;
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = tile_cost(t, ranges, cost, st_ranges, gx, gsx);
        atomicAdd(&hist[c ? 32 - __clz(c) : 0], 1u);  // bucket = bit length of the cost
        if (zero_a) {
            zero_a[t] = 0u;
            zero_b[t] = 0u;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0, heavy = 0;
        for (int b = 32; b >= 0; b--) {  // heaviest bucket first
            cur[b] = run;
            run += hist[b];
            if (b > heavy_bits) heavy += hist[b];  // cost >= 2^heavy_bits
        }
        nheavy[blockIdx.x] = heavy;
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = tile_cost(t, ranges, cost, st_ranges, gx, gsx);
#ifdef GSR_NATURAL_ORDER
        order[lo + i] = t;
#else
        order[lo + atomicAdd(&cur[c ? 32 - __clz(c) : 0], 1u)] = t;
#endif
    }
}

void launch_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost, uint32_t* order, uint32_t* nheavy,
                       int heavy_bits, hipStream_t s) {
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, ntile, ranges, cost, order, nheavy, heavy_bits,
                       (const uint2*)nullptr, 0u, 0u, (uint32_t*)nullptr, (uint32_t*)nullptr);
}

void launch_tile_order_st(unsigned ntile, unsigned gx, unsigned gsx, const uint2* st_ranges, uint32_t* order,
                          uint32_t* nheavy, int heavy_bits, uint32_t* zero_a, uint32_t* zero_b, hipStream_t s) {
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, ntile, (const uint2*)nullptr, (const uint32_t*)nullptr,
                       order, nheavy, heavy_bits, st_ranges, gx, gsx, zero_a, zero_b);
}

}  // namespace gsr
