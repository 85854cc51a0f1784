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

// Cost bucket: the bit length of c and its next two bits (4 buckets per octave), 0 for c = 0.
#ifdef GSR_COARSE_BUCKETS
constexpr int NBUCKET = 33;
__device__ __forceinline__ int cost_bucket(uint32_t c) { return c ? 32 - __clz(c) : 0; }
__device__ __forceinline__ int bucket_heavy_from(int heavy_bits) { return heavy_bits + 1; }
#else
#ifndef GSR_BUCKET_BITS
#define GSR_BUCKET_BITS 3
#endif
constexpr int BUCKET_FRAC = GSR_BUCKET_BITS;  // 2^BUCKET_FRAC buckets per octave
constexpr int NBUCKET = 33 << BUCKET_FRAC;
__device__ __forceinline__ int cost_bucket(uint32_t c) {
    if (!c) return 0;
    const int L = 32 - __clz(c);
    const uint32_t fm = (1u << BUCKET_FRAC) - 1u;
    const uint32_t f = L > BUCKET_FRAC ? (c >> (L - 1 - BUCKET_FRAC)) & fm : (c << (BUCKET_FRAC + 1 - L)) & fm;
    return (L << BUCKET_FRAC) + (int)f;
}
__device__ __forceinline__ int bucket_heavy_from(int heavy_bits) { return (heavy_bits + 1) << BUCKET_FRAC; }
#endif

__global__ void __launch_bounds__(1024) k_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost,
                                                      uint32_t* order, uint32_t* nheavy, int heavy_bits,
                                                      const uint2* st_ranges, unsigned gx, unsigned gsx,
                                                      uint32_t* zero_a, uint32_t* zero_b, uint32_t* zero_c) {
    __shared__ uint32_t hist[NBUCKET];
    __shared__ uint32_t cur[NBUCKET];
    unsigned lo, len;
    band_of(blockIdx.x, ntile, lo, len);
    if (threadIdx.x < NBUCKET) hist[threadIdx.x] = 0;
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = tile_cost(t, ranges, cost, st_ranges, gx, gsx);
        atomicAdd(&hist[cost_bucket(c)], 1u);
        if (zero_a) {
            zero_a[t] = 0u;
            zero_b[t] = 0u;
            if (zero_c) zero_c[t] = 0u;
        }
    }
    __syncthreads();
    // cur[b] = tiles in buckets above b (heaviest bucket first): a block scan over the
    // buckets in descending order, thread j holding bucket NBUCKET - 1 - j
    __shared__ uint32_t scan[1024];
    static_assert(NBUCKET <= 1024, "one thread per bucket");
    const int j = threadIdx.x, bj = NBUCKET - 1 - j;
    const uint32_t hj = bj >= 0 ? hist[bj] : 0u;
    scan[j] = hj;
    __syncthreads();
    for (int o = 1; o < NBUCKET; o <<= 1) {
        const uint32_t v = j >= o ? scan[j - o] : 0u;
        __syncthreads();
        scan[j] += v;
        __syncthreads();
    }
    if (bj >= 0) cur[bj] = scan[j] - hj;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int hb = bucket_heavy_from(heavy_bits);
        nheavy[blockIdx.x] = hb < NBUCKET ? cur[hb] + hist[hb] : 0u;  // cost >= 2^heavy_bits
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = tile_cost(t, ranges, cost, st_ranges, gx, gsx);
#ifdef GSR_NATURAL_ORDER
        order[lo + i] = t;
#else
        order[lo + atomicAdd(&cur[cost_bucket(c)], 1u)] = t;
#endif
    }
}

void launch_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost, uint32_t* order, uint32_t* nheavy,
                       int heavy_bits, hipStream_t s) {
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, ntile, ranges, cost, order, nheavy, heavy_bits,
                       (const uint2*)nullptr, 0u, 0u, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr);
}

void launch_tile_order_st(unsigned ntile, unsigned gx, unsigned gsx, const uint2* st_ranges, uint32_t* order,
                          uint32_t* nheavy, int heavy_bits, uint32_t* zero_a, uint32_t* zero_b, uint32_t* zero_c,
                          hipStream_t s) {
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, ntile, (const uint2*)nullptr, (const uint32_t*)nullptr,
                       order, nheavy, heavy_bits, st_ranges, gx, gsx, zero_a, zero_b, zero_c);
}

}  // namespace gsr
