// gsr_schedule.hip -- tile work queues for the persistent tile passes.
//
// The tile passes run one wave per tile, but tiles differ in cost by an order of magnitude
// (list length, early saturation), and a grid of one workgroup per tile leaves the chip's
// tail waiting on a few heavy tiles dispatched last.  Here each XCD gets a queue of its band
// of the image (the bands of xcd_remap: neighbouring tiles share Gaussian records in that
// XCD's L2), ordered heaviest-first by a log2 bucketing of a cost estimate; the passes
// launch as many waves as the chip holds and each wave pulls tiles from its own XCD's
// queue, then from the others' (longest-processing-time-first with stealing).
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

// One workgroup per band: order[lo .. lo+len) = the band's tiles, cost buckets descending.
__global__ void __launch_bounds__(1024) k_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost,
                                                      uint32_t* order) {
    __shared__ uint32_t hist[33];
    __shared__ uint32_t cur[33];
    unsigned lo, len;
    band_of(blockIdx.x, ntile, lo, len);
    if (threadIdx.x < 33) hist[threadIdx.x] = 0;
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = cost ? cost[t] : ranges[t].y - ranges[t].x;
        atomicAdd(&hist[c ? 32 - __clz(c) : 0], 1u);  // bucket = bit length of the cost
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int b = 32; b >= 0; b--) {  // heaviest bucket first
            cur[b] = run;
            run += hist[b];
        }
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = cost ? cost[t] : ranges[t].y - ranges[t].x;
#ifdef GSR_NATURAL_ORDER
        order[lo + i] = t;
#else
        order[lo + atomicAdd(&cur[c ? 32 - __clz(c) : 0], 1u)] = t;
#endif
    }
}

void launch_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost, uint32_t* order, uint32_t* queue,
                       hipStream_t s) {
    (void)hipMemsetAsync(queue, 0, 8 * sizeof(uint32_t), s);
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_tile_order, dim3(8), dim3(1024), 0, s, ntile, ranges, cost, order);
}

int resident_waves(int per_simd) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    return cus * 4 * per_simd;
}

}  // namespace gsr
