// gsr_block.hpp -- wave64 / workgroup scan and reduction primitives (CDNA4: 64-lane waves,
// 64-bit ballots).  Workgroups are 256 threads = 4 waves unless stated otherwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
    const int lane = __lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T n = __shfl_up(v, o, 64);
        if (lane >= o) v += n;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive scan of one value per thread across a 256-thread workgroup.
// `sh` must hold 4 elements of T.  Returns the exclusive prefix; *total gets the sum.
template <typename T>
__device__ __forceinline__ T block256_exclusive_scan(T v, T* sh, T* total) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    T inc = wave_inclusive_scan(v);
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    T w0 = sh[0], w1 = sh[1], w2 = sh[2], w3 = sh[3];
    T off = (wave > 0 ? w0 : T(0)) + (wave > 1 ? w1 : T(0)) + (wave > 2 ? w2 : T(0));
    if (total) *total = w0 + w1 + w2 + w3;
    __syncthreads();
    return off + inc - v;
}

// Exclusive scan of one value per thread across a workgroup of NW waves; `sh` holds NW
// elements of T.  Returns the exclusive prefix; *total gets the sum.
template <int NW, typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* sh, T* total) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const T inc = wave_inclusive_scan(v);
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    T off = T(0), tot = T(0);
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const T x = sh[w];
        off += w < wave ? x : T(0);
        tot += x;
    }
    if (total) *total = tot;
    __syncthreads();
    return off + inc - v;
}

}  // namespace gsr
