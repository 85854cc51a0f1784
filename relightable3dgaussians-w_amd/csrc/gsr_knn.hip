// gsr_knn.hip -- mean squared distance to the 3 nearest neighbours of every point, the
// `distCUDA2` of submodules/simple-knn (simple_knn.cu:119-220, used by
// gaussian_model.py:189,249 to initialise scales).
//
// Same algorithm and arithmetic as the reference, so results are bit-identical:
//   bounds   min / max over the points with the reference's {0,0,0} seed (cub Reduce with
//            init 0, simple_knn.cu:190-200: the box always contains the origin);
//   Morton   10 bits per axis of (c - min) / (max - min) * 1023 (truncating), interleaved;
//   sort     stable LSD radix sort of (code, index) on 30 bits (gsr_sort.hip);
//   boxes    min / max of every 1024 consecutive sorted points;
//   search   per point: the 3rd-best squared distance among its +-3 sorted neighbours is
//            a rejection bound, then boxes in index order are skipped when their distance
//            exceeds the bound or the current 3rd best, otherwise scanned in index order
//            with the reference's sorted-insertion update.
// One addition: a 32-box "super box" level.  A super box is skipped only when its distance
// (never more than any member box's, computed with the same monotone float operations)
// exceeds the current bound, in which case the reference would skip every member box, so
// the scanned set and order are unchanged.
// Sums of squares are written as fma(z, z, fma(y, y, x * x)), the contraction nvcc applies
// to the reference's `x*x + y*y + z*z` (simple_knn.cu:115,124).
#pragma clang fp contract(off)
#include <float.h>

#include "gsr_block.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

constexpr int KNN_BOX = 1024;
constexpr int KNN_SUPER = 32;  // boxes per super box

struct KBox {
    float3 mn, mx;
};

__device__ __forceinline__ float sq3(float x, float y, float z) { return __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)); }

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
// float -> u32 as cvt.rzi.u32.f32: truncation, saturation, NaN -> 0
__device__ __forceinline__ uint32_t f2u(float f) {
    if (!(f > 0.f)) return 0u;
    if (f >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// ---- bounds (seeded with 0 like the reference's Reduce init) -----------------------------
__global__ void __launch_bounds__(256) k_knn_bounds_partial(int P, const float* pts, float* part) {
    __shared__ float sh[6][4];
    float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // min xyz, max xyz
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
        const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
        v[0] = fminf(v[0], x);
        v[1] = fminf(v[1], y);
        v[2] = fminf(v[2], z);
        v[3] = fmaxf(v[3], x);
        v[4] = fmaxf(v[4], y);
        v[5] = fmaxf(v[5], z);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 6; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float t = __shfl_xor(v[k], o, 64);
            v[k] = k < 3 ? fminf(v[k], t) : fmaxf(v[k], t);
        }
        if (lane == 0) sh[k][wave] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float r = sh[k][0];
        for (int w = 1; w < 4; w++) r = k < 3 ? fminf(r, sh[k][w]) : fmaxf(r, sh[k][w]);
        part[6 * blockIdx.x + k] = r;
    }
}

__global__ void __launch_bounds__(64) k_knn_bounds_final(int nb, const float* part, float* bounds) {
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float r = 0.f;
        for (int b = 0; b < nb; b++) r = k < 3 ? fminf(r, part[6 * b + k]) : fmaxf(r, part[6 * b + k]);
        bounds[k] = r;
    }
}

// ---- Morton codes (simple_knn.cu:53-71) ---------------------------------------------------
__global__ void __launch_bounds__(256) k_knn_morton(int P, const float* pts, const float* bounds, uint32_t* codes,
                                                     uint32_t* ids) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float mnx = bounds[0], mny = bounds[1], mnz = bounds[2];
    const float mxx = bounds[3], mxy = bounds[4], mxz = bounds[5];
    const uint32_t x = prep_morton(f2u(((pts[3 * i] - mnx) / (mxx - mnx)) * 1023.f));
    const uint32_t y = prep_morton(f2u(((pts[3 * i + 1] - mny) / (mxy - mny)) * 1023.f));
    const uint32_t z = prep_morton(f2u(((pts[3 * i + 2] - mnz) / (mxz - mnz)) * 1023.f));
    codes[i] = x | (y << 1) | (z << 2);
    ids[i] = (uint32_t)i;
}

// sorted copy of the points (float4 rows) so the scans read contiguous memory
__global__ void __launch_bounds__(256) k_knn_gather(int P, const float* pts, const uint32_t* sorted_ids, float4* spts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint32_t j = sorted_ids[i];
    spts[i] = make_float4(pts[3 * j], pts[3 * j + 1], pts[3 * j + 2], 0.f);
}

// box min / max over KNN_BOX sorted points (simple_knn.cu:79-113): one workgroup per box
__global__ void __launch_bounds__(256) k_knn_boxes(int P, const float4* spts, KBox* boxes) {
    __shared__ float sh[6][4];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    const int b0 = blockIdx.x * KNN_BOX;
    for (int t = threadIdx.x; t < KNN_BOX; t += blockDim.x) {
        const int i = b0 + t;
        if (i < P) {
            const float4 p = spts[i];
            v[0] = fminf(v[0], p.x);
            v[1] = fminf(v[1], p.y);
            v[2] = fminf(v[2], p.z);
            v[3] = fmaxf(v[3], p.x);
            v[4] = fmaxf(v[4], p.y);
            v[5] = fmaxf(v[5], p.z);
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 6; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float t = __shfl_xor(v[k], o, 64);
            v[k] = k < 3 ? fminf(v[k], t) : fmaxf(v[k], t);
        }
        if (lane == 0) sh[k][wave] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float r[6];
        for (int k = 0; k < 6; k++) {
            r[k] = sh[k][0];
            for (int w = 1; w < 4; w++) r[k] = k < 3 ? fminf(r[k], sh[k][w]) : fmaxf(r[k], sh[k][w]);
        }
        boxes[blockIdx.x] = KBox{make_float3(r[0], r[1], r[2]), make_float3(r[3], r[4], r[5])};
    }
}

__global__ void __launch_bounds__(64) k_knn_super(int nbox, const KBox* boxes, KBox* supers) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int nsup = (nbox + KNN_SUPER - 1) / KNN_SUPER;
    if (s >= nsup) return;
    KBox r{make_float3(FLT_MAX, FLT_MAX, FLT_MAX), make_float3(-FLT_MAX, -FLT_MAX, -FLT_MAX)};
    for (int b = s * KNN_SUPER; b < min(nbox, (s + 1) * KNN_SUPER); b++) {
        const KBox x = boxes[b];
        r.mn = make_float3(fminf(r.mn.x, x.mn.x), fminf(r.mn.y, x.mn.y), fminf(r.mn.z, x.mn.z));
        r.mx = make_float3(fmaxf(r.mx.x, x.mx.x), fmaxf(r.mx.y, x.mx.y), fmaxf(r.mx.z, x.mx.z));
    }
    supers[s] = r;
}

// simple_knn.cu:115-126 distBoxPoint
__device__ __forceinline__ float box_dist(const KBox& b, float4 p) {
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < b.mn.x || p.x > b.mx.x) dx = fminf(fabsf(p.x - b.mn.x), fabsf(p.x - b.mx.x));
    if (p.y < b.mn.y || p.y > b.mx.y) dy = fminf(fabsf(p.y - b.mn.y), fabsf(p.y - b.mx.y));
    if (p.z < b.mn.z || p.z > b.mx.z) dz = fminf(fabsf(p.z - b.mn.z), fabsf(p.z - b.mx.z));
    return sq3(dx, dy, dz);
}

// simple_knn.cu:128-142 updateKBest<3>
__device__ __forceinline__ void update3(float4 ref, float4 p, float& b0, float& b1, float& b2) {
    float d = sq3(p.x - ref.x, p.y - ref.y, p.z - ref.z);
    float t;
    if (b0 > d) { t = b0; b0 = d; d = t; }
    if (b1 > d) { t = b1; b1 = d; d = t; }
    if (b2 > d) { b2 = d; }
}

// simple_knn.cu:144-181 boxMeanDist (one thread per sorted point)
__global__ void __launch_bounds__(256) k_knn_search(int P, const float4* spts, const uint32_t* sorted_ids,
                                                     const KBox* boxes, const KBox* supers, int nbox, float* dists) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float4 point = spts[idx];
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    for (int i = max(0, idx - 3); i <= min(P - 1, idx + 3); i++)
        if (i != idx) update3(point, spts[i], b0, b1, b2);
    const float reject = b2;
    b0 = b1 = b2 = FLT_MAX;
    const int nsup = (nbox + KNN_SUPER - 1) / KNN_SUPER;
    for (int s = 0; s < nsup; s++) {
        const float ds = box_dist(supers[s], point);
        if (ds > reject || ds > b2) continue;  // every member box would be skipped
        for (int b = s * KNN_SUPER; b < min(nbox, (s + 1) * KNN_SUPER); b++) {
            const float dist = box_dist(boxes[b], point);
            if (dist > reject || dist > b2) continue;
            const int i1 = min(P, (b + 1) * KNN_BOX);
            for (int i = b * KNN_BOX; i < i1; i++)
                if (i != idx) update3(point, spts[i], b0, b1, b2);
        }
    }
    dists[sorted_ids[idx]] = (b0 + b1 + b2) / 3.0f;
}

size_t knn_workspace_bytes(int P) {
    const size_t n = (size_t)(P > 0 ? P : 0);
    const size_t nbox = (n + KNN_BOX - 1) / KNN_BOX;
    const size_t nsup = (nbox + KNN_SUPER - 1) / KNN_SUPER;
    return 256 * 8 + 6 * 4 * 256 + 4 * 4 * n + radix_sort_temp_bytes((long long)n) + 16 * n + sizeof(KBox) * (nbox + nsup) +
           1024;
}

void launch_knn(int P, const float* pts, float* dists, void* ws, hipStream_t s) {
    if (P <= 0) return;
    auto take = [&](size_t bytes) {
        char* p = reinterpret_cast<char*>(ws);
        ws = p + ((bytes + 255) & ~(size_t)255);
        return reinterpret_cast<void*>(p);
    };
    const int nbp = 256;
    float* part = reinterpret_cast<float*>(take(6 * 4 * nbp));
    float* bounds = reinterpret_cast<float*>(take(64));
    uint32_t* codes = reinterpret_cast<uint32_t*>(take(4 * (size_t)P));
    uint32_t* ids = reinterpret_cast<uint32_t*>(take(4 * (size_t)P));
    uint32_t* codes2 = reinterpret_cast<uint32_t*>(take(4 * (size_t)P));
    uint32_t* ids2 = reinterpret_cast<uint32_t*>(take(4 * (size_t)P));
    void* sort_tmp = take(radix_sort_temp_bytes(P));
    float4* spts = reinterpret_cast<float4*>(take(16 * (size_t)P));
    const int nbox = (P + KNN_BOX - 1) / KNN_BOX;
    const int nsup = (nbox + KNN_SUPER - 1) / KNN_SUPER;
    KBox* boxes = reinterpret_cast<KBox*>(take(sizeof(KBox) * nbox));
    KBox* supers = reinterpret_cast<KBox*>(take(sizeof(KBox) * nsup));
    const int grid = (P + 255) / 256;
    hipLaunchKernelGGL(k_knn_bounds_partial, dim3(nbp), dim3(256), 0, s, P, pts, part);
    hipLaunchKernelGGL(k_knn_bounds_final, dim3(1), dim3(64), 0, s, nbp, part, bounds);
    hipLaunchKernelGGL(k_knn_morton, dim3(grid), dim3(256), 0, s, P, pts, bounds, codes, ids);
    const int flip = radix_sort_pairs(P, codes, ids, codes2, ids2, 30, sort_tmp, s);
    const uint32_t* sorted_ids = flip ? ids2 : ids;
    hipLaunchKernelGGL(k_knn_gather, dim3(grid), dim3(256), 0, s, P, pts, sorted_ids, spts);
    hipLaunchKernelGGL(k_knn_boxes, dim3(nbox), dim3(256), 0, s, P, spts, boxes);
    hipLaunchKernelGGL(k_knn_super, dim3((nsup + 63) / 64), dim3(64), 0, s, nbox, boxes, supers);
    hipLaunchKernelGGL(k_knn_search, dim3(grid), dim3(256), 0, s, P, spts, sorted_ids, boxes, supers, nbox, dists);
}

}  // namespace gsr
