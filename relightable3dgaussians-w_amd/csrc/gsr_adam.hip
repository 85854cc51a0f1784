// gsr_adam.hip -- one fused Adam step over a flat parameter buffer (the data-parallel
// training step).
//
// The reference keeps one torch.optim.Adam param group per Gaussian attribute
// (gaussian_model.py:264-274, relit3DGW_model.py:149: eps 1e-15) and steps each group with
// ~6 foreach kernels (lerp, mul, addcmul, sqrt, div, add, addcdiv), i.e. the 28 B per
// element of a fused step read and written several times over.  Here every per-Gaussian
// attribute lives in one flat buffer (gsr/train.py FlatParams), its gradient in one flat
// buffer (the one RCCL all-reduce bucket), and a single launch applies the update with the
// group's learning rate from a by-value segment table:
//     g  = grad * grad_scale                      (1/views: the all-reduced sum -> mean)
//     m  = m + (1 - b1) (g - m)                   (torch lerp_, weight < 0.5 branch)
//     v  = b2 v + (1 - b2) g g
//     p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound: 16 B read + 12 B written per element, float4 streams, grid-stride.
#include "gsr_kernels.hpp"

namespace gsr {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamSegs& s, long long i) {
    int k = 0;
#pragma unroll 1
    while (k + 1 < s.n && i >= s.end[k]) k++;
    g *= s.grad_scale;
    m = m + s.one_minus_b1 * (g - m);
    v = v * s.b2 + s.one_minus_b2 * g * g;
    const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
    p = p - s.step_size[k] * (m / denom);
}

// elements [lo, hi) (lo a multiple of 4): the data-parallel step pipelines the update chunk by
// chunk behind the gradient all-reduce (gsr.dp.finish_step)
__global__ void __launch_bounds__(256) k_adam(long long lo, long long hi, AdamSegs s, float* __restrict__ p,
                                              const float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v) {
    const long long q0 = lo >> 2, q1 = hi >> 2;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long q = q0 + (long long)blockIdx.x * blockDim.x + threadIdx.x; q < q1; q += stride) {
        float4 P = reinterpret_cast<float4*>(p)[q];
        const float4 G = reinterpret_cast<const float4*>(g)[q];
        float4 Mv = reinterpret_cast<float4*>(m)[q];
        float4 V = reinterpret_cast<float4*>(v)[q];
        const long long i = 4 * q;
        adam_one(P.x, G.x, Mv.x, V.x, s, i);
        adam_one(P.y, G.y, Mv.y, V.y, s, i + 1);
        adam_one(P.z, G.z, Mv.z, V.z, s, i + 2);
        adam_one(P.w, G.w, Mv.w, V.w, s, i + 3);
        reinterpret_cast<float4*>(p)[q] = P;
        reinterpret_cast<float4*>(m)[q] = Mv;
        reinterpret_cast<float4*>(v)[q] = V;
    }
    // tail (hi % 4 elements)
    const long long t = 4 * q1 + (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < hi && blockIdx.x == 0) adam_one(p[t], g[t], m[t], v[t], s, t);
}

void launch_adam(long long lo, long long hi, const AdamSegs& s, float* p, const float* g, float* m, float* v,
                 hipStream_t st) {
    if (hi <= lo) return;
    const long long n4 = (hi - lo + 3) >> 2;
    // ~8 float4 per thread: enough bytes in flight per CU without an oversized grid
    long long blocks = (n4 + 256 * 8 - 1) / (256 * 8);
    if (blocks < 1) blocks = 1;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, lo, hi, s, p, g, m, v);
}

}  // namespace gsr
