// gsr_ssim.hip -- the training loss's SSIM (utils/loss_utils.py:53-96) fused into one
// forward and one backward kernel.
//
// The reference computes SSIM with five depthwise 11x11 conv2d calls (mu1, mu2, E[x^2],
// E[y^2], E[xy]) plus ~15 elementwise kernels, and autograd replays the convolutions
// backward: at 1080p that is the largest cost of a training iteration (8 MIOpen
// convolutions per view).  Here:
//   forward   one 32x16 output tile per workgroup, both images staged with a 5-pixel zero
//             halo in LDS, the separable Gaussian window (11 taps, sigma 1.5, the
//             reference's normalised fp32 weights) applied as a horizontal then a
//             vertical pass over the five moments; per pixel the SSIM value is
//             multiplied by the mask and summed per workgroup (a fixed-order partial,
//             summed by the host wrapper: deterministic), and the three derivatives of
//             the SSIM value w.r.t. the moments it reads (mu1, E[x^2], E[xy]; the
//             dependence through sigma is folded in) are written, mask-weighted, for the
//             backward;
//   backward  dL/dx(p) = s * sum_q w(q - p) [d_mu1(q) + 2 x(p) d_xx(q) + y(p) d_xy(q)]:
//             the same separable window over the three derivative maps (zero outside the
//             image, as conv2d's zero padding), combined per pixel, times the scalar
//             s = dL/dloss / #mask (a device pointer: no host synchronisation).
// Both are image-space stencils over C*H*W pixels: HBM-bound (forward reads 2 images,
// writes 3 maps; backward reads 3 maps + 2 images, writes 1).
#include "gsr_kernels.hpp"

namespace gsr {

constexpr int SS_TW = 32, SS_TH = 16, SS_R = 5, SS_K = 2 * SS_R + 1;
constexpr int SS_LW = SS_TW + 2 * SS_R, SS_LH = SS_TH + 2 * SS_R;  // 42 x 26 staged pixels

__device__ __forceinline__ float ld_zero(const float* p, int x, int y, int W, int H) {
    return (x >= 0 && x < W && y >= 0 && y < H) ? p[(size_t)y * W + x] : 0.f;
}

__global__ void __launch_bounds__(256) k_ssim_fwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ mask,
                                                  long long mask_cstride, SsimWindow win, float C1, float C2,
                                                  float* __restrict__ block_sums, float* __restrict__ dmaps) {
    __shared__ float s1[SS_LH][SS_LW], s2[SS_LH][SS_LW];
    __shared__ float hm[5][SS_LH][SS_TW + 1];
    __shared__ float red[4];
    const int c = blockIdx.z;
    const size_t plane = (size_t)H * W;
    const float* a = img1 + c * plane;
    const float* b = img2 + c * plane;
    const int x0 = blockIdx.x * SS_TW - SS_R, y0 = blockIdx.y * SS_TH - SS_R;
    for (int i = threadIdx.x; i < SS_LH * SS_LW; i += 256) {
        const int ly = i / SS_LW, lx = i - ly * SS_LW;
        s1[ly][lx] = ld_zero(a, x0 + lx, y0 + ly, W, H);
        s2[ly][lx] = ld_zero(b, x0 + lx, y0 + ly, W, H);
    }
    __syncthreads();
    // horizontal pass: the five moments over 11 columns, for every staged row
    for (int i = threadIdx.x; i < SS_LH * SS_TW; i += 256) {
        const int ly = i / SS_TW, lx = i - ly * SS_TW;
        float m1 = 0.f, m2 = 0.f, m11 = 0.f, m22 = 0.f, m12 = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float u = s1[ly][lx + k], v = s2[ly][lx + k], g = win.w[k];
            m1 += g * u;
            m2 += g * v;
            m11 += g * (u * u);
            m22 += g * (v * v);
            m12 += g * (u * v);
        }
        hm[0][ly][lx] = m1;
        hm[1][ly][lx] = m2;
        hm[2][ly][lx] = m11;
        hm[3][ly][lx] = m22;
        hm[4][ly][lx] = m12;
    }
    __syncthreads();
    float acc = 0.f;
    const float* mk = mask ? mask + c * mask_cstride : nullptr;
    for (int i = threadIdx.x; i < SS_TH * SS_TW; i += 256) {
        const int ty = i / SS_TW, tx = i - ty * SS_TW;
        const int x = blockIdx.x * SS_TW + tx, y = blockIdx.y * SS_TH + ty;
        if (x >= W || y >= H) continue;
        float mu1 = 0.f, mu2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float g = win.w[k];
            mu1 += g * hm[0][ty + k][tx];
            mu2 += g * hm[1][ty + k][tx];
            e11 += g * hm[2][ty + k][tx];
            e22 += g * hm[3][ty + k][tx];
            e12 += g * hm[4][ty + k][tx];
        }
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
        const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu12;
        const float A = 2.f * mu12 + C1, B = 2.f * s12 + C2;
        const float Cc = mu1_sq + mu2_sq + C1, D = s11 + s22 + C2;
        const float inv = 1.f / (Cc * D);
        const float map = (A * B) * inv;
        const size_t pix = (size_t)y * W + x;
        const float m = mk ? mk[pix] : 1.f;
        acc += map * m;
        if (dmaps) {
            // d map / d mu1 (through A, B, Cc, D), d map / d E[x^2], d map / d E[xy]
            const float d_mu1 = 2.f * mu2 * (B - A) * inv - 2.f * mu1 * map * (1.f / Cc - 1.f / D);
            const float d_xx = -map / D;
            const float d_xy = 2.f * A * inv;
            const size_t o = c * plane + pix;  // maps are [3][C][H][W]
            dmaps[o] = m * d_mu1;
            dmaps[(size_t)gridDim.z * plane + o] = m * d_xx;
            dmaps[(size_t)2 * gridDim.z * plane + o] = m * d_xy;
        }
    }
    // fixed-order workgroup sum (deterministic)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0)
        block_sums[((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] =
            (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) k_ssim_bwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ dmaps,
                                                  const float* __restrict__ gscale, SsimWindow win,
                                                  float* __restrict__ dimg1) {
    __shared__ float s[3][SS_LH][SS_LW];
    __shared__ float hm[3][SS_LH][SS_TW + 1];
    const int c = blockIdx.z;
    const size_t plane = (size_t)H * W;
    const size_t cs = (size_t)gridDim.z * plane;
    const int x0 = blockIdx.x * SS_TW - SS_R, y0 = blockIdx.y * SS_TH - SS_R;
    for (int i = threadIdx.x; i < SS_LH * SS_LW; i += 256) {
        const int ly = i / SS_LW, lx = i - ly * SS_LW;
#pragma unroll
        for (int k = 0; k < 3; k++) s[k][ly][lx] = ld_zero(dmaps + k * cs + c * plane, x0 + lx, y0 + ly, W, H);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SS_LH * SS_TW; i += 256) {
        const int ly = i / SS_TW, lx = i - ly * SS_TW;
        float q0 = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float g = win.w[k];
            q0 += g * s[0][ly][lx + k];
            q1 += g * s[1][ly][lx + k];
            q2 += g * s[2][ly][lx + k];
        }
        hm[0][ly][lx] = q0;
        hm[1][ly][lx] = q1;
        hm[2][ly][lx] = q2;
    }
    __syncthreads();
    const float sc = *gscale;
    for (int i = threadIdx.x; i < SS_TH * SS_TW; i += 256) {
        const int ty = i / SS_TW, tx = i - ty * SS_TW;
        const int x = blockIdx.x * SS_TW + tx, y = blockIdx.y * SS_TH + ty;
        if (x >= W || y >= H) continue;
        float q0 = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float g = win.w[k];
            q0 += g * hm[0][ty + k][tx];
            q1 += g * hm[1][ty + k][tx];
            q2 += g * hm[2][ty + k][tx];
        }
        const size_t o = c * plane + (size_t)y * W + x;
        dimg1[o] = sc * (q0 + 2.f * img1[o] * q1 + img2[o] * q2);
    }
}

dim3 ssim_grid(int C, int H, int W) { return dim3((W + SS_TW - 1) / SS_TW, (H + SS_TH - 1) / SS_TH, C); }

void launch_ssim_fwd(int C, int H, int W, const float* img1, const float* img2, const float* mask,
                     long long mask_cstride, const SsimWindow& win, float C1, float C2, float* block_sums,
                     float* dmaps, hipStream_t s) {
    hipLaunchKernelGGL(k_ssim_fwd, ssim_grid(C, H, W), dim3(256), 0, s, H, W, img1, img2, mask, mask_cstride, win, C1,
                       C2, block_sums, dmaps);
}

void launch_ssim_bwd(int C, int H, int W, const float* img1, const float* img2, const float* dmaps,
                     const float* gscale, const SsimWindow& win, float* dimg1, hipStream_t s) {
    hipLaunchKernelGGL(k_ssim_bwd, ssim_grid(C, H, W), dim3(256), 0, s, H, W, img1, img2, dmaps, gscale, win, dimg1);
}

}  // namespace gsr
