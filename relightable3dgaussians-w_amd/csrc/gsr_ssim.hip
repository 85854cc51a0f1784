// gsr_ssim.hip -- the training loss's SSIM (utils/loss_utils.py:53-96) fused into one
// forward and one backward kernel.
//
// The reference computes SSIM with five depthwise 11x11 conv2d calls (mu1, mu2, E[x^2],
// E[y^2], E[xy]) plus ~15 elementwise kernels, and autograd replays the convolutions
// backward: at 1080p that is the largest cost of a training iteration (8 MIOpen
// convolutions per view).  Here:
//   forward   one 32x32 output tile per workgroup, both images staged with a 5-pixel zero
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

// One 32x32 output tile per workgroup.  The window passes slide in registers: a horizontal
// task produces 4 consecutive columns of one staged row from 14 loaded pixels, a vertical
// task 4 consecutive rows of one column from 14 loaded row values (about a third of the LDS
// reads of one output per task).  The summation order per output is the plain 11-tap order.
constexpr int SS_TW = 32, SS_TH = 32, SS_R = 5, SS_K = 2 * SS_R + 1, SS_HX = 4, SS_VY = 4;
constexpr int SS_LW = SS_TW + 2 * SS_R, SS_LH = SS_TH + 2 * SS_R;  // 42 x 42 staged pixels
constexpr int SS_HTASKS = SS_LH * (SS_TW / SS_HX);                 // 336 horizontal tasks
static_assert((SS_TW / 1) * (SS_TH / SS_VY) == 256, "one vertical task per thread");

__device__ __forceinline__ float ld_zero(const float* p, int x, int y, int W, int H) {
    return (x >= 0 && x < W && y >= 0 && y < H) ? p[(size_t)y * W + x] : 0.f;
}

// A workgroup can walk a strip of SS_CH 32-row chunks down one 32-column band: the window's
// horizontal results (hm) of the 10 halo rows carry over from one chunk to the next (a
// staged row is loaded and filtered horizontally once, not 1.31 times), and the next chunk's
// 32 new rows load into registers while the current chunk's vertical pass runs.  Measured at
// 3x1080x1920 (tools/bench_ssim.py): one chunk per workgroup 77.7 / 61.5 us (forward /
// backward), four chunks 78.0 / 66.6 us, four without the prefetch 79.6 / 64.6 us; the
// single-tile kernel that staged its window with interleaved loads and LDS stores took 89.3 /
// 64.6 us.  The gain is the window's loads issued all at once into registers: one chunk per
// workgroup (SS_CH; the loops below serve any strip length, with the next chunk's rows loaded
// during the vertical pass).  Per output the arithmetic and its order are the same either way.
constexpr int SS_CH = 1;
constexpr int SS_NEW = SS_TH * SS_LW;                            // raw values of one chunk's new rows
constexpr int SS_PF = (SS_NEW + 255) / 256;                      // per thread

// the raw values of window rows [r0, SS_LH) of the chunk whose first window row is image row y0
template <int NIMG>
__device__ __forceinline__ void ss_fetch(const float* const (&src)[NIMG], int x0, int y0, int r0, int W, int H,
                                         float (&v)[NIMG][SS_PF]) {
#pragma unroll
    for (int i = 0; i < SS_PF; i++) {
        const int e = (int)threadIdx.x + 256 * i;
        const int ly = r0 + e / SS_LW, lx = e % SS_LW;
        const bool ok = e < (SS_LH - r0) * SS_LW;
#pragma unroll
        for (int m = 0; m < NIMG; m++) v[m][i] = ok ? ld_zero(src[m], x0 + lx, y0 + ly, W, H) : 0.f;
    }
}
template <int NIMG>
__device__ __forceinline__ void ss_stage(float (*dst)[SS_LH][SS_LW], int r0, const float (&v)[NIMG][SS_PF]) {
#pragma unroll
    for (int i = 0; i < SS_PF; i++) {
        const int e = (int)threadIdx.x + 256 * i;
        if (e < (SS_LH - r0) * SS_LW) {
            const int ly = r0 + e / SS_LW, lx = e % SS_LW;
#pragma unroll
            for (int m = 0; m < NIMG; m++) dst[m][ly][lx] = v[m][i];
        }
    }
}

__global__ void __launch_bounds__(256) k_ssim_fwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ mask,
                                                  long long mask_cstride, SsimWindow win, float C1, float C2,
                                                  float* __restrict__ block_sums, float* __restrict__ dmaps) {
    __shared__ float sr[2][SS_LH][SS_LW];
    __shared__ float hm[5][SS_LH][SS_TW + 1];
    __shared__ float red[8];
    const int c = blockIdx.z;
    const size_t plane = (size_t)H * W;
    const float* const src[2] = {img1 + c * plane, img2 + c * plane};
    const int x0 = blockIdx.x * SS_TW - SS_R;
    const float* mk = mask ? mask + c * mask_cstride : nullptr;
    float acc = 0.f, cnt = 0.f;  // sum(map * mask) and #(mask == 1) over the strip
    const int ty_first = blockIdx.y * SS_CH * SS_TH;
    float pf[2][SS_PF];
    // the first chunk's whole window (its 10 leading rows first, the 32 new ones prefetched)
    {
        float head[2][SS_PF];
        ss_fetch<2>(src, x0, ty_first - SS_R, 0, W, H, head);  // rows 0..41 needs two rounds:
        ss_stage<2>(sr, 0, head);                             // rows 0 .. SS_PF*256/SS_LW
    }
    ss_fetch<2>(src, x0, ty_first - SS_R, SS_LH - SS_TH, W, H, pf);
#pragma unroll 1
    for (int j = 0; j < SS_CH; j++) {
        const int ty = ty_first + j * SS_TH;
        if (ty >= H) break;  // block-uniform
        const int r0 = j == 0 ? 0 : SS_LH - SS_TH;  // window rows [r0, SS_LH) are new
        ss_stage<2>(sr, SS_LH - SS_TH, pf);
        __syncthreads();
        // horizontal pass over the new window rows: the five moments over 11 columns
        for (int t = threadIdx.x; t < (SS_LH - r0) * (SS_TW / SS_HX); t += 256) {
            const int ly = r0 + t / (SS_TW / SS_HX), lx = (t % (SS_TW / SS_HX)) * SS_HX;
            float u[SS_K + SS_HX - 1], v[SS_K + SS_HX - 1];
#pragma unroll
            for (int k = 0; k < SS_K + SS_HX - 1; k++) {
                u[k] = sr[0][ly][lx + k];
                v[k] = sr[1][ly][lx + k];
            }
#pragma unroll
            for (int o = 0; o < SS_HX; o++) {
                float m1 = 0.f, m2 = 0.f, m11 = 0.f, m22 = 0.f, m12 = 0.f;
#pragma unroll
                for (int k = 0; k < SS_K; k++) {
                    const float uu = u[o + k], vv = v[o + k], g = win.w[k];
                    m1 += g * uu;
                    m2 += g * vv;
                    m11 += g * (uu * uu);
                    m22 += g * (vv * vv);
                    m12 += g * (uu * vv);
                }
                hm[0][ly][lx + o] = m1;
                hm[1][ly][lx + o] = m2;
                hm[2][ly][lx + o] = m11;
                hm[3][ly][lx + o] = m22;
                hm[4][ly][lx + o] = m12;
            }
        }
        __syncthreads();
        // the next chunk's new rows load while this chunk's vertical pass runs
        if (j + 1 < SS_CH && ty + SS_TH < H)
            ss_fetch<2>(src, x0, ty + SS_TH - SS_R, SS_LH - SS_TH, W, H, pf);
        {
            const int tx = threadIdx.x % SS_TW, ty0 = (threadIdx.x / SS_TW) * SS_VY;
            float col[5][SS_K + SS_VY - 1];
#pragma unroll
            for (int k = 0; k < SS_K + SS_VY - 1; k++) {
#pragma unroll
                for (int q = 0; q < 5; q++) col[q][k] = hm[q][ty0 + k][tx];
            }
            const int x = blockIdx.x * SS_TW + tx;
#pragma unroll
            for (int o = 0; o < SS_VY; o++) {
                const int y = ty + ty0 + o;
                if (x >= W || y >= H) continue;
                float mu1 = 0.f, mu2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
                for (int k = 0; k < SS_K; k++) {
                    const float g = win.w[k];
                    mu1 += g * col[0][o + k];
                    mu2 += g * col[1][o + k];
                    e11 += g * col[2][o + k];
                    e22 += g * col[3][o + k];
                    e12 += g * col[4][o + k];
                }
                const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
                const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu12;
                const float A = 2.f * mu12 + C1, B = 2.f * s12 + C2;
                const float Cc = mu1_sq + mu2_sq + C1, D = s11 + s22 + C2;
                // v_rcp_f32 (1 ulp) instead of four IEEE divisions: the loss value and its
                // gradient stay within the tests' 1e-5 of the conv2d formulation
                const float rC = __builtin_amdgcn_rcpf(Cc), rD = __builtin_amdgcn_rcpf(D);
                const float inv = rC * rD;
                const float map = (A * B) * inv;
                const size_t pix = (size_t)y * W + x;
                const float m = mk ? mk[pix] : 1.f;
                acc += map * m;
                cnt += m == 1.f ? 1.f : 0.f;
                if (dmaps) {
                    // d map / d mu1 (through A, B, Cc, D), d map / d E[x^2], d map / d E[xy]
                    const float d_mu1 = 2.f * mu2 * (B - A) * inv - 2.f * mu1 * map * (rC - rD);
                    const float d_xx = -map * rD;
                    const float d_xy = 2.f * A * inv;
                    const size_t oo = c * plane + pix;  // maps are [3][C][H][W]
                    dmaps[oo] = m * d_mu1;
                    dmaps[(size_t)gridDim.z * plane + oo] = m * d_xx;
                    dmaps[(size_t)2 * gridDim.z * plane + oo] = m * d_xy;
                }
            }
        }
        __syncthreads();
        // the window's last 10 rows are the next window's first 10
        for (int i = threadIdx.x; i < 5 * (SS_LH - SS_TH) * (SS_TW + 1); i += 256) {
            const int q = i / ((SS_LH - SS_TH) * (SS_TW + 1)), r = i % ((SS_LH - SS_TH) * (SS_TW + 1));
            const int ly = r / (SS_TW + 1), lx = r % (SS_TW + 1);
            hm[q][ly][lx] = hm[q][SS_TH + ly][lx];
        }
    }
    // fixed-order workgroup sums (deterministic); the count is exact (< 2^24 per strip)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = acc;
        red[4 + (threadIdx.x >> 6)] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const size_t bid = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        block_sums[2 * bid] = (red[0] + red[1]) + (red[2] + red[3]);
        block_sums[2 * bid + 1] = (red[4] + red[5]) + (red[6] + red[7]);
    }
}

__global__ void __launch_bounds__(256) k_ssim_bwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ dmaps,
                                                  const float* __restrict__ gscale, SsimWindow win,
                                                  float* __restrict__ dimg1, int accumulate,
                                                  const float* __restrict__ occ, const float* __restrict__ l1k) {
    __shared__ float sr[3][SS_LH][SS_LW];
    __shared__ float hm[3][SS_LH][SS_TW + 1];
    const int c = blockIdx.z;
    const size_t plane = (size_t)H * W;
    const size_t cs = (size_t)gridDim.z * plane;
    const float* const src[3] = {dmaps + c * plane, dmaps + cs + c * plane, dmaps + 2 * cs + c * plane};
    const int x0 = blockIdx.x * SS_TW - SS_R;
    const float sc = *gscale;
    const float k0 = l1k ? *l1k : 0.f;
    const int ty_first = blockIdx.y * SS_CH * SS_TH;
    float pf[3][SS_PF];
    {
        float head[3][SS_PF];
        ss_fetch<3>(src, x0, ty_first - SS_R, 0, W, H, head);
        ss_stage<3>(sr, 0, head);
    }
    ss_fetch<3>(src, x0, ty_first - SS_R, SS_LH - SS_TH, W, H, pf);
#pragma unroll 1
    for (int j = 0; j < SS_CH; j++) {
        const int ty = ty_first + j * SS_TH;
        if (ty >= H) break;  // block-uniform
        const int r0 = j == 0 ? 0 : SS_LH - SS_TH;
        ss_stage<3>(sr, SS_LH - SS_TH, pf);
        __syncthreads();
        for (int t = threadIdx.x; t < (SS_LH - r0) * (SS_TW / SS_HX); t += 256) {
            const int ly = r0 + t / (SS_TW / SS_HX), lx = (t % (SS_TW / SS_HX)) * SS_HX;
            float r[3][SS_K + SS_HX - 1];
#pragma unroll
            for (int k = 0; k < SS_K + SS_HX - 1; k++) {
#pragma unroll
                for (int q = 0; q < 3; q++) r[q][k] = sr[q][ly][lx + k];
            }
#pragma unroll
            for (int o = 0; o < SS_HX; o++) {
                float q0 = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll
                for (int k = 0; k < SS_K; k++) {
                    const float g = win.w[k];
                    q0 += g * r[0][o + k];
                    q1 += g * r[1][o + k];
                    q2 += g * r[2][o + k];
                }
                hm[0][ly][lx + o] = q0;
                hm[1][ly][lx + o] = q1;
                hm[2][ly][lx + o] = q2;
            }
        }
        __syncthreads();
        if (j + 1 < SS_CH && ty + SS_TH < H)
            ss_fetch<3>(src, x0, ty + SS_TH - SS_R, SS_LH - SS_TH, W, H, pf);
        {
            const int tx = threadIdx.x % SS_TW, ty0 = (threadIdx.x / SS_TW) * SS_VY;
            float col[3][SS_K + SS_VY - 1];
#pragma unroll
            for (int k = 0; k < SS_K + SS_VY - 1; k++) {
#pragma unroll
                for (int q = 0; q < 3; q++) col[q][k] = hm[q][ty0 + k][tx];
            }
            const int x = blockIdx.x * SS_TW + tx;
#pragma unroll
            for (int o = 0; o < SS_VY; o++) {
                const int y = ty + ty0 + o;
                if (x >= W || y >= H) continue;
                float q0 = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll
                for (int k = 0; k < SS_K; k++) {
                    const float g = win.w[k];
                    q0 += g * col[0][o + k];
                    q1 += g * col[1][o + k];
                    q2 += g * col[2][o + k];
                }
                const size_t oo = c * plane + (size_t)y * W + x;
                const float x1 = img1[oo], x2 = img2[oo];
                const float d = sc * (q0 + 2.f * x1 * q1 + x2 * q2);
                if (l1k) {  // the L1 term's gradient made here (gsr_view_loss_backward's, same order)
                    const float o = occ[(size_t)y * W + x];
                    const float a = x1 * o - x2 * o;
                    const float l1 = __fmul_rn(k0 * (a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f)), o);
                    dimg1[oo] = __fadd_rn(l1, d);  // no contraction: the unfused path's two roundings
                } else {
                    dimg1[oo] = accumulate ? dimg1[oo] + d : d;  // accumulate: onto the pointwise terms' gradient
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 3 * (SS_LH - SS_TH) * (SS_TW + 1); i += 256) {
            const int q = i / ((SS_LH - SS_TH) * (SS_TW + 1)), r = i % ((SS_LH - SS_TH) * (SS_TW + 1));
            const int ly = r / (SS_TW + 1), lx = r % (SS_TW + 1);
            hm[q][ly][lx] = hm[q][SS_TH + ly][lx];
        }
    }
}

dim3 ssim_grid(int C, int H, int W) {
    const int chunks = (H + SS_TH - 1) / SS_TH;
    return dim3((W + SS_TW - 1) / SS_TW, (chunks + SS_CH - 1) / SS_CH, C);
}

void launch_ssim_fwd(int C, int H, int W, const float* img1, const float* img2, const float* mask,
                     long long mask_cstride, const SsimWindow& win, float C1, float C2, float* block_sums,
                     float* dmaps, hipStream_t s) {
    hipLaunchKernelGGL(k_ssim_fwd, ssim_grid(C, H, W), dim3(256), 0, s, H, W, img1, img2, mask, mask_cstride, win, C1,
                       C2, block_sums, dmaps);
}

void launch_ssim_bwd(int C, int H, int W, const float* img1, const float* img2, const float* dmaps,
                     const float* gscale, const SsimWindow& win, float* dimg1, int accumulate, hipStream_t s, const float* occ,
                     const float* l1k) {
    hipLaunchKernelGGL(k_ssim_bwd, ssim_grid(C, H, W), dim3(256), 0, s, H, W, img1, img2, dmaps, gscale, win, dimg1,
                       accumulate, occ, l1k);
}

}  // namespace gsr
