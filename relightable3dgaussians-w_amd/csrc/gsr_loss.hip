// gsr_loss.hip -- the pointwise terms of the training loss (train.py:77-99) fused into one
// forward and one backward kernel over the view's images.
//
// The reference composes them from ~40 PyTorch kernels each way over [3,H,W] images
// (utils/loss_utils.py:27-35 l1_loss with masks, the sky-BRDF terms, the normal
// consistency term); at 1080p that is most of the training iteration outside the
// rasterizer.  Here one thread handles one pixel (all channels):
//   forward   per workgroup, fixed-order partial sums of
//               [0] sum |img o - gt o|                 (reconstruction L1, occluder mask o)
//               [1] #(o == 1)                           (its denominator, per channel element)
//               [2] sum |diff ns| + |spec ns|          (sky-BRDF L1s, ns = 1 - sky)
//               [3] #(ns == 1)
//               [4] sum_pixels sum_c (n_c o s)(nr_c o s)  (normal consistency dot)
//             the host wrapper adds the partials and forms the loss (gsr/train.py);
//   backward  every input gradient in one pass from the five scalar coefficients the
//             wrapper computes on the device (no host synchronisation):
//               d img  = k0 sign(img o - gt o) o
//               d diff = k2 sign(diff ns) ns,  d spec = k2 sign(spec ns) ns
//               d n_c  = k4 nr_c (o s)^2,      d nr_c = k4 n_c (o s)^2
//             (torch's abs backward: sign(0) = 0).
// HBM-bound: 6 three-channel images + 2 masks in; 5 gradients out.
//   objective one workgroup turns the pointwise partials and the SSIM partials into the
//             view's loss and the backward's four coefficients on the device (the ~25 scalar
//             PyTorch ops of the wrapper, one launch).
#include "gsr_kernels.hpp"

namespace gsr {

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ void __launch_bounds__(256) k_view_loss_fwd(int npix, const float* __restrict__ img,
                                                       const float* __restrict__ gt, const float* __restrict__ diff,
                                                       const float* __restrict__ spec, const float* __restrict__ nrm,
                                                       const float* __restrict__ nref, const float* __restrict__ sky,
                                                       const float* __restrict__ occ, float* __restrict__ partials) {
    __shared__ float red[5][4];
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = blockIdx.x * 256 + threadIdx.x; p < npix; p += gridDim.x * 256) {
        const float o = occ[p], s = sky[p], ns = 1.f - s, os = o * s;
        const bool o1 = o == 1.f, ns1 = ns == 1.f;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const size_t i = (size_t)c * npix + p;
            acc[0] += fabsf(img[i] * o - gt[i] * o);
            acc[2] += fabsf(diff[i] * ns) + fabsf(spec[i] * ns);
            acc[4] += (nrm[i] * os) * (nref[i] * os);
        }
        acc[1] += o1 ? 3.f : 0.f;
        acc[3] += ns1 ? 3.f : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 5; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 64);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x < 5)
        partials[(size_t)blockIdx.x * 5 + threadIdx.x] =
            (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

__global__ void __launch_bounds__(256) k_view_loss_bwd(int npix, const float* __restrict__ img,
                                                       const float* __restrict__ gt, const float* __restrict__ diff,
                                                       const float* __restrict__ spec, const float* __restrict__ nrm,
                                                       const float* __restrict__ nref, const float* __restrict__ sky,
                                                       const float* __restrict__ occ, const float* __restrict__ coef,
                                                       float* __restrict__ d_img, float* __restrict__ d_diff,
                                                       float* __restrict__ d_spec, float* __restrict__ d_nrm,
                                                       float* __restrict__ d_nref) {
    const float k0 = coef[0], k2 = coef[1], k4 = coef[2];
    for (int p = blockIdx.x * 256 + threadIdx.x; p < npix; p += gridDim.x * 256) {
        const float o = occ[p], s = sky[p], ns = 1.f - s, os = o * s, os2 = os * os;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const size_t i = (size_t)c * npix + p;
            if (d_img) d_img[i] = k0 * sgnf(img[i] * o - gt[i] * o) * o;
            if (d_diff) d_diff[i] = k2 * sgnf(diff[i] * ns) * ns;
            if (d_spec) d_spec[i] = k2 * sgnf(spec[i] * ns) * ns;
            const float a = nrm[i], b = nref[i];
            if (d_nrm) d_nrm[i] = k4 * b * os2;
            if (d_nref) d_nref[i] = k4 * a * os2;
        }
    }
}

// loss = pw + l_dssim (1 - ssim) as gsr/train.py composes it in PyTorch:
//   S = sum of the pointwise partials (double), k0 = (1 - l_dssim) / S1 (0 if S1 == 0),
//   k2 = l_sky / S3 (0 if S3 == 0), pw = (float)(k0 S0 + k2 S2 + l_normal (1 - S4 / npix));
//   value = (float) sum of the SSIM map partials, N = the mask count (double),
//   ssim = N > 0 ? (float)(value / N) : 1, loss = pw + (float)l_dssim * (1 - ssim) in float.
// coef = (k0, k2, -l_normal / npix, -(float)l_dssim / N (0 if N == 0)): the gradient
// coefficients of the pointwise terms and of the SSIM map sum, before the upstream gradient.
__global__ void __launch_bounds__(256) k_view_objective(int nvl, const float* __restrict__ vl, int nss,
                                                        const float* __restrict__ ss, int npix, double l_dssim,
                                                        double l_sky, double l_normal, float* __restrict__ loss,
                                                        float* __restrict__ coef) {
#pragma clang fp contract(off)
    __shared__ double red[7][4];
    double a[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // each thread's partials in the plain strided order, their loads issued 8 iterations at a
    // time (one workgroup: the latency of one dependent load per iteration was the kernel)
#pragma unroll 8
    for (int i = threadIdx.x; i < nvl; i += 256) {
#pragma unroll
        for (int k = 0; k < 5; k++) a[k] += (double)vl[(size_t)i * 5 + k];
    }
#pragma unroll 8
    for (int i = threadIdx.x; i < nss; i += 256) {
        a[5] += (double)ss[(size_t)i * 2];
        a[6] += (double)ss[(size_t)i * 2 + 1];
    }
#pragma unroll
    for (int k = 0; k < 7; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = a[k];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double S[7];
#pragma unroll
    for (int k = 0; k < 7; k++) S[k] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    const double k0 = S[1] > 0.0 ? (1.0 - l_dssim) / S[1] : 0.0;
    const double k2 = S[3] > 0.0 ? l_sky / S[3] : 0.0;
    const float pw = (float)(k0 * S[0] + k2 * S[2] + l_normal * (1.0 - S[4] / (double)npix));
    const float value = (float)S[5];
    const float ssim = S[6] > 0.0 ? (float)((double)value / S[6]) : 1.f;
    const float ld = (float)l_dssim;
    loss[0] = pw + ld * (1.f - ssim);
    coef[0] = (float)k0;
    coef[1] = (float)k2;
    coef[2] = (float)(0.0 - l_normal / (double)npix);
    coef[3] = S[6] > 0.0 ? (float)(-(double)ld / S[6]) : 0.f;
}

void launch_view_objective(int nvl, const float* vl, int nss, const float* ss, int npix, double l_dssim, double l_sky,
                           double l_normal, float* loss, float* coef, hipStream_t s) {
    hipLaunchKernelGGL(k_view_objective, dim3(1), dim3(256), 0, s, nvl, vl, nss, ss, npix, l_dssim, l_sky, l_normal,
                       loss, coef);
}

int view_loss_blocks(int npix) {
    const int b = (npix + 256 * 4 - 1) / (256 * 4);
    return b < 1 ? 1 : (b > 4096 ? 4096 : b);
}

void launch_view_loss_fwd(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, float* partials,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_view_loss_fwd, dim3(view_loss_blocks(npix)), dim3(256), 0, s, npix, img, gt, diff, spec, nrm,
                       nref, sky, occ, partials);
}

void launch_view_loss_bwd(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, const float* coef,
                          float* d_img, float* d_diff, float* d_spec, float* d_nrm, float* d_nref, hipStream_t s) {
    hipLaunchKernelGGL(k_view_loss_bwd, dim3(view_loss_blocks(npix)), dim3(256), 0, s, npix, img, gt, diff, spec, nrm,
                       nref, sky, occ, coef, d_img, d_diff, d_spec, d_nrm, d_nref);
}

}  // namespace gsr
