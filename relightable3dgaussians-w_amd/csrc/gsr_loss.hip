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
