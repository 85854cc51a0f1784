/*
 * gsr.h -- C ABI of libgsr.so, the MI355X-native (gfx950) differentiable Gaussian
 * rasterizer and relighting shade.  Plain pointers and sizes only; every float / int
 * pointer is DEVICE memory unless stated; `stream` is a hipStream_t (NULL = default).
 *
 * Each entry point replaces one reference interface (paths relative to the reference
 * checkout, submodules/diff-gaussian-rasterization/ abbreviated "dgr/"):
 *
 *   gsr_forward        dgr/cuda_rasterizer/rasterizer.h:33-55  Rasterizer::forward
 *                      (driven from dgr/rasterize_points.cu:35-113 RasterizeGaussiansCUDA)
 *   gsr_backward       dgr/cuda_rasterizer/rasterizer.h:57-82  Rasterizer::backward
 *                      (driven from dgr/rasterize_points.cu:115-192)
 *   gsr_mark_visible   dgr/cuda_rasterizer/rasterizer.h:23-29  Rasterizer::markVisible
 *                      (dgr/rasterize_points.cu:194-213)
 *   gsr_shade_forward  scene/NVDIFFREC/light.py:131-193 EnvironmentLight.shade (forward)
 *   gsr_shade_backward autograd backward of the same (PyTorch + nvdiffrast in the reference)
 *   gsr_forward_reuse  colours-only re-render over an earlier call's geometry (the 6-10
 *                      same-geometry calls of gaussian_renderer/__init__.py:160-264)
 *   gsr_knn_mean_dist  submodules/simple-knn/spatial.cu:14-26 distCUDA2
 *   gsr_relit_features / gsr_relit_features_backward
 *                      render()'s per-Gaussian colour preparation (normals, shade, sky
 *                      colour, depth; gaussian_renderer/__init__.py:120-200) fused into
 *                      the composite's feature rows
 *   gsr_adam_step      torch.optim.Adam.step over the per-Gaussian param groups
 *   gsr_adam_step_range  the same over one element range (the pipelined data-parallel step)
 *                      (train.py:191, relit3DGW_model.py:149) as one fused launch over a
 *                      flat parameter buffer (the data-parallel training step)
 *   gsr_view_loss_forward / gsr_view_loss_backward
 *                      the pointwise loss terms of train.py:77-99 (masked L1, sky-BRDF,
 *                      normal consistency) fused into one kernel each way
 *   gsr_view_regularisers_forward / _backward, gsr_densify_stats
 *                      the per-Gaussian view regularisers (utils/loss_utils.py:140-148,
 *                      210-220) and densification statistics (gaussian_model.py:627-629)
 *                      of V views in one pass each
 *   gsr_sh_basis       utils/sh_utils.py:81-151 eval_sh's basis at directions (envlight
 *                      regulariser, train.py:96)
 *   gsr_sky_xyz_forward / _backward
 *                      the sky Gaussians' shell positions (gaussian_model.py:95-103,159-169)
 *   gsr_view_objective the view's loss and backward coefficients from both partials
 *   gsr_activations_forward / _backward
 *                      the model's activations (gaussian_model.py:69-103) in one pass each
 *                      way, the backward into the optimizer's flat gradient
 *   gsr_ssim_forward / gsr_ssim_backward
 *                      the training loss's SSIM (utils/loss_utils.py:53-96, train.py:78)
 *                      as one fused stencil kernel each way
 *   gsr_relit_epilogue / gsr_relit_epilogue_backward
 *                      render()'s image-space tail: normal remap + sky mask and normal_ref
 *                      from the depth image (gaussian_renderer/__init__.py:226-276,
 *                      utils/graphics_utils.py:141-169)
 *   gsr_texture2d_forward / gsr_texture2d_backward
 *                      nvdiffrast's dr.texture (2D, linear/nearest, wrap/clamp/zero) as
 *                      the reference calls it (scene/NVDIFFREC/light.py:170, util.py:117);
 *                      backs the drop-in `nvdiffrast.torch.texture`
 *   gsr_forward_channels / gsr_backward_channels
 *                      the 6-10 same-geometry rasterizer calls of one render()
 *                      (gaussian_renderer/__init__.py:160-264) as ONE composite of all
 *                      their colour channels (multi-channel alternative)
 *
 * Error convention: every function returns 0 on success and a negative GSR_E* code on
 * failure; gsr_last_error() returns a thread-local message.  The reference's conditions
 * map as follows: AT_ERROR on a bad means3D shape is raised by the host wrapper; a
 * prefiltered point that fails the near test (the reference's device printf + __trap,
 * auxiliary.h:156-160) returns GSR_E_PREFILTERED instead of killing the context.
 */
#ifndef GSR_H_INCLUDED
#define GSR_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_OK 0
#define GSR_E_HIP (-1)
#define GSR_E_ARG (-2)
#define GSR_E_PREFILTERED (-3)
#define GSR_E_ALLOC (-4)
#define GSR_E_OVERFLOW (-5)
#define GSR_E_DEVICE_CHECK (-6) /* a GSR_DEBUG invariant or the deterministic gather failed */

/* Buffer growth callback: must return a device pointer to at least `nbytes` bytes that
 * stays valid until the matching backward call (the reference's resizeFunctional,
 * dgr/rasterize_points.cu:27-33, which resizes a torch uint8 tensor). */
typedef void* (*gsr_resize_fn)(void* ctx, size_t nbytes);

/* Forward rasterization.  Absent inputs are NULL (the reference passes empty tensors,
 * i.e. nullptr data pointers).  out_color [3,H,W] and radii [P] are fully written.
 * *num_rendered receives R, the number of (Gaussian, tile) instances. */
int gsr_forward(gsr_resize_fn geometry_buffer, void* geometry_ctx, gsr_resize_fn binning_buffer, void* binning_ctx,
                gsr_resize_fn image_buffer, void* image_ctx, int P, int D, int M, const float* background, int width,
                int height, const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                float tan_fovx, float tan_fovy, int prefiltered, float* out_color, int* radii, void* stream,
                int* num_rendered);

/* Forward rasterization of NEW colours over the geometry of an earlier gsr_forward call
 * (the reference's render() rasterizes the same Gaussians 6-10 times per view with
 * different colors_precomp, gaussian_renderer/__init__.py:160-264).  src_geom_buffer,
 * binning_buffer and image_buffer are that call's buffers, src_radii its radii; every
 * input that shapes the geometry (means, scales, rotations, cov3D, opacities, matrices,
 * image size, scale_modifier) must be unchanged -- the caller owns that check.  Writes a new
 * geometry buffer (colours replaced in the render records; the binning and image buffers
 * are shared, read-only except for identical re-writes of final_T / n_contrib),
 * out_color [3,H,W] and radii [P].  Output equals a full gsr_forward call bit for bit.
 * The returned geometry buffer pairs with the shared binning/image buffers in gsr_backward. */
int gsr_forward_reuse(gsr_resize_fn geometry_buffer, void* geometry_ctx, const void* src_geom_buffer,
                      const int* src_radii, void* binning_buffer, void* image_buffer, int P, int R,
                      const float* background, int width, int height, const float* colors_precomp, float* out_color,
                      int* radii, void* stream);

/* Backward rasterization.  geom/binning/img buffers are the ones the forward filled.
 * dL_dpix is [3,H,W].  All nine gradient outputs are fully written (no zero-fill needed):
 * dL_dmean2D [P,3] (z = 0), dL_dconic [P,2,2] (may be NULL: the reference's _C returns it to
 * no one), dL_dopacity [P], dL_dcolor [P,3] (may be NULL: not stored),
 * dL_dmean3D [P,3], dL_dcov3D [P,6] (may be NULL: not stored), dL_dsh [P,M,3] (may be NULL
 * if M == 0), dL_dscale [P,3], dL_drot [P,4].  The reference's RasterizeGaussiansBackwardCUDA
 * (rasterize_points.cu:115-192) fills all of them; an autograd caller skips the gradients of
 * inputs that need none (an empty colors_precomp or cov3D_precomp). */
int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                 const float* shs, const float* colors_precomp, const float* scales, float scale_modifier,
                 const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                 void* geom_buffer, void* binning_buffer, void* img_buffer, const float* dL_dpix, float* dL_dmean2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                 float* dL_dsh, float* dL_dscale, float* dL_drot, void* stream);

/* Multi-channel forward: gsr_forward's geometry (preprocess, depth sort, binning) once,
 * then one composite of nch per-Gaussian feature channels (16 per tile pass).  features is
 * [P][feature_stride] floats, 16-B aligned, feature_stride >= nch and a multiple of 4;
 * background [nch]; out [nch,H,W].  Channel c of out equals a gsr_forward call whose
 * colors_precomp holds feature c (bit for bit; the blend decisions do not depend on the
 * colours).  The buffers pair with gsr_backward_channels. */
int gsr_forward_channels(gsr_resize_fn geometry_buffer, void* geometry_ctx, gsr_resize_fn binning_buffer,
                         void* binning_ctx, gsr_resize_fn image_buffer, void* image_ctx, int P, int nch,
                         int feature_stride, const float* features, const float* background, int width, int height,
                         const float* means3D, const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                         const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                         int prefiltered, float* out, int* radii, void* stream, int* num_rendered);

/* Backward of gsr_forward_channels: dL_dout [nch,H,W] -> dL_dfeatures [P][feature_stride]
 * (padding columns zero) and the geometric gradients of gsr_backward (their sum over the
 * channels' separate calls).  dL_dcov3D may be null (no cov3D_precomp).  `accumulate`: bits
 * GSR_ACC_MEAN3D / _SCALE / _ROT / _OPACITY add those gradients into the given buffers
 * instead of overwriting them (several views' gradients summed by the kernel that makes
 * them). */
#define GSR_ACC_MEAN3D 1u
#define GSR_ACC_SCALE 2u
#define GSR_ACC_ROT 4u
#define GSR_ACC_OPACITY 8u
int gsr_backward_channels(int P, int nch, int feature_stride, const float* features, int R, const float* background,
                          int width, int height, const float* means3D, const float* scales, float scale_modifier,
                          const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                          const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                          const int* radii, void* geom_buffer, void* binning_buffer, void* img_buffer,
                          const float* dL_dout, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                          float* dL_dfeatures, float* dL_dmean3D, float* dL_dcov3D, float* dL_dscale, float* dL_drot,
                          unsigned accumulate, void* stream);

/* render()'s per-Gaussian channels in one pass (gaussian_renderer/__init__.py:120-200):
 * features [P][16] = [rgb, diffuse, specular, depth, 0.5 n + 0.5, 1, 0, 0], with
 *   n     = the minimum-scale axis of build_rotation(rotation), flipped towards the camera;
 *   depth = view-space z (world_view_transform viewmatrix, row-major 4x4);
 *   rgb/diffuse/specular = EnvironmentLight.shade of the foreground Gaussians (base
 *           [(deg+1)^2,3], fg_lut [256,256,2], roughness/metalness [N_fg], metalness
 *           nullable), and for sky Gaussians clamp_min(eval_sh(sky_deg, sky_sh, dir) + 0.5, 0)
 *           (sky_deg = -1: 1, fix_sky) with diffuse = specular = 0.
 * fg_rank [P] holds each Gaussian's rank among the foreground ones (-1: sky) and fg_rows
 * [N_fg] the inverse map (validated, not read: one kernel runs over all P by fg_rank).
 * workspace: gsr_relit_workspace_bytes, scratch for the backward's per-workgroup partial
 * sums (the forward leaves it untouched; the backward recomputes the normals).  features
 * must be 16-B aligned (each 64-B row is written whole by one thread). */
size_t gsr_relit_workspace_bytes(int P, int N_fg, int deg, int sky_deg);
int gsr_relit_features(int P, int N_fg, const float* xyz, const float* rotation, const float* scaling,
                       const int* fg_rank, const int* fg_rows, const float* albedo, const float* roughness,
                       const float* metalness, int deg, const float* base, const float* fg_lut, int specular,
                       int sky_deg, const float* sky_sh, const float* campos, const float* viewmatrix,
                       float* features, void* workspace, void* stream);
/* Backward: dL_dfeatures [P][16] -> d_xyz [P,3], d_rotation [P,4], d_albedo [N_fg,3],
 * d_roughness / d_metalness [N_fg] (may be NULL), d_base, d_sky_sh (may be NULL).  The
 * scaling gets no gradient (the axis is an argmin).  `accumulate`: bits GSR_ACC_MEAN3D
 * (d_xyz), GSR_ACC_ROT (d_rotation), GSR_ACC_ALBEDO / _ROUGH / _METAL add into those
 * buffers instead of overwriting them. */
#define GSR_ACC_ALBEDO 16u
#define GSR_ACC_ROUGH 32u
#define GSR_ACC_METAL 64u
int gsr_relit_features_backward(int P, int N_fg, const float* xyz, const float* rotation, const float* scaling,
                                const int* fg_rank, const int* fg_rows, const float* albedo, const float* roughness,
                                const float* metalness, int deg, const float* base, const float* fg_lut, int specular,
                                int sky_deg, const float* sky_sh, const float* campos, const float* viewmatrix,
                                const float* dL_dfeatures, float* d_xyz, float* d_rotation, float* d_albedo,
                                float* d_roughness, float* d_metalness, float* d_base, float* d_sky_sh,
                                void* workspace, unsigned accumulate, void* stream);

/* render()'s image-space tail over the composite's images ([H,W] planes, [3,H,W] for n01):
 *   normal     = ((n01 - 0.5) * 2 * (normal_view ? -1 : 1)) * sky + (1 - sky)
 *   normal_ref = normalize(cross(p[y+1] - p[y-1], p[x+1] - p[x-1])) * alpha + (1 - sky),
 *                zero normals on the one-pixel border, p = (depth * sky) * rays + centre.
 * cam12 (host memory): rows M0, M1, M2 of K^-1^T R^T (rays = x M0 + y M1 + M2) and the
 * camera centre.  The backward gives dL/dn01 and dL/ddepth (alpha gets none: the
 * reference detaches it). */
int gsr_relit_epilogue(int width, int height, const float* cam12, const float* n01, const float* depth,
                       const float* alpha, const float* sky_mask, int normal_view, float* normal, float* normal_ref,
                       void* stream);
int gsr_relit_epilogue_backward(int width, int height, const float* cam12, const float* depth, const float* alpha,
                                const float* sky_mask, int normal_view, const float* g_normal,
                                const float* g_normal_ref, float* d_n01, float* d_depth, void* stream);

/* One Adam step (torch.optim.Adam semantics, relit3DGW_model.py:149 / gaussian_model.py:264-274)
 * over a flat fp32 parameter buffer whose param groups are consecutive segments:
 * segment k = [seg_end[k-1], seg_end[k]) with learning rate seg_lr[k] (host arrays, nseg <= 16,
 * seg_end[nseg-1] == n).  grad is scaled by grad_scale first (1/views after a SUM all-reduce).
 * step is the 1-based step count after this update.  param, grad, exp_avg, exp_avg_sq: n floats
 * on the device, 16-B aligned. */
int gsr_adam_step(long long n, int nseg, const long long* seg_end, const double* seg_lr, double beta1, double beta2,
                  double eps, int step, float grad_scale, float* param, const float* grad, float* exp_avg,
                  float* exp_avg_sq, void* stream);
/* The same update over elements [lo, hi) only (lo a multiple of 4): the data-parallel step
 * runs it chunk by chunk, each chunk right after its slice of the gradient all-reduce lands
 * (gsr.dp.finish_step), so the update of chunk i overlaps the exchange of chunk i + 1.
 * gsr_adam_step(...) == gsr_adam_step_range(n, 0, n, ...). */
int gsr_adam_step_range(long long n, long long lo, long long hi, int nseg, const long long* seg_end,
                        const double* seg_lr, double beta1, double beta2, double eps, int step, float grad_scale,
                        float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* stream);

/* SSIM of the training loss (utils/loss_utils.py:53-96: 11x11 Gaussian window, sigma 1.5,
 * zero padding, C1 = 0.01^2, C2 = 0.03^2) over img1, img2 [C,H,W].  window: the 11 normalised
 * 1-D weights (host).  mask: null or [C,H,W] / [1,H,W] (mask_cstride = H*W or 0).
 * block_sums: 2 * gsr_ssim_partials(C,H,W) floats, per workgroup a fixed-order partial of
 * sum(map * mask) and of #(mask == 1) (the caller adds them).  dmaps: null (no backward) or 3*C*H*W floats kept for the backward.
 * The backward writes dL/dimg1 = gscale[0] * (window^T applied to dmaps) (img2 gets none:
 * it is the ground truth), or adds it to dimg1 when `accumulate` is non-zero; gscale is a
 * device scalar, dL/dloss / #mask. */
long long gsr_ssim_partials(int C, int height, int width);
int gsr_ssim_forward(int C, int height, int width, const float* img1, const float* img2, const float* mask,
                     long long mask_cstride, const float* window, float* block_sums, float* dmaps, void* stream);
int gsr_ssim_backward(int C, int height, int width, const float* img1, const float* img2, const float* dmaps,
                      const float* gscale, const float* window, float* dimg1, int accumulate, void* stream);
/* gsr_ssim_backward that also makes the loss's L1 term's image gradient (train.py:78 through
 * gsr_view_loss_backward's d_img: l1_coef[0] * sign(img1 * occ - img2 * occ) * occ, occ the
 * [H,W] occluder mask) and writes the sum (the same two roundings as gsr_view_loss_backward's
 * d_img followed by gsr_ssim_backward with accumulate): one pass over dimg1 instead of a write
 * and a read-modify-write.  l1_coef: device pointer. */
int gsr_ssim_l1_backward(int C, int height, int width, const float* img1, const float* img2, const float* dmaps,
                         const float* gscale, const float* window, const float* occ, const float* l1_coef,
                         float* dimg1, void* stream);

/* The pointwise terms of the training loss (train.py:77-99) over one view: images img, gt,
 * diff, spec, nrm, nref are [3,H,W] (npix = H*W), the sky and occluder masks [H,W].
 * Forward: gsr_view_loss_partials(npix) x 5 partial sums (see csrc/gsr_loss.hip) that the
 * caller adds.  Backward: coef (device) = (k_img, k_brdf, k_normal); any gradient pointer
 * may be null. */
int gsr_view_loss_partials(int npix);
/* One view's training objective from the partial sums of gsr_view_loss_forward and
 * gsr_ssim_forward (with the occluder mask): loss[0] = the pointwise terms +
 * lambda_dssim (1 - SSIM) (train.py:77-99), and coef[4] = the backward coefficients before the
 * upstream gradient: (k_img, k_brdf, k_normal) for gsr_view_loss_backward and the SSIM map
 * sum's for gsr_ssim_backward.  One workgroup; sums in double (counts exact at 4K). */
int gsr_view_objective(int n_loss_partials, const float* loss_partials, long long n_ssim_partials,
                       const float* ssim_partials, int npix, double lambda_dssim, double lambda_sky,
                       double lambda_normal, float* loss, float* coef, void* stream);
int gsr_view_loss_forward(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, float* partials,
                          void* stream);
int gsr_view_loss_backward(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                           const float* nrm, const float* nref, const float* sky, const float* occ, const float* coef,
                           float* d_img, float* d_diff, float* d_spec, float* d_nrm, float* d_nref, void* stream);

/* Training-step bookkeeping over V <= 8 views at once (csrc/gsr_trainaux.hip).
 * radii / grad_means2D: arrays of V device pointers (host arrays) to each view's [P] int32
 * radii and [P,3] means2D gradient.  depth_cols [V][4] (device): the view's depth column,
 * depth = xyz . c[0:3] + c[3].  Forward: gsr_view_regularisers_partials(P) x 5V partial sums
 * per view v: [0] #visible foreground, [1] #visible sky, [2] sum min-scale over visible
 * foreground, [3] sum depth over visible sky, [4] sum depth over visible foreground.
 * Backward: grad_sums [5V] (device) are the sums' upstream gradients; d_xyz / d_scaling
 * (either may be null) are overwritten, or added to with GSR_ACC_MEAN3D / GSR_ACC_SCALE in
 * `accumulate`.  gsr_densify_stats updates accum / denom /
 * max_radii [P] in place over the views in order; with accum = denom = NULL (grad_means2D
 * may then be NULL too) it updates max_radii alone (train.py:130 runs every iteration, the
 * sums only below densify_until_iter, train.py:143-144). */
int gsr_view_regularisers_partials(int P);
int gsr_view_regularisers_forward(int P, int V, const float* xyz, const float* scaling, const int* const* radii,
                                  const unsigned char* is_sky, const float* depth_cols, float* partials,
                                  void* stream);
int gsr_view_regularisers_backward(int P, int V, const float* scaling, const int* const* radii,
                                   const unsigned char* is_sky, const float* depth_cols, const float* grad_sums,
                                   float* d_xyz, float* d_scaling, unsigned accumulate, void* stream);
int gsr_densify_stats(int P, int V, const float* const* grad_means2D, const int* const* radii, float* accum,
                      float* denom, float* max_radii, void* stream);
/* The regularisers' per-view tail (train.py:99-118) from gsr_view_regularisers_forward's
 * summed sums [V][5], the SH basis [V*n_samples][25] at the envlight directions (gsr_sh_basis)
 * and the environment SH [V][25][3]: total[v] = envl (when lambda_env > 0) + lambda_scale
 * min-scale mean + (depth_on) lambda_depth exp(-gamma (sky depth mean - foreground depth
 * mean)).  The backward writes d_sums [V][5] (the counts and the detached foreground mean
 * get 0) and d_env_sh [V][25][3] from grad_total [V].  One workgroup; V <= 8, n_samples <= 32. */
int gsr_view_regularisers_tail_forward(int V, int n_samples, const float* sums, const float* basis, const float* env_sh,
                                       float lambda_env, float lambda_scale, float lambda_depth, float gamma,
                                       int depth_on, float* total, void* stream);
int gsr_view_regularisers_tail_backward(int V, int n_samples, const float* sums, const float* basis,
                                        const float* env_sh, float lambda_env, float lambda_scale, float lambda_depth,
                                        float gamma, int depth_on, const float* grad_total, float* d_sums,
                                        float* d_env_sh, void* stream);
/* Real SH basis [N][(deg+1)^2] at the normalised directions dirs [N,3], deg 0..4. */
int gsr_sh_basis(int N, int deg, const float* dirs, float* out, void* stream);
/* Sky shell: angles [N,2] (theta, phi; clamped to [0,pi/2] and [-pi/2,pi/2]), radius [1],
 * center [3] (device) -> xyz [N,3] = r (sin t sin p, -cos t, sin t cos p) + center.
 * Backward writes d_angles [N,2] and gsr_sky_xyz_partials(N) partial sums of d radius. */
int gsr_sky_xyz_partials(int N);
int gsr_sky_xyz_forward(int N, const float* angles, const float* radius, const float* center, float* xyz,
                        void* stream);
int gsr_sky_xyz_backward(int N, const float* angles, const float* radius, const float* grad_xyz, float* d_angles,
                         float* d_radius_partials, void* stream);

/* The model's activations (gaussian_model.py:69-103) over P = n_fg + n_sky Gaussians:
 * xyz [P,3] = the foreground rows xyz_fg [n_fg,3] and the sky shell points from angles
 * [n_sky,2], radius [1], center [3] (gsr_sky_xyz_forward), placed by src [P] (the foreground
 * row >= 0, or -1 - the sky row; null: the first n_fg rows are the foreground); scale =
 * exp(scale_raw), rot = rot_raw / max(|rot_raw|, 1e-12), op = sigmoid(op_raw) [P]; alb, rough,
 * metal = sigmoid of the raw [n_fg] rows.  The backward writes (not adds) the raw parameters'
 * gradients from the activations' upstream gradients (any g_* may be null: zero);
 * radius_partials: gsr_activations_partials(P, n_fg) floats of scratch. */
int gsr_activations_partials(int P, int n_fg);
int gsr_activations_forward(int P, int n_fg, int n_sky, const int* src, const float* xyz_fg, const float* angles,
                            const float* radius, const float* center, const float* scale_raw, const float* rot_raw,
                            const float* op_raw, const float* alb_raw, const float* rough_raw, const float* metal_raw,
                            float* xyz, float* scale, float* rot, float* op, float* alb, float* rough, float* metal,
                            void* stream);
int gsr_activations_backward(int P, int n_fg, int n_sky, const int* src, const float* xyz_fg, const float* angles,
                             const float* radius, const float* center, const float* scale_raw, const float* rot_raw,
                             const float* op_raw, const float* alb_raw, const float* rough_raw, const float* metal_raw,
                             const float* scale, const float* rot, const float* op, const float* alb,
                             const float* rough, const float* metal, const float* g_xyz, const float* g_scale,
                             const float* g_rot, const float* g_op, const float* g_alb, const float* g_rough,
                             const float* g_metal, float* d_xyz_fg, float* d_angles, float* d_radius,
                             float* radius_partials, float* d_scale_raw, float* d_rot_raw, float* d_op_raw,
                             float* d_alb_raw, float* d_rough_raw, float* d_metal_raw, void* stream);

/* 2D texture lookups with nvdiffrast.torch.texture semantics (csrc/gsr_texture.hip).
 * tex [tex_nb][tex_h][tex_w][C] (tex_nb == 1 broadcasts over the minibatch, else == nb);
 * uv [nb][npix][2]; out [nb][npix][C].  filter: 0 nearest, 1 linear; boundary: 0 wrap,
 * 1 clamp, 2 zero.  Backward: dout [nb][npix][C] -> d_uv [nb][npix][2] (may be NULL) and
 * d_tex (may be NULL; ACCUMULATED into, the caller zero-fills it). */
int gsr_texture2d_forward(int nb, int npix, int tex_nb, int tex_h, int tex_w, int C, const float* tex,
                          const float* uv, int filter, int boundary, float* out, void* stream);
int gsr_texture2d_backward(int nb, int npix, int tex_nb, int tex_h, int tex_w, int C, const float* tex,
                           const float* uv, int filter, int boundary, const float* dout, float* d_uv, float* d_tex,
                           void* stream);

/* present[i] = (view * means3D[i]).z > 0.2 (uint8 0/1). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/* Relighting shade for N foreground Gaussians (light.py:131-193).  pos, normal, albedo,
 * view_pos: [N,3]; kr: [N]; km: [N] or NULL (F0 = 0.04); base: [(deg+1)^2, 3];
 * fg_lut: [256,256,2] (the split-sum LUT).  Outputs rgb, diffuse, specular: [N,3]. */
int gsr_shade_forward(int N, int deg, const float* pos, const float* normal, const float* albedo,
                      const float* view_pos, const float* kr, const float* km, const float* base,
                      const float* fg_lut, int specular, float* rgb, float* diffuse, float* specular_out,
                      void* stream);

/* Backward of gsr_shade_forward given upstream gradients g_rgb, g_diffuse, g_specular
 * ([N,3] each, any may be NULL = zero).  Outputs (any may be NULL = not needed):
 * d_pos, d_normal, d_albedo, d_view_pos [N,3]; d_kr, d_km [N]; d_base [(deg+1)^2,3]
 * (reduced over N; fully written).  `workspace` must hold gsr_shade_workspace_bytes(N, deg)
 * bytes of device memory. */
size_t gsr_shade_workspace_bytes(int N, int deg);
int gsr_shade_backward(int N, int deg, const float* pos, const float* normal, const float* albedo,
                       const float* view_pos, const float* kr, const float* km, const float* base,
                       const float* fg_lut, int specular, const float* g_rgb, const float* g_diffuse,
                       const float* g_specular, float* d_pos, float* d_normal, float* d_albedo, float* d_view_pos,
                       float* d_kr, float* d_km, float* d_base, void* workspace, void* stream);

/* Mean squared distance to the 3 nearest other points, for P points [P,3] (simple-knn's
 * distCUDA2, submodules/simple-knn/spatial.cu:14-26 -> simple_knn.cu:185-220, used by
 * gaussian_model.py:189,249).  Same Morton/box algorithm and arithmetic, bit-identical
 * output.  `workspace`: gsr_knn_workspace_bytes(P) bytes of device memory. */
size_t gsr_knn_workspace_bytes(int P);
int gsr_knn_mean_dist(int P, const float* points, float* mean_dists, void* workspace, void* stream);

/* Private-buffer introspection for tests and profiling: byte offsets of the arrays the
 * forward leaves in its three buffers (layout is private between forward and backward). */
typedef struct gsr_layout {
    size_t geom_bytes, img_bytes, bin_bytes;  /* bin_bytes: the fixed part (header + super-tile ranges) */
    size_t geom_radii, geom_tiles, geom_depth_key, geom_rect, geom_rec, geom_acc;
    size_t img_final_T, img_n_contrib, img_ranges, img_tile_nmax, img_tile_emax;
    size_t bin_st_ranges, bin_entries;
    /* the backward's dispatch order (appended in round 4): the forward's per-tile cost estimate
     * [T] and its per-tile-row sums [tiles_y], the order [T], and the band tables (u32 [80]: the
     * backward's table at word 8 and the forward's at word 40, each relative to its start: band
     * heavy counts [0..8), balanced band bounds [8..17), band costs [24..32)) */
    size_t img_tile_cost, img_row_cost, img_order_bwd, img_nheavy;
    /* the forward's survivor lists (appended in round 5): per tile the count (u32 [T],
     * 0xFFFFFFFF: none stored) and the list (u32 pairs [T][surv_cap]), the last region of the
     * image buffer, reserved only while the survivor lists are on (img_bytes counts them then) */
    size_t img_surv_n, img_surv, surv_cap;
} gsr_layout;
int gsr_get_layout(int P, long long R, int width, int height, gsr_layout* out);

/* Stage profiling: when enabled, every stage (preprocess, compact, depth_sort, offsets_scan,
 * st_emit, st_sort, tile_lists, render_fwd, bwd_zero, render_bwd, preprocess_bwd, shade_fwd,
 * shade_bwd) is bracketed by hipEvents on the call's stream.  gsr_profile_read() waits for
 * the recorded events and returns accumulated milliseconds and launch counts per stage. */
int gsr_profile_enable(int on);
/* Restrict the timed stages to the set bits of mask (bit i = stage i; default all), so a
 * timed loop can bracket only the kernel it reports with events. */
int gsr_profile_stages(unsigned mask);
int gsr_profile_stage_count(void);
const char* gsr_profile_stage_name(int i);
int gsr_profile_read(double* ms, long long* counts, int n, int reset);

/* Deterministic backward (default off, or GSR_DETERMINISTIC=1 in the
 * environment): the tile passes write each (tile, Gaussian) pair's partial gradient sums to a
 * per-instance row instead of adding them with float atomics (the reference's
 * backward.cu:523,545-554 atomics are run-order dependent, and so are this library's), heavy
 * tiles are not split, and one pass sums every Gaussian's rows in a fixed order (its tiles
 * row-major).  Gradients are then bit-reproducible.  Costs a 48 B (3 channels) or
 * 4*(6+nch) B row per instance of device scratch and a stream synchronisation per backward.
 * Set it before the forward whose backward should be deterministic. */
int gsr_set_deterministic(int on);
int gsr_get_deterministic(void);
/* Survivor lists (default on; GSR_SURV_LISTS=0 in the environment turns them off): the forward
 * tile pass stores each tile's surviving list entries in the image buffer and the backward walks
 * them instead of filtering the tile's super-tile list again.  Results are identical either way
 * (the same evaluations in the same order); a switch for tests and A/B timing.  Set it before
 * the forward. */
int gsr_set_survivor_lists(int on);
int gsr_get_survivor_lists(void);
/* Exact blend mode (default off; GSR_EXACT_BLEND=1 in the environment turns it on): the tile passes
 * evaluate every (pixel, Gaussian) pair with the reference's float arithmetic bit for bit -- the
 * exponent in forward.cu:335's operation order, glibc's expf (the oracle's libm), alpha =
 * min(0.99, o G), the colour sum in forward.cu:359's order -- so the forward's colours,
 * transmittance and n_contrib equal the canonical oracle's exactly (the default arithmetic
 * differs by rounding, and decides a pair or two per frame within ulps of a threshold the other
 * way).  The backward replays the forward's mode (recorded per image buffer).  Slower: a
 * double-precision exp per evaluation.  Set it before the forward. */
int gsr_set_exact_blend(int on);
int gsr_get_exact_blend(void);
/* The backward's heavy-tile threshold: tiles whose estimated cost (the forward's evaluation
 * count) reaches 2^bits run as four quadrant units (a negative value restores the build's
 * default, 13).  Results agree either way within the atomic-order tolerance; a switch for tests
 * (the parity cases' tiles stay below the default) and A/B timing.  Set it before the backward. */
int gsr_set_backward_heavy_bits(int bits);
/* 1 when this library was built with -DGSR_DEBUG (`make debug` -> lib/debug/libgsr.so): every
 * forward then verifies its tile lists against the preprocess (ids, culling, rect coverage,
 * (depth, index) order, per-Gaussian instance counts, total R, n_contrib bounds) with a
 * stream synchronisation, and fails with GSR_E_DEVICE_CHECK naming the first violation. */
int gsr_debug_build(void);
/* The binning buffer holds super-tile lists: every (visible Gaussian, super-tile (8x4 tiles; 8x8 in large frames) its
 * rect touches) entry, per super-tile in (depth, index) order with the entry's local tile rect;
 * the tile passes filter a tile's list from them.  This writes the reference's point_list [R]
 * (binningState.point_list after the sort, rasterizer_impl.cu:79-99,303-308) and the tile
 * ranges [T] (imgState.ranges, identifyTileRanges, rasterizer_impl.cu:101-138) from them:
 * tests, the GSR_DEBUG checks and the deterministic backward.  Synchronous. */
int gsr_materialize_lists(int R, int width, int height, void* binning_buffer, unsigned* point_list, unsigned* ranges,
                          void* stream);
/* The same verification on demand, over a forward's three buffers (any build; synchronous). */
int gsr_check_buffers(int P, int R, int width, int height, const int* radii, void* geom_buffer, void* binning_buffer,
                      void* img_buffer, void* stream);

const char* gsr_last_error(void);
const char* gsr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H_INCLUDED */
