// gsr_trainaux.hip -- the training iteration's per-Gaussian bookkeeping fused into single
// passes (train.py:101-131 around the rasterizer; gsr/train.py):
//
//  * view regularisers (utils/loss_utils.py:140-148 depth_loss_gaussians, :210-220
//    min_scale_loss) for V views at once.  PyTorch composes them from ~30 [V,P] kernels each
//    way (masks, column selects whose backward is a zero tensor + copy, products, V x 5 full
//    reductions); here one forward pass writes per-workgroup partial sums per view
//        [0] #visible foreground  [1] #visible sky  [2] sum smin over visible foreground
//        [3] sum depth over visible sky  [4] sum depth over visible foreground
//    (smin = min over the three scales, depth = x . c_v + c_v3 with c_v the view's depth
//    column), and one backward pass writes d xyz and d scaling from V x 5 upstream gradients;
//  * densification statistics (gaussian_model.py:627-629, train.py:130) of V views at once:
//    max_radii2D = max(max_radii2D, radii_v), accum += |dL/dmean2D_v [:2]|, denom += 1 on each
//    view's visible Gaussians, in view order;
//  * the real SH basis (utils/sh_utils.py:81-151, degrees 0-4) at normalised directions (the
//    envlight regulariser's random directions);
//  * the sky Gaussians' shell positions (gaussian_model.py:95-103,159-169) and their backward;
//  * the model's activations (gaussian_model.py:69-80,84-103: exp scaling, normalised
//    rotation, sigmoid opacity and materials, get_xyz's scatter of the foreground rows and
//    the shell) in one pass, and one backward pass writing the raw parameters' gradients
//    straight into the optimizer's flat gradient (no autograd accumulation kernels).
// All HBM-bound streaming kernels, FMA contraction off where a result is compared with
// PyTorch's elementwise arithmetic.
#include "gsr_kernels.hpp"

#pragma clang fp contract(off)

namespace gsr {

constexpr int REG_THREADS = 256;

__global__ void __launch_bounds__(REG_THREADS) k_view_regs_fwd(int P, int V, const float* __restrict__ xyz,
                                                               const float* __restrict__ scaling,
                                                               const ViewPtrs<int> radii,
                                                               const unsigned char* __restrict__ is_sky,
                                                               const float* __restrict__ dcol, float* __restrict__ part) {
    __shared__ float red[REG_THREADS / 64][REG_MAXV * 5];
    float acc[REG_MAXV * 5];
#pragma unroll
    for (int k = 0; k < REG_MAXV * 5; k++) acc[k] = 0.f;
    float c[REG_MAXV][4];
#pragma unroll
    for (int v = 0; v < REG_MAXV; v++)
#pragma unroll
        for (int j = 0; j < 4; j++) c[v][j] = v < V ? dcol[4 * v + j] : 0.f;
    for (int i = blockIdx.x * REG_THREADS + threadIdx.x; i < P; i += gridDim.x * REG_THREADS) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        const float smin = fminf(fminf(scaling[3 * i], scaling[3 * i + 1]), scaling[3 * i + 2]);
        const bool sky = is_sky[i] != 0;
#pragma unroll
        for (int v = 0; v < REG_MAXV; v++) {
            if (v >= V || radii.p[v][i] <= 0) continue;
            // x c0 + y c1 + z c2 + c3, as PyTorch evaluates the elementwise expression
            const float depth = ((x * c[v][0] + y * c[v][1]) + z * c[v][2]) + c[v][3];
            if (sky) {
                acc[5 * v + 1] += 1.f;
                acc[5 * v + 3] += depth;
            } else {
                acc[5 * v + 0] += 1.f;
                acc[5 * v + 2] += smin;
                acc[5 * v + 4] += depth;
            }
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < REG_MAXV * 5; k++) {
        float a = k < 5 * V ? acc[k] : 0.f;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) red[wave][k] = a;
    }
    __syncthreads();
    if (threadIdx.x < 5 * V)
        part[(size_t)blockIdx.x * 5 * V + threadIdx.x] =
            (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// g[5 v + k]: upstream gradient of sum k of view v (k = 2: smin over foreground, 3: depth over
// sky, 4: depth over foreground; the counts have none).  d scaling goes to the first minimum
// column (torch.min's backward), d xyz = sum over views of the depth sums' gradients x c_v.
__global__ void __launch_bounds__(REG_THREADS) k_view_regs_bwd(int P, int V, const float* __restrict__ scaling,
                                                               const ViewPtrs<int> radii,
                                                               const unsigned char* __restrict__ is_sky,
                                                               const float* __restrict__ dcol,
                                                               const float* __restrict__ g, float* __restrict__ d_xyz,
                                                               float* __restrict__ d_scaling, unsigned acc) {
    const int i = blockIdx.x * REG_THREADS + threadIdx.x;
    if (i >= P) return;
    const bool sky = is_sky[i] != 0;
    float gs = 0.f, gx = 0.f, gy = 0.f, gz = 0.f;
    for (int v = 0; v < V; v++) {
        if (radii.p[v][i] <= 0) continue;
        const float gd = sky ? g[5 * v + 3] : g[5 * v + 4];
        if (!sky) gs += g[5 * v + 2];
        gx += gd * dcol[4 * v];
        gy += gd * dcol[4 * v + 1];
        gz += gd * dcol[4 * v + 2];
    }
    if (d_xyz) {
        const bool add = (acc & ACC_MEAN3D) != 0;
        d_xyz[3 * i] = add ? d_xyz[3 * i] + gx : gx;
        d_xyz[3 * i + 1] = add ? d_xyz[3 * i + 1] + gy : gy;
        d_xyz[3 * i + 2] = add ? d_xyz[3 * i + 2] + gz : gz;
    }
    if (d_scaling) {
        const float s0 = scaling[3 * i], s1 = scaling[3 * i + 1], s2 = scaling[3 * i + 2];
        const int am = (s1 < s0) ? ((s2 < s1) ? 2 : 1) : ((s2 < s0) ? 2 : 0);  // first index of the minimum
        if (acc & ACC_SCALE) {
            d_scaling[3 * i + am] += gs;
        } else {
            d_scaling[3 * i] = am == 0 ? gs : 0.f;
            d_scaling[3 * i + 1] = am == 1 ? gs : 0.f;
            d_scaling[3 * i + 2] = am == 2 ? gs : 0.f;
        }
    }
}

__global__ void __launch_bounds__(256) k_densify_stats(int P, int V, const ViewPtrs<float> g2d,
                                                       const ViewPtrs<int> radii, float* __restrict__ accum,
                                                       float* __restrict__ denom, float* __restrict__ maxr) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    // accum == nullptr: the max radii alone (train.py:130 runs every iteration, the sums of
    // add_densification_stats only below densify_until_iter, train.py:143-144)
    const bool sums = accum != nullptr;
    float a = sums ? accum[i] : 0.f, d = sums ? denom[i] : 0.f, m = maxr[i];
    for (int v = 0; v < V; v++) {
        const int r = radii.p[v][i];
        if (r <= 0) continue;
        if (sums) {
            const float gx = g2d.p[v][3 * i], gy = g2d.p[v][3 * i + 1];
            a += sqrtf(gx * gx + gy * gy);
            d += 1.f;
        }
        m = fmaxf(m, (float)r);
    }
    if (sums) {
        accum[i] = a;
        denom[i] = d;
    }
    maxr[i] = m;
}

// basis [N][(deg+1)^2] at the directions d / |d| (utils/sh_utils.py:81-151, the reference's
// constants and polynomial order; degrees 0-4)
__global__ void k_sh_basis(int N, int deg, const float* __restrict__ dirs, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float dx = dirs[3 * i], dy = dirs[3 * i + 1], dz = dirs[3 * i + 2];
    const float n = sqrtf(dx * dx + dy * dy + dz * dz);
    const float x = dx / n, y = dy / n, z = dz / n;
    const int K = (deg + 1) * (deg + 1);
    float* o = out + (size_t)i * K;
    o[0] = 0.28209479177387814f;
    if (deg < 1) return;
    const float C1 = 0.4886025119029199f;
    o[1] = -C1 * y;
    o[2] = C1 * z;
    o[3] = -C1 * x;
    if (deg < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.31539156525252005f * (2.0f * zz - xx - yy);
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.5462742152960396f * (xx - yy);
    if (deg < 3) return;
    o[9] = -0.5900435899266435f * y * (3.0f * xx - yy);
    o[10] = 2.890611442640554f * xy * z;
    o[11] = -0.4570457994644658f * y * (4.0f * zz - xx - yy);
    o[12] = 0.3731763325901154f * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
    o[13] = -0.4570457994644658f * x * (4.0f * zz - xx - yy);
    o[14] = 1.445305721320277f * z * (xx - yy);
    o[15] = -0.5900435899266435f * x * (xx - 3.0f * yy);
    if (deg < 4) return;
    o[16] = 2.5033429417967046f * xy * (xx - yy);
    o[17] = -1.7701307697799304f * yz * (3.0f * xx - yy);
    o[18] = 0.9461746957575601f * xy * (7.0f * zz - 1.0f);
    o[19] = -0.6690465435572892f * yz * (7.0f * zz - 3.0f);
    o[20] = 0.10578554691520431f * (zz * (35.0f * zz - 30.0f) + 3.0f);
    o[21] = -0.6690465435572892f * xz * (7.0f * zz - 3.0f);
    o[22] = 0.47308734787878004f * (xx - yy) * (7.0f * zz - 1.0f);
    o[23] = -1.7701307697799304f * xz * (xx - 3.0f * yy);
    o[24] = 0.6258357354491761f * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy));
}

// the sky shell: angles [N,2] (theta clamped to [0, pi/2], phi to [-pi/2, pi/2]) ->
// out [N,3] = r (sin t sin p, -cos t, sin t cos p) + c, written at row stride 3
constexpr float SKY_HALF_PI = 1.57079632679489661923f;
__global__ void __launch_bounds__(256) k_sky_xyz_fwd(int N, const float* __restrict__ ang, const float* __restrict__ radius,
                                                     const float* __restrict__ center, float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const float t = fminf(fmaxf(ang[2 * i], 0.f), SKY_HALF_PI);
    const float p = fminf(fmaxf(ang[2 * i + 1], -SKY_HALF_PI), SKY_HALF_PI);
    const float r = radius[0];
    const float st = sinf(t), ct = cosf(t), sp = sinf(p), cp = cosf(p);
    out[3 * i] = r * (st * sp) + center[0];
    out[3 * i + 1] = r * (-ct) + center[1];
    out[3 * i + 2] = r * (st * cp) + center[2];
}

// d angles [N,2] (zero where the angle was clamped: torch.clamp's backward passes the gradient
// at the bounds themselves), per-workgroup partials of d radius
__global__ void __launch_bounds__(256) k_sky_xyz_bwd(int N, const float* __restrict__ ang, const float* __restrict__ radius,
                                                     const float* __restrict__ g, float* __restrict__ d_ang,
                                                     float* __restrict__ d_rad_part) {
    __shared__ float red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    float dr = 0.f;
    if (i < N) {
        const float t0 = ang[2 * i], p0 = ang[2 * i + 1];
        const float t = fminf(fmaxf(t0, 0.f), SKY_HALF_PI), p = fminf(fmaxf(p0, -SKY_HALF_PI), SKY_HALF_PI);
        const float r = radius[0];
        const float st = sinf(t), ct = cosf(t), sp = sinf(p), cp = cosf(p);
        const float gx = g[3 * i], gy = g[3 * i + 1], gz = g[3 * i + 2];
        dr = (gx * (st * sp) + gy * (-ct)) + gz * (st * cp);
        const float dt = r * ((gx * (ct * sp) + gy * st) + gz * (ct * cp));
        const float dp = r * (gx * (st * cp) - gz * (st * sp));
        d_ang[2 * i] = (t0 >= 0.f && t0 <= SKY_HALF_PI) ? dt : 0.f;
        d_ang[2 * i + 1] = (p0 >= -SKY_HALF_PI && p0 <= SKY_HALF_PI) ? dp : 0.f;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dr += __shfl_xor(dr, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dr;
    __syncthreads();
    if (threadIdx.x == 0) d_rad_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- activations (ActArgs, gsr_kernels.hpp) ----------------------------------------------
__device__ __forceinline__ float act_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }  // as torch's kernel
constexpr float ACT_NORM_EPS = 1e-12f;  // F.normalize's eps

__global__ void __launch_bounds__(256) k_activations_fwd(ActArgs a, ActOutW o) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t < a.P) {
        // position: a foreground row or a point on the sky shell
        const int r = a.src ? a.src[t] : (t < a.Nfg ? t : -1 - (t - a.Nfg));
        float x, y, z;
        if (r >= 0) {
            x = a.xyz_fg[3 * r];
            y = a.xyz_fg[3 * r + 1];
            z = a.xyz_fg[3 * r + 2];
        } else {
            const int j = -1 - r;
            const float th = fminf(fmaxf(a.angles[2 * j], 0.f), SKY_HALF_PI);
            const float ph = fminf(fmaxf(a.angles[2 * j + 1], -SKY_HALF_PI), SKY_HALF_PI);
            const float rad = a.radius[0];
            const float st = sinf(th), ct = cosf(th), sp = sinf(ph), cp = cosf(ph);
            x = rad * (st * sp) + a.center[0];
            y = rad * (-ct) + a.center[1];
            z = rad * (st * cp) + a.center[2];
        }
        o.xyz[3 * t] = x;
        o.xyz[3 * t + 1] = y;
        o.xyz[3 * t + 2] = z;
#pragma unroll
        for (int k = 0; k < 3; k++) o.scale[3 * t + k] = expf(a.scale_raw[3 * t + k]);
        const float4 q = *reinterpret_cast<const float4*>(a.rot_raw + 4 * t);
        const float n = sqrtf(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w);
        const float d = fmaxf(n, ACT_NORM_EPS);
        *reinterpret_cast<float4*>(o.rot + 4 * t) = make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
        o.op[t] = act_sigmoid(a.op_raw[t]);
    }
    if (t < a.Nfg) {
#pragma unroll
        for (int k = 0; k < 3; k++) o.alb[3 * t + k] = act_sigmoid(a.alb_raw[3 * t + k]);
        o.rough[t] = act_sigmoid(a.rough_raw[t]);
        o.metal[t] = act_sigmoid(a.metal_raw[t]);
    }
}

// upstream gradients g (any may be null: zero) of the activations o -> the raw parameters'
// gradients d (written, not added), with torch's backward formulas: exp: g y; sigmoid:
// g (1 - y) y; normalize (y = x / max(|x|, eps)): g / d - x (g . x) / d^2 / |x| (the second
// term only when |x| > eps); shell: d angles zero where clamped, per-workgroup partials of
// d radius (k_sum_into adds them)
__global__ void __launch_bounds__(256) k_activations_bwd(ActArgs a, ActOut o, ActOut g, ActGrad d) {
    __shared__ float red[4];
    const int t = blockIdx.x * 256 + threadIdx.x;
    float drad = 0.f;
    if (t < a.P) {
        const int r = a.src ? a.src[t] : (t < a.Nfg ? t : -1 - (t - a.Nfg));
        const float gx = g.xyz ? g.xyz[3 * t] : 0.f, gy = g.xyz ? g.xyz[3 * t + 1] : 0.f,
                    gz = g.xyz ? g.xyz[3 * t + 2] : 0.f;
        if (r >= 0) {
            d.xyz_fg[3 * r] = gx;
            d.xyz_fg[3 * r + 1] = gy;
            d.xyz_fg[3 * r + 2] = gz;
        } else {
            const int j = -1 - r;
            const float t0 = a.angles[2 * j], p0 = a.angles[2 * j + 1];
            const float th = fminf(fmaxf(t0, 0.f), SKY_HALF_PI), ph = fminf(fmaxf(p0, -SKY_HALF_PI), SKY_HALF_PI);
            const float rad = a.radius[0];
            const float st = sinf(th), ct = cosf(th), sp = sinf(ph), cp = cosf(ph);
            drad = (gx * (st * sp) + gy * (-ct)) + gz * (st * cp);
            const float dt = rad * ((gx * (ct * sp) + gy * st) + gz * (ct * cp));
            const float dp = rad * (gx * (st * cp) - gz * (st * sp));
            d.angles[2 * j] = (t0 >= 0.f && t0 <= SKY_HALF_PI) ? dt : 0.f;
            d.angles[2 * j + 1] = (p0 >= -SKY_HALF_PI && p0 <= SKY_HALF_PI) ? dp : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) d.scale_raw[3 * t + k] = g.scale ? g.scale[3 * t + k] * o.scale[3 * t + k] : 0.f;
        if (g.rot) {
            const float4 x = *reinterpret_cast<const float4*>(a.rot_raw + 4 * t);
            const float4 gr = *reinterpret_cast<const float4*>(g.rot + 4 * t);
            const float n = sqrtf(((x.x * x.x + x.y * x.y) + x.z * x.z) + x.w * x.w);
            const float dd = fmaxf(n, ACT_NORM_EPS);
            const float c = n > ACT_NORM_EPS ? (((gr.x * x.x + gr.y * x.y) + gr.z * x.z) + gr.w * x.w) / (dd * dd) / n : 0.f;
            *reinterpret_cast<float4*>(d.rot_raw + 4 * t) =
                make_float4(gr.x / dd - x.x * c, gr.y / dd - x.y * c, gr.z / dd - x.z * c, gr.w / dd - x.w * c);
        } else {
            *reinterpret_cast<float4*>(d.rot_raw + 4 * t) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        d.op_raw[t] = g.op ? g.op[t] * (1.f - o.op[t]) * o.op[t] : 0.f;
    }
    if (t < a.Nfg) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float y = o.alb[3 * t + k];
            d.alb_raw[3 * t + k] = g.alb ? g.alb[3 * t + k] * (1.f - y) * y : 0.f;
        }
        d.rough_raw[t] = g.rough ? g.rough[t] * (1.f - o.rough[t]) * o.rough[t] : 0.f;
        d.metal_raw[t] = g.metal ? g.metal[t] * (1.f - o.metal[t]) * o.metal[t] : 0.f;
    }
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) drad += __shfl_xor(drad, k, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = drad;
    __syncthreads();
    if (threadIdx.x == 0 && d.radius_part) d.radius_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = the sum of n partials in a fixed order (one workgroup)
__global__ void __launch_bounds__(256) k_sum_into(int n, const float* __restrict__ part, float* __restrict__ out) {
    __shared__ float red[4];
    float v = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) v += part[i];
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) v += __shfl_xor(v, k, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

int activation_blocks(const ActArgs& a) {
    const int n = a.P > a.Nfg ? a.P : a.Nfg;
    return (n + 255) / 256;
}

void launch_activations_fwd(const ActArgs& a, const ActOutW& o, hipStream_t s) {
    hipLaunchKernelGGL(k_activations_fwd, dim3(activation_blocks(a)), dim3(256), 0, s, a, o);
}

void launch_activations_bwd(const ActArgs& a, const ActOut& o, const ActOut& g, const ActGrad& d, float* d_radius,
                            hipStream_t s) {
    const int nb = activation_blocks(a);
    hipLaunchKernelGGL(k_activations_bwd, dim3(nb), dim3(256), 0, s, a, o, g, d);
    if (d.radius_part && d_radius) hipLaunchKernelGGL(k_sum_into, dim3(1), dim3(256), 0, s, nb, d.radius_part, d_radius);
}

// ---- the regularisers' per-view scalar tail (gsr/train.py view_regularisers) ---------------
// From the per-view sums [V][5] (k_view_regs_fwd), the SH basis at the envlight directions
// [V*NS][25] and the environment SH [V][25][3]: total[v] = el + ls ms + (depth_on) ld dl, with
// ms = S2 / S0, dl = exp(-gamma (S3 / S1 - S4 / S0)) (the foreground mean detached), and el
// the mean squared negative part of vals = basis . env (0 when none is negative), as the
// PyTorch composition it replaces; one workgroup, V <= 8, NS <= 32.
constexpr int TAIL_K = 25;

__device__ __forceinline__ void tail_vals(const RegsTail& t, float* vals, float* cnt, float* sq) {
    // vals [V][NS][3] and per view the negative count and sum of squares (LDS), 256 threads
    for (int i = threadIdx.x; i < t.V * t.NS * 3; i += 256) {
        const int v = i / (t.NS * 3), r = i - v * t.NS * 3, n = r / 3, c = r - 3 * n;
        const float* b = t.basis + ((size_t)v * t.NS + n) * TAIL_K;
        const float* e = t.env + (size_t)v * TAIL_K * 3 + c;
        float a = 0.f;
        for (int k = 0; k < TAIL_K; k++) a = __builtin_fmaf(b[k], e[3 * k], a);
        vals[i] = a;
    }
    __syncthreads();
    if (threadIdx.x < t.V) {
        const int v = threadIdx.x;
        float nn = 0.f, q = 0.f;
        for (int j = 0; j < t.NS * 3; j++) {
            const float x = vals[v * t.NS * 3 + j];
            if (x < 0.f) {
                nn += 1.f;
                q += x * x;
            }
        }
        cnt[v] = nn;
        sq[v] = q;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_regs_tail_fwd(RegsTail t, float* __restrict__ total) {
    __shared__ float vals[8 * 32 * 3], cnt[8], sq[8];
    tail_vals(t, vals, cnt, sq);
    if (threadIdx.x < t.V) {
        const int v = threadIdx.x;
        const float* S = t.sums + 5 * v;
        const float ms = S[2] / S[0];
        const float dl = expf(-t.gamma * (S[3] / S[1] - S[4] / S[0]));
        const float el = cnt[v] > 0.f ? sq[v] / fmaxf(cnt[v], 1.f) : 0.f;
        float tot = 0.f;
        if (t.lam_env > 0.f) tot = tot + el;
        if (t.lam_scale > 0.f) tot = tot + t.lam_scale * ms;
        if (t.depth_on && t.lam_depth > 0.f) tot = tot + t.lam_depth * dl;
        total[v] = tot;
    }
}

// g [V]: dL/dtotal.  d_sums [V][5] (the counts and the detached foreground depth get 0),
// d_env [V][25][3]
__global__ void __launch_bounds__(256) k_regs_tail_bwd(RegsTail t, const float* __restrict__ g,
                                                       float* __restrict__ d_sums, float* __restrict__ d_env) {
    __shared__ float vals[8 * 32 * 3], cnt[8], sq[8];
    tail_vals(t, vals, cnt, sq);
    if (threadIdx.x < t.V) {
        const int v = threadIdx.x;
        const float* S = t.sums + 5 * v;
        const float gv = g[v];
        const float dl = expf(-t.gamma * (S[3] / S[1] - S[4] / S[0]));
        float* D = d_sums + 5 * v;
        D[0] = 0.f;
        D[1] = 0.f;
        D[2] = t.lam_scale > 0.f ? t.lam_scale * gv / S[0] : 0.f;
        D[3] = (t.depth_on && t.lam_depth > 0.f) ? (t.lam_depth * gv) * dl * -t.gamma / S[1] : 0.f;
        D[4] = 0.f;
    }
    // d vals = g 2 x / n on the negative entries; d env[k][c] = sum_n basis[n][k] d vals[n][c]
    for (int i = threadIdx.x; i < t.V * TAIL_K * 3; i += 256) {
        const int v = i / (TAIL_K * 3), r = i - v * TAIL_K * 3, k = r / 3, c = r - 3 * k;
        float a = 0.f;
        if (t.lam_env > 0.f && cnt[v] > 0.f) {
            const float s = g[v] / fmaxf(cnt[v], 1.f);
            for (int n = 0; n < t.NS; n++) {
                const float x = vals[(v * t.NS + n) * 3 + c];
                a = __builtin_fmaf(t.basis[((size_t)v * t.NS + n) * TAIL_K + k], x < 0.f ? 2.f * x * s : 0.f, a);
            }
        }
        d_env[i] = a;
    }
}

void launch_regs_tail_fwd(const RegsTail& t, float* total, hipStream_t s) {
    hipLaunchKernelGGL(k_regs_tail_fwd, dim3(1), dim3(256), 0, s, t, total);
}
void launch_regs_tail_bwd(const RegsTail& t, const float* g, float* d_sums, float* d_env, hipStream_t s) {
    hipLaunchKernelGGL(k_regs_tail_bwd, dim3(1), dim3(256), 0, s, t, g, d_sums, d_env);
}

int view_regs_blocks(int P) {
    const int b = (P + REG_THREADS * 8 - 1) / (REG_THREADS * 8);
    return b < 1 ? 1 : (b > 2048 ? 2048 : b);
}

void launch_view_regs_fwd(int P, int V, const float* xyz, const float* scaling, const ViewPtrs<int>& radii,
                          const unsigned char* is_sky, const float* dcol, float* partials, hipStream_t s) {
    hipLaunchKernelGGL(k_view_regs_fwd, dim3(view_regs_blocks(P)), dim3(REG_THREADS), 0, s, P, V, xyz, scaling, radii,
                       is_sky, dcol, partials);
}

void launch_view_regs_bwd(int P, int V, const float* scaling, const ViewPtrs<int>& radii, const unsigned char* is_sky,
                          const float* dcol, const float* g, float* d_xyz, float* d_scaling, unsigned acc,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_view_regs_bwd, dim3((P + REG_THREADS - 1) / REG_THREADS), dim3(REG_THREADS), 0, s, P, V,
                       scaling, radii, is_sky, dcol, g, d_xyz, d_scaling, acc);
}

void launch_densify_stats(int P, int V, const ViewPtrs<float>& g2d, const ViewPtrs<int>& radii, float* accum,
                          float* denom, float* maxr, hipStream_t s) {
    hipLaunchKernelGGL(k_densify_stats, dim3((P + 255) / 256), dim3(256), 0, s, P, V, g2d, radii, accum, denom, maxr);
}

void launch_sh_basis(int N, int deg, const float* dirs, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_basis, dim3((N + 63) / 64), dim3(64), 0, s, N, deg, dirs, out);
}

int sky_blocks(int N) { return (N + 255) / 256; }

void launch_sky_xyz_fwd(int N, const float* ang, const float* radius, const float* center, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_sky_xyz_fwd, dim3(sky_blocks(N)), dim3(256), 0, s, N, ang, radius, center, out);
}

void launch_sky_xyz_bwd(int N, const float* ang, const float* radius, const float* g, float* d_ang, float* d_rad_part,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_sky_xyz_bwd, dim3(sky_blocks(N)), dim3(256), 0, s, N, ang, radius, g, d_ang, d_rad_part);
}

}  // namespace gsr
