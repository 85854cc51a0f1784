// gsr_preprocess.hip -- forward per-Gaussian preprocess (forward.cu:155-256) and
// checkFrustum (rasterizer_impl.cu:54-66), re-designed for gfx950:
//  * one thread per Gaussian, 256-thread blocks (4 waves of 64);
//  * camera matrices are wave-uniform scalar loads;
//  * output is one packed 48-B render record per Gaussian (Rec) + a 32-bit depth key
//    + a packed tile rect, so the binning and tile passes gather one row per Gaussian;
//  * FMA contraction is OFF in this TU: radii, rects, depths, conics and SH colours are
//    bit-identical to oracle/gsr_oracle.c (the reference's op order).
#pragma clang fp contract(off)
#include "gsr_exact.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

// LDS ordering within one wave (wave-private LDS rows)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One Gaussian's inputs, loaded up front (all of them unconditionally, so that a wave has
// every global load in flight at once instead of one dependent round trip per stage).
struct GaussIn {
    float3 p;
    float4 rot;
    float3 scale;
    float opacity;
    float3 col;
    float cov[6];
};

__device__ __forceinline__ void load_gauss(const PreprocessArgs& a, const int idx, GaussIn& g) {
    g.p = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    g.opacity = a.opacities[idx];
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) g.cov[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        g.rot = *reinterpret_cast<const float4*>(a.rotations + 4 * idx);
        g.scale = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
    }
    if (a.colors_precomp)
        g.col = make_float3(a.colors_precomp[3 * idx], a.colors_precomp[3 * idx + 1], a.colors_precomp[3 * idx + 2]);
}

// One Gaussian (forward.cu:155-256).  Every output is stored once; returns the tile and
// super-tile counts (0 when culled).
template <int MAXD = 3>
__device__ __forceinline__ void preprocess_one(const PreprocessArgs& a, const int idx, const GaussIn& g,
                                               uint32_t& tiles, uint32_t& stc, const float* sh_row, uint32_t& key_out,
                                               bool& err) {
    tiles = stc = 0;
    int irad = 0;
    uint32_t key = 0xFFFFFFFFu;  // culled Gaussians sort after every visible depth
    do {
        const float3 p_orig = g.p;
        // in_frustum (auxiliary.h:139-164): near cull only
        const float3 p_view = xform_point4x3(p_orig, a.viewmatrix);
        if (p_view.z <= 0.2f) {
            if (a.prefiltered) err = true;
            break;
        }
        const float4 p_hom = xform_point4x4(p_orig, a.projmatrix);
        const float p_w = 1.0f / (p_hom.w + 0.0000001f);
        const float3 p_proj = make_float3(p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w);

        float cov3[6];
        if (a.cov3D_precomp) {
#pragma unroll
            for (int i = 0; i < 6; i++) cov3[i] = g.cov[i];
        } else {
            cov3d_from(g.scale.x, g.scale.y, g.scale.z, a.scale_modifier, g.rot, cov3);
        }
        const float3 cov = cov2d_from(p_orig, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, cov3, a.viewmatrix);
        const float det = (cov.x * cov.z - cov.y * cov.y);
        if (det == 0.0f) break;
        const float det_inv = 1.f / det;
        const float3 conic = make_float3(cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv);
        const float mid = 0.5f * (cov.x + cov.z);
        const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        const float2 point_image = make_float2(ndc2pix(p_proj.x, a.W), ndc2pix(p_proj.y, a.H));
        uint2 rmin, rmax;
        const int r_ = f2i(my_radius);
        get_rect(point_image, r_, a.grid_x, a.grid_y, rmin, rmax);
        const unsigned area = (rmax.x - rmin.x) * (rmax.y - rmin.y);
        if (area == 0) break;

        float3 rgb;
        if (a.colors_precomp) {
            rgb = g.col;
        } else if (a.shs) {
            const float3 raw = sh_to_rgb_raw<MAXD>(a.D, p_orig, a.campos, sh_row);
            rgb = make_float3(raw.x < 0 ? 0.f : raw.x, raw.y < 0 ? 0.f : raw.y, raw.z < 0 ? 0.f : raw.z);
            if (a.shjac) {
                // the SH backward's view-direction Jacobian and clamp flags (backward.cu:20-139),
                // stored so the backward reads 40 B instead of the 12 M-byte SH row
                float3 dir = make_float3(p_orig.x - a.campos[0], p_orig.y - a.campos[1], p_orig.z - a.campos[2]);
                const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
                float ddx[3], ddy[3], ddz[3];
                sh_dir_jacobian<MAXD>(a.D, dir.x / len, dir.y / len, dir.z / len, sh_row, ddx, ddy, ddz);
                const float fl = __uint_as_float((raw.x < 0 ? 1u : 0u) | (raw.y < 0 ? 2u : 0u) | (raw.z < 0 ? 4u : 0u));
                const size_t P = (size_t)a.P;
                float* jp = a.shjac + idx;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    jp[(size_t)c * P] = ddx[c];
                    jp[(size_t)(3 + c) * P] = ddy[c];
                    jp[(size_t)(6 + c) * P] = ddz[c];
                }
                jp[9 * P] = fl;
            }
        } else {
            rgb = make_float3(0.f, 0.f, 0.f);  // multi-channel composite: features live outside the record
        }
        Rec r;
        r.a = make_float4(point_image.x, point_image.y, conic.x, conic.y);
        r.b = make_float4(conic.z, g.opacity, rgb.x, rgb.y);
        r.c = make_float4(rgb.z, __logf(255.0f * g.opacity), 0.f, 0.f);
        a.rec[idx] = r;
        a.rect[idx] = make_uint2(rmin.x | (rmax.x << 16), rmin.y | (rmax.y << 16));
        key = __float_as_uint(p_view.z);
        irad = r_;
        tiles = area;
        const unsigned sth = st_sth(a.grid_x, a.grid_y);
        stc = ((rmax.x + GSR_ST_W - 1) / GSR_ST_W - rmin.x / GSR_ST_W) *
              (((rmax.y + (1u << sth) - 1) >> sth) - (rmin.y >> sth));
    } while (false);
    if (irad == 0) {
        // culled: defaults into the record, rect and Jacobian rows nobody reads, so that every
        // cache line of them is written whole (a partly written line costs the memory a
        // read-modify-write when culled and visible Gaussians interleave)
        Rec r;
        r.a = r.b = r.c = make_float4(0.f, 0.f, 0.f, 0.f);
        a.rec[idx] = r;
        a.rect[idx] = make_uint2(0u, 0u);
        if (!a.colors_precomp && a.shs && a.shjac) {
            const size_t P = (size_t)a.P;
#pragma unroll
            for (int k = 0; k < SHJAC_ROWS; k++) a.shjac[(size_t)k * P + idx] = 0.f;
        }
    }
    a.depth_key[idx] = key;
    key_out = key;
    a.radii[idx] = irad;
    a.tiles[idx] = tiles;
    a.st_count[idx] = stc;
}

// Workgroup epilogue: the workgroup's totals (visible, R, S, error), a plain store -- no
// atomics and no zero-filled buffer: the depth sort's first histogram launch sums them.
__device__ __forceinline__ void preprocess_block_out(const PreprocessArgs& a, uint32_t tiles, uint32_t stc, bool err) {
    __shared__ uint32_t s_w[4][PRE_THREADS / 64];
    uint32_t v[4] = {tiles > 0 ? 1u : 0u, tiles, stc, err ? 1u : 0u};
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 4; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
        if (lane == 0) s_w[k][wave] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0 && a.blk_tot) {
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = s_w[k][0] + s_w[k][1] + s_w[k][2] + s_w[k][3];
        a.blk_tot[blockIdx.x] = make_uint4(t[0], t[1], t[2], t[3]);
    }
}

// Preprocess + the per-workgroup totals.
// The workgroup's SH rows (256 x M x 3 floats, contiguous) are first copied to LDS with
// 16-B coalesced loads (row stride M*3+1 against bank conflicts); each thread then reads
// its own row from LDS instead of 12 strided 16-B loads.
__global__ void __launch_bounds__(256) k_preprocess(PreprocessArgs a) {
    extern __shared__ float s_sh[];
    const int g0 = blockIdx.x * blockDim.x;
    const int idx = g0 + threadIdx.x;
    const int M3 = a.M * 3, stride = M3 + 1;
    const bool staged = a.shs && !a.colors_precomp;
    GaussIn gin;
    if (idx < a.P) load_gauss(a, idx, gin);  // issued before the SH staging: one wait for all
    if (staged) {
        const int rows = min((int)blockDim.x, a.P - g0);
        const float* src = a.shs + (size_t)g0 * M3;
        const int n = rows * M3;
        if ((M3 & 3) == 0) {
            const float4* s4 = reinterpret_cast<const float4*>(src);
            for (int f = threadIdx.x; f < (n >> 2); f += blockDim.x) {
                const float4 v = s4[f];
                const int e0 = f * 4, r = e0 / M3;
                float* d = s_sh + r * stride + (e0 - r * M3);
                d[0] = v.x;
                d[1] = v.y;
                d[2] = v.z;
                d[3] = v.w;
            }
        } else {
            for (int f = threadIdx.x; f < n; f += blockDim.x) {
                const int r = f / M3;
                s_sh[r * stride + f - r * M3] = src[f];
            }
        }
        __syncthreads();
    }
    uint32_t tiles = 0, stc = 0, key = 0;
    bool err = false;
    if (idx < a.P)
        preprocess_one(a, idx, gin, tiles, stc, staged ? s_sh + threadIdx.x * stride : nullptr, key, err);
    preprocess_block_out(a, tiles, stc, err);
}

// (Round 4 also measured the SH rows staged per wave through LDS with coalesced 16-B loads: its
// single call was faster -- preprocess 0.107 -> 0.094 ms at cfg2 -- but its 53 KB of LDS per
// workgroup starved the overlapping views' kernels and the default 3-stream bench dropped 3 %,
// profiles/r4zj_ab_preprocess_default_bench.txt.)
// SH path with M in {1, 4, 9, 16}: each thread loads its own SH row into registers with
// the other inputs (16-B loads when 3M is a multiple of 4) -- no LDS, so occupancy is
// bounded by registers only (16 coefficients: 102 vs 130 us at cfg2 against the
// LDS-staged k_preprocess, which serves any other M).
template <int M>
__global__ void __launch_bounds__(256) k_preprocess_regsh(PreprocessArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    GaussIn gin;
    float shr[3 * M];
    if (idx < a.P) {
        load_gauss(a, idx, gin);
        if constexpr ((3 * M) % 4 == 0) {
            const float4* s4 = reinterpret_cast<const float4*>(a.shs + (size_t)idx * 3 * M);
#pragma unroll
            for (int k = 0; k < 3 * M / 4; k++) {
                const float4 v = s4[k];  // (non-temporal here: the preprocess 0.107 -> 0.20 ms, r4zj)
                shr[4 * k] = v.x;
                shr[4 * k + 1] = v.y;
                shr[4 * k + 2] = v.z;
                shr[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3 * M; k++) shr[k] = a.shs[(size_t)idx * 3 * M + k];
        }
    }
    uint32_t tiles = 0, stc = 0, key = 0;
    bool err = false;
    if (idx < a.P)
        preprocess_one<(M >= 16 ? 3 : M >= 9 ? 2 : M >= 4 ? 1 : 0)>(a, idx, gin, tiles, stc, shr, key, err);
    preprocess_block_out(a, tiles, stc, err);
}

__global__ void __launch_bounds__(256) k_mark_visible(int P, const float* means3D, const float* viewmatrix,
                                                       bool* present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float3 p = make_float3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    present[idx] = !(xform_point4x3(p, viewmatrix).z <= 0.2f);
}

// Same geometry, new colours (the geometry cache across a render()'s rasterizer calls):
// copy each visible Gaussian's record with its colour replaced, and the radii.
__global__ void __launch_bounds__(256) k_recolor(int P, const int* radii_src, const Rec* src, const float* colors,
                                                  Rec* dst, int* radii_out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const int r = radii_src[idx];
    radii_out[idx] = r;
    if (r > 0) {
        Rec v = src[idx];
        v.b.z = colors[3 * idx];
        v.b.w = colors[3 * idx + 1];
        v.c.x = colors[3 * idx + 2];
        dst[idx] = v;
    }
}

void launch_recolor(int P, const int* radii_src, const Rec* src, const float* colors, Rec* dst, int* radii_out,
                    hipStream_t s) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_recolor, dim3((P + 255) / 256), dim3(256), 0, s, P, radii_src, src, colors, dst, radii_out);
}

void launch_preprocess(const PreprocessArgs& a, hipStream_t s) {
    if (a.P == 0) return;
    const int maxd = a.M >= 16 ? 3 : a.M >= 9 ? 2 : a.M >= 4 ? 1 : 0;
    if (a.shs && !a.colors_precomp && a.D <= maxd) {
        const dim3 grid((a.P + 255) / 256), blk(256);
        const bool al16 = (reinterpret_cast<uintptr_t>(a.shs) & 15u) == 0;
        switch (a.M) {
            case 1: hipLaunchKernelGGL(k_preprocess_regsh<1>, grid, blk, 0, s, a); return;
            case 4: if (al16) { hipLaunchKernelGGL(k_preprocess_regsh<4>, grid, blk, 0, s, a); return; } break;
            case 9: hipLaunchKernelGGL(k_preprocess_regsh<9>, grid, blk, 0, s, a); return;
            case 16:
                if (al16) { hipLaunchKernelGGL(k_preprocess_regsh<16>, grid, blk, 0, s, a); return; }
                break;
            default: break;
        }
    }
    const size_t lds = (a.shs && !a.colors_precomp) ? sizeof(float) * 256 * (size_t)(3 * a.M + 1) : 0;
    hipLaunchKernelGGL(k_preprocess, dim3((a.P + 255) / 256), dim3(256), lds, s, a);
}

void launch_mark_visible(int P, const float* means3D, const float* viewmatrix, bool* present, hipStream_t s) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, viewmatrix, present);
}

}  // namespace gsr
