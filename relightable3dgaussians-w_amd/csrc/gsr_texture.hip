// gsr_texture.hip -- 2D texture sampling with gradients: the operation nvdiffrast's
// `dr.texture(tex, uv, filter_mode, boundary_mode)` performs for the reference's live path
// (scene/NVDIFFREC/light.py:170, the split-sum FG LUT fetch; util.py:117 latlong maps).
// nvdiffrast is third-party (not vendored, unpinned); its published 2D semantics are
// restated here (parity unpinned beyond its call sites):
//
//   texel space   u' = u * w - 0.5, v' = v * h - 0.5 (texel centres at (i + 0.5) / size),
//                 wrap mode first takes u - floor(u);
//   clamp         u' clamped to [0, w - 1] before the floor, so outside the square the
//                 sample is the edge texel and its uv gradient is zero;
//   wrap          indices taken modulo the size;  zero: taps outside the square read 0;
//   linear        bilerp(t00, t10, t01, t11) = lerp(lerp(t00, t10, fu), lerp(t01, t11, fu), fv);
//   nearest       texel floor(u * w) (clamped / wrapped), no uv gradient.
//
// One thread per output pixel; a pixel's channels are contiguous (tex [nb][h][w][C]).
// HBM-bound on large lookups; the 512 KiB LUT stays resident in L2.
#include <hip/hip_runtime.h>

#include "gsr_common.hpp"

// evaluated in source order without FMA contraction, as the oracle (-ffp-contract=off):
// lookups and uv gradients are bit-identical to orc_texture2d
#pragma clang fp contract(off)

namespace gsr {

enum { TEX_NEAREST = 0, TEX_LINEAR = 1 };
enum { TEX_WRAP = 0, TEX_CLAMP = 1, TEX_ZERO = 2 };

struct TexTaps {
    int i00, i10, i01, i11;  // texel indices within one texture layer (-1 = reads zero)
    float fu, fv;
};

__device__ __forceinline__ TexTaps tex_taps_linear(float u, float v, int w, int h, int boundary) {
    if (boundary == TEX_WRAP) {
        u = u - floorf(u);
        v = v - floorf(v);
    }
    u = u * (float)w - 0.5f;
    v = v * (float)h - 0.5f;
    bool cu = false, cv = false;
    if (boundary == TEX_CLAMP) {
        u = fminf(fmaxf(u, 0.f), (float)(w - 1));
        v = fminf(fmaxf(v, 0.f), (float)(h - 1));
        cu = (u == 0.f || u == (float)(w - 1));
        cv = (v == 0.f || v == (float)(h - 1));
    }
    int iu0 = (int)floorf(u), iv0 = (int)floorf(v);
    int iu1 = iu0 + (cu ? 0 : 1), iv1 = iv0 + (cv ? 0 : 1);
    TexTaps t;
    t.fu = u - (float)iu0;
    t.fv = v - (float)iv0;
    if (boundary == TEX_WRAP) {
        if (iu0 < 0) iu0 += w;
        if (iv0 < 0) iv0 += h;
        if (iu1 >= w) iu1 -= w;
        if (iv1 >= h) iv1 -= h;
    }
    const bool u0o = iu0 < 0 || iu0 >= w, u1o = iu1 < 0 || iu1 >= w;
    const bool v0o = iv0 < 0 || iv0 >= h, v1o = iv1 < 0 || iv1 >= h;
    // clamp / wrap never leave the square; zero mode drops the taps that do
    t.i00 = (u0o || v0o) ? -1 : iv0 * w + iu0;
    t.i10 = (u1o || v0o) ? -1 : iv0 * w + iu1;
    t.i01 = (u0o || v1o) ? -1 : iv1 * w + iu0;
    t.i11 = (u1o || v1o) ? -1 : iv1 * w + iu1;
    return t;
}

__device__ __forceinline__ int tex_tap_nearest(float u, float v, int w, int h, int boundary) {
    if (boundary == TEX_WRAP) {
        u = u - floorf(u);
        v = v - floorf(v);
    }
    int iu = (int)floorf(u * (float)w), iv = (int)floorf(v * (float)h);
    if (boundary == TEX_CLAMP || boundary == TEX_WRAP) {  // wrap: u in [0,1) up to rounding at 1
        iu = min(max(iu, 0), w - 1);
        iv = min(max(iv, 0), h - 1);
    }
    return (iu < 0 || iu >= w || iv < 0 || iv >= h) ? -1 : iv * w + iu;
}

__device__ __forceinline__ float tex_at(const float* t, int i, int C, int c) { return i < 0 ? 0.f : t[(size_t)i * C + c]; }

__global__ void __launch_bounds__(256) k_texture_fwd(int n, int npix, int tex_nb, int h, int w, int C,
                                                     const float* __restrict__ tex, const float* __restrict__ uv,
                                                     int filter, int boundary, float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int b = i / npix;
    const float* t = tex + (size_t)(tex_nb == 1 ? 0 : b) * h * w * C;
    const float2 q = reinterpret_cast<const float2*>(uv)[i];
    float* o = out + (size_t)i * C;
    if (filter == TEX_NEAREST) {
        const int k = tex_tap_nearest(q.x, q.y, w, h, boundary);
        for (int c = 0; c < C; c++) o[c] = tex_at(t, k, C, c);
        return;
    }
    const TexTaps tp = tex_taps_linear(q.x, q.y, w, h, boundary);
    for (int c = 0; c < C; c++) {
        const float a00 = tex_at(t, tp.i00, C, c), a10 = tex_at(t, tp.i10, C, c);
        const float a01 = tex_at(t, tp.i01, C, c), a11 = tex_at(t, tp.i11, C, c);
        const float x0 = a00 + tp.fu * (a10 - a00);
        const float x1 = a01 + tp.fu * (a11 - a01);
        o[c] = x0 + tp.fv * (x1 - x0);
    }
}

__global__ void __launch_bounds__(256) k_texture_bwd(int n, int npix, int tex_nb, int h, int w, int C,
                                                     const float* __restrict__ tex, const float* __restrict__ uv,
                                                     int filter, int boundary, const float* __restrict__ dout,
                                                     float* __restrict__ d_uv, float* __restrict__ d_tex) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int b = i / npix;
    const size_t layer = (size_t)(tex_nb == 1 ? 0 : b) * h * w * C;
    const float* t = tex + layer;
    float* dt = d_tex ? d_tex + layer : nullptr;
    const float2 q = reinterpret_cast<const float2*>(uv)[i];
    const float* g = dout + (size_t)i * C;
    if (filter == TEX_NEAREST) {
        const int k = tex_tap_nearest(q.x, q.y, w, h, boundary);
        if (dt && k >= 0)
            for (int c = 0; c < C; c++) atomicAdd(dt + (size_t)k * C + c, g[c]);
        if (d_uv) reinterpret_cast<float2*>(d_uv)[i] = make_float2(0.f, 0.f);
        return;
    }
    const TexTaps tp = tex_taps_linear(q.x, q.y, w, h, boundary);
    float gu = 0.f, gv = 0.f;
    for (int c = 0; c < C; c++) {
        const float gc = g[c];
        const float a00 = tex_at(t, tp.i00, C, c), a10 = tex_at(t, tp.i10, C, c);
        const float a01 = tex_at(t, tp.i01, C, c), a11 = tex_at(t, tp.i11, C, c);
        gu += gc * ((a10 - a00) * (1.f - tp.fv) + (a11 - a01) * tp.fv);
        gv += gc * ((a01 - a00) * (1.f - tp.fu) + (a11 - a10) * tp.fu);
        if (dt) {
            const float wu0 = 1.f - tp.fu, wv0 = 1.f - tp.fv;
            if (tp.i00 >= 0) atomicAdd(dt + (size_t)tp.i00 * C + c, gc * wu0 * wv0);
            if (tp.i10 >= 0) atomicAdd(dt + (size_t)tp.i10 * C + c, gc * tp.fu * wv0);
            if (tp.i01 >= 0) atomicAdd(dt + (size_t)tp.i01 * C + c, gc * wu0 * tp.fv);
            if (tp.i11 >= 0) atomicAdd(dt + (size_t)tp.i11 * C + c, gc * tp.fu * tp.fv);
        }
    }
    if (d_uv) reinterpret_cast<float2*>(d_uv)[i] = make_float2(gu * (float)w, gv * (float)h);
}

void launch_texture_fwd(int nb, int npix, int tex_nb, int h, int w, int C, const float* tex, const float* uv,
                        int filter, int boundary, float* out, hipStream_t s) {
    const int n = nb * npix;
    if (n == 0) return;
    hipLaunchKernelGGL(k_texture_fwd, dim3((n + 255) / 256), dim3(256), 0, s, n, npix, tex_nb, h, w, C, tex, uv,
                       filter, boundary, out);
}

void launch_texture_bwd(int nb, int npix, int tex_nb, int h, int w, int C, const float* tex, const float* uv,
                        int filter, int boundary, const float* dout, float* d_uv, float* d_tex, hipStream_t s) {
    const int n = nb * npix;
    if (n == 0) return;
    hipLaunchKernelGGL(k_texture_bwd, dim3((n + 255) / 256), dim3(256), 0, s, n, npix, tex_nb, h, w, C, tex, uv,
                       filter, boundary, dout, d_uv, d_tex);
}

}  // namespace gsr
