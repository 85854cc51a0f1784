// refalgo.hip -- the reference rasterizer's ALGORITHM STRUCTURE on gfx950, as a measured
// GPU baseline (BASELINE.md §2 "reference-algorithm GPU path").  Not the product: the
// product is relightable3dgaussians-w_amd/csrc (libgsr.so).  This library exists so that
// bench.py can time "the reference rasterizer on an MI355X" next to the gfx950 design.
// The reference CUDA code cannot be built or run here, so this file
// re-creates its stage structure in plain HIP:
//
//   forward  (rasterizer_impl.cu:198-336)
//     preprocess                one thread per Gaussian            [shared with libgsr, see below]
//     inclusive scan            hipcub::DeviceScan::InclusiveSum   (rasterizer_impl.cu:276-281)
//     num_rendered              one blocking D2H copy              (:281)
//     duplicateWithKeys         one thread per Gaussian, R 64-bit (tile << 32 | depth) keys (:70-111)
//     radix sort                hipcub::DeviceRadixSort::SortPairs on bits [0, 32 + msb(T)) (:300-308)
//     identifyTileRanges        memset + one thread per instance   (:116-138, :310-318)
//     render                    16x16 blocks, one thread per pixel, rounds of 256 Gaussians
//                               staged in shared memory, __syncthreads_count early exit
//                               (forward.cu:261-374)
//   backward (backward.cu)
//     zero-fill of the gradient accumulators                      (rasterize_points.cu:153-161)
//     render backward           16x16 blocks, one thread per pixel, back to front, shared
//                               staging incl. colours, 9 global float atomics per
//                               contributing (pixel, Gaussian) pair (backward.cu:399-557)
//     cov2D + preprocess bwd    one thread per Gaussian            [shared with libgsr]
//
// The per-Gaussian stages reuse libgsr's one-thread-per-Gaussian kernels (launch_preprocess,
// launch_preprocess_bwd): the reference's are the same design with more arrays stored, so
// sharing them can only make this baseline faster than a faithful one.  Likewise the
// render backward's 9 atomics land in libgsr's 64-B accumulator line instead of four
// separate arrays (same atomic count, better locality).  The baseline is therefore an
// upper bound on the reference structure's speed on MI355X; speed-ups quoted against it
// are lower bounds.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "gsr_kernels.hpp"

#define REF_BLOCK 16
#define REF_PIX 256

namespace {

// rasterizer_impl.cu:35-50: bits needed to hold the largest tile id
uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

__global__ void k_dup_keys(int P, const int* radii, const uint32_t* offsets, const uint2* rect,
                           const uint32_t* depth_key, unsigned gx, uint64_t* keys, uint32_t* vals) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P || radii[idx] <= 0) return;
    uint32_t off = idx == 0 ? 0u : offsets[idx - 1];
    const uint2 r = rect[idx];
    const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
    const uint64_t d = depth_key[idx];
    for (uint32_t y = y0; y < y1; y++)
        for (uint32_t x = x0; x < x1; x++) {
            keys[off] = ((uint64_t)(y * gx + x) << 32) | d;
            vals[off] = (uint32_t)idx;
            off++;
        }
}

__global__ void k_tile_ranges(int R, const uint64_t* keys, uint2* ranges) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const uint32_t t = (uint32_t)(keys[i] >> 32);
    if (i == 0) ranges[t].x = 0;
    else {
        const uint32_t p = (uint32_t)(keys[i - 1] >> 32);
        if (t != p) {
            ranges[p].y = i;
            ranges[t].x = i;
        }
    }
    if (i == R - 1) ranges[t].y = R;
}

__global__ void __launch_bounds__(REF_PIX) k_render_fwd(int W, int H, unsigned gx, const uint2* ranges,
                                                        const uint32_t* point_list, const gsr::Rec* rec,
                                                        const float* bg, float* final_T, uint32_t* n_contrib,
                                                        float* out) {
    const uint32_t px = blockIdx.x * REF_BLOCK + threadIdx.x % REF_BLOCK;
    const uint32_t py = blockIdx.y * REF_BLOCK + threadIdx.x / REF_BLOCK;
    const uint32_t pix = W * py + px;
    const float2 pixf = make_float2((float)px, (float)py);
    const bool inside = px < (uint32_t)W && py < (uint32_t)H;
    bool done = !inside;
    const uint2 range = ranges[blockIdx.y * gx + blockIdx.x];
    const int rounds = ((int)(range.y - range.x) + REF_PIX - 1) / REF_PIX;
    int todo = range.y - range.x;

    __shared__ int s_id[REF_PIX];
    __shared__ float2 s_xy[REF_PIX];
    __shared__ float4 s_co[REF_PIX];
    float T = 1.0f;
    uint32_t contributor = 0, last_contributor = 0;
    float C[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < rounds; i++, todo -= REF_PIX) {
        if (__syncthreads_count(done) == REF_PIX) break;
        const int progress = i * REF_PIX + threadIdx.x;
        if (range.x + progress < range.y) {
            const int id = point_list[range.x + progress];
            const gsr::Rec r = rec[id];
            s_id[threadIdx.x] = id;
            s_xy[threadIdx.x] = make_float2(r.a.x, r.a.y);
            s_co[threadIdx.x] = make_float4(r.a.z, r.a.w, r.b.x, r.b.y);
        }
        __syncthreads();
        const int n = todo < REF_PIX ? todo : REF_PIX;
        for (int j = 0; !done && j < n; j++) {
            contributor++;
            const float2 xy = s_xy[j];
            const float dx = xy.x - pixf.x, dy = xy.y - pixf.y;
            const float4 co = s_co[j];
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, co.w * expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            // colours from global memory, as the reference's features[] (forward.cu:350)
            const gsr::Rec& g = rec[s_id[j]];
            const float w = alpha * T;
            C[0] += g.b.z * w;
            C[1] += g.b.w * w;
            C[2] += g.c.x * w;
            T = test_T;
            last_contributor = contributor;
        }
    }
    if (inside) {
        final_T[pix] = T;
        n_contrib[pix] = last_contributor;
        for (int ch = 0; ch < 3; ch++) out[ch * H * W + pix] = C[ch] + T * bg[ch];
    }
}

__global__ void __launch_bounds__(REF_PIX) k_render_bwd(int W, int H, unsigned gx, const uint2* ranges,
                                                        const uint32_t* point_list, const gsr::Rec* rec,
                                                        const float* bg, const float* final_T,
                                                        const uint32_t* n_contrib, const float* dL_dpix, float* acc) {
    const uint32_t px = blockIdx.x * REF_BLOCK + threadIdx.x % REF_BLOCK;
    const uint32_t py = blockIdx.y * REF_BLOCK + threadIdx.x / REF_BLOCK;
    const uint32_t pix = W * py + px;
    const float2 pixf = make_float2((float)px, (float)py);
    const bool inside = px < (uint32_t)W && py < (uint32_t)H;
    const uint2 range = ranges[blockIdx.y * gx + blockIdx.x];
    const int rounds = ((int)(range.y - range.x) + REF_PIX - 1) / REF_PIX;
    bool done = !inside;
    int todo = range.y - range.x;

    __shared__ int s_id[REF_PIX];
    __shared__ float2 s_xy[REF_PIX];
    __shared__ float4 s_co[REF_PIX];
    __shared__ float s_col[3 * REF_PIX];

    const float T_final = inside ? final_T[pix] : 0.f;
    float T = T_final;
    uint32_t contributor = todo;
    const uint32_t last_contributor = inside ? n_contrib[pix] : 0u;
    float accum_rec[3] = {0.f, 0.f, 0.f}, dpix[3] = {0.f, 0.f, 0.f}, last_color[3] = {0.f, 0.f, 0.f};
    if (inside)
        for (int ch = 0; ch < 3; ch++) dpix[ch] = dL_dpix[ch * H * W + pix];
    float last_alpha = 0.f;
    const float ddelx = 0.5f * W, ddely = 0.5f * H;

    for (int i = 0; i < rounds; i++, todo -= REF_PIX) {
        __syncthreads();
        const int progress = i * REF_PIX + threadIdx.x;
        if (range.x + progress < range.y) {
            const int id = point_list[range.y - progress - 1];
            const gsr::Rec r = rec[id];
            s_id[threadIdx.x] = id;
            s_xy[threadIdx.x] = make_float2(r.a.x, r.a.y);
            s_co[threadIdx.x] = make_float4(r.a.z, r.a.w, r.b.x, r.b.y);
            s_col[threadIdx.x] = r.b.z;
            s_col[REF_PIX + threadIdx.x] = r.b.w;
            s_col[2 * REF_PIX + threadIdx.x] = r.c.x;
        }
        __syncthreads();
        const int n = todo < REF_PIX ? todo : REF_PIX;
        for (int j = 0; !done && j < n; j++) {
            contributor--;
            if (contributor >= last_contributor) continue;
            const float2 xy = s_xy[j];
            const float dx = xy.x - pixf.x, dy = xy.y - pixf.y;
            const float4 co = s_co[j];
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            if (power > 0.0f) continue;
            const float G = expf(power);
            const float alpha = fminf(0.99f, co.w * G);
            if (alpha < 1.0f / 255.0f) continue;
            T = T / (1.f - alpha);
            const float dchannel_dcolor = alpha * T;
            float dL_dalpha = 0.0f;
            const int gid = s_id[j];
            float* line = acc + (size_t)gid * gsr::ACC_STRIDE;
            for (int ch = 0; ch < 3; ch++) {
                const float c = s_col[ch * REF_PIX + j];
                accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                last_color[ch] = c;
                dL_dalpha += (c - accum_rec[ch]) * dpix[ch];
                atomicAdd(line + 6 + ch, dchannel_dcolor * dpix[ch]);
            }
            dL_dalpha *= T;
            last_alpha = alpha;
            float bg_dot = 0.f;
            for (int ch = 0; ch < 3; ch++) bg_dot += bg[ch] * dpix[ch];
            dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
            const float dL_dG = co.w * dL_dalpha;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * co.x - gdy * co.y;
            const float dG_ddely = -gdy * co.z - gdx * co.y;
            atomicAdd(line + 0, dL_dG * dG_ddelx * ddelx);
            atomicAdd(line + 1, dL_dG * dG_ddely * ddely);
            atomicAdd(line + 2, -0.5f * gdx * dx * dL_dG);
            atomicAdd(line + 3, -0.5f * gdx * dy * dL_dG);
            atomicAdd(line + 4, -0.5f * gdy * dy * dL_dG);
            atomicAdd(line + 5, G * dL_dalpha);
        }
    }
}

struct Grow {
    void* p = nullptr;
    size_t n = 0;
    void* get(size_t need) {
        if (need > n) {
            if (p) (void)hipFree(p);
            p = nullptr;
            n = 0;
            if (hipMalloc(&p, need) != hipSuccess) return nullptr;
            n = need;
        }
        return p;
    }
};

}  // namespace

struct GsrRefCtx {
    Grow geom_rec, geom_aux, keys, vals, keys_alt, vals_alt, sort_tmp, scan_tmp, img, acc, shjac;
    int P = 0, W = 0, H = 0, R = 0;
    float* final_T = nullptr;
    uint32_t* n_contrib = nullptr;
    uint2* ranges = nullptr;
    uint32_t* point_list = nullptr;
    gsr::Rec* rec = nullptr;
    char err[256] = {0};
};

namespace {
int ref_fail(GsrRefCtx* c, const char* msg, int code = -1) {
    snprintf(c->err, sizeof(c->err), "%s", msg);
    return code;
}
#define REF_HIP(x)                                                                     \
    do {                                                                               \
        hipError_t _e = (x);                                                           \
        if (_e != hipSuccess) return ref_fail(ctx, hipGetErrorString(_e), -2);         \
    } while (0)
size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

extern "C" {

GsrRefCtx* gsr_ref_create() { return new GsrRefCtx(); }

void gsr_ref_destroy(GsrRefCtx* c) {
    if (!c) return;
    for (Grow* g : {&c->geom_rec, &c->geom_aux, &c->keys, &c->vals, &c->keys_alt, &c->vals_alt, &c->sort_tmp,
                    &c->scan_tmp, &c->img, &c->acc})
        if (g->p) (void)hipFree(g->p);
    delete c;
}

const char* gsr_ref_last_error(GsrRefCtx* c) { return c ? c->err : "null context"; }

// Forward: out_color [3,H,W], radii [P]; returns num_rendered via *num_rendered.
int gsr_ref_forward(GsrRefCtx* ctx, void* stream, int P, int D, int M, const float* bg, int W, int H,
                    const float* means3D, const float* shs, const float* colors_precomp, const float* opacities,
                    const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                    const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                    float tan_fovy, float* out_color, int* radii, int* num_rendered) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    *num_rendered = 0;
    ctx->P = P; ctx->W = W; ctx->H = H; ctx->R = 0;
    const unsigned gx = (W + REF_BLOCK - 1) / REF_BLOCK, gy = (H + REF_BLOCK - 1) / REF_BLOCK;
    const size_t T = (size_t)gx * gy, npix = (size_t)W * H;
    // image state: final_T, n_contrib, ranges
    char* img = (char*)ctx->img.get(al(4 * npix) + al(4 * npix) + al(8 * T));
    if (!img) return ref_fail(ctx, "alloc img");
    ctx->final_T = (float*)img;
    ctx->n_contrib = (uint32_t*)(img + al(4 * npix));
    ctx->ranges = (uint2*)(img + 2 * al(4 * npix));
    REF_HIP(hipMemsetAsync(out_color, 0, 12 * npix, s));
    if (P == 0) return 0;
    // geometry state
    ctx->rec = (gsr::Rec*)ctx->geom_rec.get(sizeof(gsr::Rec) * (size_t)P);
    const size_t naux = 4 * al(4 * (size_t)P) + al(8 * (size_t)P);
    char* aux = (char*)ctx->geom_aux.get(naux);
    if (!ctx->rec || !aux) return ref_fail(ctx, "alloc geom");
    uint32_t* tiles = (uint32_t*)aux;
    uint32_t* offsets = (uint32_t*)(aux + al(4 * (size_t)P));
    uint32_t* st_count = (uint32_t*)(aux + 2 * al(4 * (size_t)P));
    uint32_t* depth_key = (uint32_t*)(aux + 3 * al(4 * (size_t)P));
    uint2* rect = (uint2*)(aux + 4 * al(4 * (size_t)P));

    gsr::PreprocessArgs pa{};
    memset(&pa, 0, sizeof(pa));
    pa.P = P; pa.D = D; pa.M = M;
    pa.means3D = means3D; pa.scales = scales; pa.scale_modifier = scale_modifier; pa.rotations = rotations;
    pa.opacities = opacities; pa.shs = shs; pa.cov3D_precomp = cov3D_precomp; pa.colors_precomp = colors_precomp;
    pa.viewmatrix = viewmatrix; pa.projmatrix = projmatrix; pa.campos = campos;
    pa.W = W; pa.H = H; pa.tan_fovx = tan_fovx; pa.tan_fovy = tan_fovy;
    pa.focal_x = W / (2.0f * tan_fovx); pa.focal_y = H / (2.0f * tan_fovy);
    pa.grid_x = gx; pa.grid_y = gy; pa.prefiltered = 0;
    pa.radii = radii; pa.tiles = tiles; pa.st_count = st_count; pa.depth_key = depth_key; pa.rect = rect;
    pa.rec = ctx->rec;  // blk_tot / hist0 null: this baseline scans tiles_touched itself
    pa.shjac = (shs && !colors_precomp) ? (float*)ctx->shjac.get(sizeof(float) * gsr::SHJAC_ROWS * (size_t)P) : nullptr;
    gsr::launch_preprocess(pa, s);

    size_t scan_bytes = 0;
    REF_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, tiles, offsets, P, s));
    void* scan_tmp = ctx->scan_tmp.get(scan_bytes);
    if (!scan_tmp) return ref_fail(ctx, "alloc scan");
    REF_HIP(hipcub::DeviceScan::InclusiveSum(scan_tmp, scan_bytes, tiles, offsets, P, s));
    uint32_t R = 0;
    REF_HIP(hipMemcpyAsync(&R, offsets + P - 1, 4, hipMemcpyDeviceToHost, s));
    REF_HIP(hipStreamSynchronize(s));
    ctx->R = (int)R;
    *num_rendered = (int)R;
    REF_HIP(hipMemsetAsync(ctx->ranges, 0, 8 * T, s));
    if (R == 0) {
        ctx->point_list = nullptr;
    } else {
        uint64_t* k0 = (uint64_t*)ctx->keys.get(8 * (size_t)R);
        uint32_t* v0 = (uint32_t*)ctx->vals.get(4 * (size_t)R);
        uint64_t* k1 = (uint64_t*)ctx->keys_alt.get(8 * (size_t)R);
        uint32_t* v1 = (uint32_t*)ctx->vals_alt.get(4 * (size_t)R);
        if (!k0 || !v0 || !k1 || !v1) return ref_fail(ctx, "alloc binning");
        hipLaunchKernelGGL(k_dup_keys, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, offsets, rect, depth_key,
                           gx, k0, v0);
        const int bit = (int)higher_msb((uint32_t)T);
        size_t sort_bytes = 0;
        REF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, k0, k1, v0, v1, (int)R, 0, 32 + bit, s));
        void* sort_tmp = ctx->sort_tmp.get(sort_bytes);
        if (!sort_tmp) return ref_fail(ctx, "alloc sort");
        REF_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp, sort_bytes, k0, k1, v0, v1, (int)R, 0, 32 + bit, s));
        hipLaunchKernelGGL(k_tile_ranges, dim3((R + 255) / 256), dim3(256), 0, s, (int)R, k1, ctx->ranges);
        ctx->point_list = v1;
    }
    hipLaunchKernelGGL(k_render_fwd, dim3(gx, gy), dim3(REF_PIX), 0, s, W, H, gx, ctx->ranges, ctx->point_list,
                       ctx->rec, bg, ctx->final_T, ctx->n_contrib, out_color);
    REF_HIP(hipGetLastError());
    return 0;
}

// Backward of the last forward on this context; output arrays as the reference's
// rasterize_gaussians_backward (dL_dsh may be null when M == 0).
int gsr_ref_backward(GsrRefCtx* ctx, void* stream, int D, int M, const float* bg, const float* means3D,
                     const float* shs, const float* scales, float scale_modifier, const float* rotations,
                     const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                     const float* campos, float tan_fovx, float tan_fovy, const int* radii, const float* dL_dpix,
                     float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D,
                     float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int P = ctx->P, W = ctx->W, H = ctx->H;
    if (P == 0) return 0;
    const unsigned gx = (W + REF_BLOCK - 1) / REF_BLOCK, gy = (H + REF_BLOCK - 1) / REF_BLOCK;
    float* acc = (float*)ctx->acc.get(sizeof(float) * gsr::ACC_STRIDE * (size_t)P);
    if (!acc) return ref_fail(ctx, "alloc acc");
    REF_HIP(hipMemsetAsync(acc, 0, sizeof(float) * gsr::ACC_STRIDE * (size_t)P, s));
    if (ctx->R > 0)
        hipLaunchKernelGGL(k_render_bwd, dim3(gx, gy), dim3(REF_PIX), 0, s, W, H, gx, ctx->ranges, ctx->point_list,
                           ctx->rec, bg, ctx->final_T, ctx->n_contrib, dL_dpix, acc);
    gsr::PreprocessBwdArgs pb;
    memset(&pb, 0, sizeof(pb));
    pb.P = P; pb.D = D; pb.M = M;
    pb.means3D = means3D; pb.radii = radii; pb.shs = shs; pb.scales = scales; pb.rotations = rotations;
    pb.scale_modifier = scale_modifier; pb.cov3D_precomp = cov3D_precomp;
    pb.viewmatrix = viewmatrix; pb.projmatrix = projmatrix; pb.campos = campos;
    pb.tan_fovx = tan_fovx; pb.tan_fovy = tan_fovy;
    pb.focal_x = W / (2.0f * tan_fovx); pb.focal_y = H / (2.0f * tan_fovy);
    pb.acc = acc;
    pb.shjac = (const float*)ctx->shjac.get(sizeof(float) * gsr::SHJAC_ROWS * (size_t)P);
    pb.dL_dmean2D = dL_dmean2D; pb.dL_dconic = dL_dconic; pb.dL_dopacity = dL_dopacity; pb.dL_dcolor = dL_dcolor;
    pb.dL_dmean3D = dL_dmean3D; pb.dL_dcov3D = dL_dcov3D; pb.dL_dsh = M > 0 ? dL_dsh : nullptr;
    pb.dL_dscale = dL_dscale; pb.dL_drot = dL_drot;
    gsr::launch_preprocess_bwd(pb, s);
    REF_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
