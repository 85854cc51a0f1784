// gsr_preprocess_bwd.hip -- fused per-Gaussian backward: computeCov2DCUDA
// (backward.cu:144-274) + preprocessCUDA (backward.cu:346-396) with the SH backward
// (:20-139) and the cov3D backward (:278-341), plus the unpacking of the render
// backward's 64-B accumulator line into the reference's output tensors.
//
// One kernel instead of two + nine memsets: every output element is written here
// (zeros for culled Gaussians), so the caller's buffers need no zero-fill.  cov3D is
// recomputed with the forward's exact (contraction-off) code instead of being stored and
// re-read.  The SH part never reads the SH rows: the forward preprocess stored each visible
// Gaussian's d(colour)/d(view direction) and clamp flags (40 B, gsr_preprocess.hip), and
// dL/dsh = basis(dir) x dL/dcolour is written from the basis and the masked colour gradient
// staged per Gaussian in LDS (80 B) by a coalesced 16-B writer.
#pragma clang fp contract(off)
#include "gsr_exact.hpp"

#include "gsr_kernels.hpp"

namespace gsr {

// One Gaussian's inputs, all loads issued up front.
struct BwdIn {
    float4 l0, l1;  // accumulator line [0..8)
    float l2;       // [8]
    int radius;
    float3 mean;
    float4 rot;
    float3 scl;
    float cov[6];
    float jac[9];   // SH path: ddx[c], ddy[c], ddz[c] from the forward
    uint32_t clampf;
};

// The accumulator lines and the Jacobian rows are read for the last time here: non-temporal
// loads were measured neutral at cfg2 and slower at cfg5 (+20 us a call,
// profiles/r4zi_ab_prebwd_nt.txt), so these are plain loads.
template <typename T>
__device__ __forceinline__ T last_load(const T* p) {
    return *p;
}
__device__ __forceinline__ float4 last_load4(const float* p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v t = last_load(reinterpret_cast<const f4v*>(p));
    return make_float4(t.x, t.y, t.z, t.w);
}

__device__ __forceinline__ void load_bwd_in(const PreprocessBwdArgs& a, int idx, BwdIn& in) {
    const float* line = a.acc + (size_t)idx * ACC_STRIDE;
    in.l0 = last_load4(line);
    in.l1 = last_load4(line + 4);
    in.l2 = last_load(line + 8);
    in.radius = a.radii[idx];
    in.mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) in.cov[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        in.rot = *reinterpret_cast<const float4*>(a.rotations + 4 * idx);
        in.scl = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
    }
    if (a.shs) {
        const size_t P = (size_t)a.P;  // coalesced SoA rows
#pragma unroll
        for (int k = 0; k < 9; k++) in.jac[k] = last_load(a.shjac + (size_t)k * P + idx);
        in.clampf = __float_as_uint(last_load(a.shjac + 9 * P + idx));
    }
}

__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdArgs& a, int idx, const BwdIn& in, float* brow);

// auxiliary.h:107-117
__device__ __forceinline__ float3 dnormvdv3(float3 v, float3 dv) {
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    float3 o;
    o.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    o.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    o.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return o;
}

// LDS row per Gaussian for the dL/dsh writer: the 16 SH basis values (zero above the
// evaluated degree, and for culled Gaussians), the masked colour gradient g[3], one pad
constexpr int BROW = 20;

__global__ void __launch_bounds__(256) k_preprocess_bwd(PreprocessBwdArgs a) {
    __shared__ float s_b[256 * BROW];
    const int g0 = blockIdx.x * blockDim.x;
    const int idx = g0 + threadIdx.x;
    BwdIn in;
    if (idx < a.P) load_bwd_in(a, idx, in);
    if (idx < a.P) preprocess_bwd_one(a, idx, in, s_b + threadIdx.x * BROW);
    if (a.dL_dsh) {
        // dL/dsh[k][c] = basis[k] g[c] (backward.cu:20-139): the workgroup's rows ([M][3] floats
        // each, contiguous) leave as 16-B stores, each element from its Gaussian's LDS row
        __syncthreads();
        const int M3 = a.M * 3;
        const int rows = (a.P - g0) < (int)blockDim.x ? (a.P - g0) : (int)blockDim.x;
        float* out = a.dL_dsh + (size_t)g0 * M3;
        const int n = rows * M3;
        if ((M3 & 3) == 0) {
            // a float4 never straddles two rows (3M % 4 == 0): its row from one float
            // multiply (exact for these small indices), its (coefficient, channel) pairs from
            // the first one
            const int F4 = M3 >> 2;
            const float invF4 = 1.0f / (float)F4;
            float4* o4 = reinterpret_cast<float4*>(out);
            for (int f = threadIdx.x; f < (n >> 2); f += blockDim.x) {
                const int r = (int)(((float)f + 0.5f) * invF4);
                const unsigned w0 = 4u * (unsigned)(f - r * F4), k0 = w0 / 3u, c0 = w0 - 3u * k0;
                const float* b = s_b + r * BROW;
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const unsigned c = c0 + i, hi = c >= 3u ? 1u : 0u, k = k0 + hi, cc = c - 3u * hi;
                    v[i] = k < 16u ? b[k] * b[16 + cc] : 0.f;
                }
                // non-temporal: the 12M-byte rows are written once and read by the optimizer
                // later; caching them evicted the next forward's inputs from the Infinity Cache
                // (next preprocess 0.126 -> 0.112 ms, this kernel +4 us)
                typedef float f4v __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store((f4v){v[0], v[1], v[2], v[3]}, reinterpret_cast<f4v*>(o4 + f));
            }
        } else {
            for (int e = threadIdx.x; e < n; e += blockDim.x) {
                const int r = e / M3, w = e - r * M3, k = w / 3, c = w - 3 * k;
                const float* b = s_b + r * BROW;
                out[e] = k < 16 ? b[k] * b[16 + c] : 0.f;
            }
        }
    }
}

// One Gaussian: every per-Gaussian output, and (with dL_dsh) its LDS row for the dL/dsh
// writer.  (A register SH row cost 182 VGPRs; the LDS-staged SH rows of round 1 held the
// occupancy to 3 waves per SIMD.)
// a gradient output: stored, or added to what earlier views left there (acc_mask)
__device__ __forceinline__ void put(float* p, float v, bool add) { *p = add ? *p + v : v; }
__device__ __forceinline__ void put3(float* p, float x, float y, float z, bool add) {
    put(p, x, add);
    put(p + 1, y, add);
    put(p + 2, z, add);
}
__device__ __forceinline__ void put4(float* p, float4 v, bool add) {
    if (add) {
        const float4 o = *reinterpret_cast<const float4*>(p);
        v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
    }
    *reinterpret_cast<float4*>(p) = v;
}

__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdArgs& a, int idx, const BwdIn& in, float* brow) {
    const bool am = (a.acc_mask & ACC_MEAN3D) != 0, as = (a.acc_mask & ACC_SCALE) != 0,
               ar = (a.acc_mask & ACC_ROT) != 0, ao = (a.acc_mask & ACC_OPACITY) != 0;
    // ---- unpack the render-backward accumulator line ------------------------------
    const float4 l0 = in.l0, l1 = in.l1;
    const float l2 = in.l2;
    // raw lines (acc_raw): dL/dconic = -1/2 op sum G dL/dalpha (dx dx, dx dy, dy dy)
    // (backward.cu:548-550; the tile passes applied op), dL/dmean2D once the conic is known below
    const float cs = a.acc_raw ? -0.5f : 1.f;
    float dm2x = l0.x, dm2y = l0.y;
    const float dcx = cs * l0.z, dcy = cs * l0.w, dcw = cs * l1.x, dop = l1.y;
    const float dcol0 = l1.z, dcol1 = l1.w, dcol2 = l2;
    if (!a.acc_raw || !(in.radius > 0)) {  // (a culled Gaussian's line is zero)
        a.dL_dmean2D[3 * idx + 0] = a.acc_raw ? 0.f : dm2x;
        a.dL_dmean2D[3 * idx + 1] = a.acc_raw ? 0.f : dm2y;
        a.dL_dmean2D[3 * idx + 2] = 0.f;
    }
    if (a.dL_dconic)  // the reference allocates it but returns it to no one (rasterize_points.cu:145,186)
        *reinterpret_cast<float4*>(a.dL_dconic + 4 * idx) = make_float4(dcx, dcy, 0.f, dcw);
    put(a.dL_dopacity + idx, dop, ao);
    if (a.dL_dcolor) {  // absent for the multi-channel composite (its features have their own gradient)
        a.dL_dcolor[3 * idx + 0] = dcol0;
        a.dL_dcolor[3 * idx + 1] = dcol1;
        a.dL_dcolor[3 * idx + 2] = dcol2;
    }

    float dcov[6];  // dL/dcov3D, stored to dL_dcov3D when the caller wants it
    const bool want_dsh = a.dL_dsh != nullptr;
    if (!(in.radius > 0)) {
        if (!am) put3(a.dL_dmean3D + 3 * idx, 0.f, 0.f, 0.f, false);
        if (a.dL_dcov3D) {
#pragma unroll
            for (int i = 0; i < 6; i++) a.dL_dcov3D[6 * idx + i] = 0.f;
        }
        if (want_dsh) {
#pragma unroll
            for (int i = 0; i < BROW; i++) brow[i] = 0.f;
        }
        if (a.dL_dscale) {
            if (!as) put3(a.dL_dscale + 3 * idx, 0.f, 0.f, 0.f, false);
            if (!ar) put4(a.dL_drot + 4 * idx, make_float4(0.f, 0.f, 0.f, 0.f), false);
        }
        return;
    }
    const float3 mean = in.mean;
    float cov3[6];
    float4 rot = make_float4(0.f, 0.f, 0.f, 0.f);
    float3 scl = make_float3(0.f, 0.f, 0.f);
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) cov3[i] = in.cov[i];
    } else {
        rot = in.rot;
        scl = in.scl;
        cov3d_from(scl.x, scl.y, scl.z, a.scale_modifier, rot, cov3);
    }

    // ---- computeCov2DCUDA (backward.cu:144-274) --------------------------------------
    const float* v = a.viewmatrix;
    const float h_x = a.focal_x, h_y = a.focal_y;
    float3 t = xform_point4x3(mean, v);
    const float limx = 1.3f * a.tan_fovx;
    const float limy = 1.3f * a.tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
    const M3 J = mcols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0.f,
                       0.f, 0.f);
    const M3 W = mcols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    const M3 Vrk = mcols(cov3[0], cov3[1], cov3[2], cov3[1], cov3[3], cov3[4], cov3[2], cov3[4], cov3[5]);
    const M3 T = mmul(W, J);
    M3 cov2D = mmul(mmul(mtrans(T), mtrans(Vrk)), T);
    const float ca = cov2D.m[0][0] += 0.3f;
    const float cb = cov2D.m[0][1];
    const float cc = cov2D.m[1][1] += 0.3f;
    const float denom = ca * cc - cb * cb;
    if (a.acc_raw) {
        // the conic exactly as the forward computed it (forward.cu:219-222: det, 1/det, products;
        // contraction off in both TUs, so the record's bits), then dL/dmean2D in NDC units
        // (backward.cu:540-545): -(W/2) (a M1 + b M2), -(H/2) (b M1 + c M2) with M = op sum G dL/dalpha d
        const float det_inv = 1.f / denom;
        const float ka = cc * det_inv, kb = -cb * det_inv, kc = ca * det_inv;
        dm2x = -0.5f * (float)a.W * (ka * l0.x + kb * l0.y);
        dm2y = -0.5f * (float)a.H * (kb * l0.x + kc * l0.y);
        a.dL_dmean2D[3 * idx + 0] = dm2x;
        a.dL_dmean2D[3 * idx + 1] = dm2y;
        a.dL_dmean2D[3 * idx + 2] = 0.f;
    }
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
#define TT(i, j) T.m[i][j]
    if (denom2inv != 0.f) {
        dL_da = denom2inv * (-cc * cc * dcx + 2 * cb * cc * dcy + (denom - ca * cc) * dcw);
        dL_dc = denom2inv * (-ca * ca * dcw + 2 * ca * cb * dcy + (denom - ca * cc) * dcx);
        dL_db = denom2inv * 2 * (cb * cc * dcx - (denom + 2 * cb * cb) * dcy + ca * cb * dcw);
        dcov[0] = (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc);
        dcov[3] = (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc);
        dcov[5] = (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc);
        dcov[1] = 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 1) * dL_dc;
        dcov[2] = 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 2) * dL_dc;
        dcov[4] = 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                  2 * TT(1, 1) * TT(1, 2) * dL_dc;
    } else {
#pragma unroll
        for (int i = 0; i < 6; i++) dcov[i] = 0.f;
    }
#define VV(i, j) Vrk.m[i][j]
    const float dL_dT00 = 2 * (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_da +
                          (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_db;
    const float dL_dT01 = 2 * (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_da +
                          (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_db;
    const float dL_dT02 = 2 * (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_da +
                          (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_db;
    const float dL_dT10 = 2 * (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_dc +
                          (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_db;
    const float dL_dT11 = 2 * (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_dc +
                          (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_db;
    const float dL_dT12 = 2 * (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_dc +
                          (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_db;
#undef VV
#undef TT
#define WW(i, j) W.m[i][j]
    const float dL_dJ00 = WW(0, 0) * dL_dT00 + WW(0, 1) * dL_dT01 + WW(0, 2) * dL_dT02;
    const float dL_dJ02 = WW(2, 0) * dL_dT00 + WW(2, 1) * dL_dT01 + WW(2, 2) * dL_dT02;
    const float dL_dJ11 = WW(1, 0) * dL_dT10 + WW(1, 1) * dL_dT11 + WW(1, 2) * dL_dT12;
    const float dL_dJ12 = WW(2, 0) * dL_dT10 + WW(2, 1) * dL_dT11 + WW(2, 2) * dL_dT12;
#undef WW
    const float tz = 1.f / t.z;
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    const float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                         (2 * h_y * t.y) * tz3 * dL_dJ12;
    float3 dm = make_float3(v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz, v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz,
                            v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz);

    // ---- preprocessCUDA backward (backward.cu:366-396) -------------------------------
    const float* proj = a.projmatrix;
    const float4 m_hom = xform_point4x4(mean, proj);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
    const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
    dm.x += (proj[0] * m_w - proj[3] * mul1) * dm2x + (proj[1] * m_w - proj[3] * mul2) * dm2y;
    dm.y += (proj[4] * m_w - proj[7] * mul1) * dm2x + (proj[5] * m_w - proj[7] * mul2) * dm2y;
    dm.z += (proj[8] * m_w - proj[11] * mul1) * dm2x + (proj[9] * m_w - proj[11] * mul2) * dm2y;

    if (a.shs) {
        // backward.cu:20-139 from the forward's Jacobian and clamp flags
        const float3 dir_orig = make_float3(mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]);
        const float g[3] = {dcol0 * ((in.clampf & 1u) ? 0 : 1), dcol1 * ((in.clampf & 2u) ? 0 : 1),
                            dcol2 * ((in.clampf & 4u) ? 0 : 1)};
        const float3 dL_ddir = make_float3(in.jac[0] * g[0] + in.jac[1] * g[1] + in.jac[2] * g[2],
                                           in.jac[3] * g[0] + in.jac[4] * g[1] + in.jac[5] * g[2],
                                           in.jac[6] * g[0] + in.jac[7] * g[1] + in.jac[8] * g[2]);
        const float3 d = dnormvdv3(dir_orig, dL_ddir);
        dm.x += d.x;
        dm.y += d.y;
        dm.z += d.z;
        if (want_dsh) {
            // the SH basis at the view direction (the factors of dL/dsh, backward.cu:72-136);
            // coefficients above the evaluated degree get zero (torch::zeros in the reference)
            const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
            const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
            const int deg = a.D;
            float b[16];
            b[0] = SH_C0;
#pragma unroll
            for (int k = 1; k < 16; k++) b[k] = 0.f;
            if (deg > 0) {
                b[1] = -SH_C1 * y;
                b[2] = SH_C1 * z;
                b[3] = -SH_C1 * x;
                if (deg > 1) {
                    const float xx = x * x, yy = y * y, zz = z * z;
                    const float xy = x * y, yz = y * z, xz = x * z;
                    b[4] = SH_C2_0 * xy;
                    b[5] = SH_C2_1 * yz;
                    b[6] = SH_C2_2 * (2.f * zz - xx - yy);
                    b[7] = SH_C2_3 * xz;
                    b[8] = SH_C2_4 * (xx - yy);
                    if (deg > 2) {
                        b[9] = SH_C3_0 * y * (3.f * xx - yy);
                        b[10] = SH_C3_1 * xy * z;
                        b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
                        b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                        b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
                        b[14] = SH_C3_5 * z * (xx - yy);
                        b[15] = SH_C3_6 * x * (xx - 3.f * yy);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 16; k++) brow[k] = b[k];
            brow[16] = g[0];
            brow[17] = g[1];
            brow[18] = g[2];
        }
    } else if (want_dsh) {
#pragma unroll
        for (int i = 0; i < BROW; i++) brow[i] = 0.f;
    }
    put3(a.dL_dmean3D + 3 * idx, dm.x, dm.y, dm.z, am);
    if (a.dL_dcov3D) {
#pragma unroll
        for (int i = 0; i < 6; i++) a.dL_dcov3D[6 * idx + i] = dcov[i];
    }

    if (a.dL_dscale) {
        if (!a.scales) {
            if (!as) put3(a.dL_dscale + 3 * idx, 0.f, 0.f, 0.f, false);
            if (!ar) put4(a.dL_drot + 4 * idx, make_float4(0.f, 0.f, 0.f, 0.f), false);
            return;
        }
        // ---- computeCov3D backward (backward.cu:278-341) ------------------------------
        const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
        const M3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                           2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                           2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
        M3 S = mcols(1.0f, 0.f, 0.f, 0.f, 1.0f, 0.f, 0.f, 0.f, 1.0f);
        const float s0 = a.scale_modifier * scl.x, s1 = a.scale_modifier * scl.y, s2 = a.scale_modifier * scl.z;
        S.m[0][0] = s0;
        S.m[1][1] = s1;
        S.m[2][2] = s2;
        const M3 M = mmul(S, R);
        const M3 dL_dSigma = mcols(dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                                   0.5f * dcov[2], 0.5f * dcov[4], dcov[5]);
        M3 M2;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) M2.m[i][j] = 2.0f * M.m[i][j];
        const M3 dL_dM = mmul(M2, dL_dSigma);
        const M3 Rt = mtrans(R);
        M3 D = mtrans(dL_dM);
        put3(a.dL_dscale + 3 * idx, Rt.m[0][0] * D.m[0][0] + Rt.m[0][1] * D.m[0][1] + Rt.m[0][2] * D.m[0][2],
             Rt.m[1][0] * D.m[1][0] + Rt.m[1][1] * D.m[1][1] + Rt.m[1][2] * D.m[1][2],
             Rt.m[2][0] * D.m[2][0] + Rt.m[2][1] * D.m[2][1] + Rt.m[2][2] * D.m[2][2], as);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            D.m[0][j] *= s0;
            D.m[1][j] *= s1;
            D.m[2][j] *= s2;
        }
#define DD(i, j) D.m[i][j]
        float4 dq;
        dq.x = 2 * z * (DD(0, 1) - DD(1, 0)) + 2 * y * (DD(2, 0) - DD(0, 2)) + 2 * x * (DD(1, 2) - DD(2, 1));
        dq.y = 2 * y * (DD(1, 0) + DD(0, 1)) + 2 * z * (DD(2, 0) + DD(0, 2)) + 2 * r * (DD(1, 2) - DD(2, 1)) -
               4 * x * (DD(2, 2) + DD(1, 1));
        dq.z = 2 * x * (DD(1, 0) + DD(0, 1)) + 2 * r * (DD(2, 0) - DD(0, 2)) + 2 * z * (DD(1, 2) + DD(2, 1)) -
               4 * y * (DD(2, 2) + DD(0, 0));
        dq.w = 2 * r * (DD(0, 1) - DD(1, 0)) + 2 * x * (DD(2, 0) + DD(0, 2)) + 2 * y * (DD(1, 2) + DD(2, 1)) -
               4 * z * (DD(1, 1) + DD(0, 0));
#undef DD
        put4(a.dL_drot + 4 * idx, dq, ar);
    }
}

void launch_preprocess_bwd(const PreprocessBwdArgs& a, hipStream_t s) {
    if (a.P == 0) return;
    hipLaunchKernelGGL(k_preprocess_bwd, dim3((a.P + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace gsr
