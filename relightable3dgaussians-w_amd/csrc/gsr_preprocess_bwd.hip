// gsr_preprocess_bwd.hip -- fused per-Gaussian backward: computeCov2DCUDA
// (backward.cu:144-274) + preprocessCUDA (backward.cu:346-396) with the SH backward
// (:20-139) and the cov3D backward (:278-341), plus the unpacking of the render
// backward's 64-B accumulator line into the reference's output tensors.
//
// One kernel instead of two + nine memsets: every output element is written here
// (zeros for culled Gaussians), so the caller's buffers need no zero-fill.  cov3D and
// the SH clamp flags are recomputed with the forward's exact (contraction-off) code
// instead of being stored and re-read.
#pragma clang fp contract(off)
#include "gsr_exact.hpp"

#include "gsr_kernels.hpp"

namespace gsr {

// One Gaussian's inputs, loaded before the workgroup's SH rows are staged (every global load
// of the thread in flight at once instead of one dependent round trip after the barrier).
struct BwdIn {
    float4 l0, l1;  // accumulator line [0..8)
    float l2;       // [8]
    int radius;
    float3 mean;
    float4 rot;
    float3 scl;
    float cov[6];
};

__device__ __forceinline__ void load_bwd_in(const PreprocessBwdArgs& a, int idx, BwdIn& in) {
    const float4* line = reinterpret_cast<const float4*>(a.acc + (size_t)idx * ACC_STRIDE);
    in.l0 = line[0];
    in.l1 = line[1];
    in.l2 = a.acc[(size_t)idx * ACC_STRIDE + 8];
    in.radius = a.radii[idx];
    in.mean = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) in.cov[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        in.rot = *reinterpret_cast<const float4*>(a.rotations + 4 * idx);
        in.scl = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
    }
}

template <int MC, bool DO_SH = true>
__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdArgs& a, int idx, const BwdIn& in, float* row);

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

// SH rows ([M][3] floats = 192 B at degree 3) of the workgroup's Gaussians are one
// contiguous block in HBM: it is moved as a flat array of 16-B words (every lane busy,
// many loads in flight) and scattered into LDS rows of stride M*3+1 (odd: conflict-free
// per-thread row access); the gradient rows go back out the same way.
__device__ __forceinline__ void load_rows(float* s, int stride, const float* g, int rows, int width) {
    const int n = rows * width;
    if ((width & 3) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(g);
        for (int f = threadIdx.x; f < (n >> 2); f += blockDim.x) {
            const float4 v = g4[f];
            const int e0 = f * 4, r = e0 / width, e = e0 - r * width;
            float* d = s + r * stride + e;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
    } else {
        for (int f = threadIdx.x; f < n; f += blockDim.x) {
            const int r = f / width;
            s[r * stride + f - r * width] = g[f];
        }
    }
}
__device__ __forceinline__ void store_rows(float* g, const float* s, int stride, int rows, int width) {
    const int n = rows * width;
    if ((width & 3) == 0) {
        float4* g4 = reinterpret_cast<float4*>(g);
        for (int f = threadIdx.x; f < (n >> 2); f += blockDim.x) {
            const int e0 = f * 4, r = e0 / width, e = e0 - r * width;
            const float* d = s + r * stride + e;
            g4[f] = make_float4(d[0], d[1], d[2], d[3]);
        }
    } else {
        for (int f = threadIdx.x; f < n; f += blockDim.x) {
            const int r = f / width;
            g[f] = s[r * stride + f - r * width];
        }
    }
}

__global__ void __launch_bounds__(256) k_preprocess_bwd(PreprocessBwdArgs a) {
    extern __shared__ float s_sh[];
    const int M3 = a.M * 3, sh_stride = M3 + 1;
    const int g0 = blockIdx.x * blockDim.x;
    const int rows = (a.P - g0) < (int)blockDim.x ? (a.P - g0) : (int)blockDim.x;
    BwdIn in;
    if (g0 + (int)threadIdx.x < a.P) load_bwd_in(a, g0 + threadIdx.x, in);
    if (a.shs) {
        load_rows(s_sh, sh_stride, a.shs + (size_t)g0 * M3, rows, M3);
        __syncthreads();
    }
    const int idx = g0 + threadIdx.x;
    if (idx < a.P) preprocess_bwd_one<0>(a, idx, in, s_sh + threadIdx.x * sh_stride);
    if (a.dL_dsh) {
        __syncthreads();
        store_rows(a.dL_dsh + (size_t)g0 * M3, s_sh, sh_stride, rows, M3);
    }
}

// backward.cu:20-139 for one Gaussian: reads the SH coefficients from `row`, overwrites
// them with dL/dsh (each degree block reads its coefficients before overwriting them) and
// returns the view-direction part of dL/dmean3D.  MC as preprocess_bwd_one.
template <int MC>
__device__ __forceinline__ float3 sh_bwd_row(const PreprocessBwdArgs& a, float3 mean, float* row, float dcol0,
                                             float dcol1, float dcol2) {
    // backward.cu:20-139 on this Gaussian's LDS row (coalesced in/out, see below);
    // each degree block reads its coefficients before overwriting them with dL/dsh.
    float* sh = row;
    constexpr int MAXD = MC == 0 ? 3 : (MC >= 16 ? 3 : MC >= 9 ? 2 : MC >= 4 ? 1 : 0);
    const float3 raw = sh_to_rgb_raw<MAXD>(a.D, mean, a.campos, sh);  // clamp flags, as the forward
    const float3 dir_orig = make_float3(mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]);
    const float len = sqrtf(dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z);
    const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
    float g[3] = {dcol0 * (raw.x < 0 ? 0 : 1), dcol1 * (raw.y < 0 ? 0 : 1), dcol2 * (raw.z < 0 ? 0 : 1)};
    float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
    const int deg = a.D;
    float* dsh = sh;
#define SHC(k, c) sh[3 * (k) + (c)]
#pragma unroll
    for (int c = 0; c < 3; c++) dsh[c] = SH_C0 * g[c];
    if ((MC == 0 || MC >= 4) && deg > 0) {
        const float b1 = -SH_C1 * y, b2 = SH_C1 * z, b3 = -SH_C1 * x;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            ddx[c] = -SH_C1 * SHC(3, c);
            ddy[c] = -SH_C1 * SHC(1, c);
            ddz[c] = SH_C1 * SHC(2, c);
            dsh[3 + c] = b1 * g[c];
            dsh[6 + c] = b2 * g[c];
            dsh[9 + c] = b3 * g[c];
        }
        if ((MC == 0 || MC >= 9) && deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            const float b4 = SH_C2_0 * xy, b5 = SH_C2_1 * yz, b6 = SH_C2_2 * (2.f * zz - xx - yy);
            const float b7 = SH_C2_3 * xz, b8 = SH_C2_4 * (xx - yy);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                ddx[c] += SH_C2_0 * y * SHC(4, c) + SH_C2_2 * 2.f * -x * SHC(6, c) + SH_C2_3 * z * SHC(7, c) +
                          SH_C2_4 * 2.f * x * SHC(8, c);
                ddy[c] += SH_C2_0 * x * SHC(4, c) + SH_C2_1 * z * SHC(5, c) + SH_C2_2 * 2.f * -y * SHC(6, c) +
                          SH_C2_4 * 2.f * -y * SHC(8, c);
                ddz[c] += SH_C2_1 * y * SHC(5, c) + SH_C2_2 * 2.f * 2.f * z * SHC(6, c) + SH_C2_3 * x * SHC(7, c);
                dsh[12 + c] = b4 * g[c];
                dsh[15 + c] = b5 * g[c];
                dsh[18 + c] = b6 * g[c];
                dsh[21 + c] = b7 * g[c];
                dsh[24 + c] = b8 * g[c];
            }
            if ((MC == 0 || MC >= 16) && deg > 2) {
                const float b9 = SH_C3_0 * y * (3.f * xx - yy);
                const float b10 = SH_C3_1 * xy * z;
                const float b11 = SH_C3_2 * y * (4.f * zz - xx - yy);
                const float b12 = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                const float b13 = SH_C3_4 * x * (4.f * zz - xx - yy);
                const float b14 = SH_C3_5 * z * (xx - yy);
                const float b15 = SH_C3_6 * x * (xx - 3.f * yy);
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    ddx[c] += (SH_C3_0 * SHC(9, c) * 3.f * 2.f * xy + SH_C3_1 * SHC(10, c) * yz +
                               SH_C3_2 * SHC(11, c) * -2.f * xy + SH_C3_3 * SHC(12, c) * -3.f * 2.f * xz +
                               SH_C3_4 * SHC(13, c) * (-3.f * xx + 4.f * zz - yy) +
                               SH_C3_5 * SHC(14, c) * 2.f * xz + SH_C3_6 * SHC(15, c) * 3.f * (xx - yy));
                    ddy[c] += (SH_C3_0 * SHC(9, c) * 3.f * (xx - yy) + SH_C3_1 * SHC(10, c) * xz +
                               SH_C3_2 * SHC(11, c) * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3_3 * SHC(12, c) * -3.f * 2.f * yz + SH_C3_4 * SHC(13, c) * -2.f * xy +
                               SH_C3_5 * SHC(14, c) * -2.f * yz + SH_C3_6 * SHC(15, c) * -3.f * 2.f * xy);
                    ddz[c] += (SH_C3_1 * SHC(10, c) * xy + SH_C3_2 * SHC(11, c) * 4.f * 2.f * yz +
                               SH_C3_3 * SHC(12, c) * 3.f * (2.f * zz - xx - yy) +
                               SH_C3_4 * SHC(13, c) * 4.f * 2.f * xz + SH_C3_5 * SHC(14, c) * (xx - yy));
                    dsh[27 + c] = b9 * g[c];
                    dsh[30 + c] = b10 * g[c];
                    dsh[33 + c] = b11 * g[c];
                    dsh[36 + c] = b12 * g[c];
                    dsh[39 + c] = b13 * g[c];
                    dsh[42 + c] = b14 * g[c];
                    dsh[45 + c] = b15 * g[c];
                }
            }
        }
    }
#undef SHC
    // coefficients above the evaluated degree get zero gradient (torch::zeros in the reference)
    const int kmin = deg < 0 ? 0 : (deg > 3 ? 16 : (deg + 1) * (deg + 1));
    if constexpr (MC > 0) {
#pragma unroll
        for (int k = 0; k < MC; k++)
            if (k >= kmin) dsh[3 * k] = dsh[3 * k + 1] = dsh[3 * k + 2] = 0.f;
    } else {
        for (int k = kmin; k < a.M; k++) {
            dsh[3 * k] = 0.f;
            dsh[3 * k + 1] = 0.f;
            dsh[3 * k + 2] = 0.f;
        }
    }
    const float3 dL_ddir = make_float3(ddx[0] * g[0] + ddx[1] * g[1] + ddx[2] * g[2],
                                       ddy[0] * g[0] + ddy[1] * g[1] + ddy[2] * g[2],
                                       ddz[0] * g[0] + ddz[1] * g[1] + ddz[2] * g[2]);
    return dnormvdv3(dir_orig, dL_ddir);
}

// `row` holds the Gaussian's SH coefficients (MC > 0: a register array of 3 MC floats; MC
// == 0: an LDS row of a.M * 3 floats, k_preprocess_bwd).  The SH backward reads the
// coefficients from the row and overwrites them with dL/dsh.  (Measured slower at cfg2:
// register rows, 242 vs 199 us -- 182 VGPRs leave 2 waves per SIMD; and a split into a
// geometry kernel + a register-row SH kernel, 63 + 196 us -- its strided 16-B row stores
// write partial lines, where the LDS-staged rows leave the workgroup as whole lines.)
template <int MC, bool DO_SH>
__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdArgs& a, int idx, const BwdIn& in, float* row) {
    // ---- unpack the render-backward accumulator line ------------------------------
    const float4 l0 = in.l0, l1 = in.l1;
    const float l2 = in.l2;
    const float dm2x = l0.x, dm2y = l0.y, dcx = l0.z, dcy = l0.w, dcw = l1.x, dop = l1.y;
    const float dcol0 = l1.z, dcol1 = l1.w, dcol2 = l2;
    a.dL_dmean2D[3 * idx + 0] = dm2x;
    a.dL_dmean2D[3 * idx + 1] = dm2y;
    a.dL_dmean2D[3 * idx + 2] = 0.f;
    if (a.dL_dconic)  // the reference allocates it but returns it to no one (rasterize_points.cu:145,186)
        *reinterpret_cast<float4*>(a.dL_dconic + 4 * idx) = make_float4(dcx, dcy, 0.f, dcw);
    a.dL_dopacity[idx] = dop;
    if (a.dL_dcolor) {  // absent for the multi-channel composite (its features have their own gradient)
        a.dL_dcolor[3 * idx + 0] = dcol0;
        a.dL_dcolor[3 * idx + 1] = dcol1;
        a.dL_dcolor[3 * idx + 2] = dcol2;
    }

    float* dcov = a.dL_dcov3D + 6 * idx;
    float* dsh = row;  // written back by the caller when dL_dsh is requested
    const bool want_dsh = DO_SH && a.dL_dsh != nullptr;
    if (!(in.radius > 0)) {
        a.dL_dmean3D[3 * idx + 0] = 0.f;
        a.dL_dmean3D[3 * idx + 1] = 0.f;
        a.dL_dmean3D[3 * idx + 2] = 0.f;
#pragma unroll
        for (int i = 0; i < 6; i++) dcov[i] = 0.f;
        if (want_dsh) {
            if constexpr (MC > 0) {
#pragma unroll
                for (int i = 0; i < 3 * MC; i++) dsh[i] = 0.f;
            } else {
                for (int i = 0; i < a.M * 3; i++) dsh[i] = 0.f;
            }
        }
        if (a.dL_dscale) {
            a.dL_dscale[3 * idx + 0] = 0.f;
            a.dL_dscale[3 * idx + 1] = 0.f;
            a.dL_dscale[3 * idx + 2] = 0.f;
            *reinterpret_cast<float4*>(a.dL_drot + 4 * idx) = make_float4(0.f, 0.f, 0.f, 0.f);
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

    if (DO_SH && a.shs) {
        const float3 d = sh_bwd_row<MC>(a, mean, row, dcol0, dcol1, dcol2);
        dm.x += d.x;
        dm.y += d.y;
        dm.z += d.z;
    }
    a.dL_dmean3D[3 * idx + 0] = dm.x;
    a.dL_dmean3D[3 * idx + 1] = dm.y;
    a.dL_dmean3D[3 * idx + 2] = dm.z;

    if (a.dL_dscale) {
        if (!a.scales) {
            a.dL_dscale[3 * idx + 0] = 0.f;
            a.dL_dscale[3 * idx + 1] = 0.f;
            a.dL_dscale[3 * idx + 2] = 0.f;
            *reinterpret_cast<float4*>(a.dL_drot + 4 * idx) = make_float4(0.f, 0.f, 0.f, 0.f);
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
        float* ds = a.dL_dscale + 3 * idx;
        ds[0] = Rt.m[0][0] * D.m[0][0] + Rt.m[0][1] * D.m[0][1] + Rt.m[0][2] * D.m[0][2];
        ds[1] = Rt.m[1][0] * D.m[1][0] + Rt.m[1][1] * D.m[1][1] + Rt.m[1][2] * D.m[1][2];
        ds[2] = Rt.m[2][0] * D.m[2][0] + Rt.m[2][1] * D.m[2][1] + Rt.m[2][2] * D.m[2][2];
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
        *reinterpret_cast<float4*>(a.dL_drot + 4 * idx) = dq;
    }
}

void launch_preprocess_bwd(const PreprocessBwdArgs& a, hipStream_t s) {
    if (a.P == 0) return;
    // 256 Gaussians per workgroup while their SH rows fit 64 KiB of LDS, else 64
    const size_t row = a.shs ? (size_t)(a.M * 3 + 1) * sizeof(float) : 0;
    const int threads = row * 256 <= 65536 ? 256 : 64;
    hipLaunchKernelGGL(k_preprocess_bwd, dim3((a.P + threads - 1) / threads), dim3(threads), row * threads, s, a);
}

}  // namespace gsr
