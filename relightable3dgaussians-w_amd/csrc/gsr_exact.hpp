// gsr_exact.hpp -- the bit-exact per-Gaussian geometry of the forward preprocess.
//
// Include ONLY after `#pragma clang fp contract(off)`: every expression below is written
// in the reference's evaluation order (forward.cu:20-256, auxiliary.h:41-164, glm's
// column-major mat3 semantics) and must round exactly as oracle/gsr_oracle.c does.
#pragma once
#include "gsr_common.hpp"

namespace gsr {

// glm type_mat3x3.inl operator*: R[c][r] = A[0][r]B[c][0] + A[1][r]B[c][1] + A[2][r]B[c][2]
__device__ __forceinline__ M3 mmul(const M3& A, const M3& B) {
    M3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return R;
}

__device__ __forceinline__ M3 mtrans(const M3& A) {
    M3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) R.m[c][r] = A.m[r][c];
    return R;
}

// auxiliary.h:58-66
__device__ __forceinline__ float3 xform_point4x3(float3 p, const float* m) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}

// auxiliary.h:68-77
__device__ __forceinline__ float4 xform_point4x4(float3 p, const float* m) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// auxiliary.h:41-44 -- evaluated in double
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

// auxiliary.h:46-56 (p + r + 16 - 1 evaluated left to right in float)
__device__ __forceinline__ void get_rect(float2 p, int max_radius, unsigned gx, unsigned gy, uint2& rmin,
                                         uint2& rmax) {
    int a;
    a = f2i((p.x - (float)max_radius) / (float)GSR_BLOCK_X);
    a = a > 0 ? a : 0;
    rmin.x = (unsigned)a < gx ? (unsigned)a : gx;
    a = f2i((p.y - (float)max_radius) / (float)GSR_BLOCK_Y);
    a = a > 0 ? a : 0;
    rmin.y = (unsigned)a < gy ? (unsigned)a : gy;
    a = f2i((p.x + (float)max_radius + (float)GSR_BLOCK_X - 1.0f) / (float)GSR_BLOCK_X);
    a = a > 0 ? a : 0;
    rmax.x = (unsigned)a < gx ? (unsigned)a : gx;
    a = f2i((p.y + (float)max_radius + (float)GSR_BLOCK_Y - 1.0f) / (float)GSR_BLOCK_Y);
    a = a > 0 ? a : 0;
    rmax.y = (unsigned)a < gy ? (unsigned)a : gy;
}

// forward.cu:118-152 (quaternion used as given, :127)
__device__ __forceinline__ void cov3d_from(float sx, float sy, float sz, float mod, float4 rot, float* cov) {
    M3 S = mcols(1.0f, 0.f, 0.f, 0.f, 1.0f, 0.f, 0.f, 0.f, 1.0f);
    S.m[0][0] = mod * sx;
    S.m[1][1] = mod * sy;
    S.m[2][2] = mod * sz;
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    M3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y), 2.f * (x * y + r * z),
                 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x), 2.f * (x * z - r * y), 2.f * (y * z + r * x),
                 1.f - 2.f * (x * x + y * y));
    M3 M = mmul(S, R);
    M3 Sig = mmul(mtrans(M), M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

// forward.cu:74-113
__device__ __forceinline__ float3 cov2d_from(float3 mean, float fx, float fy, float tanx, float tany, const float* c3,
                                             const float* v) {
    float3 t = xform_point4x3(mean, v);
    const float limx = 1.3f * tanx;
    const float limy = 1.3f * tany;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    M3 J = mcols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0.f, 0.f, 0.f);
    M3 W = mcols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    M3 T = mmul(W, J);
    M3 Vrk = mcols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    M3 cov = mmul(mmul(mtrans(T), mtrans(Vrk)), T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    return make_float3(cov.m[0][0], cov.m[0][1], cov.m[1][1]);
}

// forward.cu:20-71: SH (deg <= 3) -> RGB before clamping.  sh: this Gaussian's [M][3].
// MAXD: the largest degree the row can hold (register rows of fewer than 16 coefficients
// prune the higher blocks at compile time); deg must not exceed it.
template <int MAXD = 3>
__device__ __forceinline__ float3 sh_to_rgb_raw(int deg, float3 pos, const float* campos, const float* sh) {
    float3 dir = make_float3(pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]);
    const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x = dir.x / len;
    dir.y = dir.y / len;
    dir.z = dir.z / len;
    float res[3];
#pragma unroll
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh[c];
    if (MAXD > 0 && deg > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
#pragma unroll
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - SH_C1 * y * sh[3 + c] + SH_C1 * z * sh[6 + c] - SH_C1 * x * sh[9 + c];
        if (MAXD > 1 && deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + SH_C2_0 * xy * sh[12 + c] + SH_C2_1 * yz * sh[15 + c] +
                         SH_C2_2 * (2.0f * zz - xx - yy) * sh[18 + c] + SH_C2_3 * xz * sh[21 + c] +
                         SH_C2_4 * (xx - yy) * sh[24 + c];
            if (MAXD > 2 && deg > 2) {
#pragma unroll
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + SH_C3_0 * y * (3.0f * xx - yy) * sh[27 + c] + SH_C3_1 * xy * z * sh[30 + c] +
                             SH_C3_2 * y * (4.0f * zz - xx - yy) * sh[33 + c] +
                             SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[36 + c] +
                             SH_C3_4 * x * (4.0f * zz - xx - yy) * sh[39 + c] +
                             SH_C3_5 * z * (xx - yy) * sh[42 + c] + SH_C3_6 * x * (xx - 3.0f * yy) * sh[45 + c];
            }
        }
    }
    return make_float3(res[0] + 0.5f, res[1] + 0.5f, res[2] + 0.5f);
}

// d(SH colour)/d(unit view direction) per channel (backward.cu:61-113, the dRGBdx/dy/dz of
// the SH backward) at the direction (x, y, z), from the SH row `sh` ([M][3]).  The forward
// preprocess evaluates it once and stores it for the backward (gsr_preprocess.hip); both TUs
// compile with contraction off, so it is the arithmetic the backward would do, bit for bit.
template <int MAXD = 3>
__device__ __forceinline__ void sh_dir_jacobian(int deg, float x, float y, float z, const float* sh, float (&ddx)[3],
                                                float (&ddy)[3], float (&ddz)[3]) {
#define SHC(k, c) sh[3 * (k) + (c)]
#pragma unroll
    for (int c = 0; c < 3; c++) ddx[c] = ddy[c] = ddz[c] = 0.f;
    if (MAXD > 0 && deg > 0) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            ddx[c] = -SH_C1 * SHC(3, c);
            ddy[c] = -SH_C1 * SHC(1, c);
            ddz[c] = SH_C1 * SHC(2, c);
        }
        if (MAXD > 1 && deg > 1) {
#pragma unroll
            for (int c = 0; c < 3; c++) {
                ddx[c] += SH_C2_0 * y * SHC(4, c) + SH_C2_2 * 2.f * -x * SHC(6, c) + SH_C2_3 * z * SHC(7, c) +
                          SH_C2_4 * 2.f * x * SHC(8, c);
                ddy[c] += SH_C2_0 * x * SHC(4, c) + SH_C2_1 * z * SHC(5, c) + SH_C2_2 * 2.f * -y * SHC(6, c) +
                          SH_C2_4 * 2.f * -y * SHC(8, c);
                ddz[c] += SH_C2_1 * y * SHC(5, c) + SH_C2_2 * 2.f * 2.f * z * SHC(6, c) + SH_C2_3 * x * SHC(7, c);
            }
            if (MAXD > 2 && deg > 2) {
                const float xx = x * x, yy = y * y, zz = z * z;
                const float xy = x * y, yz = y * z, xz = x * z;
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
                }
            }
        }
    }
#undef SHC
}

}  // namespace gsr
