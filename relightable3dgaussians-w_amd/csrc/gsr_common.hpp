// gsr_common.hpp -- shared device helpers for the MI355X (gfx950) Gaussian rasterizer.
//
// The preprocess / binning math must be bit-identical to the reference's
// (cuda_rasterizer/auxiliary.h, forward.cu) as restated in oracle/gsr_oracle.c, so every
// translation unit that includes this header with GSR_EXACT defined compiles its float
// arithmetic with FMA contraction off and IEEE (correctly rounded) div/sqrt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GSR_BLOCK_X 16
#define GSR_BLOCK_Y 16
#define GSR_TILE_PIX 256
// super-tile (binning granularity): GSR_ST_W tiles wide and 2^sth tiles high, sth chosen per
// frame by st_sth (below)
#define GSR_ST_W 8u

namespace gsr {

// A super-tile entry's local tile rect (the tiles of its super-tile the Gaussian's rect
// covers): cx0 | (cx1 - 1) << ST_XB | cy0 << 2 ST_XB | (cy1 - 1) << (2 ST_XB + ST_YB), with
// [cx0, cx1) x [cy0, cy1) tile offsets inside the super-tile (fields sized for the tallest
// super-tile).
constexpr uint32_t ST_XB = 3u, ST_YB = 3u;
static_assert((1u << ST_XB) == GSR_ST_W, "super-tile width");
constexpr uint32_t ST_CODE_BITS = 2u * (ST_XB + ST_YB);
constexpr int ST_TILES = 64;  // tiles of the tallest super-tile (8 x 8), one lane each
// Super-tile height: 8x4 tiles (sth = 2) while the frame has at most ST_SMALL_MAX of them, the
// binning scatter's limit for 8 waves per workgroup in 64 KiB of LDS (st_waves); larger
// frames (4K: 1020 8x4 super-tiles) take 8x8 (sth = 3): fewer entries per Gaussian (cfg5:
// 3.2 instead of 4.7) and half the per-wave scatter state, for a little more filtering in
// the tile passes.  A pure function of the tile grid, evaluated on the host and in the
// kernels alike.
constexpr unsigned ST_SMALL_MAX = 682;
__host__ __device__ __forceinline__ unsigned st_sth(unsigned gx, unsigned gy) {
    const unsigned long long ns4 = (unsigned long long)((gx + GSR_ST_W - 1u) / GSR_ST_W) * ((gy + 3u) / 4u);
    return ns4 > ST_SMALL_MAX ? 3u : 2u;
}

// auxiliary.h:22-39 (same decimal literals as the reference)
__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

// Render record: one 48-byte row per Gaussian, written by preprocess, gathered by the
// tile passes into LDS.  a = (x, y, conic.a, conic.b), b = (conic.c, opacity, r, g),
// c = (b, ln(255*opacity), 0, 0).
struct __align__(16) Rec {
    float4 a, b, c;
};

// Per-Gaussian gradient accumulator line (64 B, 64-B aligned; one atomic instruction per
// (tile, Gaussian)): [0] dL/dmean2D.x [1] .y [2] dL/dconic.x [3] .y [4] .w [5] dL/dopacity
// [6..8] dL/dcolor [9..15] unused.  The float atomics execute at the memory side in 64-B
// requests: with 48-B lines half of a Gaussian's 9-value atomics straddled two 64-B segments.
// 64-B lines (measured at cfg2, rocprofv3 kernel trace): render_bwd 351 -> 334 us, the
// preprocess backward 122 -> 131 us (33 % more accumulator bytes to read; a coalesced LDS
// hand-out of the lines measured the same), the call pair -16 us.
constexpr int ACC_STRIDE = 16;

// The forward tile pass's survivor lists (RenderFwdArgs::surv): at most SURV_CAP entries per
// tile (cfg2: 285 at most, the clustered cfg2c 749), a count of SURV_NONE sends the backward
// back to its super-tile list.
constexpr uint32_t SURV_CAP = 1024;
constexpr uint32_t SURV_NONE = 0xffffffffu;

// Gradient outputs added into (instead of overwritten): the backward kernels' accumulate
// bits (include/gsr.h GSR_ACC_*), so several views' gradients are summed where they are made.
constexpr unsigned ACC_MEAN3D = 1u, ACC_SCALE = 2u, ACC_ROT = 4u, ACC_OPACITY = 8u, ACC_ALBEDO = 16u, ACC_ROUGH = 32u,
                   ACC_METAL = 64u;

// float -> int exactly as v_cvt_i32_f32 / the reference's implicit conversions
// (forward.cu:235, :251): truncation, saturation, NaN -> 0.
__device__ __forceinline__ int f2i(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

// glm::mat3, column-major m[c][r]
struct M3 {
    float m[3][3];
};

__device__ __forceinline__ M3 mcols(float a0, float a1, float a2, float b0, float b1, float b2, float c0, float c1,
                                    float c2) {
    M3 R;
    R.m[0][0] = a0; R.m[0][1] = a1; R.m[0][2] = a2;
    R.m[1][0] = b0; R.m[1][1] = b1; R.m[1][2] = b2;
    R.m[2][0] = c0; R.m[2][1] = c1; R.m[2][2] = c2;
    return R;
}

}  // namespace gsr

// HIP error plumbing for the C ABI (gsr_capi.cpp)
#define GSR_LAUNCH_CHECK()                                       \
    do {                                                         \
        hipError_t _e = hipGetLastError();                       \
        if (_e != hipSuccess) return gsr_fail_hip(_e, __LINE__); \
    } while (0)
