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
// kernels alike.  GSR_ST_STH forces one height (experiments).
constexpr unsigned ST_SMALL_MAX = 682;
__host__ __device__ __forceinline__ unsigned st_sth(unsigned gx, unsigned gy) {
#ifdef GSR_ST_STH
    (void)gx;
    (void)gy;
    return GSR_ST_STH;
#else
    const unsigned long long ns4 = (unsigned long long)((gx + GSR_ST_W - 1u) / GSR_ST_W) * ((gy + 3u) / 4u);
    return ns4 > ST_SMALL_MAX ? 3u : 2u;
#endif
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
// hand-out of the lines measured the same), the call pair -16 us.  GSR_ACC_STRIDE=12 builds
// the 48-B layout.
#ifndef GSR_ACC_STRIDE
#define GSR_ACC_STRIDE 16
#endif
constexpr int ACC_STRIDE = GSR_ACC_STRIDE;
static_assert(ACC_STRIDE % 4 == 0 && ACC_STRIDE >= 12, "accumulator lines hold 9 floats, 16-B aligned");

// The forward tile pass's survivor lists (RenderFwdArgs::surv): at most SURV_CAP entries per
// tile (cfg2: 285 at most, the clustered cfg2c 749), a count of SURV_NONE sends the backward
// back to its super-tile list.  GSR_SURV_CAP=0 builds without them.
#ifndef GSR_SURV_CAP
#define GSR_SURV_CAP 1024
#endif
constexpr uint32_t SURV_CAP = GSR_SURV_CAP;
constexpr uint32_t SURV_NONE = 0xffffffffu;
// Quadrant lists (GSR_QLIST): the forward's quadrant units of a tile whose super-tile list holds
// at least GSR_QL_MIN entries store their own quadrant's survivors, each to a list of SURV_CAP
// slots of their own (qsurv, indexed by the unit's slot: tile_unit), and the tile's count word
// becomes SURV_QFLAG | slot; the backward merges the four lists in windows of 64 positions
// instead of re-filtering the whole super-tile list (cfg2c: its slowest backward units are these
// tiles, 400+ us each).  Measured in round 5 (profiles/r5z_qlist_ab.txt): cfg2c render_bwd 0.432
// -> 0.418 ms, cfg2 0.314 -> 0.311, single calls unchanged, but the 3-stream throughput -3.8 %
// (cfg2) / -2.6 % (cfg2c): the backward at 110 VGPRs (104 without) and the forward's extra
// stores; walked one quadrant after another instead (each survivor reduced per quadrant):
// render_bwd 0.31 -> 0.41 ms.  Off.
#ifndef GSR_QLIST
#define GSR_QLIST 0
#endif
#ifndef GSR_QL_MIN
#define GSR_QL_MIN 4096
#endif
constexpr uint32_t SURV_QFLAG = 0x80000000u;
// (the tile passes' split counts, gsr_tile.hpp, here for the host's layout)
#ifndef GSR_HEAVY_CAP
#define GSR_HEAVY_CAP 64
#endif
#ifndef GSR_FWD_TAIL
#define GSR_FWD_TAIL 128
#endif
// the forward's quadrant-unit slots (tile_unit's qslot)
constexpr unsigned QL_SLOTS = 8u * (GSR_HEAVY_CAP + GSR_FWD_TAIL);
// Backward chunks (GSR_CK_SURV > 0): the forward checkpoints a whole tile's per-pixel state (T and
// the colour so far) after the batch at which another CK_SURV survivors have been stored, at most
// CK_MAX times; the backward then runs a tile as one unit per chunk of its survivor list, each
// starting from its checkpoint (T, and the recurrence from the final colour), in parallel.
#ifndef GSR_CK_SURV
#define GSR_CK_SURV 0
#endif
#ifndef GSR_CK_MAX
#define GSR_CK_MAX 3
#endif
constexpr uint32_t CK_SURV = GSR_CK_SURV;
constexpr uint32_t CK_MAX = GSR_CK_MAX;
// backward units per tile at most: its chunks, or four quadrants of a heavy tile without a list
constexpr uint32_t UNITS_MAX = (CK_MAX + 1) > 4 ? (CK_MAX + 1) : 4;
// unit codes (the top 8 bits of an expanded order entry): chunk index, a quadrant, the whole tile
constexpr uint32_t UNIT_QUAD = 0xF0u, UNIT_WHOLE = 0xFFu;

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
