// gsr_tile.hpp -- helpers shared by the forward and backward tile passes.
#pragma once
#include "gsr_common.hpp"

namespace gsr {

// bijective XCD-aware block -> tile remap: blocks b and b+8 run on the same XCD (private
// L2), so each XCD gets a contiguous band of tiles whose Gaussian records overlap.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n) {
    const unsigned q = n >> 3, r = n & 7u, x = b & 7u;
    const unsigned base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

// exp as the tile loops evaluate it, identical in forward and backward so that the
// backward replays exactly the forward's blend decisions (v_exp_f32 on x*log2(e)).
__device__ __forceinline__ float tile_exp(float x) { return __expf(x); }

// Minimum over the pixel box [dx0,dx1]x[dy0,dy1] (offsets from the Gaussian centre) of
// q(d) = a dx^2 + 2 b dx dy + c dy^2, for a positive-definite conic (a, b, c).
__device__ __forceinline__ float qmin_box(float a, float b, float c, float dx0, float dx1, float dy0, float dy1) {
    if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return 0.f;
    // edges dx = const: argmin dy = -b dx / c ; edges dy = const: argmin dx = -b dy / a
    const float ic = 1.f / c, ia = 1.f / a;
    float q = 3.4e38f;
    {
        const float X = dx0;
        const float y = fminf(fmaxf(-b * X * ic, dy0), dy1);
        q = fminf(q, a * X * X + 2.f * b * X * y + c * y * y);
    }
    {
        const float X = dx1;
        const float y = fminf(fmaxf(-b * X * ic, dy0), dy1);
        q = fminf(q, a * X * X + 2.f * b * X * y + c * y * y);
    }
    {
        const float Y = dy0;
        const float x = fminf(fmaxf(-b * Y * ia, dx0), dx1);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    {
        const float Y = dy1;
        const float x = fminf(fmaxf(-b * Y * ia, dx0), dx1);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    return q;
}

// Conservative test: can this Gaussian reach alpha >= 1/255 at any integer pixel of the
// box?  The render loops evaluate alpha = min(0.99, o * exp(-q/2)) and skip alpha < 1/255,
// so a Gaussian with o * exp(-qmin/2) < 1/255 contributes nothing to any pixel of the box
// (in the forward, the backward, n_contrib or T).  `lnthr` = ln(255 * o).  The margin
// covers the float rounding of q at the pixels (relative to the magnitude of its terms)
// and of the exp/threshold evaluation, so the skip is never wrong.
__device__ __forceinline__ bool box_reachable(float a, float b, float c, float lnthr, float dx0, float dx1, float dy0,
                                              float dy1) {
    const float q = qmin_box(a, b, c, dx0, dx1, dy0, dy1);
    const float mx = fmaxf(fabsf(dx0), fabsf(dx1)), my = fmaxf(fabsf(dy0), fabsf(dy1));
    const float S = a * mx * mx + 2.f * fabsf(b) * mx * my + c * my * my;
    return q <= 2.f * lnthr + 1e-2f + 1e-4f * S;
}

// All-lane wave64 float sum on the VALU: 4 DPP row steps + the gfx950 permlane swaps.
template <int ctrl>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, true));
}
// Every lane receives the sum over its 16-lane DPP row (4 fused v_add_f32_dpp).
__device__ __forceinline__ float row_sum(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x124>(v);
    return v + dpp<0x128>(v);
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x124>(v);  // row_ror:4
    v += dpp<0x128>(v);  // row_ror:8   -> every lane holds its 16-lane row sum
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(s[0]) + __uint_as_float(s[1]);  // rows (0,1) and (2,3)
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);  // halves
}

// ---- batch staging shared by the forward and backward tile passes ---------------------
struct TileStageLDS {
    float4 a[256];           // (x, y, conic.a, conic.b)
    float4 b[256];           // (conic.c, opacity, r, g)
    float c[256];            // b
    uint32_t pos[256];       // position in the tile's range
    uint32_t id[256];        // Gaussian index
    uint16_t qidx[4][256];   // per-quadrant lists of slots, in range order
    uint32_t qcnt[4];        // per-quadrant list length
    uint32_t cnt;            // slots used
    uint32_t wcnt[4][5];     // per-wave ballot counts: kept, quadrant 0..3
};

struct TileStage {
    int px, py;
    bool inside;
    float pfx, pfy, tx0, ty0, wmax, hmax;
    uint64_t lt;

    __device__ __forceinline__ void init(unsigned tile, unsigned gx, int W, int H) {
        const unsigned bx = tile % gx, by = tile / gx;
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        px = bx * GSR_BLOCK_X + (wave & 1) * 8 + (lane & 7);
        py = by * GSR_BLOCK_Y + (wave >> 1) * 8 + (lane >> 3);
        inside = px < W && py < H;
        pfx = (float)px;
        pfy = (float)py;
        tx0 = (float)(bx * GSR_BLOCK_X);
        ty0 = (float)(by * GSR_BLOCK_Y);
        wmax = (float)(W - 1);
        hmax = (float)(H - 1);
        lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    }

    // Gather this thread's candidate record (if `valid`), keep it if it can reach any pixel
    // of a quadrant, and compact the survivors (in thread order, i.e. range order) into the
    // LDS slots and the four quadrant lists.  Contains two workgroup barriers; the caller
    // must have passed a barrier since the previous batch's last read of `sm`.
    // `qlimit` (optional, LDS): quadrant q only keeps positions < qlimit[q].
    __device__ __forceinline__ void stage(TileStageLDS& sm, bool valid, uint32_t position, uint32_t gid,
                                          const Rec* rec, const uint32_t* qlimit = nullptr) {
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        Rec r;
        uint32_t qmask = 0;
        if (valid) {
            r = rec[gid];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float qx0 = tx0 + (q & 1) * 8.f, qy0 = ty0 + (q >> 1) * 8.f;
                const float qx1 = fminf(qx0 + 7.f, wmax), qy1 = fminf(qy0 + 7.f, hmax);
                if (qx0 <= wmax && qy0 <= hmax && (!qlimit || position < qlimit[q]) &&
                    box_reachable(r.a.z, r.a.w, r.b.x, r.c.y, qx0 - r.a.x, qx1 - r.a.x, qy0 - r.a.y, qy1 - r.a.y))
                    qmask |= 1u << q;
            }
        }
        const bool keep = qmask != 0;
        const uint64_t bk = __ballot(keep);
        uint64_t bq[4];
#pragma unroll
        for (int q = 0; q < 4; q++) bq[q] = __ballot((qmask >> q) & 1u);
        if (lane == 0) {
            sm.wcnt[wave][0] = (uint32_t)__popcll(bk);
#pragma unroll
            for (int q = 0; q < 4; q++) sm.wcnt[wave][1 + q] = (uint32_t)__popcll(bq[q]);
        }
        __syncthreads();
        if (keep) {
            uint32_t slot = (uint32_t)__popcll(bk & lt);
            for (int w = 0; w < wave; w++) slot += sm.wcnt[w][0];
            sm.a[slot] = r.a;
            sm.b[slot] = r.b;
            sm.c[slot] = r.c.x;
            sm.pos[slot] = position;
            sm.id[slot] = gid;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if ((qmask >> q) & 1u) {
                    uint32_t qp = (uint32_t)__popcll(bq[q] & lt);
                    for (int w = 0; w < wave; w++) qp += sm.wcnt[w][1 + q];
                    sm.qidx[q][qp] = (uint16_t)slot;
                }
            }
        }
        if (tid < 4) sm.qcnt[tid] = sm.wcnt[0][1 + tid] + sm.wcnt[1][1 + tid] + sm.wcnt[2][1 + tid] + sm.wcnt[3][1 + tid];
        if (tid == 4) sm.cnt = sm.wcnt[0][0] + sm.wcnt[1][0] + sm.wcnt[2][0] + sm.wcnt[3][0];
        __syncthreads();
    }
};

}  // namespace gsr
