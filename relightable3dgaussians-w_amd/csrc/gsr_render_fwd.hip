// gsr_render_fwd.hip -- per-tile front-to-back alpha compositing (forward.cu:261-374).
//
// gfx950 design:
//  * one 256-thread workgroup per 16x16 tile, each wave owns an 8x8 quadrant (compact
//    footprint -> coherent early exit); tiles are remapped so each XCD's L2 serves a
//    contiguous band of the image (xcd_remap);
//  * staging: each thread gathers one 48-B record of the batch, tests it conservatively
//    against the tile and its four quadrants (box_reachable), and the survivors are
//    compacted into LDS with wave ballots -- the inner loop never sees a Gaussian that
//    cannot reach alpha >= 1/255 in this tile, and a wave skips (uniformly) the ones that
//    miss its quadrant.  The original range position travels with the record, so
//    n_contrib (the reference's last_contributor) is unchanged;
//  * inner loop: broadcast LDS reads, v_exp_f32, colour from LDS (the reference re-reads
//    colours from global memory per pixel);
//  * block-wide early exit with __syncthreads_count exactly as the reference.
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

__global__ void __launch_bounds__(256) k_render_fwd(RenderFwdArgs a) {
    __shared__ float4 s_a[256];
    __shared__ float4 s_b[256];
    __shared__ float s_c[256];
    __shared__ uint32_t s_meta[256];
    __shared__ uint32_t s_wcnt[4];
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap(blockIdx.x, ntile);
    const unsigned bx = tile % a.grid_x, by = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int px = bx * GSR_BLOCK_X + (wave & 1) * 8 + (lane & 7);
    const int py = by * GSR_BLOCK_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    // pixel boxes (integer pixel coordinates) of the tile's four quadrants, clipped to the image
    const float tx0 = (float)(bx * GSR_BLOCK_X), ty0 = (float)(by * GSR_BLOCK_Y);
    const float wmax = (float)(a.W - 1), hmax = (float)(a.H - 1);
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    bool done = !inside;
    float T = 1.0f;
    uint32_t last_contributor = 0;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    for (int b0 = 0; b0 < n; b0 += 256) {
        if (__syncthreads_count(done) == 256) break;
        const int j = b0 + tid;
        bool keep = false;
        uint32_t qmask = 0;
        Rec r;
        if (j < n) {
            const uint32_t id = a.point_list[range.x + j];
            r = a.rec[id];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float qx0 = tx0 + (q & 1) * 8.f, qy0 = ty0 + (q >> 1) * 8.f;
                const float qx1 = fminf(qx0 + 7.f, wmax), qy1 = fminf(qy0 + 7.f, hmax);
                if (qx0 <= wmax && qy0 <= hmax &&
                    box_reachable(r.a.z, r.a.w, r.b.x, r.c.y, qx0 - r.a.x, qx1 - r.a.x, qy0 - r.a.y, qy1 - r.a.y))
                    qmask |= 1u << q;
            }
            keep = qmask != 0;
        }
        const uint64_t bal = __ballot(keep);
        if (lane == 0) s_wcnt[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        const uint32_t w0 = s_wcnt[0], w1 = s_wcnt[1], w2 = s_wcnt[2], w3 = s_wcnt[3];
        const int cnt = (int)(w0 + w1 + w2 + w3);
        if (keep) {
            const uint32_t off = (wave > 0 ? w0 : 0u) + (wave > 1 ? w1 : 0u) + (wave > 2 ? w2 : 0u);
            const uint32_t slot = off + (uint32_t)__popcll(bal & lt);
            s_a[slot] = r.a;
            s_b[slot] = r.b;
            s_c[slot] = r.c.x;
            s_meta[slot] = ((uint32_t)j << 4) | qmask;
        }
        __syncthreads();
        if (!done) {
            for (int k = 0; k < cnt; k++) {
                const uint32_t meta = s_meta[k];
                if (!((meta >> wave) & 1u)) continue;  // wave-uniform: misses this quadrant
                const float4 A = s_a[k];
                const float4 B = s_b[k];
                const float dx = A.x - pfx, dy = A.y - pfy;
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, B.y * tile_exp(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = T * (1 - alpha);
                if (test_T < 0.0001f) {
                    done = true;
                    break;
                }
                const float w = alpha * T;
                C0 += B.z * w;
                C1 += B.w * w;
                C2 += s_c[k] * w;
                T = test_T;
                last_contributor = (meta >> 4) + 1u;  // position in the range, 1-based
            }
        }
    }
    if (inside) {
        const int pix = a.W * py + px;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last_contributor;
        const int HW = a.H * a.W;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[HW + pix] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix] = C2 + T * a.bg[2];
    }
}

void launch_render_fwd(const RenderFwdArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_render_fwd, dim3(ntile), dim3(256), 0, s, a);
}

}  // namespace gsr
