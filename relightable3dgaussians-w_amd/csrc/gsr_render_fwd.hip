// gsr_render_fwd.hip -- per-tile front-to-back alpha compositing (forward.cu:261-374).
//
// gfx950 design:
//  * one 256-thread workgroup per 16x16 tile, each wave owns an 8x8 quadrant (compact
//    footprint -> coherent early exit); tiles are remapped so each XCD's L2 serves a
//    contiguous band of the image (xcd_remap);
//  * staging: each thread gathers one 48-B record of the batch and tests it
//    conservatively against the four quadrants (box_reachable).  Survivors are compacted
//    into LDS with wave ballots, and every quadrant gets its own index list, so each wave
//    iterates only over Gaussians that can reach alpha >= 1/255 somewhere in its 8x8
//    pixels.  The original range position travels with the record, so n_contrib (the
//    reference's last_contributor) is unchanged;
//  * inner loop: branch-free (predicated) blend on broadcast LDS reads, v_exp_f32, colour
//    from LDS (the reference re-reads colours from global memory per pixel); the wave
//    leaves the loop as soon as all its pixels are saturated;
//  * block-wide early exit with __syncthreads_count exactly as the reference.
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

__global__ void __launch_bounds__(256) k_render_fwd(RenderFwdArgs a) {
    TileStage st;
    __shared__ TileStageLDS sm;
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap(blockIdx.x, ntile);
    st.init(tile, a.grid_x, a.W, a.H);
    const int tid = threadIdx.x, wave = tid >> 6;
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    bool done = !st.inside;
    float T = 1.0f;
    uint32_t last_contributor = 0;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    for (int b0 = 0; b0 < n; b0 += 256) {
        if (__syncthreads_count(done) == 256) break;
        const int j = b0 + tid;
        uint32_t id = 0;
        if (j < n) id = a.point_list[range.x + j];
        st.stage(sm, j < n, j, id, a.rec);
        if (!__all(done)) {
            const int cnt = sm.qcnt[wave];
            for (int k = 0; k < cnt; k++) {
                const int s = sm.qidx[wave][k];
                const float4 A = sm.a[s];
                const float4 B = sm.b[s];
                const float dx = A.x - st.pfx, dy = A.y - st.pfy;
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                const float alpha = fminf(0.99f, B.y * tile_exp(power));
                const bool hit = !done && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
                const float test_T = T * (1 - alpha);
                const bool sat = hit && test_T < 0.0001f;  // saturating Gaussian is not blended
                const bool blend = hit && !sat;
                done = done || sat;
                const float w = blend ? alpha * T : 0.f;
                C0 += B.z * w;
                C1 += B.w * w;
                C2 += sm.c[s] * w;
                T = blend ? test_T : T;
                last_contributor = blend ? sm.pos[s] + 1u : last_contributor;
                if (__all(done)) break;
            }
        }
    }
    if (st.inside) {
        const int pix = a.W * st.py + st.px;
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
