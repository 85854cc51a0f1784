// gsr_render_bwd.hip -- per-tile back-to-front gradient replay (backward.cu:399-557).
//
// gfx950 design (the reference issues 9 float atomics to global memory per contributing
// (pixel, Gaussian) pair, backward.cu:523,545-554):
//  * the replay starts at the tile's largest n_contrib (positions past every pixel's last
//    contributor are skipped by the reference too) and stages records from the back with
//    the forward's conservative quadrant culling into per-quadrant LDS lists (TileStage);
//  * the per-pixel recurrence (T, accum_rec, last_alpha, last_color) is evaluated
//    branch-free with predicated updates;
//  * per Gaussian, each 16-lane row of the wave reduces its 9 partial gradients on the
//    VALU (4 fused DPP adds per value) -- skipped when no lane of the wave contributes --
//    and 36 lanes (9 per row) add the row sums into the tile's LDS row with one ds_add;
//  * after each batch the tile flushes one 9-float row per Gaussian to the 64-B
//    per-Gaussian accumulator line; one wave-instruction covers 4 whole lines.
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs a) {
    TileStage st;
    __shared__ TileStageLDS sm;
    __shared__ float s_acc[256][9];
    __shared__ uint32_t s_qmax[4];
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap(blockIdx.x, ntile);
    st.init(tile, a.grid_x, a.W, a.H);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint2 range = a.ranges[tile];
    const int pix = a.W * st.py + st.px;
    const int HW = a.H * a.W;

    const float T_final = st.inside ? a.final_T[pix] : 0.f;
    float T = T_final;
    const uint32_t last_contributor = st.inside ? a.n_contrib[pix] : 0u;
    float dpx0 = 0.f, dpx1 = 0.f, dpx2 = 0.f;
    if (st.inside) {
        dpx0 = a.dL_dpix[pix];
        dpx1 = a.dL_dpix[HW + pix];
        dpx2 = a.dL_dpix[2 * HW + pix];
    }
    const float bg_dot = a.bg[0] * dpx0 + a.bg[1] * dpx1 + a.bg[2] * dpx2;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;
    float last_alpha = 0.f;
    const float ddelx_dx = 0.5f * a.W;
    const float ddely_dy = 0.5f * a.H;

    uint32_t m = last_contributor;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = __shfl_xor(m, o, 64);
        m = t > m ? t : m;
    }
    // each quadrant (wave) only replays positions below its own largest n_contrib
    if (lane == 0) s_qmax[wave] = m;
    __syncthreads();
    const int nmax = (int)max(max(s_qmax[0], s_qmax[1]), max(s_qmax[2], s_qmax[3]));

    for (int b0 = 0; b0 < nmax; b0 += 256) {
        const int nb = (nmax - b0) < 256 ? (nmax - b0) : 256;
        __syncthreads();  // the previous batch's flush is done with sm / s_acc
        const int p = nmax - 1 - (b0 + tid);
        uint32_t id = 0;
        if (tid < nb) id = a.point_list[range.x + p];
#pragma unroll
        for (int v = 0; v < 9; v++) s_acc[tid][v] = 0.f;
        st.stage(sm, tid < nb, (uint32_t)p, id, a.rec, s_qmax);
        const int cnt = sm.qcnt[wave];
        for (int k = 0; k < cnt; k++) {
            const int s = sm.qidx[wave][k];
            const float4 A = sm.a[s];
            const float4 B = sm.b[s];
            const float c2 = sm.c[s];
            const uint32_t pos = sm.pos[s];
            const float dx = A.x - st.pfx, dy = A.y - st.pfy;
            const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
            const float G = tile_exp(power);
            const float alpha = fminf(0.99f, B.y * G);
            const bool active = pos < last_contributor && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            if (__ballot(active) == 0ull) continue;  // wave-uniform
            const float inv = __builtin_amdgcn_rcpf(1.f - alpha);
            const float Tn = T * inv;
            const float dchannel_dcolor = alpha * Tn;
            const float c0 = B.z, c1 = B.w;
            const float na0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
            const float na1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
            const float na2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
            float dL_dalpha = ((c0 - na0) * dpx0 + (c1 - na1) * dpx1 + (c2 - na2) * dpx2) * Tn;
            dL_dalpha += (-T_final * inv) * bg_dot;
            const float dL_dG = B.y * dL_dalpha;
            const float gdx = G * dx;
            const float gdy = G * dy;
            const float dG_ddelx = -gdx * A.z - gdy * A.w;
            const float dG_ddely = -gdy * B.x - gdx * A.w;
            const float h = -0.5f * dL_dG;
            float g0 = active ? dL_dG * dG_ddelx * ddelx_dx : 0.f;
            float g1 = active ? dL_dG * dG_ddely * ddely_dy : 0.f;
            float g2 = active ? h * gdx * dx : 0.f;
            float g3 = active ? h * gdx * dy : 0.f;
            float g4 = active ? h * gdy * dy : 0.f;
            float g5 = active ? G * dL_dalpha : 0.f;
            float g6 = active ? dchannel_dcolor * dpx0 : 0.f;
            float g7 = active ? dchannel_dcolor * dpx1 : 0.f;
            float g8 = active ? dchannel_dcolor * dpx2 : 0.f;
            T = active ? Tn : T;
            acc0 = active ? na0 : acc0;
            acc1 = active ? na1 : acc1;
            acc2 = active ? na2 : acc2;
            lc0 = active ? c0 : lc0;
            lc1 = active ? c1 : lc1;
            lc2 = active ? c2 : lc2;
            last_alpha = active ? alpha : last_alpha;
            // 16-lane row sums on the VALU; lanes c < 9 of every row add component c of their
            // row into the tile's LDS row (one ds_add_f32, 4 rows per address)
            g0 = row_sum(g0);
            g1 = row_sum(g1);
            g2 = row_sum(g2);
            g3 = row_sum(g3);
            g4 = row_sum(g4);
            g5 = row_sum(g5);
            g6 = row_sum(g6);
            g7 = row_sum(g7);
            g8 = row_sum(g8);
            const int c = lane & 15;
            if (c < 9) {
                float v = g0;
                v = c == 1 ? g1 : v;
                v = c == 2 ? g2 : v;
                v = c == 3 ? g3 : v;
                v = c == 4 ? g4 : v;
                v = c == 5 ? g5 : v;
                v = c == 6 ? g6 : v;
                v = c == 7 ? g7 : v;
                v = c == 8 ? g8 : v;
                atomicAdd(&s_acc[s][c], v);
            }
        }
        __syncthreads();
        const int used = (int)sm.cnt;
        for (int q = tid; q < used * 16; q += 256) {
            const int j = q >> 4, c = q & 15;
            if (c < 9) {
                const float v = s_acc[j][c];
                if (v != 0.f) atomicAdd(a.acc + (size_t)sm.id[j] * ACC_STRIDE + c, v);
            }
        }
    }
}

void launch_render_bwd(const RenderBwdArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0) return;
    hipLaunchKernelGGL(k_render_bwd, dim3(ntile), dim3(256), 0, s, a);
}

}  // namespace gsr
