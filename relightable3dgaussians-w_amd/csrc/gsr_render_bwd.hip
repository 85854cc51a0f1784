// gsr_render_bwd.hip -- per-tile back-to-front gradient replay (backward.cu:399-557).
//
// gfx950 design (the reference issues 9 float atomics to global memory per contributing
// (pixel, Gaussian) pair, backward.cu:523,545-554):
//  * the replay starts at the tile's largest n_contrib (positions past every pixel's last
//    contributor are skipped by the reference too) and stages records from the back with
//    the forward's conservative tile/quadrant culling and ballot compaction;
//  * per Gaussian, each 16-lane row of the wave reduces its 9 partial gradients on the
//    VALU (4 fused DPP adds per value) -- skipped when no lane of the wave contributes --
//    and 36 lanes (9 per row) add the row sums into the tile's LDS row with one ds_add;
//  * after each batch the tile flushes one 9-float row per Gaussian to the 64-B
//    per-Gaussian accumulator line; one wave-instruction covers 4 whole lines.
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs a) {
    __shared__ float4 s_a[256];
    __shared__ float4 s_b[256];
    __shared__ float s_c[256];
    __shared__ uint32_t s_meta[256];
    __shared__ uint32_t s_id[256];
    __shared__ float s_acc[256][9];
    __shared__ uint32_t s_wcnt[4];
    __shared__ uint32_t s_max;
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap(blockIdx.x, ntile);
    const unsigned bx = tile % a.grid_x, by = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int px = bx * GSR_BLOCK_X + (wave & 1) * 8 + (lane & 7);
    const int py = by * GSR_BLOCK_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    const float tx0 = (float)(bx * GSR_BLOCK_X), ty0 = (float)(by * GSR_BLOCK_Y);
    const float wmax = (float)(a.W - 1), hmax = (float)(a.H - 1);
    const uint2 range = a.ranges[tile];
    const int pix = a.W * py + px;
    const int HW = a.H * a.W;
    const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

    const float T_final = inside ? a.final_T[pix] : 0.f;
    float T = T_final;
    const uint32_t last_contributor = inside ? a.n_contrib[pix] : 0u;
    float dpx0 = 0.f, dpx1 = 0.f, dpx2 = 0.f;
    if (inside) {
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
    if (tid == 0) s_max = 0;
    __syncthreads();
    if (lane == 0) atomicMax(&s_max, m);
    __syncthreads();
    const int nmax = (int)s_max;

    for (int b0 = 0; b0 < nmax; b0 += 256) {
        const int nb = (nmax - b0) < 256 ? (nmax - b0) : 256;
        __syncthreads();  // previous batch's flush is done with the LDS rows
        bool keep = false;
        uint32_t qmask = 0, id = 0;
        int p = 0;
        Rec r;
        if (tid < nb) {
            p = nmax - 1 - (b0 + tid);
            id = a.point_list[range.x + p];
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
            s_meta[slot] = ((uint32_t)p << 4) | qmask;
            s_id[slot] = id;
        }
#pragma unroll
        for (int v = 0; v < 9; v++) s_acc[tid][v] = 0.f;
        __syncthreads();
        for (int k = 0; k < cnt; k++) {
            const uint32_t meta = s_meta[k];
            if (!((meta >> wave) & 1u)) continue;  // wave-uniform
            const uint32_t pos = meta >> 4;
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f, g4 = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool active = false;
            if (pos < last_contributor) {
                const float4 A = s_a[k];
                const float4 B = s_b[k];
                const float dx = A.x - pfx, dy = A.y - pfy;
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                if (!(power > 0.0f)) {
                    const float G = tile_exp(power);
                    const float alpha = fminf(0.99f, B.y * G);
                    if (!(alpha < 1.0f / 255.0f)) {
                        active = true;
                        const float inv = __builtin_amdgcn_rcpf(1.f - alpha);
                        T = T * inv;
                        const float dchannel_dcolor = alpha * T;
                        const float c0 = B.z, c1 = B.w, c2 = s_c[k];
                        acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                        acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                        acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                        lc0 = c0; lc1 = c1; lc2 = c2;
                        float dL_dalpha = (c0 - acc0) * dpx0 + (c1 - acc1) * dpx1 + (c2 - acc2) * dpx2;
                        g6 = dchannel_dcolor * dpx0;
                        g7 = dchannel_dcolor * dpx1;
                        g8 = dchannel_dcolor * dpx2;
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final * inv) * bg_dot;
                        const float dL_dG = B.y * dL_dalpha;
                        const float gdx = G * dx;
                        const float gdy = G * dy;
                        const float dG_ddelx = -gdx * A.z - gdy * A.w;
                        const float dG_ddely = -gdy * B.x - gdx * A.w;
                        g0 = dL_dG * dG_ddelx * ddelx_dx;
                        g1 = dL_dG * dG_ddely * ddely_dy;
                        const float h = -0.5f * dL_dG;
                        g2 = h * gdx * dx;
                        g3 = h * gdx * dy;
                        g4 = h * gdy * dy;
                        g5 = G * dL_dalpha;
                    }
                }
            }
            if (__ballot(active) != 0ull) {
                // 16-lane row sums on the VALU, then lanes c < 9 of every row add component c
                // of their row into the tile's LDS row (one ds_add_f32, 4 rows per address)
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
                    atomicAdd(&s_acc[k][c], v);
                }
            }
        }
        __syncthreads();
        for (int q = tid; q < cnt * 16; q += 256) {
            const int j = q >> 4, c = q & 15;
            if (c < 9) {
                const float v = s_acc[j][c];
                if (v != 0.f) atomicAdd(a.acc + (size_t)s_id[j] * ACC_STRIDE + c, v);
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
