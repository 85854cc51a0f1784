// gsr_render_bwd.hip -- per-tile back-to-front gradient replay (backward.cu:399-557).
//
// gfx950 design (the reference issues 9 float atomics to global memory per contributing
// (pixel, Gaussian) pair, backward.cu:523,545-554):
//  * per Gaussian, the 64 lanes of a wave reduce their 9 partial gradients in registers
//    (skipped entirely when no lane of the wave contributes: wave-uniform ballot);
//  * lane 0 of each wave adds the 9 wave sums into a per-tile LDS accumulator
//    (ds_add_f32), so the 4 waves of the tile meet in LDS;
//  * after each 256-Gaussian batch the tile flushes one 9-float row per Gaussian to the
//    64-B per-Gaussian accumulator line with global atomics laid out so that one
//    wave-instruction touches 4 whole lines (one request per Gaussian per tile);
//  * the replay starts at the tile's largest n_contrib instead of the range end
//    (Gaussians past every pixel's last contributor are skipped by the reference too).
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

__device__ __forceinline__ unsigned xcd_remap_b(unsigned b, unsigned n) {
    const unsigned q = n >> 3, r = n & 7u, x = b & 7u;
    const unsigned base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs a) {
    __shared__ float4 s_a[256];
    __shared__ float4 s_b[256];
    __shared__ float s_c[256];
    __shared__ uint32_t s_id[256];
    __shared__ float s_acc[256][9];
    __shared__ uint32_t s_max;
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap_b(blockIdx.x, ntile);
    const unsigned bx = tile % a.grid_x, by = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int px = bx * GSR_BLOCK_X + (wave & 1) * 8 + (lane & 7);
    const int py = by * GSR_BLOCK_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int pix = a.W * py + px;
    const int HW = a.H * a.W;

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

    // tile-wide max of n_contrib
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
        const int cnt = (nmax - b0) < 256 ? (nmax - b0) : 256;
        __syncthreads();
        if (tid < cnt) {
            const int p = nmax - 1 - (b0 + tid);
            const uint32_t id = a.point_list[range.x + p];
            const Rec r = a.rec[id];
            s_id[tid] = id;
            s_a[tid] = r.a;
            s_b[tid] = r.b;
            s_c[tid] = r.c.x;
        }
#pragma unroll
        for (int v = 0; v < 9; v++) s_acc[tid][v] = 0.f;
        __syncthreads();
        for (int k = 0; k < cnt; k++) {
            const uint32_t p = (uint32_t)(nmax - 1 - (b0 + k));
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f, g4 = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool active = false;
            if (p < last_contributor) {
                const float4 A = s_a[k];
                const float4 B = s_b[k];
                const float dx = A.x - pfx, dy = A.y - pfy;
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                if (!(power > 0.0f)) {
                    const float G = expf(power);
                    const float alpha = fminf(0.99f, B.y * G);
                    if (!(alpha < 1.0f / 255.0f)) {
                        active = true;
                        T = T / (1.f - alpha);
                        const float dchannel_dcolor = alpha * T;
                        const float c0 = B.z, c1 = B.w, c2 = s_c[k];
                        float dL_dalpha = 0.0f;
                        acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                        acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                        acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                        lc0 = c0; lc1 = c1; lc2 = c2;
                        dL_dalpha += (c0 - acc0) * dpx0;
                        dL_dalpha += (c1 - acc1) * dpx1;
                        dL_dalpha += (c2 - acc2) * dpx2;
                        g6 = dchannel_dcolor * dpx0;
                        g7 = dchannel_dcolor * dpx1;
                        g8 = dchannel_dcolor * dpx2;
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = B.y * dL_dalpha;
                        const float gdx = G * dx;
                        const float gdy = G * dy;
                        const float dG_ddelx = -gdx * A.z - gdy * A.w;
                        const float dG_ddely = -gdy * B.x - gdx * A.w;
                        g0 = dL_dG * dG_ddelx * ddelx_dx;
                        g1 = dL_dG * dG_ddely * ddely_dy;
                        g2 = -0.5f * gdx * dx * dL_dG;
                        g3 = -0.5f * gdx * dy * dL_dG;
                        g4 = -0.5f * gdy * dy * dL_dG;
                        g5 = G * dL_dalpha;
                    }
                }
            }
            if (__ballot(active) != 0ull) {
                g0 = wave_reduce_sum(g0);
                g1 = wave_reduce_sum(g1);
                g2 = wave_reduce_sum(g2);
                g3 = wave_reduce_sum(g3);
                g4 = wave_reduce_sum(g4);
                g5 = wave_reduce_sum(g5);
                g6 = wave_reduce_sum(g6);
                g7 = wave_reduce_sum(g7);
                g8 = wave_reduce_sum(g8);
                if (lane == 0) {
                    float* row = s_acc[k];
                    atomicAdd(row + 0, g0);
                    atomicAdd(row + 1, g1);
                    atomicAdd(row + 2, g2);
                    atomicAdd(row + 3, g3);
                    atomicAdd(row + 4, g4);
                    atomicAdd(row + 5, g5);
                    atomicAdd(row + 6, g6);
                    atomicAdd(row + 7, g7);
                    atomicAdd(row + 8, g8);
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
