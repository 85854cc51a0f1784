// gsr_render_fwd.hip -- per-tile front-to-back alpha compositing (forward.cu:261-374).
//
// gfx950 design:
//  * one 256-thread workgroup per 16x16 tile; each wave owns an 8x8 pixel quadrant
//    (compact footprint -> coherent early exit);
//  * tiles are remapped so that each XCD (private L2) works on a contiguous band of
//    the image: neighbouring tiles share Gaussian records through the same L2;
//  * the batch of 256 Gaussian records (48 B each: xy, conic, opacity, colour) is
//    gathered into LDS once per batch; the inner loop reads broadcast LDS words only
//    (the reference re-reads colours from global memory per pixel);
//  * block-wide early exit with __syncthreads_count exactly as the reference.
#include "gsr_kernels.hpp"

namespace gsr {

// bijective XCD-aware block -> tile remap (blocks b and b+8 share an XCD)
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n) {
    const unsigned q = n >> 3, r = n & 7u, x = b & 7u;
    const unsigned base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

__global__ void __launch_bounds__(256) k_render_fwd(RenderFwdArgs a) {
    __shared__ float4 s_a[256];
    __shared__ float4 s_b[256];
    __shared__ float s_c[256];
    const unsigned ntile = a.grid_x * a.grid_y;
    const unsigned tile = xcd_remap(blockIdx.x, ntile);
    const unsigned bx = tile % a.grid_x, by = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int px = bx * GSR_BLOCK_X + (wave & 1) * 8 + (lane & 7);
    const int py = by * GSR_BLOCK_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);
    bool done = !inside;
    float T = 1.0f;
    uint32_t contributor = 0, last_contributor = 0;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    for (int b0 = 0; b0 < n; b0 += 256) {
        if (__syncthreads_count(done) == 256) break;
        const int j = b0 + tid;
        if (j < n) {
            const uint32_t id = a.point_list[range.x + j];
            const Rec r = a.rec[id];
            s_a[tid] = r.a;
            s_b[tid] = r.b;
            s_c[tid] = r.c.x;
        }
        __syncthreads();
        const int cnt = (n - b0) < 256 ? (n - b0) : 256;
        if (!done) {
            for (int k = 0; k < cnt; k++) {
                contributor++;
                const float4 A = s_a[k];
                const float4 B = s_b[k];
                const float dx = A.x - pfx, dy = A.y - pfy;
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, B.y * expf(power));
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
                last_contributor = contributor;
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
