// gsr_epilogue.hip -- render()'s image-space tail (gaussian_renderer/__init__.py:226-276) as
// one kernel each way, after the multi-channel composite:
//   normal     = ((N01 - 0.5) * 2 * (normal_view ? -1 : 1)) * S + (1 - S)
//   normal_ref = normalize(cross(dx, dy)) * A + (1 - S)       (interior pixels; 0 * A + 1 - S
//                on the one-pixel border), with the points of depth_to_normal
//                (graphics_utils.py:141-169): p = (D * S) * rays_d + o, dx the row
//                difference p[y+1] - p[y-1], dy the column difference p[x+1] - p[x-1]
// N01 = the composited 0.5 n + 0.5 image, D = depth (channel 0), A = alpha (detached, as
// the reference), S = the sky mask; rays_d(x, y) = x M0 + y M1 + M2 and o are the camera's
// (K^-1^T R^T rows and centre, computed on the host).
// The backward gathers, per pixel, the contributions of the four neighbours whose
// differences it enters (their cross-product derivatives made once per tile in LDS), so it
// needs no atomics.
#include "gsr_kernels.hpp"

namespace gsr {

struct EpiCam {
    float m[9];  // rows M0, M1, M2
    float o[3];
};

__device__ __forceinline__ float3 epi_point(const EpiCam& c, const float* depth, const float* sky, int W, int x, int y) {
    const float d = depth[y * W + x] * sky[y * W + x];
    const float fx = (float)x, fy = (float)y;
    const float rx = fx * c.m[0] + fy * c.m[3] + c.m[6];
    const float ry = fx * c.m[1] + fy * c.m[4] + c.m[7];
    const float rz = fx * c.m[2] + fy * c.m[5] + c.m[8];
    return make_float3(d * rx + c.o[0], d * ry + c.o[1], d * rz + c.o[2]);
}

__device__ __forceinline__ float3 f3sub(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float3 f3cross(float3 a, float3 b) {
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// a = dx (rows), b = dy (columns) at interior pixel (x, y)
__device__ __forceinline__ void epi_diffs(const EpiCam& c, const float* depth, const float* sky, int W, int x, int y,
                                          float3& a, float3& b) {
    a = f3sub(epi_point(c, depth, sky, W, x, y + 1), epi_point(c, depth, sky, W, x, y - 1));
    b = f3sub(epi_point(c, depth, sky, W, x + 1, y), epi_point(c, depth, sky, W, x - 1, y));
}

__global__ void __launch_bounds__(256) k_epilogue_fwd(int W, int H, EpiCam cam, const float* n01, const float* depth,
                                                       const float* alpha, const float* sky, float nsign,
                                                       float* normal, float* normal_ref) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int HW = W * H;
    if (i >= HW) return;
    const int x = i % W, y = i / W;
    const float s = sky[i];
    const float bgk = 1.f - s;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) normal[ch * HW + i] = ((n01[ch * HW + i] - 0.5f) * 2.f * nsign) * s + bgk;
    float3 n = make_float3(0.f, 0.f, 0.f);
    if (x >= 1 && x <= W - 2 && y >= 1 && y <= H - 2) {
        float3 a, b;
        epi_diffs(cam, depth, sky, W, x, y, a, b);
        const float3 cr = f3cross(a, b);
        const float len = fmaxf(sqrtf(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z), 1e-12f);  // F.normalize eps
        n = make_float3(cr.x / len, cr.y / len, cr.z / len);
    }
    const float al = alpha[i];
    normal_ref[i] = n.x * al + bgk;
    normal_ref[HW + i] = n.y * al + bgk;
    normal_ref[2 * HW + i] = n.z * al + bgk;
}

// d(normalize(c)) for upstream g: (g - n (n.g)) / |c| (|c| above eps; else g / eps)
__device__ __forceinline__ float3 epi_dcross(float3 cr, float3 g) {
    const float l = sqrtf(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z);
    if (l <= 1e-12f) return make_float3(g.x / 1e-12f, g.y / 1e-12f, g.z / 1e-12f);
    const float3 n = make_float3(cr.x / l, cr.y / l, cr.z / l);
    const float ng = n.x * g.x + n.y * g.y + n.z * g.z;
    return make_float3((g.x - n.x * ng) / l, (g.y - n.y * ng) / l, (g.z - n.z * ng) / l);
}

// One 32x8 output tile per workgroup, in three LDS phases: the back-projected points of the
// tile plus a two-pixel margin; for every interior pixel q of the tile plus a one-pixel margin
// the derivative of its normal_ref term, dL/d(cross) -> dL/da = b x dc and dL/db = dc x a
// (each computed once instead of once per neighbour that reads it); then per pixel the four
// neighbours' contributions in the fixed order (x, y-1), (x, y+1), (x-1, y), (x+1, y).
constexpr int EPI_TW = 32, EPI_TH = 8;
constexpr int EPI_QW = EPI_TW + 2, EPI_QH = EPI_TH + 2;  // q: the tile and a 1-pixel margin
constexpr int EPI_PW = EPI_TW + 4, EPI_PH = EPI_TH + 4;  // points: a 2-pixel margin

__global__ void __launch_bounds__(256) k_epilogue_bwd(int W, int H, EpiCam cam, const float* depth,
                                                       const float* alpha, const float* sky, float nsign,
                                                       const float* g_normal, const float* g_normal_ref, float* d_n01,
                                                       float* d_depth) {
    __shared__ float3 s_p[EPI_PH][EPI_PW];
    __shared__ float3 s_ga[EPI_QH][EPI_QW], s_gb[EPI_QH][EPI_QW];
    const int HW = W * H;
    const int x0 = blockIdx.x * EPI_TW, y0 = blockIdx.y * EPI_TH;
    const int tx = threadIdx.x % EPI_TW, ty = threadIdx.x / EPI_TW;
    const int x = x0 + tx, y = y0 + ty;
    const bool in = x < W && y < H;
    const int i = y * W + x;
    const float s = in ? sky[i] : 0.f;
    if (d_n01 && in) {
#pragma unroll
        for (int ch = 0; ch < 3; ch++) d_n01[ch * HW + i] = g_normal ? g_normal[ch * HW + i] * 2.f * nsign * s : 0.f;
    }
    if (!d_depth) return;
    if (!g_normal_ref) {
        if (in) d_depth[i] = s * 0.f;
        return;
    }
    for (int e = threadIdx.x; e < EPI_PH * EPI_PW; e += 256) {
        const int px = x0 - 2 + e % EPI_PW, py = y0 - 2 + e / EPI_PW;
        s_p[e / EPI_PW][e % EPI_PW] = (px >= 0 && px < W && py >= 0 && py < H) ? epi_point(cam, depth, sky, W, px, py)
                                                                                : make_float3(0.f, 0.f, 0.f);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < EPI_QH * EPI_QW; e += 256) {
        const int lx = e % EPI_QW, ly = e / EPI_QW;  // q = (x0 - 1 + lx, y0 - 1 + ly); its points at (lx + 1, ly + 1)
        const int qx = x0 - 1 + lx, qy = y0 - 1 + ly;
        float3 ga = make_float3(0.f, 0.f, 0.f), gb = ga;
        if (qx >= 1 && qx <= W - 2 && qy >= 1 && qy <= H - 2) {
            const int j = qy * W + qx;
            const float al = alpha[j];
            const float3 g = make_float3(g_normal_ref[j] * al, g_normal_ref[HW + j] * al, g_normal_ref[2 * HW + j] * al);
            const float3 a = f3sub(s_p[ly + 2][lx + 1], s_p[ly][lx + 1]);
            const float3 b = f3sub(s_p[ly + 1][lx + 2], s_p[ly + 1][lx]);
            const float3 dc = epi_dcross(f3cross(a, b), g);
            // c = a x b: dL/da = b x dc, dL/db = dc x a
            ga = f3cross(b, dc);
            gb = f3cross(dc, a);
        }
        s_ga[ly][lx] = ga;
        s_gb[ly][lx] = gb;
    }
    __syncthreads();
    if (!in) return;
    // this pixel enters a of (x, y-1) (+) and (x, y+1) (-), b of (x-1, y) (+) and (x+1, y) (-)
    const float3 c0 = s_ga[ty][tx + 1], c1 = s_ga[ty + 2][tx + 1], c2 = s_gb[ty + 1][tx], c3 = s_gb[ty + 1][tx + 2];
    float3 gp = make_float3(0.f, 0.f, 0.f);
    gp.x += c0.x; gp.y += c0.y; gp.z += c0.z;
    gp.x += -c1.x; gp.y += -c1.y; gp.z += -c1.z;
    gp.x += c2.x; gp.y += c2.y; gp.z += c2.z;
    gp.x += -c3.x; gp.y += -c3.y; gp.z += -c3.z;
    const float fx = (float)x, fy = (float)y;
    const float rx = fx * cam.m[0] + fy * cam.m[3] + cam.m[6];
    const float ry = fx * cam.m[1] + fy * cam.m[4] + cam.m[7];
    const float rz = fx * cam.m[2] + fy * cam.m[5] + cam.m[8];
    d_depth[i] = s * (gp.x * rx + gp.y * ry + gp.z * rz);
}

void launch_epilogue_fwd(int W, int H, const float* m12, const float* n01, const float* depth, const float* alpha,
                         const float* sky, int normal_view, float* normal, float* normal_ref, hipStream_t s) {
    EpiCam c;
    for (int k = 0; k < 9; k++) c.m[k] = m12[k];
    for (int k = 0; k < 3; k++) c.o[k] = m12[9 + k];
    const int n = W * H;
    if (n == 0) return;
    hipLaunchKernelGGL(k_epilogue_fwd, dim3((n + 255) / 256), dim3(256), 0, s, W, H, c, n01, depth, alpha, sky,
                       normal_view ? -1.f : 1.f, normal, normal_ref);
}

void launch_epilogue_bwd(int W, int H, const float* m12, const float* depth, const float* alpha, const float* sky,
                         int normal_view, const float* g_normal, const float* g_normal_ref, float* d_n01,
                         float* d_depth, hipStream_t s) {
    EpiCam c;
    for (int k = 0; k < 9; k++) c.m[k] = m12[k];
    for (int k = 0; k < 3; k++) c.o[k] = m12[9 + k];
    const int n = W * H;
    if (n == 0) return;
    hipLaunchKernelGGL(k_epilogue_bwd, dim3((W + EPI_TW - 1) / EPI_TW, (H + EPI_TH - 1) / EPI_TH), dim3(256), 0, s, W, H,
                       c, depth, alpha, sky, normal_view ? -1.f : 1.f, g_normal, g_normal_ref, d_n01, d_depth);
}

}  // namespace gsr
