// gsr_det.hip -- the deterministic backward's fixed-order gradient sum (a
// reproducible alternative to the tile passes' atomics, for diffing and debugging).
//
// In deterministic mode the backward tile passes write each (tile, Gaussian) pair's partial
// gradient sums to that instance's row instead of adding them into the Gaussian's
// accumulator line (gsr_render_bwd.hip / gsr_render_mc.hip, `partial`), and heavy tiles are
// not split, so every row has exactly one writer.  This kernel then sums the rows of each
// Gaussian in one fixed order: its tiles in row-major order over its rect (the reference's
// duplicateWithKeys order, forward.cu:261-301 / rasterizer_impl.cu:79-99), its position in
// each tile's list found by binary search on (depth key, index) -- the binning's order
// (bit-exact with the reference's sort, tests/test_gpu_rasterizer.py).  Results are then
// bit-reproducible run to run.  One thread per Gaussian: a debugging path, not a fast one.
#include "gsr_kernels.hpp"

namespace gsr {

__global__ void __launch_bounds__(256) k_det_gather(DetGatherArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P || !(a.radii[idx] > 0)) return;
    const uint2 r = a.rect[idx];
    const unsigned x0 = r.x & 0xffffu, x1 = min(r.x >> 16, a.gx), y0 = r.y & 0xffffu, y1 = min(r.y >> 16, a.gy);
    const uint32_t key = a.depth_key[idx];
    float* acc = a.acc + (size_t)idx * ACC_STRIDE;
    float* feat = a.dL_dfeat ? a.dL_dfeat + (size_t)idx * a.fstride : nullptr;
    unsigned missing = 0;
    for (unsigned ty = y0; ty < y1; ty++) {
        for (unsigned tx = x0; tx < x1; tx++) {
            const uint2 rg = a.ranges[ty * a.gx + tx];
            // lower bound of (key, idx) in the tile's (depth key, index)-ordered list
            uint32_t lo = rg.x, hi = rg.y;
            while (lo < hi) {
                const uint32_t mid = lo + ((hi - lo) >> 1);
                const uint32_t g = a.point_list[mid];
                const uint32_t k = a.depth_key[g];
                if (k < key || (k == key && g < (uint32_t)idx)) lo = mid + 1;
                else hi = mid;
            }
            if (lo >= rg.y || a.point_list[lo] != (uint32_t)idx) {
                missing++;
                continue;
            }
            if (a.mode == 0) {
                const float4* row = reinterpret_cast<const float4*>(a.partial + (size_t)lo * DET_ROW3);
                const float4 p0 = row[0], p1 = row[1], p2 = row[2];
                acc[0] += p0.x;
                acc[1] += p0.y;
                acc[2] += p0.z;
                acc[3] += p0.w;
                acc[4] += p1.x;
                acc[5] += p1.y;
                acc[6] += p1.z;
                acc[7] += p1.w;
                acc[8] += ((p2.x + p2.y) + p2.z) + p2.w;
            } else {
                const float* row = a.partial + (size_t)lo * a.pstride;
                for (int j = 0; j < 6; j++) acc[j] += row[j];
                for (int c = 0; c < a.nch; c++) feat[c] += row[6 + c];
            }
        }
    }
    if (missing && a.missing) atomicAdd(a.missing, missing);
}

void launch_det_gather(const DetGatherArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    hipLaunchKernelGGL(k_det_gather, dim3((a.P + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace gsr

// ---- GSR_DEBUG invariant checks -------------------------------------------------------------
namespace gsr {

__device__ __forceinline__ void dbg_fail(DebugReport* rep, unsigned code, unsigned a, unsigned b, unsigned c) {
    if (atomicCAS(&rep->code, 0u, code) == 0u) {
        rep->a = a;
        rep->b = b;
        rep->c = c;
    }
}

// one thread per tile: the tile's range and list
__global__ void __launch_bounds__(256) k_check_tile(int P, long long R, unsigned gx, unsigned ntile, const int* radii,
                                                     const uint2* rect, const uint32_t* depth_key, const uint2* ranges,
                                                     const uint32_t* point_list, uint32_t* count,
                                                     unsigned long long* total, DebugReport* rep) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntile) return;
    const uint2 rg = ranges[t];
    if (rg.y < rg.x || (long long)rg.y > R) {
        dbg_fail(rep, DBG_RANGE, t, rg.x, rg.y);
        return;
    }
    atomicAdd(total, (unsigned long long)(rg.y - rg.x));
    const unsigned tx = t % gx, ty = t / gx;
    uint32_t pk = 0, pid = 0;
    for (uint32_t k = rg.x; k < rg.y; k++) {
        const uint32_t id = point_list[k];
        if (id >= (uint32_t)P) {
            dbg_fail(rep, DBG_ID, t, k, id);
            return;
        }
        if (!(radii[id] > 0)) {
            dbg_fail(rep, DBG_CULLED, t, k, id);
            return;
        }
        const uint2 r = rect[id];
        if (tx < (r.x & 0xffffu) || tx >= (r.x >> 16) || ty < (r.y & 0xffffu) || ty >= (r.y >> 16)) {
            dbg_fail(rep, DBG_OUTSIDE_RECT, t, k, id);
            return;
        }
        const uint32_t dk = depth_key[id];
        if (k > rg.x && !(pk < dk || (pk == dk && pid < id))) {
            dbg_fail(rep, DBG_ORDER, t, k, id);
            return;
        }
        pk = dk;
        pid = id;
        atomicAdd(count + id, 1u);
    }
}

// one thread per Gaussian: listed exactly area(rect) times
__global__ void __launch_bounds__(256) k_check_counts(int P, const int* radii, const uint2* rect, const uint32_t* count,
                                                       DebugReport* rep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    unsigned want = 0;
    if (radii[i] > 0) {
        const uint2 r = rect[i];
        want = ((r.x >> 16) - (r.x & 0xffffu)) * ((r.y >> 16) - (r.y & 0xffffu));
    }
    if (count[i] != want) dbg_fail(rep, DBG_COUNT, (unsigned)i, count[i], want);
}

// one thread per pixel: n_contrib within its tile's list; the total equals R
__global__ void __launch_bounds__(256) k_check_pixels(long long R, unsigned gx, int W, int H, const uint2* ranges,
                                                       const uint32_t* n_contrib, const unsigned long long* total,
                                                       DebugReport* rep) {
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix == 0 && (long long)*total != R) dbg_fail(rep, DBG_TOTAL, (unsigned)*total, (unsigned)R, 0u);
    if (pix >= W * H) return;
    const int x = pix % W, y = pix / W;
    const uint2 rg = ranges[(y / GSR_BLOCK_Y) * gx + x / GSR_BLOCK_X];
    if (n_contrib && n_contrib[pix] > rg.y - rg.x) dbg_fail(rep, DBG_NCONTRIB, (unsigned)pix, n_contrib[pix], rg.y - rg.x);
}

void launch_check_lists(int P, long long R, unsigned gx, unsigned gy, int W, int H, const int* radii,
                        const uint2* rect, const uint32_t* depth_key, const uint2* ranges, const uint32_t* point_list,
                        const uint32_t* n_contrib, uint32_t* count, unsigned long long* total, DebugReport* rep,
                        hipStream_t s) {
    const unsigned ntile = gx * gy;
    if (ntile) hipLaunchKernelGGL(k_check_tile, dim3((ntile + 255) / 256), dim3(256), 0, s, P, R, gx, ntile, radii, rect,
                                  depth_key, ranges, point_list, count, total, rep);
    if (P > 0) hipLaunchKernelGGL(k_check_counts, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, rect, count, rep);
    const int npix = W * H;
    if (npix > 0) hipLaunchKernelGGL(k_check_pixels, dim3((npix + 255) / 256), dim3(256), 0, s, R, gx, W, H, ranges,
                                     n_contrib, total, rep);
}

}  // namespace gsr
