// gsr_kernels.hpp -- kernel argument blocks and host launchers shared by the HIP
// translation units and the C ABI (gsr_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsr_common.hpp"

namespace gsr {

struct PreprocessArgs {
    int P, D, M;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    int W, H;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    unsigned grid_x, grid_y;
    int prefiltered;
    // outputs
    int* radii;
    uint32_t* tiles;
    uint32_t* depth_key;
    uint2* rect;
    Rec* rec;
    unsigned* err_flag;
};

void launch_preprocess(const PreprocessArgs& a, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* viewmatrix, bool* present, hipStream_t s);

// ---- scans (gsr_scan.hip) -----------------------------------------------------------
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 4096
inline int scan_blocks(long long n) { return (int)((n + SCAN_TILE - 1) / SCAN_TILE); }

// Visibility compaction: tiles[i] > 0 <=> visible.  Produces, in index order (stable),
// vis_key[j] = depth_key[i], vis_val[j] = i for the j-th visible Gaussian, and
// totals[0] = number of visible Gaussians, totals[1..2] = 64-bit sum of tiles.
// block_tmp: scan_blocks(P) * 8 bytes (u64).
void launch_compact_visible(int P, const uint32_t* tiles, const uint32_t* depth_key, uint32_t* vis_key,
                            uint32_t* vis_val, unsigned long long* block_tmp, unsigned long long* totals,
                            hipStream_t s);

// Exclusive scan (u32) of in[0..n) -> out; block_tmp: scan_blocks(n) u32;
// total (optional) receives the sum.  If gather != nullptr the input is in[gather[i]].
void launch_exclusive_scan_u32(long long n, const uint32_t* in, const uint32_t* gather, uint32_t* out,
                               uint32_t* block_tmp, uint32_t* total, hipStream_t s);

// ---- radix sort (gsr_sort.hip) ---------------------------------------------------------
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 16;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;  // 4096 keys per block
inline int sort_blocks(long long n) { return (int)((n + SORT_TILE - 1) / SORT_TILE); }
// scratch bytes for sort of n items
size_t radix_sort_temp_bytes(long long n);
// Stable LSD sort of (key, value) pairs on key bits [0, end_bit).  Ping-pongs between
// (keys, vals) and (keys_alt, vals_alt); returns 1 if the sorted result ended in the alt
// buffers, 0 if in the primary buffers.
int radix_sort_pairs(long long n, uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                     int end_bit, void* temp, hipStream_t s);

// ---- binning (gsr_binning.hip) ----------------------------------------------------------
// For the depth-sorted visible Gaussians: emit one (tile, gaussian) pair per touched tile,
// y-major then x, at offsets[s] (exclusive scan of tiles in depth order).
void launch_duplicate(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets, const uint2* rect,
                      unsigned grid_x, uint32_t* tile_keys, uint32_t* gauss_vals, hipStream_t s);
// ranges[t] = [first, last+1) over the tile-sorted keys; untouched tiles (0, 0).
void launch_ranges(long long R, int T, const uint32_t* sorted_tile_keys, uint2* ranges, hipStream_t s);

// ---- render (gsr_render_fwd.hip / gsr_render_bwd.hip) --------------------------------
struct RenderFwdArgs {
    int W, H;
    unsigned grid_x, grid_y;
    const uint2* ranges;
    const uint32_t* point_list;
    const Rec* rec;
    const float* bg;
    float* out_color;
    float* final_T;
    uint32_t* n_contrib;
};
void launch_render_fwd(const RenderFwdArgs& a, hipStream_t s);

struct RenderBwdArgs {
    int W, H;
    unsigned grid_x, grid_y;
    const uint2* ranges;
    const uint32_t* point_list;
    const Rec* rec;
    const float* colors;  // optional: colour source if not in rec (unused: rec holds colour)
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    float* acc;  // [P][ACC_STRIDE]
};
void launch_render_bwd(const RenderBwdArgs& a, hipStream_t s);

struct PreprocessBwdArgs {
    int P, D, M;
    const float* means3D;
    const int* radii;
    const float* shs;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    const float* cov3D_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    const float* acc;  // [P][ACC_STRIDE] from the render backward
    // outputs (fully written, no pre-zeroing needed)
    float* dL_dmean2D;
    float* dL_dconic;
    float* dL_dopacity;
    float* dL_dcolor;
    float* dL_dmean3D;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dscale;
    float* dL_drot;
};
void launch_preprocess_bwd(const PreprocessBwdArgs& a, hipStream_t s);

}  // namespace gsr
