// gsr_kernels.hpp -- kernel argument blocks and host launchers shared by the HIP
// translation units and the C ABI (gsr_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsr_common.hpp"

namespace gsr {

constexpr int SHJAC_ROWS = 10;
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
    uint32_t* st_count;  // super-tiles touched (binning entries)
    uint32_t* depth_key;
    uint2* rect;
    Rec* rec;
    // SH path, visible Gaussians (optional): d(colour)/d(view direction) and the clamp flags
    // for the backward, SoA [SHJAC_ROWS][P]: rows 0-8 ddx[c], ddy[c], ddz[c]; row 9 the flags
    float* shjac;
    // per 256-Gaussian workgroup (optional, null to skip): blk_tot[b] = (visible, instances
    // R, super-tile entries S, prefiltered-error flag)
    uint4* blk_tot;
};
constexpr int PRE_THREADS = 256;
inline int pre_blocks(long long P) { return (int)((P + PRE_THREADS - 1) / PRE_THREADS); }

void launch_preprocess(const PreprocessArgs& a, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* viewmatrix, bool* present, hipStream_t s);
void launch_recolor(int P, const int* radii_src, const Rec* src, const float* colors, Rec* dst, int* radii_out,
                    hipStream_t s);

// ---- scans (gsr_scan.hip) -----------------------------------------------------------
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 4096
inline int scan_blocks(long long n) { return (int)((n + SCAN_TILE - 1) / SCAN_TILE); }

// Exclusive scan (u32) of in[0..n) -> out; block_tmp: scan_blocks(n) u32;
// total (optional) receives the sum.  If gather != nullptr the input is in[gather[i]].
void launch_exclusive_scan_u32(long long n, const uint32_t* in, const uint32_t* gather, uint32_t* out,
                               uint32_t* block_tmp, uint32_t* total, hipStream_t s);

// ---- radix sort (gsr_sort.hip) ---------------------------------------------------------
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 8;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;  // 2048 keys per block
inline int sort_blocks(long long n) { return (int)((n + SORT_TILE - 1) / SORT_TILE); }
// scratch bytes for sort of n items
size_t radix_sort_temp_bytes(long long n);
// Stable LSD sort of (key, value) pairs on key bits [0, end_bit).  Ping-pongs between
// (keys, vals) and (keys_alt, vals_alt); returns 1 if the sorted result ended in the alt
// buffers, 0 if in the primary buffers.
int radix_sort_pairs(long long n, uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                     int end_bit, void* temp, hipStream_t s);
// The same with a separate, untouched input (keys_in, vals_in; vals_in == nullptr means
// the values 0..n-1); the result lands in (keys, vals) or, when 1 is returned, the alt pair.
// A non-null aux_in (8 B per pair, input order) moves with the pairs and lands in aux or,
// when 1 is returned, aux_alt.
int radix_sort_pairs_from(long long n, const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys,
                          uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, int end_bit, void* temp,
                          hipStream_t s, const uint2* aux_in = nullptr, uint2* aux = nullptr,
                          uint2* aux_alt = nullptr);

// table[d][0..nb) -> exclusive prefix within each of ndigits rows; digit_tot[d] = row total
void launch_digit_scan(int ndigits, uint32_t* table, int nb, uint32_t* digit_tot, hipStream_t s);

// The forward's depth sort of all P keys (stable LSD, 4 passes of 8 bits, values = indices,
// an 8-B side payload moving along).  The last pass also stores the visible count P_v (the
// start of the culled keys' top byte 0xFF) to *pv_out, and does not store the sorted keys
// (nothing reads them: the values and the payload are the result).  Returns 1 if the result
// is in the alt buffers.
size_t depth_sort_temp_bytes(long long P);
int depth_sort(long long P, const uint32_t* keys_in, uint32_t* keys, uint32_t* vals, uint32_t* keys_alt,
               uint32_t* vals_alt, const uint2* aux_in, uint2* aux, uint2* aux_alt, void* temp,
               unsigned long long* pv_out, hipStream_t s, void* zero = nullptr, size_t zero_bytes = 0,
               bool pack = false);
// A grid of at most 255 x 255 tiles sorts and bins its rects packed to 4 bytes (pack_rect).
inline bool rect_packable(unsigned gx, unsigned gy) { return gx <= 255u && gy <= 255u; }
// (x0 | x1 << 16, y0 | y1 << 16) <-> x0 | x1 << 8 | y0 << 16 | y1 << 24 (every bound <= 255)
__host__ __device__ inline uint32_t pack_rect(uint2 r) {
    return (r.x & 0xffu) | ((r.x >> 8) & 0xff00u) | ((r.y & 0xffu) << 16) | ((r.y << 8) & 0xff000000u);
}
__host__ __device__ inline uint2 unpack_rect(uint32_t p) {
    return make_uint2((p & 0xffu) | ((p & 0xff00u) << 8), ((p >> 16) & 0xffu) | ((p >> 8) & 0xff0000u));
}

// One pass's dispatch order (k_tile_order, or extra workgroups of the binning scatter).
struct TileOrderArgs {
    unsigned ntile, gx, gsx;
    const uint2* ranges;      // cost = list length (materialised ranges), or
    const uint32_t* cost;     // an explicit per-tile cost, or
    const uint2* st_ranges;   // the tile's super-tile entry count from its range, or
    const uint32_t* st_tot;   // from the super-tile totals
    uint32_t* order;
    uint32_t* nheavy;
    int heavy_bits;
    uint32_t *zero_a, *zero_b, *zero_c;  // optional per-tile words zeroed (the forward's targets)
    uint32_t* unset;  // optional per-tile words set to SURV_NONE (survivor counts the forward may not write)
    int balance;  // cost-balanced bands, their first tiles stored to nheavy[8..17) (tile_unit's bal)
    // per tile row: the summed cost the balanced bands read (row_cost), or zeroed by the
    // forward's order for its tile pass to raise (zero_rows); nrows = tile rows
    const uint32_t* row_cost;
    uint32_t* zero_rows;
    unsigned nrows;
};

// The forward's frame totals for the host: one workgroup sums the preprocess's per-workgroup
// (P_v, R, S, error) and stores them to host-mapped memory as (value << 16 | seq mod 2^16)
// words; the host polls until all four carry its call's tag (no copy or event on the stream:
// each left a 6-19 us bubble between kernels).  Run as an extra workgroup of the super-tile
// scatter (launch_st_bin), or on its own (launch_frame_totals).
void launch_tile_order_args(const TileOrderArgs& a, hipStream_t s);  // k_tile_order, 8 bands

struct FrameTotals {
    const uint4* blk_tot;
    int nblk;
    unsigned long long* host;  // device address of the host-mapped words
    unsigned long long seq;
};
void launch_frame_totals(const FrameTotals& ft, hipStream_t s);

// ---- binning (gsr_binning.hip) ----------------------------------------------------------
// The binning stops at SUPER-TILE lists: one entry per (visible Gaussian, super-tile (8x4 tiles, 8x8 past ST_SMALL_MAX: st_sth)
// its rect touches), entry = (local tile rect code << ST_KEY_BITS | super-tile id, Gaussian
// id), every super-tile's entries contiguous and in (depth, index) order.  A tile's list (the
// reference's point_list range) is the subsequence of its super-tile's entries whose local
// rect covers the tile; the tile passes filter it on the fly (TileList, gsr_tile.hpp), and
// launch_materialize writes the reference's point_list + ranges when asked (tests, the
// GSR_DEBUG checks, the deterministic backward).
// Super-tile keys: id in bits [0, ST_KEY_BITS), the entry's local tile rect above (so at
// most 2^20 super-tiles; the sort orders only the id bits).
constexpr int ST_KEY_BITS = 20;
static_assert(ST_KEY_BITS + ST_CODE_BITS <= 32, "super-tile key + local rect code must fit 32 bits");
constexpr uint32_t ST_KEY_MASK = (1u << ST_KEY_BITS) - 1u;
// Super-tile entries of the P_v depth-sorted Gaussians, emitted directly in super-tile
// order, plus the super-tile ranges and header[0] = S.  NS <= 1365.
// rect_sorted: the rects already in depth order (the depth sort's side payload).
size_t st_bin_temp_bytes(long long Pv, int NS);
bool st_bin_supported(int NS);
// Pv: the visible count, or (with dev_totals non-null) its upper bound P, the kernels then
// reading the visible count *dev_totals (depth_sort's pv_out) on the device.  Entries at
// positions >= cap are not written (the speculative forward detects the overflow and redoes
// the binning).  ft (optional): the frame totals run as one extra workgroup of the scatter.
void launch_st_bin(int Pv, const unsigned long long* dev_totals, const uint32_t* sorted_ids, const void* rect_sorted,
                   bool packed, unsigned gsx, unsigned sth, int NS, void* temp, uint2* ent, uint2* st_ranges,
                   unsigned long long* header,
                   uint32_t cap, hipStream_t s, const FrameTotals* ft = nullptr, const TileOrderArgs* order = nullptr);
// Large images (NS > 1365): in depth order, every visible Gaussian emits one (super-tile,
// gaussian) pair per super-tile its rect touches, at offsets[s] (exclusive scan of st_count
// in depth order); the pairs are then radix-sorted by super-tile and packed into entries.
void launch_st_emit(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets, const uint2* rect, unsigned gsx,
                    unsigned sth, uint32_t* st_keys, uint32_t* st_vals, hipStream_t s);
// ranges[k] = [first, last+1) of super-tile k in the sorted pairs ((0, 0) when absent), the
// pairs packed into ent, header[0] = n.
void launch_seg_ranges(long long n, int nseg, const uint32_t* sorted_keys, const uint32_t* sorted_vals, uint2* ranges,
                       uint2* ent, unsigned long long* header, hipStream_t s);
// The reference's point_list [R] and tile ranges [T] from the super-tile lists (S entries):
// per 1024-entry segment a count pass, a per-tile prefix over segments, a scan over tiles,
// and a write pass.  temp: materialize_temp_bytes(S, nst, T).
size_t materialize_temp_bytes(long long S, int nst, int T);
void launch_materialize(long long S, int nst, const uint2* st_ranges, const uint2* ent, unsigned gx, unsigned gy,
                        unsigned gsx, void* temp, uint32_t* point_list, uint2* ranges, long long R, hipStream_t s);

// ---- tile order (gsr_schedule.hip) ------------------------------------------------------

// order: per XCD band of tiles (xcd_remap bands), heaviest first by log2 of `cost` (or of
// the tile's list length when cost is null); nheavy[8]: per band, the leading tiles with
// cost >= 2^heavy_bits.
// row_cost [nrows] (optional): the forward's summed cost per tile row (the balanced bands)
void launch_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost, uint32_t* order, uint32_t* nheavy,
                       int heavy_bits, hipStream_t s, const uint32_t* row_cost = nullptr, unsigned nrows = 0);

// Heavy tiles (split into four quadrant units, gsr_tile.hpp tile_unit): the forward splits a
// tile from 2^16 super-tile entries (round 4: 2^14): at cfg2c, whose heaviest super-tiles hold
// 30-45k entries in hundreds of similar tiles, the whole heavy tiles beyond the split cap ran as
// long as the split ones anyway, and a split tile stores no survivor list, so its backward
// re-filtered the whole super-tile list.  Round 5 (profiles/r5z_fwd_heavy_ab.txt): no split there
// took cfg2c render_fwd 0.369 -> 0.359 ms, its call 1.227 -> 1.217 ms, its throughput +2.3 %;
// cfg2 has no such tiles.  The test PLY scene's few 86k-entry tiles (a dense centre, DESIGN §3
// "Heavy tiles") still split.  Thresholds relative to the band's mean cost measured slower on
// cfg2c (profiles/r5e_heavy_split_ab.txt): a quadrant unit redoes the list filter, the culling
// and (backward) the per-survivor reduction.
constexpr int FWD_HEAVY_BITS = 16;  // super-tile entries >= 65536
constexpr int BWD_HEAVY_BITS = 13;  // (survivor, quadrant) evaluations >= 8192

// ---- render (gsr_render_fwd.hip / gsr_render_bwd.hip) --------------------------------
// The tile passes read each tile's list from its super-tile's entries (TileList):
// st_ranges [NS], ent [S], gsx super-tiles per row.
struct RenderFwdArgs {
    int W, H;
    unsigned grid_x, grid_y;
    const uint2* st_ranges;
    const uint2* ent;
    unsigned gsx;
    const Rec* rec;
    const float* bg;
    float* out_color;
    float* final_T;
    uint32_t* n_contrib;
    const uint32_t* order;  // dispatch order (launch_tile_order)
    const uint32_t* nheavy;
    uint32_t* tile_nmax;  // out: per tile, the largest n_contrib (the backward's cost; atomicMax, zeroed)
    uint32_t* tile_emax;  // out: per tile, 1 + the entry index of that last contributor (where the backward starts)
    uint32_t* tile_cost;  // out (when non-null): per tile, its (survivor, quadrant) evaluations (atomicAdd, zeroed)
    uint32_t* row_cost;   // out (when non-null): the same summed per tile row (the backward's balanced bands)
    // when non-null: zero_n4 float4s the backward needs zeroed (the gradient accumulator lines),
    // cleared by the pass's workgroups a slice each (zero_slice): VALU-bound waves have the HBM
    // write bandwidth to spare
    float4* zero;
    long long zero_n4;
    // when non-null: each whole-tile unit stores its survivors (entries reaching a live
    // quadrant), front to back, to surv[tile * SURV_CAP ...) as (Gaussian, position << 4 | reach
    // mask) and their count to surv_n[tile] (SURV_NONE past SURV_CAP); the backward walks them
    // instead of re-filtering the super-tile list
    uint2* surv;
    uint32_t* surv_n;
    int exact;  // the reference's blend arithmetic bit for bit (gsr_tile.hpp "exact mode")
};
void launch_render_fwd(const RenderFwdArgs& a, hipStream_t s);

struct RenderBwdArgs {
    int W, H;
    unsigned grid_x, grid_y;
    const uint2* st_ranges;
    const uint2* ent;
    unsigned gsx;
    const uint32_t* tile_emax;  // the forward's: where each tile's back-to-front walk starts
    const uint32_t* tile_nmax;  // the forward's: that entry's list position + 1
    const uint2* ranges;  // deterministic mode only: the materialised tile ranges (partial row index)
    const Rec* rec;
    const float* colors;  // optional: colour source if not in rec (unused: rec holds colour)
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    float* acc;  // [P][ACC_STRIDE]
    const uint32_t* order;  // dispatch order (launch_tile_order)
    const uint32_t* nheavy;
    // deterministic mode (non-null): each (tile, Gaussian) writes its partial sums to row
    // [instance] of DET_ROW3 floats instead of adding them into acc (k_det_gather sums them)
    float* partial;
    // the forward's survivor lists (RenderFwdArgs::surv); tiles whose count is SURV_NONE (or
    // all tiles when null) filter their super-tile list
    const uint2* surv;
    const uint32_t* surv_n;
    int exact;  // the forward's exact mode, replayed
};
constexpr int DET_ROW3 = 12;  // 8 sums + the ninth's four row partials
void launch_render_bwd(const RenderBwdArgs& a, hipStream_t s);

// Multi-channel tile passes (gsr_render_mc.hip): one group of <= 16 feature channels.
struct RenderMcArgs {
    int W, H;
    unsigned grid_x, grid_y;
    const uint2* st_ranges;
    const uint2* ent;
    unsigned gsx;
    uint32_t* tile_emax;  // forward: out (atomicMax when non-null); backward: in
    const uint2* ranges;  // deterministic backward only (materialised)
    const Rec* rec;
    const float4* feat;  // group's first channel; row stride fstride4 float4
    int fstride4, fstride;
    int nch;             // channels in this group
    const float* bg;     // [nch]
    float* out;          // forward: [nch][H][W]
    float* final_T;      // forward: written when non-null
    uint32_t* n_contrib;
    uint32_t* tile_nmax;  // forward: atomicMax when non-null
    uint32_t* tile_cost;  // forward: atomicAdd of its (survivor, quadrant) evaluations when non-null
    uint32_t* row_cost;   // forward: the same per tile row when non-null
    const uint32_t* order;
    const uint32_t* nheavy;
    const float* dL_dout;  // backward: [nch][H][W]
    float* acc;            // backward: [P][ACC_STRIDE], slots 0..5
    float* dL_dfeat;       // backward: group's first channel, row stride fstride
    // deterministic mode (non-null): per-instance rows of pstride floats, [6 geometric sums
    // (added over the groups)][every channel]; pc0 = this group's first channel
    float* partial;
    int pstride, pc0;
    float4* zero;  // forward: as RenderFwdArgs::zero
    long long zero_n4;
    // survivor lists as RenderFwdArgs::surv (forward: stored when non-null) and RenderBwdArgs::surv
    uint2* surv;
    uint32_t* surv_n;
    int exact;  // exact mode (RenderFwdArgs::exact)
};
void launch_render_fwd_mc(const RenderMcArgs& a, hipStream_t s);
void launch_render_bwd_mc(const RenderMcArgs& a, hipStream_t s);

// ---- deterministic backward: fixed-order per-Gaussian sum of the per-instance rows (gsr_det.hip)
// For every Gaussian with radii > 0, its tiles in row-major order (its rect), its position in
// each tile's list by binary search on (depth key, index) -- the order the binning emits --
// and the partial row there.  mode 0: DET_ROW3 rows -> acc[0..8]; mode 1: rows of pstride
// floats -> acc[0..5] and dL_dfeat[0..nch).  acc / dL_dfeat are zeroed by the caller.
struct DetGatherArgs {
    int P;
    unsigned gx, gy;
    const int* radii;
    const uint2* rect;
    const uint32_t* depth_key;
    const uint2* ranges;
    const uint32_t* point_list;
    const float* partial;
    int mode, pstride, nch, fstride;
    float* acc;
    float* dL_dfeat;
    unsigned* missing;  // counts Gaussians' tiles whose list lacks them (must stay 0)
};
void launch_det_gather(const DetGatherArgs& a, hipStream_t s);

// ---- GSR_DEBUG invariant checks (gsr_det.hip) ----------------------------------------------
// The first failed check (code, three details) is recorded with an atomic CAS; the host reads
// it after a stream synchronisation.
struct DebugReport {
    unsigned code, a, b, c;
};
enum DebugCode : unsigned {
    DBG_OK = 0, DBG_RANGE = 1, DBG_ID = 2, DBG_CULLED = 3, DBG_OUTSIDE_RECT = 4, DBG_ORDER = 5, DBG_COUNT = 6,
    DBG_TOTAL = 7, DBG_NCONTRIB = 8
};
// Tile lists against the preprocess: every range inside [0, R), every listed id < P, visible,
// its rect covering the tile, (depth key, id) strictly increasing per tile, every visible
// Gaussian listed exactly area(rect) times, the lengths summing to R; n_contrib[pix] at most
// its tile's list length.  count: P u32 of zeroed scratch, total: one zeroed u64.
void launch_check_lists(int P, long long R, unsigned gx, unsigned gy, int W, int H, const int* radii,
                        const uint2* rect, const uint32_t* depth_key, const uint2* ranges, const uint32_t* point_list,
                        const uint32_t* n_contrib, uint32_t* count, unsigned long long* total, DebugReport* rep,
                        hipStream_t s);

// ---- fused Adam over a flat parameter buffer (gsr_adam.hip) ---------------------------
constexpr int ADAM_MAX_SEGS = 32;
struct AdamSegs {
    int n;                               // segments (param groups), <= ADAM_MAX_SEGS
    long long end[ADAM_MAX_SEGS];        // exclusive end element of each segment (ascending)
    float step_size[ADAM_MAX_SEGS];      // lr / (1 - b1^t) per segment
    float bc2_sqrt, one_minus_b1, b2, one_minus_b2, eps, grad_scale;
};
void launch_adam(long long lo, long long hi, const AdamSegs& s, float* p, const float* g, float* m, float* v,
                 hipStream_t st);  // elements [lo, hi), lo % 4 == 0

// ---- fused SSIM loss (gsr_ssim.hip) ---------------------------------------------------
struct SsimWindow {
    float w[11];  // normalised 1-D Gaussian (window 11, sigma 1.5)
};
dim3 ssim_grid(int C, int H, int W);
void launch_ssim_fwd(int C, int H, int W, const float* img1, const float* img2, const float* mask,
                     long long mask_cstride, const SsimWindow& win, float C1, float C2, float* block_sums,
                     float* dmaps, hipStream_t s);
void launch_ssim_bwd(int C, int H, int W, const float* img1, const float* img2, const float* dmaps,
                     const float* gscale, const SsimWindow& win, float* dimg1, int accumulate, hipStream_t s,
                     const float* occ = nullptr, const float* l1k = nullptr);

// ---- fused pointwise training-loss terms (gsr_loss.hip) ---------------------------------
int view_loss_blocks(int npix);
void launch_view_loss_fwd(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, float* partials,
                          hipStream_t s);
void launch_view_objective(int nvl, const float* vl, int nss, const float* ss, int npix, double l_dssim, double l_sky,
                           double l_normal, float* loss, float* coef, hipStream_t s);
void launch_view_loss_bwd(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, const float* coef,
                          float* d_img, float* d_diff, float* d_spec, float* d_nrm, float* d_nref, hipStream_t s);

// render()'s image-space tail (gsr_epilogue.hip): cam12 = rows of K^-1^T R^T, then the centre
void launch_epilogue_fwd(int W, int H, const float* cam12, const float* n01, const float* depth, const float* alpha,
                         const float* sky, int normal_view, float* normal, float* normal_ref, hipStream_t s);
void launch_epilogue_bwd(int W, int H, const float* cam12, const float* depth, const float* alpha, const float* sky,
                         int normal_view, const float* g_normal, const float* g_normal_ref, float* d_n01,
                         float* d_depth, hipStream_t s);

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
    // acc_raw: the line holds the tile passes' raw sums (gsr_render_bwd.hip): op * (sum G dL/dalpha
    // dx, ... dy, ... dx dx, ... dx dy, ... dy dy), sum G dL/dalpha, the colour sums; the conic and
    // the screen scale are applied here, once per Gaussian.  0: the line holds the reference's
    // values (dL/dmean2D, dL/dconic, dL/dopacity, dL/dcolor; baseline/refalgo.hip)
    int acc_raw, W, H;
    const float* shjac;  // [SHJAC_ROWS][P] from the forward preprocess (required with shs)
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
    // add into (instead of overwrite) dL_dmean3D (bit 0), dL_dscale (1), dL_drot (2),
    // dL_dopacity (3): several views' gradients summed in the kernels that produce them
    unsigned acc_mask;
};
void launch_preprocess_bwd(const PreprocessBwdArgs& a, hipStream_t s);

// ---- 3-nearest-neighbour mean distance (gsr_knn.hip) ------------------------------------
size_t knn_workspace_bytes(int P);
void launch_knn(int P, const float* pts, float* dists, void* ws, hipStream_t s);

// ---- 2D texture sampling, nvdiffrast dr.texture semantics (gsr_texture.hip) -------------
void launch_texture_fwd(int nb, int npix, int tex_nb, int h, int w, int C, const float* tex, const float* uv,
                        int filter, int boundary, float* out, hipStream_t s);
void launch_texture_bwd(int nb, int npix, int tex_nb, int h, int w, int C, const float* tex, const float* uv,
                        int filter, int boundary, const float* dout, float* d_uv, float* d_tex, hipStream_t s);

// ---- training-step bookkeeping over V views at once (gsr_trainaux.hip) ------------------
constexpr int REG_MAXV = 8;  // views per launch
template <typename T>
struct ViewPtrs {  // one device pointer per view, passed by value in the kernel arguments
    const T* p[REG_MAXV];
};
int view_regs_blocks(int P);
void launch_view_regs_fwd(int P, int V, const float* xyz, const float* scaling, const ViewPtrs<int>& radii,
                          const unsigned char* is_sky, const float* dcol, float* partials, hipStream_t s);
void launch_view_regs_bwd(int P, int V, const float* scaling, const ViewPtrs<int>& radii, const unsigned char* is_sky,
                          const float* dcol, const float* g, float* d_xyz, float* d_scaling, unsigned acc,
                          hipStream_t s);
void launch_densify_stats(int P, int V, const ViewPtrs<float>& g2d, const ViewPtrs<int>& radii, float* accum,
                          float* denom, float* maxr, hipStream_t s);
void launch_sh_basis(int N, int deg, const float* dirs, float* out, hipStream_t s);
int sky_blocks(int N);
// the model's activations over P Gaussians (N_fg foreground rows, N_sky sky rows)
struct ActArgs {
    int P, Nfg, Nsky;
    const int* src;  // [P]: the foreground row (>= 0) or -1 - the sky row; null: rows < Nfg are foreground
    const float *xyz_fg, *angles, *radius, *center;
    const float *scale_raw, *rot_raw, *op_raw, *alb_raw, *rough_raw, *metal_raw;
};
struct ActOut {  // activated tensors (or their upstream gradients)
    const float *xyz, *scale, *rot, *op, *alb, *rough, *metal;
};
struct ActOutW {
    float *xyz, *scale, *rot, *op, *alb, *rough, *metal;
};
struct ActGrad {  // the raw parameters' gradients
    float *xyz_fg, *angles, *radius_part, *scale_raw, *rot_raw, *op_raw, *alb_raw, *rough_raw, *metal_raw;
};
int activation_blocks(const ActArgs& a);
struct RegsTail {  // the regularisers' scalar tail (gsr_trainaux.hip)
    int V, NS, depth_on;
    float lam_env, lam_scale, lam_depth, gamma;
    const float *sums, *basis, *env;
};
void launch_regs_tail_fwd(const RegsTail& t, float* total, hipStream_t s);
void launch_regs_tail_bwd(const RegsTail& t, const float* g, float* d_sums, float* d_env, hipStream_t s);
void launch_activations_fwd(const ActArgs& a, const ActOutW& o, hipStream_t s);
void launch_activations_bwd(const ActArgs& a, const ActOut& o, const ActOut& g, const ActGrad& d, float* d_radius,
                            hipStream_t s);
void launch_sky_xyz_fwd(int N, const float* ang, const float* radius, const float* center, float* out, hipStream_t s);
void launch_sky_xyz_bwd(int N, const float* ang, const float* radius, const float* g, float* d_ang, float* d_rad_part,
                        hipStream_t s);

}  // namespace gsr
