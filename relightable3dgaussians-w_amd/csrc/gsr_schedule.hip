// gsr_schedule.hip -- heaviest-first dispatch order of the tile passes.
//
// The tile passes run one wave per tile, and tiles differ in cost by an order of magnitude
// (list length, early saturation).  Each XCD band of the image (the bands of xcd_remap:
// neighbouring tiles share Gaussian records in that XCD's L2) is ordered heaviest-first in
// 8 buckets per octave of a cost estimate (gsr_order.hpp); the passes dispatch block b on
// position b / 8 of band b mod 8, so the hardware dispatcher runs a longest-first schedule
// per XCD.  Tiles above a cost threshold (lists in the thousands: dense centres of real
// scenes) and, in the forward, each band's lightest tiles run as four one-wave units, one
// per 8x8 quadrant; the rest as one wave each (tile_unit in gsr_tile.hpp).  The forward's
// order runs inside the binning scatter (gsr_binning.hip); this file launches the others.
// (A persistent variant pulling tiles from per-XCD atomic queues measured 2x slower: the
// returning atomics cost ~13 us per pull under load.)
#include "gsr_order.hpp"

namespace gsr {

template <bool BAL>
__global__ void __launch_bounds__(512) k_tile_order(TileOrderArgs a) { tile_order_band<BAL>(blockIdx.x, a); }

void launch_tile_order_args(const TileOrderArgs& a, hipStream_t s) {
    if (a.ntile == 0) return;
    if (a.balance) hipLaunchKernelGGL(k_tile_order<true>, dim3(8), dim3(512), 0, s, a);
    else hipLaunchKernelGGL(k_tile_order<false>, dim3(8), dim3(512), 0, s, a);
}

void launch_tile_order(unsigned ntile, const uint2* ranges, const uint32_t* cost, uint32_t* order, uint32_t* nheavy,
                       int heavy_bits, hipStream_t s, const uint32_t* row_cost, unsigned nrows) {
    if (ntile == 0) return;
    TileOrderArgs a{};
    a.ntile = ntile; a.ranges = ranges; a.cost = cost; a.order = order; a.nheavy = nheavy; a.heavy_bits = heavy_bits;
    a.row_cost = row_cost; a.nrows = nrows;
    a.balance = 1;  // the backward passes' bands are cost-balanced (tile_unit_bwd)
    hipLaunchKernelGGL(k_tile_order<true>, dim3(8), dim3(512), 0, s, a);
}

}  // namespace gsr
