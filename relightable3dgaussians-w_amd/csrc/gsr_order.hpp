// gsr_order.hpp -- a tile pass's dispatch order for one XCD band (k_tile_order in
// gsr_schedule.hip, or extra workgroups of the binning scatter in gsr_binning.hip).
#pragma once
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

// The cost of tile t: cost[t]; else its super-tile's entry count (the forward: st_tot, or
// st_ranges; gx tiles per row, gsx super-tiles per row); else its list length.
__device__ __forceinline__ uint32_t tile_cost(unsigned t, const TileOrderArgs& a) {
    if (a.cost) return a.cost[t];
    if (a.st_tot || a.st_ranges) {
        const unsigned st = ((t / a.gx) >> st_sth(a.gx, a.ntile / a.gx)) * a.gsx + (t % a.gx) / GSR_ST_W;
        if (a.st_tot) return a.st_tot[st];
        const uint2 r = a.st_ranges[st];
        return r.y - r.x;
    }
    return a.ranges ? a.ranges[t].y - a.ranges[t].x : 0u;
}

// Cost bucket: the bit length of c and its next three bits (8 buckets per octave), 0 for c = 0.
// (One bucket per octave took the backward tile pass to 0.40 ms at cfg2, eight 0.38 ms; four and
// sixteen measured the same as eight.)
constexpr int BUCKET_FRAC = 3;  // 2^BUCKET_FRAC buckets per octave
constexpr int NBUCKET = 33 << BUCKET_FRAC;
__device__ __forceinline__ int cost_bucket(uint32_t c) {
    if (!c) return 0;
    const int L = 32 - __clz(c);
    const uint32_t fm = (1u << BUCKET_FRAC) - 1u;
    const uint32_t f = L > BUCKET_FRAC ? (c >> (L - 1 - BUCKET_FRAC)) & fm : (c << (BUCKET_FRAC + 1 - L)) & fm;
    return (L << BUCKET_FRAC) + (int)f;
}
__device__ __forceinline__ int bucket_heavy_from(int heavy_bits) { return (heavy_bits + 1) << BUCKET_FRAC; }

// One band's order (any block size): order[lo .. lo+len) = the band's tiles, cost buckets
// descending; nheavy[band] = how many lead the order with a cost >= 2^heavy_bits (split 4
// ways).  Also zeroes the optional per-tile targets of the forward (tile maxima, summed cost).
// Cost-balanced band b: the contiguous tile range over which the prefix of cost' = cost + a
// floor (half the mean tile cost, rounded up) crosses b / 8 and (b + 1) / 8 of its total (the floor bounds
// a band at 3 ntile / 8 + 2 tiles: tile_pass_blocks_bal).  The forward's tile pass also sums the
// costs per tile row (row_cost), so every workgroup of the order launch finds its two
// boundaries cheaply: a workgroup scan over the rows finds the row holding each boundary, a
// second over that row's tiles the tile.  Equal bands when the frame's total cost is 0 or no
// row costs exist.  (Reading every tile's cost in every workgroup made the launch 10-37 us
// longer; whole-row bounds balanced too coarsely.)
__device__ __forceinline__ void balanced_band(unsigned band, const TileOrderArgs& a, unsigned& lo, unsigned& len) {
    __shared__ unsigned long long s_scan[16];
    __shared__ unsigned long long s_rowp[2];  // cost' before the boundary rows
    __shared__ unsigned s_row[2], s_bound[2];
    const unsigned n = a.nrows, gx = n ? a.ntile / n : 0u;
    // the forward's order has no row sums: a row's cost is summed from its super-tiles' entry
    // counts (its tiles' costs), a handful of loads per row
    const bool strow = !a.row_cost && !a.cost && (a.st_ranges || a.st_tot);
    if ((!a.row_cost && !strow) || n == 0 || n > blockDim.x || gx > blockDim.x || gx * n != a.ntile ||
        blockDim.x != 512) {
        band_of(band, a.ntile, lo, len);
        return;
    }
    const unsigned r = threadIdx.x;
    unsigned long long c = 0ull;
    if (r < n) {
        if (strow) {
            for (unsigned x0 = 0; x0 < gx; x0 += GSR_ST_W)  // one super-tile's tiles of this row at a time
                c += (unsigned long long)tile_cost(r * gx + x0, a) * (gx - x0 < GSR_ST_W ? gx - x0 : GSR_ST_W);
        } else {
            c = a.row_cost[r];
        }
    }
    if (threadIdx.x < 2) {
        s_row[threadIdx.x] = 0xffffffffu;
        s_bound[threadIdx.x] = threadIdx.x == 0 ? (band > 0 ? 0xffffffffu : 0u) : (band < 7 ? 0xffffffffu : a.ntile);
    }
    unsigned long long total;
    const unsigned long long before = block_exclusive_scan<8>(c, s_scan, &total);  // 512 threads = 8 waves
    if (total == 0) {
        band_of(band, a.ntile, lo, len);
        return;
    }
    // the per-tile floor, rounded up so that total <= 2 ntile add: a band's tiles then number at
    // most 3 ntile / 8 + 2 (tile_pass_blocks_bal)
    const unsigned long long add = (total + BAL_FLOOR_DIV * a.ntile - 1) / (BAL_FLOOR_DIV * a.ntile);
    const unsigned long long tp = total + add * a.ntile;
    const unsigned long long tgt[2] = {band * tp / 8, (band + 1) * tp / 8};
    const bool need[2] = {band > 0, band < 7};
    // Each boundary is 1 + the last tile whose cost' interval starts below the target: the row
    // is the last one starting below it, then the tile the last one of that row.  Every band's
    // workgroup evaluates the same function of the same costs, so band b's upper bound is band
    // b + 1's lower bound and the bounds are monotone even if the row sums disagreed with the
    // tile costs (no per-workgroup fallback that could leave bands overlapping or gapped).
    if (r < n) {
        const unsigned long long p = before + (unsigned long long)r * gx * add, q = p + c + gx * add;
        const unsigned long long pn = q;  // the next row's start
#pragma unroll
        for (int k = 0; k < 2; k++)
            if (need[k] && p < tgt[k] && (r + 1 == n || pn >= tgt[k])) {
                s_row[k] = r;
                s_rowp[k] = p;
            }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (!need[k]) continue;  // workgroup-uniform
        const unsigned row = s_row[k];
        const unsigned long long ct = (row < n && threadIdx.x < gx) ? tile_cost(row * gx + threadIdx.x, a) + add : 0ull;
        unsigned long long rt;
        const unsigned long long bt = block_exclusive_scan<8>(ct, s_scan, &rt);
        if (row < n && threadIdx.x < gx) {
            const unsigned long long p = s_rowp[k] + bt, q = p + ct;
            if (p < tgt[k] && (threadIdx.x + 1 == gx || q >= tgt[k])) s_bound[k] = row * gx + threadIdx.x + 1;
        }
    }
    __syncthreads();
    // (a target at or below the first row's start cannot occur: tgt > 0 = the first start)
    lo = s_bound[0] == 0xffffffffu ? 0u : s_bound[0];
    len = (s_bound[1] == 0xffffffffu ? a.ntile : s_bound[1]) - lo;
}

// BAL: the band is cost-balanced (balanced_band; a template argument, so that the binning
// scatter's order workgroups carry none of its LDS)
template <bool BAL = false>
__device__ __forceinline__ void tile_order_band(unsigned band, const TileOrderArgs& a) {
    __shared__ uint32_t hist[NBUCKET];
    __shared__ uint32_t cur[NBUCKET];
    __shared__ uint32_t scan[8];  // per-wave bucket sums
    unsigned lo, len;
    if constexpr (BAL) {
        balanced_band(band, a, lo, len);
        if (threadIdx.x == 0) {
            a.nheavy[8 + band] = lo;
            if (band == 7) a.nheavy[16] = lo + len;
        }
    } else {
        band_of(band, a.ntile, lo, len);
    }
    __shared__ unsigned long long s_band_cost;
    for (int i = threadIdx.x; i < NBUCKET; i += blockDim.x) hist[i] = 0;
    if (threadIdx.x == 0) s_band_cost = 0ull;
    if (a.zero_rows && band == 0)
        for (unsigned i = threadIdx.x; i < a.nrows; i += blockDim.x) a.zero_rows[i] = 0u;
    __syncthreads();
    unsigned long long csum = 0ull;
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        const uint32_t c = tile_cost(t, a);
        csum += c;
        atomicAdd(&hist[cost_bucket(c)], 1u);
        if (a.zero_a) {
            a.zero_a[t] = 0u;
            a.zero_b[t] = 0u;
            if (a.zero_c) a.zero_c[t] = 0u;
        }
        if (a.unset) a.unset[t] = SURV_NONE;
    }
    if (csum) atomicAdd(&s_band_cost, csum);
    __syncthreads();
    // cur[b] = tiles in buckets above b (heaviest bucket first): a block scan over the
    // buckets in descending order, thread j holding bucket NBUCKET - 1 - j -- wave scans and one
    // barrier (one thread serially when the block is smaller than the bucket count)
    if (blockDim.x >= NBUCKET && blockDim.x <= 512) {
        const int j = threadIdx.x, bj = NBUCKET - 1 - j, wave = j >> 6;
        const uint32_t hj = bj >= 0 ? hist[bj] : 0u;
        const uint32_t inc = wave_inclusive_scan(hj);
        if ((j & 63) == 63) scan[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
        for (int w = 0; w < wave; w++) off += scan[w];
        if (bj >= 0) cur[bj] = off + inc - hj;
    } else if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int b = NBUCKET - 1; b >= 0; b--) {
            cur[b] = run;
            run += hist[b];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // heavy: cost >= 2^heavy_bits
        const int hb = bucket_heavy_from(a.heavy_bits);
        a.nheavy[band] = hb < NBUCKET ? cur[hb] + hist[hb] : 0u;
        // the band's estimated cost (the rotated bands: tile_unit)
        a.nheavy[24 + band] = (uint32_t)min(s_band_cost, 0xffffffffull);
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < len; i += blockDim.x) {
        const unsigned t = lo + i;
        a.order[lo + atomicAdd(&cur[cost_bucket(tile_cost(t, a))], 1u)] = t;
    }
}

}  // namespace gsr
