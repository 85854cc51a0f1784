// gsr_tile.hpp -- helpers shared by the forward and backward tile passes.
#pragma once
#include "gsr_common.hpp"

namespace gsr {

// bijective XCD-aware block -> tile remap: blocks b and b+8 run on the same XCD (private
// L2), so each XCD gets a contiguous band of tiles whose Gaussian records overlap.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n) {
    const unsigned q = n >> 3, r = n & 7u, x = b & 7u;
    const unsigned base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + (b >> 3);
}

// band x of xcd_remap: tiles [lo, lo + len)
__device__ __forceinline__ void band_of(unsigned x, unsigned n, unsigned& lo, unsigned& len) {
    const unsigned q = n >> 3, r = n & 7u;
    lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    len = q + (x < r ? 1u : 0u);
}

// Work unit of a one-wave workgroup of the tile passes: block b serves unit b / 8 of XCD
// band b mod 8.  The band's first min(nheavy, HEAVY_CAP) tiles (heaviest first) are split
// into four units, one per 8x8 quadrant; so are its last min(ntail, rest) tiles (the lightest:
// the pass's tail then drains in quarter-tile units while the chip is still full, instead of
// one whole tile per wave slot); every other tile is one unit.  Sets tile and the quadrant
// mask; false when the block has nothing to do.  (Four-wave workgroups holding a heavy
// tile's quadrants measured slower on balanced scenes: a workgroup waits for four free wave
// slots on one CU, so single waves cannot backfill.)
constexpr unsigned HEAVY_CAP = 64;  // split heavy tiles per band
// words per unit in the instrumented builds' timing records (g_fwd_times / g_bwd_times)
#define GSR_UNIT_REC 8
// Split tail tiles per band: the forward passes split their 128 lightest (render_fwd 0.247 ->
// 0.233 ms at cfg2); the backward passes none (splitting its lightest 32 / 96 per band cost 1.5 /
// 3.5 % of the throughput: a quadrant unit repeats the per-survivor reduction,
// profiles/r5z_bwd_tail_ab.txt)
constexpr unsigned FWD_TAIL_SPLIT = 128;
// Rotated bands: block b takes unit b / 8 of band (b + (b / 8 >> ROT_SHIFT)) mod 8 instead of band
// b mod 8, so each XCD (b mod 8) works through every band's order in runs of 2^ROT_SHIFT units,
// when the bands' estimated costs (nheavy[rcost + b], written by the order) are uneven: the
// largest above ROT_THR8 / 8 x their mean.  A skewed frame then no longer waits for one XCD's
// band; an even one keeps each band's L2 locality (rotating unconditionally measured cfg2c
// +1.5 %, cfg2 -0.9 %; a step per unit instead of per 32 fetched 3.4x the bytes,
// profiles/r5z_band_rotate_ab.txt).  The backward passes rotate their cost-balanced bands when
// the *forward's* equal bands had uneven costs (cfg2c render_bwd 0.434 -> 0.397 ms): the
// backward's table (nheavy) starts 32 words before the forward's, so those costs are at
// nheavy[BWD_ROT_COST + b] there.
constexpr unsigned ROT_THR8 = 10u, ROT_SHIFT = 5u;
constexpr unsigned BWD_ROT_COST = 32u + 24u;
__device__ __forceinline__ bool tile_unit(unsigned ntile, const uint32_t* order, const uint32_t* nheavy,
                                          unsigned& tile, uint32_t& qallow, unsigned ntail, bool bal, unsigned rot,
                                          unsigned rcost) {
    unsigned u = blockIdx.x >> 3, band = blockIdx.x & 7u;
    if (rot != 0u) {
        uint32_t mx = 0u;
        unsigned long long sum = 0ull;
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t c = nheavy[rcost + b];
            mx = max(mx, c);
            sum += c;
        }
        if (64ull * mx > (unsigned long long)rot * sum) band = (band + (u >> ROT_SHIFT)) & 7u;
    }
    unsigned lo, len;
    if (bal) {
        lo = nheavy[8 + band];
        len = nheavy[9 + band] - lo;
    } else {
        band_of(band, ntile, lo, len);
    }
    const unsigned h = min(min(nheavy[band], HEAVY_CAP), len);
    const unsigned t = min(ntail, len - h);
    const unsigned whole = len - h - t;
    unsigned pos;
    if (u < 4u * h) {
        pos = u >> 2;
        qallow = 1u << (u & 3u);
    } else if (u < 4u * h + whole) {
        pos = h + (u - 4u * h);
        qallow = 15u;
    } else {
        const unsigned v = u - 4u * h - whole;
        pos = h + whole + (v >> 2);
        qallow = 1u << (v & 3u);
    }
    if (pos >= len) return false;
    tile = order[lo + pos];
    return true;
}
// The forward passes' units: equal bands, their 128 lightest tiles split
__device__ __forceinline__ bool tile_unit_fwd(unsigned ntile, const uint32_t* order, const uint32_t* nheavy,
                                              unsigned& tile, uint32_t& qallow) {
    return tile_unit(ntile, order, nheavy, tile, qallow, FWD_TAIL_SPLIT, false, ROT_THR8, 24u);
}
// The backward passes' units: cost-balanced bands (balanced_band), no tail split; det: one
// writer per partial row, so no band rotation either
__device__ __forceinline__ bool tile_unit_bwd(unsigned ntile, const uint32_t* order, const uint32_t* nheavy,
                                              unsigned& tile, uint32_t& qallow, bool det) {
    return tile_unit(ntile, order, nheavy, tile, qallow, 0u, true, det ? 0u : ROT_THR8, BWD_ROT_COST);
}
// blocks of a tile pass launch: the longest band's units (heavy and tail tiles count four)
__host__ __device__ constexpr unsigned tile_pass_blocks(unsigned ntile, unsigned ntail) {
    return 8u * ((ntile + 7u) / 8u + 3u * HEAVY_CAP + 3u * ntail);
}
// the same with cost-balanced bands: a band holds at most 3 ntile / 8 + 2 tiles (balanced_band;
// the grid launches 12/4 workgroups per 8 tiles of a band: blocks past a band's units exit at
// once, and a grid of 5/4 measured the same within noise, profiles/r5q_ab_grid.txt)
__host__ __device__ constexpr unsigned tile_pass_blocks_bal(unsigned ntile, unsigned ntail) {
    return 8u * ((12u * ((ntile + 7u) / 8u) + 3u) / 4u + 2u + 3u * HEAVY_CAP + 3u * ntail);
}
// the balanced bands' per-tile floor: the mean tile cost / BAL_FLOOR_DIV (the grid bound of
// tile_pass_blocks_bal holds for 1 and 2)
constexpr unsigned long long BAL_FLOOR_DIV = 2ull;
// LDS ordering within one wave (the tile passes' waves share no LDS)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- a tile's list, read from its super-tile's entries -------------------------------------
// The binning stops at super-tile lists (gsr_binning.hip): the entries of every Gaussian that
// touches a super-tile (8x4 or 8x8 tiles, st_sth), in (depth, index) order, each carrying its local tile rect.
// A tile's list -- the reference's point_list range, entry for entry -- is the subsequence of
// its super-tile's entries whose local rect covers the tile.  TileList filters 64 entries per
// step (one 8-B load per lane, prefetched a step ahead; a rect test; a ballot) and appends the
// covering ones, with their list positions and entry indices, to a 256-slot LDS ring; the
// tile passes take full batches of 64 from the ring, so their per-batch work is what it was
// over a materialised list.  Forward: front to back from position 0.  Backward: back to front
// from a given entry (exclusive) whose preceding covering entries number pos0.
constexpr uint32_t TL_RING = 256;
struct TileListLds {  // per wave
    uint32_t id[TL_RING], e[TL_RING];
};

// FWD: front to back; the entries' list positions are consecutive, so a batch's are its first
// position (take's p0, wave-uniform) + slot.  BWD: back to front, positions p0 - slot.
// KEEP_E: also queue the entry indices (the forward records where its last contributor sits).
template <bool FWD, bool KEEP_E = FWD>
struct TileList {
    const uint2* ent;
    uint32_t e;      // FWD: next entry to filter; BWD: entries below e remain
    uint32_t lim;    // FWD: end (exclusive); BWD: bottom (inclusive)
    uint32_t head, tail;
    uint32_t tpos;   // list position of the next entry to take (BWD: counting down)
    uint32_t lx, ly;
    uint2 nx, nx2;   // this lane's entries of the next two steps (loads issued two steps ahead)

    // the step starting at eb (BWD: top eb).  Unconditional: lanes past the range read an
    // entry at its edge (the entry array has 64 slack entries, so even an empty range at the
    // end reads inside it) and step() masks them, so a prefetch register is never written
    // twice (a zero default + a masked load made the compiler wait for every load in flight)
    __device__ __forceinline__ uint2 load_step(uint32_t eb) const {
        const uint32_t lane = threadIdx.x & 63;
        if (FWD) return ent[min(eb + lane, lim)];
        return ent[max((int)eb - 1 - (int)lane, (int)lim)];
    }
    __device__ __forceinline__ uint32_t step_after(uint32_t eb) const {
        return FWD ? min(eb + 64u, lim) : (eb > lim + 64u ? eb - 64u : lim);
    }
    // st_range: the super-tile's entries [first, last); BWD: start below `top`, whose covering
    // predecessors number pos0
    // sth: the super-tile height's log2 (st_sth)
    __device__ __forceinline__ void init(const uint2* ent_, uint2 st_range, unsigned tile, unsigned gx, unsigned sth,
                                         uint32_t top, uint32_t pos0) {
        ent = ent_;
        const unsigned tx = tile % gx, ty = tile / gx;
        lx = tx % GSR_ST_W;
        ly = ty & ((1u << sth) - 1u);
        head = tail = 0;
        if (FWD) {
            e = st_range.x;
            lim = st_range.y;
            tpos = 0;
        } else {
            e = top;
            lim = st_range.x;
            tpos = pos0 - 1u;
        }
        nx = load_step(e);
        nx2 = load_step(step_after(e));
    }
    __device__ __forceinline__ bool covers(uint32_t key) const {
        constexpr uint32_t XM = (1u << ST_XB) - 1u, YM = (1u << ST_YB) - 1u;
        const uint32_t code = key >> 20, cx0 = code & XM, cx1 = (code >> ST_XB) & XM, cy0 = (code >> (2 * ST_XB)) & YM,
                       cy1 = (code >> (2 * ST_XB + ST_YB)) & YM;  // inclusive maxima
        return (lx - cx0) <= (cx1 - cx0) && (ly - cy0) <= (cy1 - cy0);  // unsigned: also lx >= cx0
    }
    __device__ __forceinline__ bool more() const { return FWD ? e < lim : e > lim; }
    __device__ __forceinline__ bool want() const { return tail - head < 64u && more(); }
    // one filter step: this lane's entry v of the step at e (advances e)
    __device__ __forceinline__ void step(TileListLds& L, const uint2 v) {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t i = FWD ? e + lane : e - 1u - lane;
        const bool valid = FWD ? i < lim : e > lim + lane;
        e = step_after(e);
        const bool c = valid && covers(v.x);
        const uint64_t cm = __ballot(c);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
        if (c) {
            const uint32_t slot = (tail + r) & (TL_RING - 1u);
            L.id[slot] = v.y;
            if (KEEP_E) L.e[slot] = i;
        }
        tail += (uint32_t)__popcll(cm);
    }
    // filter until >= 64 entries are queued or the list is exhausted, two steps at a time:
    // the two prefetch registers are consumed in a fixed order and each is reloaded right
    // after it is consumed, so no register copy waits on a load in flight (a step past the
    // end queues nothing; the ring holds the up to 63 + 128 entries this leaves queued)
    __device__ __forceinline__ void fill(TileListLds& L) {
        wave_lds_sync();
        while (want()) {
            step(L, nx);
            nx = load_step(step_after(e));
            step(L, nx2);
            nx2 = load_step(step_after(e));
        }
        wave_lds_sync();
    }
    // up to 64 queued entries: the count (wave-uniform); lanes below it get theirs; p0: the
    // batch's first list position (FWD: lane's = p0 + lane; BWD: p0 - lane)
    __device__ __forceinline__ uint32_t take(const TileListLds& L, uint32_t& id, uint32_t& ei, uint32_t& p0) {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t n = min(64u, tail - head);
        if (lane < n) {
            const uint32_t slot = (head + lane) & (TL_RING - 1u);
            id = L.id[slot];
            if (KEEP_E) ei = L.e[slot];
        }
        head += n;
        p0 = tpos;
        tpos = FWD ? tpos + n : tpos - n;
        return n;
    }
};

// The tile passes evaluate Gaussians in log2 units: the conic is pre-scaled by log2(e) when
// a record is staged (once per record and batch), so exp(power) is one v_exp_f32 (exp2) per
// evaluation with no multiply.  Forward and backward stage and evaluate identically, so the
// backward replays exactly the forward's blend decisions.
// (The backward accumulates raw sums of G dL/dalpha dx...: G is the same value in either unit.)
constexpr float TILE_LOG2E = 1.44269504088896340736f;
constexpr float TILE_LN2 = 0.69314718055994530942f;
constexpr float TILE_STAGE_AC = -0.5f * TILE_LOG2E;  // factor of conic.a and conic.c
constexpr float TILE_STAGE_B = -TILE_LOG2E;          // factor of conic.b
__device__ __forceinline__ float tile_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Minimum over the pixel box [dx0,dx1]x[dy0,dy1] (offsets from the Gaussian centre) of
// q(d) = a dx^2 + 2 b dx dy + c dy^2, for a positive-definite conic (a, b, c).
__device__ __forceinline__ float qmin_box(float a, float b, float c, float dx0, float dx1, float dy0, float dy1) {
    if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return 0.f;
    // edges dx = const: argmin dy = -b dx / c ; edges dy = const: argmin dx = -b dy / a.
    // v_rcp_f32 (1 ulp) only moves the candidate point along the edge, where q is
    // stationary; the margin in box_reachable absorbs the second-order change.
    const float ic = __builtin_amdgcn_rcpf(c), ia = __builtin_amdgcn_rcpf(a);
    float q = 3.4e38f;
    {
        const float X = dx0;
        const float y = fminf(fmaxf(-b * X * ic, dy0), dy1);
        q = fminf(q, a * X * X + 2.f * b * X * y + c * y * y);
    }
    {
        const float X = dx1;
        const float y = fminf(fmaxf(-b * X * ic, dy0), dy1);
        q = fminf(q, a * X * X + 2.f * b * X * y + c * y * y);
    }
    {
        const float Y = dy0;
        const float x = fminf(fmaxf(-b * Y * ia, dx0), dx1);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    {
        const float Y = dy1;
        const float x = fminf(fmaxf(-b * Y * ia, dx0), dx1);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    return q;
}

// Conservative test: can this Gaussian reach alpha >= 1/255 at any integer pixel of the
// box?  The render loops evaluate alpha = min(0.99, o * exp(-q/2)) and skip alpha < 1/255,
// so a Gaussian with o * exp(-qmin/2) < 1/255 contributes nothing to any pixel of the box
// (in the forward, the backward, n_contrib or T).  `lnthr` = ln(255 * o).  The margin
// covers the float rounding of q at the pixels (relative to the magnitude of its terms)
// and of the exp/threshold evaluation, so the skip is never wrong.
__device__ __forceinline__ bool box_reachable(float a, float b, float c, float lnthr, float dx0, float dx1, float dy0,
                                              float dy1) {
    const float q = qmin_box(a, b, c, dx0, dx1, dy0, dy1);
    const float mx = fmaxf(fabsf(dx0), fabsf(dx1)), my = fmaxf(fabsf(dy0), fabsf(dy1));
    const float S = a * mx * mx + 2.f * fabsf(b) * mx * my + c * my * my;
    return q <= 2.f * lnthr + 1e-2f + 1e-4f * S;
}

// All-lane wave64 float sum on the VALU: 4 DPP row steps + the gfx950 permlane swaps.
template <int ctrl>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, true));
}
// Every lane receives the sum over its 16-lane DPP row (4 fused v_add_f32_dpp).
__device__ __forceinline__ float row_sum(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x124>(v);
    return v + dpp<0x128>(v);
}
// permlane32 swap of (a, b) + add: lanes 0-31 get a[l] + a[l+32], lanes 32-63 b[l-32] + b[l].
__device__ __forceinline__ float swap32_sum(float a, float b) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// permlane16 swap of (a, b) + add: rows 0/2 get a's row pair sums, rows 1/3 b's.
__device__ __forceinline__ float swap16_sum(float a, float b) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// Wave sums of N per-lane values at once (transposed butterfly): N/2 permlane32 swaps, N/4
// permlane16 swaps, then one 16-lane DPP row sum per 4 values -- ~1.75 N operations instead
// of N full wave reductions.  On return, lane (row r, column c) with c < ceil(N/4) holds the
// sum of value wave_multi_sum_index(lane) (if < N); `out` is that lane's value.
__device__ __forceinline__ int wave_multi_sum_index(int lane) {
    const int r = lane >> 4, c = lane & 15;
    return 4 * c + (r == 0 ? 0 : r == 1 ? 2 : r == 2 ? 1 : 3);
}
template <int N>
__device__ __forceinline__ float wave_multi_sum(const float (&v)[N]) {
    constexpr int NP = (N + 1) / 2, NQ = (NP + 1) / 2;
    float Pp[2 * NQ];
#pragma unroll
    for (int t = 0; t < NP; t++) Pp[t] = swap32_sum(v[2 * t], 2 * t + 1 < N ? v[2 * t + 1] : 0.f);
#pragma unroll
    for (int t = NP; t < 2 * NQ; t++) Pp[t] = 0.f;
    const int col = threadIdx.x & 15;
    float out = 0.f;
#pragma unroll
    for (int t = 0; t < NQ; t++) {
        const float q = row_sum(swap16_sum(Pp[2 * t], Pp[2 * t + 1]));
        out = col == t ? q : out;
    }
    return out;
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x124>(v);  // row_ror:4
    v += dpp<0x128>(v);  // row_ror:8   -> every lane holds its 16-lane row sum
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(s[0]) + __uint_as_float(s[1]);  // rows (0,1) and (2,3)
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);  // halves
}

// The forward tile passes clear the backward's gradient accumulator lines: workgroup b of the
// grid stores zeros over float4s [b per, (b + 1) per), per = ceil(n4 / grid), before it takes
// its unit (so the blocks past the last unit clear their slice too).  Non-temporal: the lines
// are next touched by the backward, and the pass's records stay in the caches.
__device__ __forceinline__ void zero_slice(float4* z, long long n4) {
    if (!z) return;
    const long long per = (n4 + gridDim.x - 1) / gridDim.x;
    const long long b0 = (long long)blockIdx.x * per;
    const long long b1 = b0 + per < n4 ? b0 + per : n4;
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (long long i = b0 + (threadIdx.x & 63); i < b1; i += 64)
        __builtin_nontemporal_store((f4v){0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f4v*>(z + i));
}

// ---- one wave per 16x16 tile --------------------------------------------------------
// Lane l owns pixel (l % 8, l / 8) of each of the tile's four 8x8 quadrants q (offset
// (8 (q & 1), 8 (q >> 1))), so a wave holds the whole tile and every per-Gaussian quadrant
// decision is wave-uniform.  Batches of 64 candidates live in registers (one per lane);
// the inner loop walks the surviving lanes with s_ff1 and broadcasts each record with
// v_readlane, so the tile passes need no LDS and no workgroup barriers.
struct WaveTile {
    float pfx, pfy;          // quadrant-0 pixel of this lane
    float tx0, ty0, wmax, hmax;
    int px, py;

    __device__ __forceinline__ void init(unsigned tile, unsigned gx, int W, int H) {
        const int lane = threadIdx.x & 63;
        const unsigned bx = tile % gx, by = tile / gx;
        px = (int)(bx * GSR_BLOCK_X) + (lane & 7);
        py = (int)(by * GSR_BLOCK_Y) + (lane >> 3);
        pfx = (float)px;
        pfy = (float)py;
        tx0 = (float)(bx * GSR_BLOCK_X);
        ty0 = (float)(by * GSR_BLOCK_Y);
        wmax = (float)(W - 1);
        hmax = (float)(H - 1);
    }
    __device__ __forceinline__ bool inside(int q, int W, int H) const {
        return px + 8 * (q & 1) < W && py + 8 * (q >> 1) < H;
    }
    __device__ __forceinline__ int pixel(int q, int W) const { return W * (py + 8 * (q >> 1)) + px + 8 * (q & 1); }

    // Quadrants (bit q) the record can reach with alpha >= 1/255 (conservative, see
    // box_reachable); `limit[q]`: only positions < limit[q] are kept for quadrant q.
    // `qmask` (wave-uniform): the quadrants worth testing (a quadrant unit's own)
    __device__ __forceinline__ uint32_t reach(const Rec& r, uint32_t position, const uint32_t* limit,
                                              uint32_t qmask = 15u) const {
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (!((qmask >> q) & 1u)) continue;
            const float qx0 = tx0 + (q & 1) * 8.f, qy0 = ty0 + (q >> 1) * 8.f;
            const float qx1 = fminf(qx0 + 7.f, wmax), qy1 = fminf(qy0 + 7.f, hmax);
            if (qx0 <= wmax && qy0 <= hmax && (!limit || position < limit[q]) &&
                box_reachable(r.a.z, r.a.w, r.b.x, r.c.y, qx0 - r.a.x, qx1 - r.a.x, qy0 - r.a.y, qy1 - r.a.y))
                m |= 1u << q;
        }
        return m;
    }
};

// Exponent of the Gaussian at offset (dx, dy) from its centre, with the conic prepared as
// (na, nb, nc) = (-a/2, -b, -c/2) log2(e): power = (-(a dx^2 + c dy^2)/2 - b dx dy) log2(e).  The forward and
// backward tile passes evaluate it with this exact operation sequence, so the backward
// replays the forward's blend decisions bit for bit.
__device__ __forceinline__ float gauss_power(float na, float nb, float nc, float dx, float dy) {
    return __builtin_fmaf(na * dx, dx, __builtin_fmaf(nc * dy, dy, (nb * dx) * dy));
}

// ---- exact mode: the reference's blend arithmetic bit for bit ------------------------------
// The fast evaluation above (prescaled conic, two FMAs, v_exp_f32) decides a (pixel, Gaussian)
// pair differently from the reference's float arithmetic only where the exponent is within
// rounding of a threshold (alpha within ulps of 1/255, a transmittance within ulps of 1e-4): a
// pixel or two per frame.  A guard band around the alpha threshold -- the pairs there
// re-evaluated with the oracle's arithmetic -- measured +7.8 % on the 3-stream headline and +3 % on
// the single call (round 6: the forward to five waves per SIMD, one add and one compare per
// evaluation in both passes), and it cannot reach the transmittance decisions, which depend on
// every earlier alpha of the pixel.  So bit-parity is a mode: with gsr_set_exact_blend(1) the tile
// passes evaluate every pair as the reference does --
//   power = -0.5f * (a dx dx + c dy dy) - b dx dy  in its operation order, no contraction
//   G = expf(power)                                 glibc's algorithm (the oracle's libm), below
//   alpha = min(0.99f, o * G),  C += (colour * alpha) * T,  out = C + T * bg
// (forward.cu:335-359, oracle/gsr_oracle.c:437-456; every such block under `#pragma clang fp
// contract(off)`) -- so the forward's colours, transmittance and
// n_contrib equal the canonical oracle's bit for bit and the backward replays the same decisions
// (its gradients differ by summation order only).
// (plain operators under the pragma: HIP's __fmul_rn / __fadd_rn are operators in functions of
// their own, compiled with contraction on, so LLVM may still fuse them into FMAs once inlined)
__device__ __forceinline__ float ref_power(float a, float b, float c, float dx, float dy) {
#pragma clang fp contract(off)
    return -0.5f * (a * dx * dx + c * dy * dy) - b * dx * dy;
}
// glibc's expf (sysdeps/ieee754/flt-32/e_expf.c, the ARM optimized-routines algorithm the oracle's
// libm runs; on FMA hosts the __expf_fma build, whose contractions are reproduced here): x = (k +
// r) ln2 / 32 with k = round(x 32 / ln2), 2^(k/32) from a 32-entry table of asuint64(2^(i/32)) -
// (i << 47), 2^(r/32) by a cubic, all in double.  Equal to the host libm's expf on every float in
// [-104, 8] (2.2e9 inputs checked, tools/check_glibc_expf.c); below log(2^-150) it is 0, as glibc's
// underflow path returns.  tab: the table in LDS (gexp_table_init).
constexpr unsigned long long GEXP_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
__device__ __forceinline__ void gexp_table_init(unsigned long long* tab) {
    const int lane = threadIdx.x & 63;
    if (lane < 32) tab[lane] = GEXP_TAB[lane];
}
__device__ __forceinline__ float glibc_expf(float x, const unsigned long long* tab) {
#pragma clang fp contract(off)
    constexpr double INVLN2N = 0x1.71547652b82fep+5, SHIFT = 0x1.8p+52;
    const double xd = (double)x;
    double kd = __builtin_fma(xd, INVLN2N, SHIFT);
    const unsigned long long ki = __double_as_longlong(kd);
    kd -= SHIFT;
    const double r = __builtin_fma(xd, INVLN2N, -kd);
    const unsigned long long t = tab[ki & 31u] + (ki << 47);
    const double s = __longlong_as_double((long long)t);
    const double zz = __builtin_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
    const double r2 = r * r;
    double y = __builtin_fma(r, 0x1.62e42ff0c52d6p-6, 1.0);
    y = __builtin_fma(zz, r2, y);
    y = y * s;
    return x < -0x1.9fe368p6f ? 0.f : (float)y;
}

// Lane masks in SGPR pairs and selects on them (v_cmp_*_e64 / v_cndmask_b32_e64).  On
// gfx950 a v_cndmask_b32 that reads its mask from VCC (the VOP2 form the compiler picks
// for `c ? a : b`) issues ~5x slower than the VOP3 form reading any other SGPR pair
// (tools/micro/vcmp.hip), so the tile loops build masks and selects explicitly.
typedef uint64_t lmask;
__device__ __forceinline__ lmask m_gt0(float a) {  // a > 0
    lmask m;
    asm("v_cmp_lt_f32_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ lmask m_ge(float a, float b) {  // a >= b (false on NaN)
    lmask m;
    asm("v_cmp_ge_f32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
    return m;
}
__device__ __forceinline__ lmask m_lt1(float a) {  // a < 1
    lmask m;
    asm("v_cmp_gt_f32_e64 %0, 1.0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ lmask m_lt(float a, float b) {  // a < b
    lmask m;
    asm("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
    return m;
}
__device__ __forceinline__ lmask m_ult(uint32_t a, uint32_t b) {  // a < b, a wave-uniform
    lmask m;
    asm("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "s"(a), "v"(b));
    return m;
}
__device__ __forceinline__ lmask m_ultv(uint32_t a, uint32_t b) {  // a < b, a in a VGPR
    lmask m;
    asm("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
    return m;
}
__device__ __forceinline__ float sel(lmask m, float t, float f) {  // m ? t : f per lane
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t sel(lmask m, uint32_t t, uint32_t f) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
__device__ __forceinline__ lmask exec_mask() { return __builtin_amdgcn_read_exec(); }
// index of the lowest set bit of a wave-uniform mask, -1 when it is 0 (s_ff1_i32_b64)
__device__ __forceinline__ int sgpr_ff1(uint64_t m) {
    int r;
    asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
    return r;
}
// m with bit b cleared (s_bitset0_b64; b wave-uniform)
__device__ __forceinline__ uint64_t sgpr_clear_bit(uint64_t m, int b) {
    asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(b));
    return m;
}

// Row sums of NQ registers' 16-lane rows at once, transposed as row_sum3 (mirror steps pair
// registers, lone ones add to themselves), then quad_perm steps; lane column c returns
// register row_sums_t_reg<NQ>(c)'s row sum (-1: a duplicate or unused lane).
template <int NQ>
__device__ __forceinline__ int row_sums_t_reg(int col) {
    constexpr int NW = (NQ + 1) / 2, NX = (NW + 1) / 2;
    const int j = col & 3, b2 = (col >> 2) & 1, b3 = (col >> 3) & 1;
    if (j >= NX) return -1;
    const int w = 2 * j + 1 < NW ? 2 * j + b2 : (b2 ? -1 : 2 * j);
    if (w < 0) return -1;
    return 2 * w + 1 < NQ ? 2 * w + b3 : (b3 ? -1 : 2 * w);
}
template <int NQ>
__device__ __forceinline__ float row_sums_t(const float (&Q)[NQ], lmask mb3, lmask mb2, int col) {
    constexpr int NW = (NQ + 1) / 2, NX = (NW + 1) / 2;
    static_assert(NX <= 4, "at most 16 registers");
    float W[NW], X[NX];
#pragma unroll
    for (int i = 0; i < NW; i++)
        W[i] = 2 * i + 1 < NQ ? sel(mb3, Q[2 * i + 1], Q[2 * i]) + dpp<0x140>(sel(mb3, Q[2 * i], Q[2 * i + 1]))
                              : Q[2 * i] + dpp<0x140>(Q[2 * i]);
#pragma unroll
    for (int j = 0; j < NX; j++) {
        X[j] = 2 * j + 1 < NW ? sel(mb2, W[2 * j + 1], W[2 * j]) + dpp<0x141>(sel(mb2, W[2 * j], W[2 * j + 1]))
                              : W[2 * j] + dpp<0x141>(W[2 * j]);
        X[j] += dpp<0x4E>(X[j]);
        X[j] += dpp<0xB1>(X[j]);
    }
    float out = X[0];
#pragma unroll
    for (int j = 1; j < NX; j++) out = (col & 3) == j ? X[j] : out;
    return out;
}

// Row sums of three registers' 16-lane rows at once, transposed: row_mirror and
// row_half_mirror steps pair two registers per add (lane bit 3, then bit 2, selects which
// register a lane carries), then two quad_perm steps -- 5 DPP adds + 4 selects instead of
// 3 x 4 DPP adds.  On return the lanes of column 0 hold a's row sums, column 8 b's and
// column 4 c's.  mb3 / mb2: lane masks of column bit 3 / bit 2.
__device__ __forceinline__ float row_sum3(float a, float b, float c, lmask mb3, lmask mb2) {
    const float w = sel(mb3, b, a) + dpp<0x140>(sel(mb3, a, b));  // row_mirror: l <-> 15 - l
    const float v = c + dpp<0x140>(c);
    float x = sel(mb2, v, w) + dpp<0x141>(sel(mb2, w, v));        // row_half_mirror: l <-> 7 - l
    x += dpp<0x4E>(x);
    return x + dpp<0xB1>(x);
}

__device__ __forceinline__ float bcast(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ uint32_t bcast(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = __shfl_xor(m, o, 64);
        m = t > m ? t : m;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
}

}  // namespace gsr
