// gsr_binning.hip -- instance lists per tile (rasterizer_impl.cu:70-138 re-designed).
//
// The reference emits one 64-bit key (tile << 32 | depth) per (Gaussian, tile) pair --
// R of them, ~28M at 1.5M Gaussians/1080p -- and radix-sorts all R on 32+13 bits.  Here:
//   1. the P_v visible Gaussians are sorted once by depth (gsr_sort.hip);
//   2. in that order every Gaussian emits one entry per SUPER-TILE (8x4 tiles, 8x8 for large frames: st_sth) its rect
//      touches (k_st_emit: S ~ 1.3 P_v entries instead of R);
//   3. the S entries are stably sorted by super-tile id (one 8-bit pass at 1080p);
//   4. each super-tile list is cut into 1024-entry segments (k_seg_table); one workgroup
//      per segment keeps, for each of the super-tile's 32 tiles, the entries whose rect
//      covers it with an order-preserving wave-ballot compaction.  The entry's coverage of
//      its super-tile (a local tile rect, 10 bits) rides in the key's top bits through the
//      sort (which only orders bits [0, log2 NS)), so the filters read one coalesced word per
//      entry instead of gathering the Gaussian's rect.  A count pass
//      (k_seg_lists<false>), a per-tile prefix over segments (k_seg_prefix), a scan over
//      tiles (= the reference's ranges) and a write pass (k_seg_lists<true>) produce
//      point_list directly, in coalesced runs.
// Every step is stable, so each tile's list is exactly the reference's order
// (depth-bits ascending, Gaussian index ascending on ties), bit-exact.
#include <type_traits>

#include "gsr_block.hpp"
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"
#include "gsr_order.hpp"

namespace gsr {

// Local tile rect of a Gaussian inside super-tile (sx, sy) of height 2^sth tiles
// (gsr_common.hpp's code layout).
__device__ __forceinline__ uint32_t local_rect_code(uint2 r, uint32_t sx, uint32_t sy, uint32_t sth) {
    const int tx0 = (int)(sx * GSR_ST_W), ty0 = (int)(sy << sth);
    const int cx0 = max((int)(r.x & 0xffffu) - tx0, 0), cx1 = min((int)(r.x >> 16) - tx0, (int)GSR_ST_W);
    const int cy0 = max((int)(r.y & 0xffffu) - ty0, 0), cy1 = min((int)(r.y >> 16) - ty0, 1 << sth);
    return (uint32_t)cx0 | ((uint32_t)(cx1 - 1) << ST_XB) | ((uint32_t)cy0 << (2 * ST_XB)) |
           ((uint32_t)(cy1 - 1) << (2 * ST_XB + ST_YB));
}
// the super-tile's tiles a code covers: bit t = tile (t % ST_W, t / ST_W)
__device__ __forceinline__ uint64_t local_rect_mask(uint32_t code) {
    constexpr uint32_t XM = (1u << ST_XB) - 1u, YM = (1u << ST_YB) - 1u;
    const uint32_t cx0 = code & XM, cx1 = ((code >> ST_XB) & XM) + 1u, cy0 = (code >> (2 * ST_XB)) & YM,
                   cy1 = ((code >> (2 * ST_XB + ST_YB)) & YM) + 1u;
    const uint64_t row = ((1ull << cx1) - 1ull) & ~((1ull << cx0) - 1ull);
    uint64_t m = 0;
#pragma unroll
    for (uint32_t y = 0; y < (1u << ST_YB); y++) m |= (y >= cy0 && y < cy1) ? row << (GSR_ST_W * y) : 0ull;
    return m;
}
// the super-tile rect [sx0, sx1) x [sy0, sy1) of a tile rect, packed as the tile rects are
__device__ __forceinline__ uint2 st_rect_of(uint2 r, uint32_t sth) {
    const uint32_t sx0 = (r.x & 0xffffu) / GSR_ST_W, sx1 = ((r.x >> 16) + GSR_ST_W - 1) / GSR_ST_W;
    const uint32_t sy0 = (r.y & 0xffffu) >> sth, sy1 = ((r.y >> 16) + (1u << sth) - 1u) >> sth;
    return make_uint2(sx0 | (sx1 << 16), sy0 | (sy1 << 16));
}

// ---- 2. super-tile emission -----------------------------------------------------------
// One wave emits the entries of 64 consecutive depth-sorted Gaussians as one contiguous
// run: lane i writes entry i, i+64, ... (coalesced), locating its Gaussian by binary
// search over the wave's inclusive count prefix in LDS.
__global__ void __launch_bounds__(256) k_st_emit(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets,
                                                  const uint2* rect, unsigned gsx, unsigned sth, uint32_t* st_keys,
                                                  uint32_t* st_vals) {
    __shared__ uint32_t s_inc[4][64];
    __shared__ uint32_t s_id[4][64];
    __shared__ uint2 s_srect[4][64];
    __shared__ uint2 s_rect[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t idx = 0, cnt = 0;
    uint2 sr = make_uint2(0, 0), r = make_uint2(0, 0);
    if (s < Pv) {
        idx = sorted_ids[s];
        r = rect[idx];
        sr = st_rect_of(r, sth);
        cnt = ((sr.x >> 16) - (sr.x & 0xffffu)) * ((sr.y >> 16) - (sr.y & 0xffffu));
    }
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    s_inc[wave][lane] = inc;
    s_id[wave][lane] = idx;
    s_srect[wave][lane] = sr;
    s_rect[wave][lane] = r;
    const int s0 = blockIdx.x * blockDim.x + wave * 64;
    const uint32_t base = s0 < Pv ? offsets[s0] : 0u;
    const uint32_t total = __shfl(inc, 63, 64);
    __syncthreads();
    for (uint32_t i = lane; i < total; i += 64) {
        int lo = 0, hi = 63;  // first j with s_inc[j] > i
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_inc[wave][mid] > i) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t k = i - (lo ? s_inc[wave][lo - 1] : 0u);
        const uint2 rr = s_srect[wave][lo];
        const uint32_t x0 = rr.x & 0xffffu, w = (rr.x >> 16) - x0, y0 = rr.y & 0xffffu;
        const uint32_t yy = k / w, xx = k - yy * w;
        const uint32_t sx = x0 + xx, sy = y0 + yy;
        st_keys[base + i] = (sy * gsx + sx) | (local_rect_code(s_rect[wave][lo], sx, sy, sth) << ST_KEY_BITS);
        st_vals[base + i] = s_id[wave][lo];
    }
}

// ---- frame totals for the host (see FrameTotals) ---------------------------------------------
__device__ __forceinline__ void frame_totals(const FrameTotals& f) {
    __shared__ unsigned long long st[4][16];
    unsigned long long v[4] = {0, 0, 0, 0};
    constexpr int U = 4;  // loads in flight per thread (few registers: it rides in other kernels)
    for (int b0 = 0; b0 < f.nblk; b0 += U * (int)blockDim.x) {
        uint4 t[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int b = b0 + u * (int)blockDim.x + (int)threadIdx.x;
            t[u] = b < f.nblk ? f.blk_tot[b] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            v[0] += t[u].x;
            v[1] += t[u].y;
            v[2] += t[u].z;
            v[3] |= t[u].w;
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long u = __shfl_xor(v[k], o, 64);
            v[k] = k == 3 ? (v[k] | u) : v[k] + u;
        }
        if (lane == 0) st[k][wave] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        unsigned long long t = 0;
        for (int w = 0; w < nw; w++) t = k == 3 ? (t | st[k][w]) : t + st[k][w];
        // each word carries the call's tag in its low 16 bits, so the host needs no ordering
        // between them (a system-scope release would write back the L2)
        const unsigned long long w = (t > 0xFFFFFFFFFFFFull ? 0xFFFFFFFFFFFFull : t) << 16 | (f.seq & 0xFFFFull);
        __hip_atomic_store(f.host + k, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void __launch_bounds__(256) k_frame_totals(FrameTotals f) { frame_totals(f); }

void launch_frame_totals(const FrameTotals& ft, hipStream_t s) {
    hipLaunchKernelGGL(k_frame_totals, dim3(1), dim3(256), 0, s, ft);
}

// ---- 2+3 fused: super-tile entries emitted straight into super-tile order ----------------
// The depth-sorted visible Gaussians are cut into blocks of ST_G.  k_st_hist counts each
// block's entries per super-tile (digit-major table [NS][nb]) from the rects in depth order
// (carried through the depth sort, so nothing is gathered at random); k_digit_scan (gsr_sort.hip) turns every super-tile's row into
// block offsets + a total; k_st_scatter scans the totals into super-tile bases and ranges,
// re-enumerates each block's entries in (Gaussian, super-tile) order and
// ranks them per super-tile with wave ballots, writing each entry at its final position.
// Equivalent to emit + a stable counting sort by super-tile (the entry order within a
// super-tile is the depth order), in four launches and no entry round trip through HBM.
constexpr int ST_G = 1024;  // Gaussians per block
// waves per block in k_st_hist / k_st_scatter (ST_G / W Gaussians each): 8, or 4 when the
// per-wave LDS state of 8 waves would not fit (st_waves)


// P_v from the depth sort's last pass (depth_sort's pv_out).  The forward launches the binning before its one host synchronisation (the
// binning buffer is sized from the previous call's counts, see gsr_capi.cpp), so these
// kernels read the visible count on the device.  Block-uniform.
__device__ __forceinline__ int block_visible(int pv_host, const unsigned long long* pv) {
    if (!pv) return pv_host;
    return (int)__builtin_amdgcn_readfirstlane((int)*pv);
}

// The depth-sorted rects: 8 B each, or packed to 4 (pack_rect) on a grid of at most 255 x 255
// tiles (the depth sort moves 4 bytes less per key and pass, the binning reads 4 less).
template <bool PACKED>
__device__ __forceinline__ uint2 sorted_rect(const void* r, int p) {
    if constexpr (PACKED) return unpack_rect(reinterpret_cast<const uint32_t*>(r)[p]);
    else return reinterpret_cast<const uint2*>(r)[p];
}

// k_st_hist's LDS histograms: one per block.  (Round 3's per-wave counts stored by k_st_hist
// for the scatter were retired in round 5: k_st_hist now stores the block's entry-balanced wave
// cuts instead.)
constexpr int st_hist_count(int) { return 1; }

// A lane's super-tile rect [sx0, sx1) x [sy0, sy1) is walked by the lane itself when it holds
// at most ST_BIG super-tiles; larger rects (screen-filling Gaussians right in front of the
// camera: up to every super-tile of the frame) are walked by the whole wave, one rect at a
// time, 64 super-tiles per step, so one such Gaussian does not serialise its chunk -- its lane
// alone issued one LDS atomic per super-tile per pass, and its neighbours' lanes the same
// addresses (the clustered cfg2c frame: k_st_scatter 32 -> 113 us against cfg2).  f(sx, sy, o,
// a0, a1, a2) runs once per (lane o, super-tile) pair with lane o's values a0..a2.  Every lane
// of the wave must call it (a ballot); lanes with nothing to walk pass an empty rect.
constexpr uint32_t ST_BIG = 16u;
template <class F>
__device__ __forceinline__ void st_rect_walk(uint32_t sx0, uint32_t sx1, uint32_t sy0, uint32_t sy1, uint32_t a0,
                                             uint32_t a1, uint32_t a2, F&& f) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = sx1 > sx0 ? sx1 - sx0 : 0u, n = sy1 > sy0 ? w * (sy1 - sy0) : 0u;
    const bool big = n > ST_BIG;
    if (!big)
        for (uint32_t sy = sy0; sy < sy1; sy++)
            for (uint32_t sx = sx0; sx < sx1; sx++) f(sx, sy, lane, a0, a1, a2);
    uint64_t bm = __ballot(big);
    while (bm) {
        const int k = __builtin_ctzll(bm);
        bm &= bm - 1ull;
        const uint32_t bx = bcast(sx0, k), bw = bcast(w, k), by = bcast(sy0, k), by1 = bcast(sy1, k);
        const uint32_t b0 = bcast(a0, k), b1 = bcast(a1, k), b2 = bcast(a2, k);
        if (bw >= 64u) {  // a row per step, 64 columns at a time
            for (uint32_t sy = by; sy < by1; sy++)
                for (uint32_t sx = bx + (uint32_t)lane; sx < bx + bw; sx += 64u) f(sx, sy, k, b0, b1, b2);
        } else {  // floor(64 / bw) rows per step; one division per rect, none per step
            const uint32_t rps = 64u / bw, ro = (uint32_t)lane / bw, col = (uint32_t)lane - ro * bw;
            if (ro < rps)
                for (uint32_t sy = by + ro; sy < by1; sy += rps) f(bx + col, sy, k, b0, b1, b2);
        }
    }
}

// k_st_hist: per block of ST_G depth-sorted Gaussians, its entry count per super-tile (the
// digit scan's table) and its ST_W wave cuts for k_st_scatter.  Thread t counts Gaussians
// g0 + PER t .. + PER - 1.  The cuts split the block into contiguous wave ranges of about equal
// entry counts (super-tiles touched): cuts[blk][w] = the first Gaussian of wave w (w >= 1; wave
// 0 starts at g0, the last wave ends at the block's end).  Equal Gaussian counts gave the wave
// holding the block's nearest Gaussians (block 0: screen-filling splats right in front of the
// camera) most of the block's entries -- a 72 us wave against ~8 us for the rest at cfg2c
// (tools/unit_times.py).
template <int ST_W, bool PACKED>
__global__ void __launch_bounds__(64 * ST_W) k_st_hist(int Pv, const unsigned long long* totals, const void* rect_sorted, unsigned gsx, unsigned sth,
                                                  int NS, int nb, uint32_t* table, uint32_t* cuts) {
    constexpr int PER = ST_G / (64 * ST_W);  // consecutive Gaussians per thread
    extern __shared__ uint32_t hist[];  // [NS]
    __shared__ uint32_t s_bscan[ST_W];
    for (int i = threadIdx.x; i < NS; i += (64 * ST_W)) hist[i] = 0;
    Pv = block_visible(Pv, totals);
    __syncthreads();
    const unsigned blk = xcd_remap(blockIdx.x, nb);  // neighbouring blocks share an L2
    const int t = threadIdx.x;
    const int g0 = blk * ST_G, g1 = min(Pv, g0 + ST_G);
    uint32_t n[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {  // wave-uniform trip count (st_rect_walk's ballot)
        const int p = g0 + t * PER + j;
        const uint2 sr = p < g1 ? st_rect_of(sorted_rect<PACKED>(rect_sorted, p), sth) : make_uint2(0u, 0u);
        const uint32_t sx0 = sr.x & 0xffffu, sx1 = sr.x >> 16, sy0 = sr.y & 0xffffu, sy1 = sr.y >> 16;
        n[j] = (sx1 - sx0) * (sy1 - sy0);
        sum += n[j];
        st_rect_walk(sx0, sx1, sy0, sy1, 0u, 0u, 0u,
                     [&](uint32_t sx, uint32_t sy, int, uint32_t, uint32_t, uint32_t) { atomicAdd(&hist[sy * gsx + sx], 1u); });
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<ST_W>(sum, s_bscan, &tot);
    uint32_t* cb = cuts + (size_t)blk * ST_W;
    // s_bscan[w] = hardware wave w's entries = wave w's under equal Gaussian counts (64 threads x
    // PER = ST_G / ST_W Gaussians).  Balanced blocks keep the equal cuts: whole 64-Gaussian chunks
    // per wave (an entry-balanced cut falls mid-chunk and costs its wave a third, partial chunk:
    // +3 us on the uniform cfg2 scatter); only a block whose heaviest wave holds over twice the
    // mean is cut by entries.
    uint32_t wmax = 0;
#pragma unroll
    for (int w = 0; w < ST_W; w++) wmax = max(wmax, s_bscan[w]);
    if (tot == 0 || (unsigned long long)wmax * ST_W <= 2ull * tot) {  // equal Gaussian counts
        if (t > 0 && t < ST_W) cb[t] = (uint32_t)min(max(g0, g1), g0 + t * (ST_G / ST_W));
    } else {
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const uint32_t lo = run;
            run += n[j];
            for (int w = 1; w < ST_W; w++) {
                const uint32_t tgt = (uint32_t)(((unsigned long long)w * tot) / ST_W);
                if (lo <= tgt && tgt < run) cb[w] = (uint32_t)(g0 + t * PER + j);  // the Gaussian holding entry tgt
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NS; i += (64 * ST_W)) table[(size_t)i * nb + blk] = hist[i];
}

// Segment table of the materialised tile lists (SEG entries per segment, see k_seg_lists),
// in the materialisation scratch (seg_layout).
constexpr uint32_t SEG = 1024;
struct SegTable {
    uint32_t *seg_st, *seg_e0, *st_seg0, *nseg_total, *seg_cnt;
    uint32_t gcap;  // capacity of the table (segments)
};
__host__ __device__ inline size_t seg_capacity(long long S, int nst) { return (size_t)((S + SEG - 1) / SEG) + (size_t)nst; }
inline SegTable seg_layout(void* temp, long long S, int nst) {
    const size_t G = seg_capacity(S, nst);
    SegTable t;
    t.seg_st = reinterpret_cast<uint32_t*>(temp);
    t.seg_e0 = t.seg_st + G;
    t.st_seg0 = t.seg_e0 + G;
    t.nseg_total = t.st_seg0 + nst + 1;
    t.seg_cnt = t.nseg_total + 1;  // [G][32], becomes the segment bases in place
    t.gcap = (uint32_t)G;
    return t;
}

// Orders a wave's LDS accesses across lanes (LDS executes one wave's instructions in order)
// without the vmcnt wait a wavefront fence adds: the ranking must not wait for its own
// scattered stores or the next chunk's prefetch.
__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Per block of ST_G sorted Gaussians, ST_W waves each own ST_G / ST_W consecutive Gaussians,
// one Gaussian per lane per 64-Gaussian chunk.  k_st_hist counted each wave's entries per
// super-tile, so each wave's run of every super-tile starts at the block offset from the
// table + the counts of the block's earlier waves.  Per chunk: every lane ORs its bit into
// the 64-bit lane mask of each super-tile it touches; an entry's rank in its run is the popcount of the mask's
// lower lanes (a Gaussian touches a super-tile at most once, so the lanes in a mask are
// exactly the entries of that super-tile in depth order); the lowest lane then advances
// the run and clears the mask.  Order-independent atomics only, so the output is
// deterministic, and each super-tile's entries come out in depth order.
template <bool PACKED>
__device__ __forceinline__ void st_pass(int p0, int p1, const uint32_t* sorted_ids, const void* rect_sorted,
                                        unsigned gsx, unsigned sth, uint32_t* wcnt, unsigned long long* wmask, uint2* ent,
                                        uint32_t cap) {
    const int lane = threadIdx.x & 63;
    const unsigned long long bit = 1ull << lane, lt = bit - 1ull;
    // the next chunk's rect and id are loaded while this chunk is ranked
    uint2 r_nx = make_uint2(0u, 0u);
    uint32_t gid_nx = 0;
    if (p0 + lane < p1) {
        r_nx = sorted_rect<PACKED>(rect_sorted, p0 + lane);
        gid_nx = sorted_ids[p0 + lane];
    }
    for (int c0 = p0; c0 < p1; c0 += 64) {
        const uint2 r = r_nx;
        const uint32_t gid = gid_nx;
        const uint2 sr = (c0 + lane < p1) ? st_rect_of(r, sth) : make_uint2(0u, 0u);
        if (c0 + 64 + lane < p1) {
            r_nx = sorted_rect<PACKED>(rect_sorted, c0 + 64 + lane);
            gid_nx = sorted_ids[c0 + 64 + lane];
        }
        const uint32_t sx0 = sr.x & 0xffffu, sx1 = sr.x >> 16, sy0 = sr.y & 0xffffu, sy1 = sr.y >> 16;
        st_rect_walk(sx0, sx1, sy0, sy1, 0u, 0u, 0u, [&](uint32_t sx, uint32_t sy, int o, uint32_t, uint32_t, uint32_t) {
            atomicOr(&wmask[sy * gsx + sx], 1ull << o);
        });
        lds_order();
        st_rect_walk(sx0, sx1, sy0, sy1, r.x, r.y, gid,
                     [&](uint32_t sx, uint32_t sy, int o, uint32_t rx, uint32_t ry, uint32_t g) {
                         const uint32_t sid = sy * gsx + sx;
                         const uint32_t pos = wcnt[sid] + (uint32_t)__popcll(wmask[sid] & ((1ull << o) - 1ull));
                         if (pos < cap)  // S beyond the speculative capacity: the forward redoes the binning
                             ent[pos] = make_uint2(sid | (local_rect_code(make_uint2(rx, ry), sx, sy, sth) << ST_KEY_BITS), g);
                     });
        lds_order();
        st_rect_walk(sx0, sx1, sy0, sy1, 0u, 0u, 0u, [&](uint32_t sx, uint32_t sy, int o, uint32_t, uint32_t, uint32_t) {
            const uint32_t sid = sy * gsx + sx;
            const unsigned long long m = wmask[sid];
            if ((m & ((1ull << o) - 1ull)) == 0ull) {  // the lowest lane of the run advances it
                wcnt[sid] += (uint32_t)__popcll(m);
                wmask[sid] = 0ull;
            }
        });
        lds_order();
    }
}

// Workgroups: nb scatter blocks, then (optional) the frame totals, then (optional) the
// forward's dispatch order, one workgroup per XCD band (costs from the super-tile totals, so
// neither needs a launch of its own).  Each scatter block scans the super-tile totals into
// the super-tile bases itself (block 0 also writes the ranges and header[0] = S).
#ifdef GSR_RENDER_STATS
__device__ unsigned long long g_st_times[4 * 65536];  // per scatter wave: block start, pass start, end, block
#endif
template <int ST_W, bool PACKED>
__global__ void __launch_bounds__(64 * ST_W) k_st_scatter(int Pv, const unsigned long long* totals, const uint32_t* sorted_ids,
                                                     const void* rect_sorted, unsigned gsx, unsigned sth, int NS, int nb,
                                                     const uint32_t* table, const uint32_t* cuts,
                                                     const uint32_t* tot, uint2* st_ranges, unsigned long long* header,
                                                     uint2* ent, uint32_t cap, FrameTotals ft, TileOrderArgs ord) {
    if ((int)blockIdx.x >= nb) {
        const int x = (int)blockIdx.x - nb - (ft.host ? 1 : 0);
        if (x < 0) frame_totals(ft);  // the extra workgroup: the host's frame totals
        else tile_order_band((unsigned)x, ord);
        return;
    }
#ifdef GSR_RENDER_STATS
    const unsigned long long t_block = __builtin_amdgcn_s_memrealtime();
#endif
    extern __shared__ unsigned long long st_lds[];  // [ST_W][NS] lane masks, then [ST_W][NS] run counters
    __shared__ uint32_t s_scan[ST_W];
    unsigned long long* wmask_all = st_lds;
    uint32_t* wcnt_all = reinterpret_cast<uint32_t*>(st_lds + ST_W * NS);
    const int wave = threadIdx.x >> 6;
    Pv = block_visible(Pv, totals);
    const unsigned blk = xcd_remap(blockIdx.x, nb);  // as k_st_hist: runs of neighbours merge in L2
    const int g0 = blk * ST_G;
    // wave `wave`'s Gaussians: [p0, p1), the entry-balanced cuts k_st_hist stored
    const int gend = min(Pv, g0 + ST_G);
    const int p0 = wave == 0 ? g0 : (int)cuts[(size_t)blk * ST_W + wave];
    const int p1 = wave + 1 == ST_W ? max(g0, gend) : (int)cuts[(size_t)blk * ST_W + wave + 1];
    // super-tile s's base (exclusive scan of the totals); each wave's run of s starts there +
    // the block's offset + the counts of the block's earlier waves.  The waves count their
    // entries per super-tile again here, into the run counters, from the rects k_st_hist read
    // (4 KiB per block, L2-resident): storing k_st_hist's per-wave counts and reading them back
    // moved 4 x ST_W x NS bytes per block through HBM (80 MB each way at cfg5).
    for (int i = threadIdx.x; i < ST_W * NS; i += (64 * ST_W)) wcnt_all[i] = 0u;
    __syncthreads();
    {
        const int lane = threadIdx.x & 63;
        uint32_t* wh = wcnt_all + wave * NS;
        for (int pb = p0; pb < p1; pb += 64) {
            const int p = pb + lane;
            const uint2 sr = p < p1 ? st_rect_of(sorted_rect<PACKED>(rect_sorted, p), sth) : make_uint2(0u, 0u);
            st_rect_walk(sr.x & 0xffffu, sr.x >> 16, sr.y & 0xffffu, sr.y >> 16, 0u, 0u, 0u,
                         [&](uint32_t sx, uint32_t sy, int, uint32_t, uint32_t, uint32_t) { atomicAdd(&wh[sy * gsx + sx], 1u); });
        }
    }
    __syncthreads();
    uint32_t carry = 0;
    for (int c = 0; c < NS; c += 64 * ST_W) {
        const int i = c + (int)threadIdx.x;
        const uint32_t v = i < NS ? tot[i] : 0u;
        uint32_t t;
        const uint32_t ex = carry + block_exclusive_scan<ST_W>(v, s_scan, &t);
        if (i < NS) {
            // ranges clamped to the entry capacity (the scatter drops entries beyond it: a tile
            // pass over an overflowed binning reads only written entries, the forward redoes it)
            if (blockIdx.x == 0) st_ranges[i] = v ? make_uint2(min(ex, cap), min(ex + v, cap)) : make_uint2(0u, 0u);
            uint32_t run = ex + table[(size_t)i * nb + blk];
            for (int w = 0; w < ST_W; w++) {
                const uint32_t c = wcnt_all[w * NS + i];  // this thread's super-tile only
                wmask_all[w * NS + i] = 0ull;
                wcnt_all[w * NS + i] = run;
                run += c;
            }
        }
        carry += t;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) header[0] = min(carry, cap);
    __syncthreads();
#ifdef GSR_RENDER_STATS
    const unsigned long long t_pass = __builtin_amdgcn_s_memrealtime();
#endif
    st_pass<PACKED>(p0, p1, sorted_ids, rect_sorted, gsx, sth, wcnt_all + wave * NS, wmask_all + wave * NS, ent, cap);
#ifdef GSR_RENDER_STATS
    if ((threadIdx.x & 63) == 0 && blockIdx.x * ST_W + wave < 65536) {  // per wave: block start, pass start, end
        unsigned long long* u = g_st_times + 4 * (blockIdx.x * ST_W + wave);
        u[0] = t_block;
        u[1] = t_pass;
        u[2] = __builtin_amdgcn_s_memrealtime();
        u[3] = (unsigned long long)blk;
    }
#endif
}

#ifdef GSR_RENDER_STATS
extern "C" int gsr_debug_st_times(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_st_times), sizeof(unsigned long long) * 4 * n) == hipSuccess ? 0 : -1;
}
extern "C" int gsr_debug_st_times_reset() {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_st_times)) != hipSuccess) return -1;
    return hipMemset(p, 0, sizeof(g_st_times)) == hipSuccess ? 0 : -1;
}
#endif

static int st_waves(int NS) { return 12 * 8 * NS <= 65536 ? 8 : 4; }

size_t st_bin_temp_bytes(long long Pv, int NS) {
    const size_t nb = (size_t)((Pv + ST_G - 1) / ST_G);
    return 4 * (size_t)NS * nb + 4 * (size_t)st_waves(NS) * nb + 8 * (size_t)NS + 4 * 256 + 1024 + 256;
}

// per-wave LDS masks + counters: 12 B x waves x NS within a 64 KiB workgroup allocation
bool st_bin_supported(int NS) { return 12 * 4 * NS <= 65536; }

void launch_st_bin(int Pv, const unsigned long long* totals, const uint32_t* sorted_ids, const void* rect_sorted,
                   bool packed, unsigned gsx, unsigned sth, int NS, void* temp, uint2* ent, uint2* st_ranges,
                   unsigned long long* header, uint32_t cap, hipStream_t s, const FrameTotals* ftp,
                   const TileOrderArgs* ordp) {
    FrameTotals ft{};
    if (ftp) ft = *ftp;
    TileOrderArgs ord{};
    if (ordp) ord = *ordp;
    if (Pv <= 0) {  // otherwise the scatter writes every super-tile's range
        (void)hipMemsetAsync(st_ranges, 0, sizeof(uint2) * (size_t)NS, s);
        (void)hipMemsetAsync(header, 0, 8, s);
        if (ftp) launch_frame_totals(ft, s);
        if (ordp) {  // every tile's cost is 0: its super-tile range, zeroed above
            ord.st_ranges = st_ranges;
            ord.st_tot = nullptr;
            launch_tile_order_args(ord, s);
        }
        return;
    }
    const int nb = (Pv + ST_G - 1) / ST_G;
    const int W = st_waves(NS);
    char* t = reinterpret_cast<char*>(temp);
    auto take = [&](size_t bytes) {
        char* p = t;
        t += (bytes + 255) & ~(size_t)255;
        return p;
    };
    uint32_t* table = reinterpret_cast<uint32_t*>(take(4 * (size_t)NS * nb));
    uint32_t* tot = reinterpret_cast<uint32_t*>(take(4 * (size_t)NS));
    uint32_t* cuts = reinterpret_cast<uint32_t*>(take(4 * (size_t)W * nb));  // the blocks' wave cuts
    auto hist = [&](auto kern, int threads) {
        hipLaunchKernelGGL(kern, dim3(nb), dim3(threads), 4 * st_hist_count(threads / 64) * NS, s, Pv, totals, rect_sorted, gsx, sth,
                           NS, nb, table, cuts);
    };
    if (W == 8) packed ? hist(k_st_hist<8, true>, 512) : hist(k_st_hist<8, false>, 512);
    else packed ? hist(k_st_hist<4, true>, 256) : hist(k_st_hist<4, false>, 256);
    launch_digit_scan(NS, table, nb, tot, s);
    if (ordp) ord.st_tot = tot;
    const dim3 grid(nb + (ftp ? 1 : 0) + (ordp && ord.ntile ? 8 : 0));
    auto scatter = [&](auto kern, int threads) {
        hipLaunchKernelGGL(kern, grid, dim3(threads), 12 * (threads / 64) * NS, s, Pv, totals, sorted_ids, rect_sorted,
                           gsx, sth, NS, nb, table, cuts, tot, st_ranges, header, ent, cap, ft, ord);
    };
    if (W == 8) packed ? scatter(k_st_scatter<8, true>, 512) : scatter(k_st_scatter<8, false>, 512);
    else packed ? scatter(k_st_scatter<4, true>, 256) : scatter(k_st_scatter<4, false>, 256);
}

// super-tile segment bounds in the sorted entry list; empty super-tiles stay (0, 0)
__global__ void __launch_bounds__(256) k_seg_ranges(long long n, const uint32_t* keys, uint2* ranges) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t cur = keys[i] & ST_KEY_MASK;
    if (i == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys[i - 1] & ST_KEY_MASK;
        if (cur != prev) {
            ranges[prev].y = (uint32_t)i;
            ranges[cur].x = (uint32_t)i;
        }
    }
    if (i == n - 1) ranges[cur].y = (uint32_t)n;
}

// the non-fused path's sorted (key, id) pairs -> entries; header[0] = S
__global__ void __launch_bounds__(256) k_pack_entries(long long n, const uint32_t* keys, const uint32_t* vals,
                                                       uint2* ent, unsigned long long* header) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) header[0] = (unsigned long long)n;
    if (i < n) ent[i] = make_uint2(keys[i], vals[i]);
}

// ---- 4. tile lists from the super-tile lists (materialised for tests, the GSR_DEBUG checks
// and the deterministic backward; the tile passes filter the super-tile lists themselves) ----

struct StGeom {
    unsigned tx0, ty0, nx, ny;
};
__device__ __forceinline__ StGeom st_geom(unsigned st, unsigned gsx, unsigned gx, unsigned gy) {
    StGeom g;
    g.tx0 = (st % gsx) * GSR_ST_W;
    const unsigned sth = st_sth(gx, gy);
    g.ty0 = (st / gsx) << sth;
    g.nx = min(GSR_ST_W, gx - g.tx0);
    g.ny = min(1u << sth, gy - g.ty0);
    return g;
}

// Segment table of the materialisation.

__global__ void __launch_bounds__(256) k_seg_table(int nst, const uint2* st_ranges, uint32_t* seg_st,
                                                    uint32_t* seg_e0, uint32_t* st_seg0, uint32_t* nseg_total,
                                                    uint32_t gcap) {
    // single workgroup: exclusive scan of per-super-tile segment counts, then fill the table
    __shared__ uint32_t sh[4];
    uint32_t carry = 0;
    for (int c = 0; c < nst; c += 256) {
        const int st = c + threadIdx.x;
        uint32_t n = 0;
        uint2 r = make_uint2(0, 0);
        if (st < nst) {
            r = st_ranges[st];
            n = (r.y - r.x + SEG - 1) / SEG;
        }
        uint32_t tot;
        const uint32_t off = carry + block256_exclusive_scan(n, sh, &tot);
        if (st < nst) {
            st_seg0[st] = off;
            for (uint32_t k = 0; k < n && off + k < gcap; k++) {  // gcap: the table's capacity
                seg_st[off + k] = (uint32_t)st;
                seg_e0[off + k] = r.x + k * SEG;
            }
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        st_seg0[nst] = carry;
        *nseg_total = min(carry, gcap);
    }
}

// Count (WRITE = false) or write (WRITE = true) one segment: for each of the super-tile's
// 32 tiles, the entries whose rect covers it, ranked in list order by wave ballots.  Lane t
// of every wave holds the wave's output base for tile t, so a rank is one readlane plus
// a lane-masked popcount; lanes covering tile t store to consecutive addresses.
template <bool WRITE>
__global__ void __launch_bounds__(256) k_seg_lists(const uint32_t* nseg_total, const uint32_t* seg_st,
                                                    const uint32_t* seg_e0, const uint2* st_ranges,
                                                    const uint2* ent, unsigned gx,
                                                    unsigned gy, unsigned gsx, uint32_t* seg_cnt,
                                                    const uint32_t* seg_base, const uint32_t* tile_start,
                                                    uint32_t* point_list, uint32_t cap_s, uint32_t cap_r) {
    __shared__ uint32_t s_wc[4][ST_TILES];
    const uint32_t gseg = blockIdx.x;
    if (gseg >= *nseg_total) return;
    const unsigned st = seg_st[gseg];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t e0 = seg_e0[gseg];
    // cap_s / cap_r: the entry and list capacities (exceeded only when the forward's
    // speculative binning buffer was too small; it then redoes the binning)
    const uint32_t e1 = min(min(e0 + SEG, st_ranges[st].y), cap_s);
    // lane t < 32: running output position of tile t (block-uniform across waves): the
    // segment's base within the tile's list + the tile's list start
    uint32_t run = 0;
    if (WRITE && lane < ST_TILES) {
        run = seg_base[(size_t)gseg * ST_TILES + lane];
        const StGeom g = st_geom(st, gsx, gx, gy);
        const unsigned lx = lane % GSR_ST_W, ly = lane / GSR_ST_W;
        if (lx < g.nx && ly < g.ny) run += tile_start[(g.ty0 + ly) * gx + g.tx0 + lx];
    }
    // every batch's keys (and ids) are loaded up front: one memory latency per segment
    constexpr int NB = SEG / 256;
    uint32_t kb[NB], vb[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const uint32_t e = e0 + 256u * j + tid;
        const uint2 v = e < e1 ? ent[e] : make_uint2(0u, 0u);
        kb[j] = v.x;
        vb[j] = v.y;
    }
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const uint32_t b = e0 + 256u * j;
        if (b >= e1) break;  // block-uniform
        const uint32_t e = b + tid;
        uint32_t id = 0;
        uint64_t mask = 0;
        if (e < e1) {
            // local tile coverage mask (bit t = tile (t % ST_W, t / ST_W))
            mask = local_rect_mask(kb[j] >> ST_KEY_BITS);
            if (WRITE) id = vb[j];
        }
        uint64_t bal[ST_TILES];
        uint32_t mine = 0;
#pragma unroll
        for (int t = 0; t < ST_TILES; t++) {
            bal[t] = __ballot((uint32_t)(mask >> t) & 1u);
            mine = lane == t ? (uint32_t)__popcll(bal[t]) : mine;
        }
        if (lane < ST_TILES) s_wc[wave][lane] = mine;
        __syncthreads();
        uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        if (lane < ST_TILES) {
            c0 = s_wc[0][lane];
            c1 = s_wc[1][lane];
            c2 = s_wc[2][lane];
            c3 = s_wc[3][lane];
        }
        if (WRITE) {
            const uint32_t wbase = run + (wave > 0 ? c0 : 0u) + (wave > 1 ? c1 : 0u) + (wave > 2 ? c2 : 0u);
#pragma unroll
            for (int t = 0; t < ST_TILES; t++) {
                if ((uint32_t)(mask >> t) & 1u) {
                    const uint32_t lo = (uint32_t)bal[t], hi = (uint32_t)(bal[t] >> 32);
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
                    const uint32_t pos = bcast(wbase, t) + r;
                    if (pos < cap_r) point_list[pos] = id;
                }
            }
        }
        run += c0 + c1 + c2 + c3;
        __syncthreads();
    }
    if (!WRITE && wave == 0 && lane < ST_TILES) seg_cnt[(size_t)gseg * ST_TILES + lane] = run;
}

// Per (super-tile, local tile): prefix of the segment counts -> segment-relative bases,
// and the tile's total count.
__global__ void __launch_bounds__(256) k_seg_prefix(int nst, const uint32_t* st_seg0, unsigned gx, unsigned gy,
                                                     unsigned gsx, uint32_t* seg_cnt_to_base, uint32_t* tile_cnt,
                                                     uint32_t gcap) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nst * (int)ST_TILES) return;
    const unsigned st = i / ST_TILES, t = i % ST_TILES;
    const StGeom g = st_geom(st, gsx, gx, gy);
    const unsigned lx = t % GSR_ST_W, ly = t / GSR_ST_W;
    uint32_t run = 0;
    for (uint32_t k = st_seg0[st]; k < min(st_seg0[st + 1], gcap); k++) {
        const uint32_t c = seg_cnt_to_base[(size_t)k * ST_TILES + t];
        seg_cnt_to_base[(size_t)k * ST_TILES + t] = run;
        run += c;
    }
    if (lx < g.nx && ly < g.ny) tile_cnt[(g.ty0 + ly) * gx + g.tx0 + lx] = run;
}



// One 1024-thread workgroup: tile_start = exclusive scan of the tile counts, ranges =
// [start, start + count) (empty tiles (0, 0)), and tile_nmax zeroed for the forward's
// atomicMax.  The counts are staged in LDS (up to TS_LDS tiles; larger grids read them
// from HBM).  (The dispatch order stays its own 8-workgroup launch: its LDS atomics
// serialise when all eight bands share one CU.)
constexpr int TS_LDS = 12288;
__global__ void __launch_bounds__(1024) k_tile_scan(int T, const uint32_t* cnt, uint32_t* start, uint2* ranges,
                                                     uint32_t* tile_nmax, uint32_t cap_r) {
    __shared__ uint32_t s_cnt[TS_LDS];
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool in_lds = T <= TS_LDS;
    if (in_lds) {  // coalesced; all loads issued before the first LDS store
        uint32_t tmp[TS_LDS / 1024];
#pragma unroll
        for (int k = 0; k < TS_LDS / 1024; k++) tmp[k] = tid + 1024 * k < T ? cnt[tid + 1024 * k] : 0u;
#pragma unroll
        for (int k = 0; k < TS_LDS / 1024; k++)
            if (tid + 1024 * k < T) s_cnt[tid + 1024 * k] = tmp[k];
    }
    __syncthreads();
    uint32_t carry = 0;
    for (int c0 = 0; c0 < T; c0 += 8192) {
        const int base = c0 + tid * 8;
        uint32_t v[8], tot = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            v[k] = base + k < T ? (in_lds ? s_cnt[base + k] : cnt[base + k]) : 0u;
            tot += v[k];
        }
        uint32_t inc = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t wpre = 0, all = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            wpre += w < wave ? wsum[w] : 0u;
            all += wsum[w];
        }
        uint32_t run = carry + wpre + inc - tot;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (base + k < T) {
                start[base + k] = run;
                ranges[base + k] = v[k] ? make_uint2(min(run, cap_r), min(run + v[k], cap_r)) : make_uint2(0u, 0u);
            }
            run += v[k];
        }
        carry += all;
        __syncthreads();
    }
    if (tile_nmax)
        for (int t = tid; t < T; t += 1024) tile_nmax[t] = 0;
}

// ---- host launchers ---------------------------------------------------------------------
void launch_st_emit(int Pv, const uint32_t* sorted_ids, const uint32_t* offsets, const uint2* rect, unsigned gsx,
                    unsigned sth, uint32_t* st_keys, uint32_t* st_vals, hipStream_t s) {
    if (Pv == 0) return;
    hipLaunchKernelGGL(k_st_emit, dim3((Pv + 255) / 256), dim3(256), 0, s, Pv, sorted_ids, offsets, rect, gsx, sth,
                       st_keys, st_vals);
}

void launch_seg_ranges(long long n, int nseg, const uint32_t* sorted_keys, const uint32_t* sorted_vals, uint2* ranges,
                       uint2* ent, unsigned long long* header, hipStream_t s) {
    (void)hipMemsetAsync(ranges, 0, sizeof(uint2) * (size_t)nseg, s);
    if (n == 0) {
        (void)hipMemsetAsync(header, 0, 8, s);
        return;
    }
    const unsigned nb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_seg_ranges, dim3(nb), dim3(256), 0, s, n, sorted_keys, ranges);
    hipLaunchKernelGGL(k_pack_entries, dim3(nb), dim3(256), 0, s, n, sorted_keys, sorted_vals, ent, header);
}

size_t materialize_temp_bytes(long long S, int nst, int T) {
    const size_t G = seg_capacity(S, nst);
    return 4 * (2 * G + (nst + 1) + 1 + G * ST_TILES) + 8 * (size_t)T + 1024;
}

void launch_materialize(long long S, int nst, const uint2* st_ranges, const uint2* ent, unsigned gx, unsigned gy,
                        unsigned gsx, void* temp, uint32_t* point_list, uint2* ranges, long long R, hipStream_t s) {
    const int T = (int)(gx * gy);
    const SegTable tab = seg_layout(temp, S, nst);
    const size_t G = tab.gcap;
    uint32_t* tile_cnt = tab.seg_cnt + G * ST_TILES;
    uint32_t* tile_start = tile_cnt + T;
    hipLaunchKernelGGL(k_seg_table, dim3(1), dim3(256), 0, s, nst, st_ranges, tab.seg_st, tab.seg_e0, tab.st_seg0,
                       tab.nseg_total, (uint32_t)G);
    if (G > 0)
        hipLaunchKernelGGL(k_seg_lists<false>, dim3((unsigned)G), dim3(256), 0, s, tab.nseg_total, tab.seg_st,
                           tab.seg_e0, st_ranges, ent, gx, gy, gsx, tab.seg_cnt, (const uint32_t*)nullptr,
                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t)S, (uint32_t)R);
    // k_seg_prefix writes every tile's count (the super-tiles partition the grid)
    const int np = nst * (int)ST_TILES;
    hipLaunchKernelGGL(k_seg_prefix, dim3((np + 255) / 256), dim3(256), 0, s, nst, tab.st_seg0, gx, gy, gsx,
                       tab.seg_cnt, tile_cnt, (uint32_t)G);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, T, tile_cnt, tile_start, ranges, (uint32_t*)nullptr,
                       (uint32_t)(R < 0xFFFFFFFFll ? R : 0xFFFFFFFFll));
    if (G > 0)
        hipLaunchKernelGGL(k_seg_lists<true>, dim3((unsigned)G), dim3(256), 0, s, tab.nseg_total, tab.seg_st,
                           tab.seg_e0, st_ranges, ent, gx, gy, gsx, (uint32_t*)nullptr, tab.seg_cnt, tile_start,
                           point_list, (uint32_t)S, (uint32_t)R);
}

}  // namespace gsr
