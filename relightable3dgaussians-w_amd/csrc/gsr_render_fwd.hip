// gsr_render_fwd.hip -- per-tile front-to-back alpha compositing (forward.cu:261-374).
//
// gfx950 design:
//  * one wave per 16x16 tile (WaveTile): each lane owns 4 pixels, one per 8x8 quadrant;
//    tiles are remapped so each XCD's L2 serves a contiguous band of the image (xcd_remap);
//  * the tile's list comes from its super-tile's entries (TileList, gsr_tile.hpp), filtered
//    and queued in LDS; batches of 64 list entries: each lane gathers one 48-B record and tests it
//    conservatively against the four quadrants (box_reachable); the wave then walks the
//    surviving lanes in list order (s_ff1), broadcasting each record with v_readlane, and
//    blends it only into the quadrants it can reach (wave-uniform branches).  The range
//    position travels with the record, so n_contrib (the reference's last_contributor)
//    is unchanged;
//  * a quadrant leaves the loop as soon as all its pixels are saturated, the tile as soon
//    as all four are (the reference's block-wide __syncthreads_count exit).
// Blend decisions and arithmetic order per pixel are the reference's, so colours, T and
// n_contrib match it exactly.
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

// six waves per SIMD
constexpr int FWD_WAVES = 6;

namespace gsr {

#ifdef GSR_RENDER_STATS
__device__ unsigned long long g_fwd_stats[8];
// per unit (workgroup): start, end (s_memrealtime), hw id, tile, quadrant mask, cost estimate, evaluations, -
__device__ unsigned long long g_fwd_times[GSR_UNIT_REC * 65536];
#ifdef GSR_TIMES_ONLY  // per-tile timing only (tools/xcd_balance.py): no per-evaluation counters
#define FWD_STAT(k, v)
#else
#define FWD_STAT(k, v) st[k] += (v)
#endif
#else
#define FWD_STAT(k, v)
#endif

// EXACT: the reference's blend arithmetic bit for bit (gsr_tile.hpp "exact mode"): the raw conic
// staged, the reference-order power, glibc's expf, the reference's colour order
template <bool EXACT>
__device__ __forceinline__ void render_fwd_tile(const RenderFwdArgs& a, const unsigned tile, const uint32_t qallow) {
    WaveTile wt;
    wt.init(tile, a.grid_x, a.W, a.H);
    const int lane = threadIdx.x;
    const unsigned sth = st_sth(a.grid_x, a.grid_y);
    const unsigned sti = ((tile / a.grid_x) >> sth) * a.gsx + (tile % a.grid_x) / GSR_ST_W;
    __shared__ TileListLds s_list;
    TileList<true> tl;
    const uint2 str = a.st_ranges[sti];
    tl.init(a.ent, str, tile, a.grid_x, sth, 0u, 0u);

    const float pxq[2] = {wt.pfx, wt.pfx + 8.f}, pyq[2] = {wt.pfy, wt.pfy + 8.f};
    __shared__ float4 s_a[64], s_b[64];
    __shared__ float4 s_c[64];  // (colour b, quadrant mask, -, -): 16-B rows, one LDS address for all three reads
    __shared__ uint32_t s_e[64];  // entry index
    __shared__ unsigned long long s_gexp[EXACT ? 32 : 1];  // exact mode: glibc_expf's table
    if (EXACT) gexp_table_init(s_gexp);
    float T[4], C0[4], C1[4], C2[4];
    float lim[4];  // alpha a Gaussian must reach to blend: 1/255, or +inf once the pixel is done
    uint32_t last[4];
    uint32_t live = 0;  // quadrants with a pixel still blending (wave-uniform)
#pragma unroll
    for (int q = 0; q < 4; q++) {
        T[q] = 1.f;
        C0[q] = C1[q] = C2[q] = 0.f;
        last[q] = 0;
        const bool in = wt.inside(q, a.W, a.H);
        lim[q] = in ? 1.0f / 255.0f : __builtin_inff();
        if (((qallow >> q) & 1u) && __ballot(in)) live |= 1u << q;
    }
#ifdef GSR_RENDER_STATS
    unsigned long long st[8] = {};
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t elast = 0;  // entry index of the latest Gaussian that blended anywhere (wave-uniform)
    // survivors stored so far (whole-tile units; SURV_NONE: none stored, or past SURV_CAP)
    uint32_t scnt = (a.surv && qallow == 15u) ? 0u : SURV_NONE;
    uint2* const sl = a.surv + (size_t)tile * SURV_CAP;
    // (survivor, quadrant) evaluations: the backward's cost estimate (its dispatch order, heaviest
    // first, and its balanced bands).  Round 5 (profiles/r5z_eval_cost_ab.txt): against the sum of
    // the quadrants' largest n_contrib, cfg2c render_bwd 0.465 -> 0.429 ms (its bands balance by the
    // work the backward repeats, not by list positions), cfg2 and training unchanged
    uint32_t nev = 0;
    while (live) {
        tl.fill(s_list);
        uint32_t id = 0, ei = 0, p0 = 0;
        const uint32_t nb = tl.take(s_list, id, ei, p0);
        if (nb == 0) break;
        const uint32_t j = p0 + (uint32_t)lane;  // list position
        uint32_t qm = 0;
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
        float rc = 0.f;
        if ((uint32_t)lane < nb) {
            const Rec r = a.rec[id];
            // a quadrant unit culls its batch against its own quadrant only (k_render_fwd 238.1 ->
            // 236.9 us, profiles/r5z_reach_own_ab.txt)
            qm = wt.reach(r, j, nullptr, qallow);
            // conic as gauss_power takes it: (-a/2, -b, -c/2) log2(e) (exact mode: raw)
            ra = EXACT ? r.a : make_float4(r.a.x, r.a.y, TILE_STAGE_AC * r.a.z, TILE_STAGE_B * r.a.w);
            rb = EXACT ? r.b : make_float4(TILE_STAGE_AC * r.b.x, r.b.y, r.b.z, r.b.w);
            rc = r.c.x;
        }
        // the batch's records go to LDS; the walk below reads each survivor's record with
        // broadcast LDS loads (LDS pipe) instead of 11 v_readlane (VALU), the next
        // survivor's loads issued before the current one is blended
        wave_lds_sync();
        s_a[lane] = ra;
        s_b[lane] = rb;
        s_c[lane] = make_float4(rc, __uint_as_float(qm), __uint_as_float(id), 0.f);
        s_e[lane] = ei;
        wave_lds_sync();
        const uint64_t todo0 = __ballot((qm & live) != 0);
        if (scnt != SURV_NONE) {  // the backward's list: (Gaussian, position << 4 | reach mask)
            const uint32_t n = (uint32_t)__popcll(todo0);
            if (scnt + n > SURV_CAP) {
                scnt = SURV_NONE;
            } else {
                if ((qm & live) != 0) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(todo0 >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)todo0, 0u));
                    sl[scnt + r] = make_uint2(id, (j << 4) | qm);
                }
                scnt += n;
            }
        }
        FWD_STAT(0, nb);
        FWD_STAT(1, __popcll(todo0));
        if (!todo0) continue;
        // blend one survivor (record A, B, Cq at batch slot k) into the four quadrants
        int klast = -1;  // batch slot of the latest survivor that blended anywhere
        uint64_t todo = todo0;
        auto blend_one = [&](const float4& A, const float4& B, const float4& Cq, int k) __attribute__((always_inline)) {
            const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(Cq.y)) & live;
            nev += (uint32_t)__popc(m);
            // the list position + 1 in a VGPR once per survivor (the selects below cannot read
            // it from an SGPR beside their SGPR mask: one constant-bus read per VOP3 on gfx950)
            uint32_t pos1;
            asm("v_mov_b32 %0, %1" : "=v"(pos1) : "s"(p0 + (uint32_t)k + 1u));
            lmask blended = 0;
            FWD_STAT(5, m == 15u);
            FWD_STAT(6, m != 0u);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!((m >> q) & 1u)) continue;
                const float dx = A.x - pxq[q & 1], dy = A.y - pyq[q >> 1];
                float power, alpha;
                if (EXACT) {  // forward.cu:335-343
#pragma clang fp contract(off)
                    power = ref_power(A.z, A.w, B.x, dx, dy);
                    alpha = fminf(0.99f, B.y * glibc_expf(power, s_gexp));
                } else {
                    power = gauss_power(A.z, A.w, B.x, dx, dy);
                    alpha = fminf(0.99f, B.y * tile_exp2(power));
                }
                // hit: !(power > 0) && alpha >= lim (masks and selects in SGPR pairs, see m_ge)
                // (compare results are 0 on inactive lanes, and the walk runs with every lane on:
                // no exec masking; each mask op below is one SALU instruction)
                const lmask hit = m_ge(alpha, lim[q]) & ~m_gt0(power);
                FWD_STAT(2, 1);
                FWD_STAT(3, hit != 0ull);
                FWD_STAT(4, __popcll(hit));
                const float test_T = T[q] * (1 - alpha);
                const lmask lt = m_lt(test_T, 0.0001f);  // saturating Gaussian is not blended
                const lmask blend = hit & ~lt, sat = hit & lt;
                if (EXACT) {  // forward.cu:359: C += feature * alpha * T, left to right
#pragma clang fp contract(off)
                    C0[q] = sel(blend, C0[q] + B.z * alpha * T[q], C0[q]);
                    C1[q] = sel(blend, C1[q] + B.w * alpha * T[q], C1[q]);
                    C2[q] = sel(blend, C2[q] + Cq.x * alpha * T[q], C2[q]);
                } else {
                    const float w = sel(blend, alpha * T[q], 0.f);
                    C0[q] += B.z * w;
                    C1[q] += B.w * w;
                    C2[q] += Cq.x * w;
                }
                T[q] = sel(blend, test_T, T[q]);
                last[q] = sel(blend, pos1, last[q]);
                blended |= blend;
                if (sat) {  // rare: pixels finish
                    lim[q] = sel(sat, __builtin_inff(), lim[q]);
                    if (!(m_lt(lim[q], 1.f) & exec_mask())) {
                        live &= ~(1u << q);
                        if (!live) todo = 0;  // the walk ends at the next survivor it would take
                    }
                }
            }
            if (blended) klast = k;
        };
        // survivors in pairs over two register sets (the next survivor's record is read
        // while the current one blends, and no register copies between them); the walk's
        // bookkeeping is a handful of SALU ops per survivor (s_ff1 gives -1 when none is left,
        // s_bitset0 clears the taken bit, the record rows share one LDS address)
        int k = sgpr_ff1(todo);
        todo = sgpr_clear_bit(todo, k);
        float4 A = s_a[k], B = s_b[k], Cq = s_c[k];
        for (;;) {
            const int kn = sgpr_ff1(todo), kl = kn > 0 ? kn : 0;
            todo = sgpr_clear_bit(todo, kl);
            const float4 An = s_a[kl], Bn = s_b[kl], Cn = s_c[kl];
            blend_one(A, B, Cq, k);
            if (kn < 0) break;
            k = sgpr_ff1(todo);
            const int kl2 = k > 0 ? k : 0;
            todo = sgpr_clear_bit(todo, kl2);
            A = s_a[kl2];
            B = s_b[kl2];
            Cq = s_c[kl2];
            blend_one(An, Bn, Cn, kn);
            if (k < 0) break;
        }
        if (klast >= 0) elast = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_e[klast]);
    }
#ifdef GSR_RENDER_STATS
    if (lane == 0) {
        for (int k = 0; k < 7; k++) atomicAdd(&g_fwd_stats[k], st[k]);
        if (blockIdx.x < 65536) {
            unsigned long long* u = g_fwd_times + GSR_UNIT_REC * blockIdx.x;
            u[0] = t_start;
            u[1] = __builtin_amdgcn_s_memrealtime();
            u[2] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
            u[3] = tile;
            u[4] = qallow;
            u[5] = a.st_ranges[sti].y - a.st_ranges[sti].x;
            u[6] = nev;
        }
    }
#endif
    const int HW = a.H * a.W;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (((qallow >> q) & 1u) && wt.inside(q, a.W, a.H)) {
            const int pix = wt.pixel(q, a.W);
            a.final_T[pix] = T[q];
            a.n_contrib[pix] = last[q];
            if (EXACT) {  // forward.cu:372
#pragma clang fp contract(off)
                a.out_color[pix] = C0[q] + T[q] * a.bg[0];
                a.out_color[HW + pix] = C1[q] + T[q] * a.bg[1];
                a.out_color[2 * HW + pix] = C2[q] + T[q] * a.bg[2];
            } else {
                a.out_color[pix] = C0[q] + T[q] * a.bg[0];
                a.out_color[HW + pix] = C1[q] + T[q] * a.bg[1];
                a.out_color[2 * HW + pix] = C2[q] + T[q] * a.bg[2];
            }
        }
    }
    if (lane == 0 && a.surv && qallow == 15u) a.surv_n[tile] = scnt;
    uint32_t nm = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t m = ((qallow >> q) & 1u) ? wave_max_u32(last[q]) : 0u;
        nm = m > nm ? m : nm;
    }
    if (lane == 0 && nm) {
        atomicMax(&a.tile_nmax[tile], nm);
        atomicMax(&a.tile_emax[tile], elast + 1u);
        if (a.tile_cost) atomicAdd(&a.tile_cost[tile], nev);
        if (a.row_cost) atomicAdd(&a.row_cost[tile / a.grid_x], nev);
    }
}


// One wave per unit of the dispatch order (tile_unit): a quadrant of a heavy tile or a
// whole tile.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FWD_WAVES, FWD_WAVES)))
k_render_fwd(RenderFwdArgs a) {
    unsigned tile;
    uint32_t qallow;
    zero_slice(a.zero, a.zero_n4);
    if (!tile_unit_fwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow)) return;
    render_fwd_tile<false>(a, tile, qallow);
}
// exact mode (gsr_set_exact_blend): the registers its double-precision expf needs, no occupancy target
__global__ void __launch_bounds__(64) k_render_fwd_exact(RenderFwdArgs a) {
    unsigned tile;
    uint32_t qallow;
    zero_slice(a.zero, a.zero_n4);
    if (!tile_unit_fwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow)) return;
    render_fwd_tile<true>(a, tile, qallow);
}

#ifdef GSR_RENDER_STATS
// zero the per-unit records (blocks without a unit write none)
extern "C" int gsr_debug_fwd_times_reset() {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_fwd_times)) != hipSuccess) return -1;
    return hipMemset(p, 0, sizeof(g_fwd_times)) == hipSuccess ? 0 : -1;
}
extern "C" int gsr_debug_fwd_times(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fwd_times), sizeof(unsigned long long) * GSR_UNIT_REC * n) == hipSuccess ? 0 : -1;
}
extern "C" int gsr_debug_fwd_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fwd_stats), sizeof(g_fwd_stats)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

void launch_render_fwd(const RenderFwdArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0) return;
    // one block per unit of the longest band (heavy tiles count four); the rest exit
    if (a.exact) hipLaunchKernelGGL(k_render_fwd_exact, dim3(tile_pass_blocks(ntile, FWD_TAIL_SPLIT)), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_render_fwd, dim3(tile_pass_blocks(ntile, FWD_TAIL_SPLIT)), dim3(64), 0, s, a);
}

}  // namespace gsr
