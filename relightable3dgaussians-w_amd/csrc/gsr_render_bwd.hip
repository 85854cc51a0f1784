// gsr_render_bwd.hip -- per-tile back-to-front gradient replay (backward.cu:399-557).
//
// gfx950 design (the reference issues 9 float atomics to global memory per contributing
// (pixel, Gaussian) pair, backward.cu:523,545-554):
//  * one wave per 16x16 tile (WaveTile), each lane owns one pixel of each 8x8 quadrant;
//    quadrant q replays only positions below its largest n_contrib (positions past every
//    pixel's last contributor are skipped by the reference too);
//  * the tile's list from its super-tile's entries (TileList, gsr_tile.hpp), back to front
//    from the forward's last contributor; batches of 64 list entries: each lane gathers one
//    record and tests it
//    against the four quadrants (box_reachable, limited by the quadrant's n_contrib); the
//    wave walks the surviving lanes (s_ff1 + v_readlane broadcasts);
//  * per Gaussian, the reachable quadrants run the reference's per-pixel recurrence
//    (T, accum_rec, last_alpha, last_color) branch-free with predicated updates and sum
//    their 9 partial gradients in-lane; the wave then reduces the 9 values once: 16-lane
//    DPP row sums (4 fused v_add_f32_dpp each), lane c of each row keeps value c, and two
//    permlane swaps add the four rows.  Lanes 0..8 issue one 9-lane atomic to the
//    Gaussian's 64-B accumulator line -- one request per (tile, Gaussian).
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"


namespace gsr {

#ifdef GSR_RENDER_STATS
__device__ unsigned long long g_bwd_stats[8];
// per unit (workgroup): start, end (s_memrealtime), hw id, tile, quadrant mask, largest n_contrib, survivors, -
__device__ unsigned long long g_bwd_times[GSR_UNIT_REC * 65536];
#ifdef GSR_TIMES_ONLY  // per-tile timing only (tools/xcd_balance.py): no per-evaluation counters
#define BWD_STAT(k, v)
#else
#define BWD_STAT(k, v) st[k] += (v)
#endif
#else
#define BWD_STAT(k, v)
#endif

// EXACT: the forward's exact mode replayed (gsr_tile.hpp): the same power, G and alpha bits
template <bool DET, bool EXACT>
__device__ __forceinline__ void render_bwd_tile(const RenderBwdArgs& a, const unsigned tile, const uint32_t qallow) {
    WaveTile wt;
    wt.init(tile, a.grid_x, a.W, a.H);
    const int lane = threadIdx.x;
    const int HW = a.H * a.W;

    const float pxq[2] = {wt.pfx, wt.pfx + 8.f}, pyq[2] = {wt.pfy, wt.pfy + 8.f};
    __shared__ float4 s_a[64], s_b[64], s_c[64];
    __shared__ unsigned long long s_gexp[EXACT ? 32 : 1];  // exact mode: glibc_expf's table
    if (EXACT) gexp_table_init(s_gexp);
    // per quadrant pixel state: T, dL/dpix, the background term, and the recurrence of
    // backward.cu:514-537 carried as one dot product with dL/dpix: Sr = accum_rec . dL/dpix
    // of the Gaussians behind the current one.  The reference updates accum_rec one step
    // late from (last_alpha, last_color); Sr is updated right after each Gaussian,
    // Sr = alpha cd + (1 - alpha) Sr = Sr + alpha (cd - Sr) -- the same recurrence, and a no-op
    // for a lane whose alpha is 0, so no per-lane selects are needed.
    float T[4], Tb[4], dp0[4], dp1[4], dp2[4], Sr[4];
    uint32_t last[4], qlim[4];
    uint32_t nmax = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const bool in = wt.inside(q, a.W, a.H);
        const int pix = in ? wt.pixel(q, a.W) : 0;
        const float Tf = in ? a.final_T[pix] : 0.f;
        last[q] = in ? a.n_contrib[pix] : 0u;
        dp0[q] = in ? a.dL_dpix[pix] : 0.f;
        dp1[q] = in ? a.dL_dpix[HW + pix] : 0.f;
        dp2[q] = in ? a.dL_dpix[2 * HW + pix] : 0.f;
        T[q] = Tf;
        // -T_final * bg . dL/dpix, the background term of dL/dalpha (backward.cu:533-537)
        Tb[q] = -Tf * (a.bg[0] * dp0[q] + a.bg[1] * dp1[q] + a.bg[2] * dp2[q]);
        Sr[q] = 0.f;
        qlim[q] = ((qallow >> q) & 1u) ? wave_max_u32(last[q]) : 0u;  // other quadrants: another wave
        nmax = qlim[q] > nmax ? qlim[q] : nmax;
    }
    // Reduction layout (see the end of the loop): lane 16 r + 8 j, j < 2, ends up holding
    // value 4 j + {0,2,1,3}[r] of the Gaussian's 9 gradient sums; lanes 4 + 16 r hold four
    // partial sums of value 8.
    const int row = lane >> 4, col = lane & 15;
    const int vrow = row == 0 ? 0 : row == 1 ? 2 : row == 2 ? 1 : 3;
    const int vidx = col == 0 ? vrow : col == 8 ? 4 + vrow : col == 4 ? 8 : -1;
    const lmask mb3 = __ballot((col & 8) != 0), mb2 = __ballot((col & 4) != 0);
    // values 0-4 (the conic-weighted sums) carry the opacity; the conic, -1/2 and the screen
    // scale are applied once per Gaussian by the preprocess backward (acc_raw)
    const bool vop = vidx >= 0 && vidx <= 4;
    // deterministic mode: the slot of this lane's value in the instance's partial row
    // (values 0..7, then value 8's four row partials)
    const int pslot = vidx < 8 ? vidx : 8 + row;

#ifdef GSR_RENDER_STATS
    unsigned long long st[8] = {};
    uint32_t nsurv = 0;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
    // the tile's list back to front from its last contributor (the forward's tile_emax and
    // tile_nmax: the entry and, over the whole tile, its list position + 1)
    const unsigned sth = st_sth(a.grid_x, a.grid_y);
    const unsigned sti = ((tile / a.grid_x) >> sth) * a.gsx + (tile % a.grid_x) / GSR_ST_W;
    __shared__ TileListLds s_list;
    // the forward's survivor list when it stored one (wave-uniform): batches of 64 back to front,
    // each lane's entry loaded a batch ahead (its record one batch ahead too measured the same
    // call and a slower 3-stream headline: 113 VGPRs); else the super-tile list, filtered and
    // culled again
    const uint32_t sn = a.surv ? a.surv_n[tile] : SURV_NONE;
    const uint2* sl = a.surv + (size_t)tile * SURV_CAP;
    const bool lst = sn != SURV_NONE;
    uint32_t li = lst ? sn : 0u;  // list entries left
    uint2 nv = lst ? sl[max((int)li - 1 - lane, 0)] : make_uint2(0u, 0u);
    TileList<false> tl;
    if (!lst)
        tl.init(a.ent, a.st_ranges[sti], tile, a.grid_x, sth, nmax ? a.tile_emax[tile] : 0u, nmax ? a.tile_nmax[tile] : 0u);
    const uint32_t rbase = DET ? a.ranges[tile].x : 0u;  // deterministic rows: the materialised list start
    for (;;) {
        uint32_t id = 0, nb, p, qm = 0;  // p: list position (back to front)
        if (lst) {
            nb = min(64u, li);
            if (nb == 0) break;
            const uint2 v = nv;
            li -= nb;
            nv = sl[max((int)li - 1 - lane, 0)];
            id = v.x;
            p = v.y >> 4;
            if ((uint32_t)lane < nb) {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (p < qlim[q]) qm |= v.y & (1u << q);
            }
        } else {
            tl.fill(s_list);
            uint32_t ei = 0, p0 = 0;
            nb = tl.take(s_list, id, ei, p0);
            if (nb == 0) break;
            p = p0 - (uint32_t)lane;
        }
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
        float rc = 0.f;
        if ((uint32_t)lane < nb) {
            const Rec r = a.rec[id];
            if (!lst) qm = wt.reach(r, p, qlim);
            // conic as gauss_power takes it: (-a/2, -b, -c/2) log2(e) (exact mode: raw)
            ra = EXACT ? r.a : make_float4(r.a.x, r.a.y, TILE_STAGE_AC * r.a.z, TILE_STAGE_B * r.a.w);
            rb = EXACT ? r.b : make_float4(TILE_STAGE_AC * r.b.x, r.b.y, r.b.z, r.b.w);
            rc = r.c.x;
        }
        // records to LDS; survivors are read back with broadcast LDS loads (LDS pipe)
        // instead of v_readlane (VALU), the next survivor's issued before the current one
        wave_lds_sync();
        s_a[lane] = ra;
        s_b[lane] = rb;
        // (position << 4 | reach mask): one word, one readfirstlane per survivor for both
        s_c[lane] = make_float4(rc, __uint_as_float((p << 4) | qm), __uint_as_float(id), 0.f);
        wave_lds_sync();
        uint64_t todo = __ballot(qm != 0);
        BWD_STAT(0, nb);
        BWD_STAT(1, __popcll(todo));
#ifdef GSR_RENDER_STATS
        nsurv += __popcll(todo);
#endif
        if (!todo) continue;
        // one survivor (record A, B, Cq at batch slot k), back to front
        auto grad_one = [&](const float4& A, const float4& B, const float4& Cq, int k) __attribute__((always_inline)) {
            const uint32_t mp = (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(Cq.y));
            const uint32_t m = mp & 15u;
            const float ax = A.x, ay = A.y, ka = A.z, kb = A.w, kc = B.x, op = B.y;
            const float c0 = B.z, c1 = B.w, c2 = Cq.x;
            const uint32_t pos = mp >> 4;  // list position
            // per-lane sums over the quadrants: M1 = sum G dL/dalpha dx, M2 = ... dy,
            // S2/S3/S4 = sum G dL/dalpha (dx dx, dx dy, dy dy), S5 = sum G dL/dalpha,
            // S6..8 = sum alpha T dL/dpix
            float M1 = 0.f, M2 = 0.f, S2 = 0.f, S3 = 0.f, S4 = 0.f, S5 = 0.f, S6 = 0.f, S7 = 0.f, S8 = 0.f;
            bool any = false;
            // one reachable quadrant: the exponent and the blend decision (pre), then the
            // recurrence and this Gaussian's sums (post); inactive lanes run post with alpha =
            // G = 0, leaving T, the sums and the gradients unchanged
            auto pre = [&](int q, float& dx, float& dy, float& G, float& alpha, lmask& act) __attribute__((always_inline)) {
                BWD_STAT(2, 1);
                dx = ax - pxq[q & 1];
                dy = ay - pyq[q >> 1];
                float power;
                if (EXACT) {  // backward.cu:494-500 with the forward's exact bits
#pragma clang fp contract(off)
                    power = ref_power(ka, kb, kc, dx, dy);
                    G = glibc_expf(power, s_gexp);
                    alpha = fminf(0.99f, op * G);
                } else {
                    power = gauss_power(ka, kb, kc, dx, dy);
                    G = tile_exp2(power);
                    alpha = fminf(0.99f, op * G);
                }
                // active: pos < last && !(power > 0) && !(alpha < 1/255)
                // (compare results are 0 on inactive lanes, and every lane is on: no exec masking)
                act = (m_ult(pos, last[q]) & ~m_gt0(power)) & ~m_lt(alpha, 1.0f / 255.0f);
            };
            auto post = [&](int q, float dx, float dy, float G, float alpha, lmask act) __attribute__((always_inline)) {
                BWD_STAT(3, 1);
                BWD_STAT(4, __popcll(act));
                const float ae = sel(act, alpha, 0.f);
                const float Ge = sel(act, G, 0.f);
                const float inv = __builtin_amdgcn_rcpf(1.f - ae);
                const float Tn = T[q] * inv;
                const float dch = ae * Tn;
                const float cdp = __builtin_fmaf(c2, dp2[q], __builtin_fmaf(c1, dp1[q], c0 * dp0[q]));
                const float dcs = cdp - Sr[q];
                const float dLda = __builtin_fmaf(Tn, dcs, inv * Tb[q]);
                Sr[q] = __builtin_fmaf(ae, dcs, Sr[q]);
                const float Gd = Ge * dLda;
                S5 += Gd;
                const float wdx = Gd * dx, wdy = Gd * dy;
                M1 += wdx;
                M2 += wdy;
                S2 = __builtin_fmaf(wdx, dx, S2);
                S3 = __builtin_fmaf(wdx, dy, S3);
                S4 = __builtin_fmaf(wdy, dy, S4);
                S6 = __builtin_fmaf(dch, dp0[q], S6);
                S7 = __builtin_fmaf(dch, dp1[q], S7);
                S8 = __builtin_fmaf(dch, dp2[q], S8);
                T[q] = Tn;
            };
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!((m >> q) & 1u)) continue;
                float dx, dy, G, al;
                lmask k;
                pre(q, dx, dy, G, al, k);
                if (k == 0ull) continue;  // wave-uniform
                any = true;
                post(q, dx, dy, G, al, k);
            }
            if (any) {
            BWD_STAT(5, 1);
            // raw sums (the line's layout, acc_raw): M1, M2 -- dL/dmean2D is -(a M1 + b M2),
            // -(b M1 + c M2) in pixels (backward.cu:540-545), formed per Gaussian by the
            // preprocess backward, as is the conic's -1/2 and the NDC scale
            // wave reduction: permlane32 swaps pair (M1,M2),(S2,S3),(S4,S5),(S6,S7)
            // into half-wave sums, permlane16 swaps pair those into row sums of four values
            // per register, then the three registers' 16-lane rows sum transposed (row_sum3)
            float P0 = swap32_sum(M1, M2), P1 = swap32_sum(S2, S3), P2 = swap32_sum(S4, S5);
            float P3 = swap32_sum(S6, S7);
            // S8 skips both swap stages: its four row sums go to the atomic as partial sums
            // (lanes 4, 20, 36, 52)
            const float Q0 = swap16_sum(P0, P1), Q1 = swap16_sum(P2, P3), Q2 = S8;
            float v = row_sum3(Q0, Q1, Q2, mb3, mb2);
            v = vop ? v * op : v;
            if (DET) {  // one row per instance, summed per Gaussian in tile order (k_det_gather)
                if (vidx >= 0 && v != 0.f) a.partial[(size_t)(rbase + pos) * DET_ROW3 + pslot] = v;
            } else if (vidx >= 0 && v != 0.f) {
                atomicAdd(a.acc + (size_t)__float_as_uint(Cq.z) * ACC_STRIDE + vidx, v);
            }
            }
        };
        // survivors in pairs over two register sets (the next survivor's record is read
        // while the current one runs, and no register copies between them); s_ff1 gives -1
        // when none is left, s_bitset0 clears the taken bit
        int k = sgpr_ff1(todo);
        todo = sgpr_clear_bit(todo, k);
        float4 A = s_a[k], B = s_b[k], Cq = s_c[k];
        for (;;) {
            const int kn = sgpr_ff1(todo), kl = kn > 0 ? kn : 0;
            todo = sgpr_clear_bit(todo, kl);
            const float4 An = s_a[kl], Bn = s_b[kl], Cn = s_c[kl];
            grad_one(A, B, Cq, k);
            if (kn < 0) break;
            k = sgpr_ff1(todo);
            const int kl2 = k > 0 ? k : 0;
            todo = sgpr_clear_bit(todo, kl2);
            A = s_a[kl2];
            B = s_b[kl2];
            Cq = s_c[kl2];
            grad_one(An, Bn, Cn, kn);
            if (k < 0) break;
        }
    }
#ifdef GSR_RENDER_STATS
    if (lane == 0) {
        for (int k = 0; k < 6; k++) atomicAdd(&g_bwd_stats[k], st[k]);
        if (blockIdx.x < 65536) {
            unsigned long long* u = g_bwd_times + GSR_UNIT_REC * blockIdx.x;
            u[0] = t_start;
            u[1] = __builtin_amdgcn_s_memrealtime();
            u[2] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
            u[3] = tile;
            u[4] = qallow;
            u[5] = nmax;
            u[6] = nsurv;
        }
    }
#endif
}


// One wave per unit of the dispatch order (tile_unit): a quadrant of a heavy tile or a
// whole tile.  Four waves per SIMD: the kernel alone is faster at five (336.6-337.1 ->
// 330.4-332.5 us at cfg2, tools/r3_check44.sh), but in the bench's throughput mode -- views on
// 3 HIP streams, this pass overlapping other views' forward and geometry kernels -- four leave
// them room: the headline +0.9 % at cfg2 and +1.3 % at cfg5, the isolated call pair +7 / +22 us
// (profiles/r4zo_ab_bwd_waves_default_bench.txt).
constexpr int BWD_WAVES = 4;
template <bool DET>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BWD_WAVES, BWD_WAVES)))
k_render_bwd(RenderBwdArgs a) {
    unsigned tile;
    uint32_t qallow;
    if (!tile_unit_bwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow, DET)) return;
    render_bwd_tile<DET, false>(a, tile, qallow);
}
template <bool DET>
__global__ void __launch_bounds__(64) k_render_bwd_exact(RenderBwdArgs a) {
    unsigned tile;
    uint32_t qallow;
    if (!tile_unit_bwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow, DET)) return;
    render_bwd_tile<DET, true>(a, tile, qallow);
}

#ifdef GSR_RENDER_STATS
// zero the per-unit records (blocks without a unit write none)
extern "C" int gsr_debug_bwd_times_reset() {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_bwd_times)) != hipSuccess) return -1;
    return hipMemset(p, 0, sizeof(g_bwd_times)) == hipSuccess ? 0 : -1;
}
extern "C" int gsr_debug_bwd_times(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_times), sizeof(unsigned long long) * GSR_UNIT_REC * n) == hipSuccess ? 0 : -1;
}
extern "C" int gsr_debug_bwd_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_stats), sizeof(g_bwd_stats)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

void launch_render_bwd(const RenderBwdArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0) return;
    // one block per unit of the longest band (heavy tiles count four); the rest exit
    const dim3 grid(tile_pass_blocks_bal(ntile, 0u));
    if (a.exact) {
        if (a.partial) hipLaunchKernelGGL(k_render_bwd_exact<true>, grid, dim3(64), 0, s, a);
        else hipLaunchKernelGGL(k_render_bwd_exact<false>, grid, dim3(64), 0, s, a);
    } else {
        if (a.partial) hipLaunchKernelGGL(k_render_bwd<true>, grid, dim3(64), 0, s, a);
        else hipLaunchKernelGGL(k_render_bwd<false>, grid, dim3(64), 0, s, a);
    }
}

}  // namespace gsr
