// gsr_render_mc.hip -- multi-channel tile passes: one forward / backward composite of up
// to 16 per-Gaussian feature channels over one geometry.
//
// render() (gaussian_renderer/__init__.py:160-264) rasterizes the same Gaussians 6-10 times
// with different colours (image, diffuse, specular, depth, normal, alpha, ...).  Every call
// repeats the per-(pixel, Gaussian) alpha evaluation, the transmittance recurrence and the
// backward's geometric gradient reduction; only the three colour FMAs differ.  Here all
// channels are composited in one pass: alpha, T and the blend decisions are evaluated once
// and applied to every channel.  The blend arithmetic per channel is the forward tile
// pass's (gsr_render_fwd.hip), so each channel equals what a separate 3-channel call of the
// same features produces, bit for bit; the backward's geometric gradients are the sum of
// the separate calls' (the recurrence is carried as dot products over all channels).
//
// Layout: features [P][fstride] floats, fstride a multiple of 4; the pass handles one group
// of <= 16 channels (NC4 float4 per Gaussian), the host loops over groups.  Per batch of 64
// list entries the group's features go to LDS with the records and survivors read them by
// broadcast ds_read_b128.  Backward: 6 geometric sums + 4 NC4 feature sums reduce with the
// same permlane32 / permlane16 / DPP tree as the 3-channel pass; geometric sums go to the
// Gaussian's accumulator line, feature sums to dL/dfeatures (one atomic per value per
// (tile, Gaussian)).
#include <type_traits>

#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

// NCH: channels composited (<= 4 NC4; render()'s layout has 14, so its group skips the two
// padding channels' FMAs and reduction slots)
// EXACT: the reference's blend arithmetic bit for bit (gsr_tile.hpp "exact mode")
template <int NC4, int NCH = 4 * NC4, bool EXACT = false>
__device__ __forceinline__ void render_fwd_mc_tile(const RenderMcArgs& a, const unsigned tile, const uint32_t qallow) {
    WaveTile wt;
    wt.init(tile, a.grid_x, a.W, a.H);
    const int lane = threadIdx.x;
    const unsigned sth = st_sth(a.grid_x, a.grid_y);
    const unsigned st = ((tile / a.grid_x) >> sth) * a.gsx + (tile % a.grid_x) / GSR_ST_W;
    __shared__ TileListLds s_list;
    TileList<true> tl;
    tl.init(a.ent, a.st_ranges[st], tile, a.grid_x, sth, 0u, 0u);

    const float pxq[2] = {wt.pfx, wt.pfx + 8.f}, pyq[2] = {wt.pfy, wt.pfy + 8.f};
    __shared__ float4 s_a[64], s_b[64];
    __shared__ float4 s_f[NC4][64];
    __shared__ uint32_t s_q[64], s_e[64];  // quadrant mask, entry index
    __shared__ unsigned long long s_gexp[EXACT ? 32 : 1];  // exact mode: glibc_expf's table
    if (EXACT) gexp_table_init(s_gexp);
    float T[4], Cc[4][NCH], lim[4];
    uint32_t last[4];
    uint32_t live = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        T[q] = 1.f;
#pragma unroll
        for (int c = 0; c < NCH; c++) Cc[q][c] = 0.f;
        last[q] = 0;
        const bool in = wt.inside(q, a.W, a.H);
        lim[q] = in ? 1.0f / 255.0f : __builtin_inff();
        if (((qallow >> q) & 1u) && __ballot(in)) live |= 1u << q;
    }
    uint32_t elast = 0;  // entry index of the latest Gaussian that blended anywhere
    uint32_t nev = 0;    // (survivor, quadrant) evaluations: the backward's cost estimate
    // the backward's survivor list (as gsr_render_fwd.hip): whole-tile units only
    uint32_t scnt = (a.surv && qallow == 15u) ? 0u : SURV_NONE;
    uint2* const sl = a.surv + (size_t)tile * SURV_CAP;
    while (live) {
        tl.fill(s_list);
        uint32_t id = 0, ei = 0, p0 = 0;
        const uint32_t nb = tl.take(s_list, id, ei, p0);
        if (nb == 0) break;
        const uint32_t j = p0 + (uint32_t)lane;
        uint32_t qm = 0;
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
        float4 f[NC4];
#pragma unroll
        for (int g = 0; g < NC4; g++) f[g] = ra;
        if ((uint32_t)lane < nb) {
            const Rec r = a.rec[id];
            qm = wt.reach(r, j, nullptr, qallow);  // (a quadrant unit tests its own only)
            ra = EXACT ? r.a : make_float4(r.a.x, r.a.y, TILE_STAGE_AC * r.a.z, TILE_STAGE_B * r.a.w);
            rb = make_float4(EXACT ? r.b.x : TILE_STAGE_AC * r.b.x, r.b.y, 0.f, 0.f);
#pragma unroll
            for (int g = 0; g < NC4; g++) f[g] = a.feat[(size_t)id * a.fstride4 + g];
        }
        wave_lds_sync();
        s_a[lane] = ra;
        s_b[lane] = rb;
        s_q[lane] = qm;
        s_e[lane] = ei;
#pragma unroll
        for (int g = 0; g < NC4; g++) s_f[g][lane] = f[g];
        wave_lds_sync();
        uint64_t todo = __ballot((qm & live) != 0);
        if (scnt != SURV_NONE) {
            const uint32_t n = (uint32_t)__popcll(todo);
            if (scnt + n > SURV_CAP) {
                scnt = SURV_NONE;
            } else {
                if ((qm & live) != 0) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(todo >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)todo, 0u));
                    sl[scnt + r] = make_uint2(id, (j << 4) | qm);
                }
                scnt += n;
            }
        }
        int klast = -1;  // batch slot of the latest survivor that blended anywhere
        while (todo && live) {
            const int k = sgpr_ff1(todo);
            todo = sgpr_clear_bit(todo, k);
            const float4 A = s_a[k], B = s_b[k];
            float4 F[NC4];
#pragma unroll
            for (int g = 0; g < NC4; g++) F[g] = s_f[g][k];
            const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[k]) & live;
            nev += (uint32_t)__popc(m);
            const uint32_t pos1 = p0 + (uint32_t)k + 1u;
            lmask blended = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!((m >> q) & 1u)) continue;
                const float dx = A.x - pxq[q & 1], dy = A.y - pyq[q >> 1];
                float power, alpha;
                if (EXACT) {
#pragma clang fp contract(off)
                    power = ref_power(A.z, A.w, B.x, dx, dy);
                    alpha = fminf(0.99f, B.y * glibc_expf(power, s_gexp));
                } else {
                    power = gauss_power(A.z, A.w, B.x, dx, dy);
                    alpha = fminf(0.99f, B.y * tile_exp2(power));
                }
                // (compare results are 0 on inactive lanes, and the walk runs with every lane on:
                // no exec masking; each mask op below is one SALU instruction)
                const lmask hit = m_ge(alpha, lim[q]) & ~m_gt0(power);
                const float test_T = T[q] * (1 - alpha);
                const lmask lt = m_lt(test_T, 0.0001f);
                const lmask blend = hit & ~lt, sat = hit & lt;
                float Fs[4 * NC4];
#pragma unroll
                for (int g = 0; g < NC4; g++) {
                    Fs[4 * g + 0] = F[g].x;
                    Fs[4 * g + 1] = F[g].y;
                    Fs[4 * g + 2] = F[g].z;
                    Fs[4 * g + 3] = F[g].w;
                }
                if (EXACT) {  // forward.cu:359: C += feature * alpha * T, left to right
#pragma clang fp contract(off)
#pragma unroll
                    for (int c = 0; c < NCH; c++)
                        Cc[q][c] = sel(blend, Cc[q][c] + Fs[c] * alpha * T[q], Cc[q][c]);
                } else {
                    const float w = sel(blend, alpha * T[q], 0.f);
#pragma unroll
                    for (int c = 0; c < NCH; c++) Cc[q][c] += Fs[c] * w;
                }
                T[q] = sel(blend, test_T, T[q]);
                last[q] = sel(blend, pos1, last[q]);
                blended |= blend;
                if (sat) {  // rare: pixels finish
                    lim[q] = sel(sat, __builtin_inff(), lim[q]);
                    if (!(m_lt(lim[q], 1.f) & exec_mask())) live &= ~(1u << q);
                }
            }
            if (blended) klast = k;
        }
        if (klast >= 0) elast = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_e[klast]);
    }
    if (threadIdx.x == 0 && a.surv && qallow == 15u) a.surv_n[tile] = scnt;
    const int HW = a.H * a.W;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (((qallow >> q) & 1u) && wt.inside(q, a.W, a.H)) {
            const int pix = wt.pixel(q, a.W);
            if (a.final_T) {
                a.final_T[pix] = T[q];
                a.n_contrib[pix] = last[q];
            }
#pragma unroll
            for (int c = 0; c < NCH; c++)
                if (c < a.nch) {
                    if (EXACT) {
#pragma clang fp contract(off)
                        a.out[c * HW + pix] = Cc[q][c] + T[q] * a.bg[c];
                    } else {
                        a.out[c * HW + pix] = Cc[q][c] + T[q] * a.bg[c];
                    }
                }
        }
    }
    if (a.tile_nmax) {
        uint32_t nm = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t mq = ((qallow >> q) & 1u) ? wave_max_u32(last[q]) : 0u;
            nm = mq > nm ? mq : nm;
        }
        if (lane == 0 && nm) {
            atomicMax(&a.tile_nmax[tile], nm);
            atomicMax(&a.tile_emax[tile], elast + 1u);
            if (a.tile_cost) atomicAdd(&a.tile_cost[tile], nev);
            if (a.row_cost) atomicAdd(&a.row_cost[tile / a.grid_x], nev);
        }
    }
}

// The composite backward's LDS (declared once per kernel: the walks below share it).
template <int NC4>
struct McBwdLds {
    float4 a[64], b[64];
    float4 f[NC4][64];
    uint2 q[64];  // (list position << 4 | quadrant mask, Gaussian id)
    TileListLds list;
};

// The back-to-front walk of one tile over its NL = NCH channels.
template <int NC4, int NCH, bool DET, bool EXACT>
__device__ __forceinline__ void mc_bwd_walk(const RenderMcArgs& a, const unsigned tile, const WaveTile& wt,
                                            McBwdLds<NC4>& sm, float (&T)[4], const float (&Tb)[4],
                                            const float (&dpl)[4][NCH], const uint32_t (&last)[4],
                                            const uint32_t (&qlim)[4], const uint32_t nmax) {
    constexpr int NL = NCH;
    constexpr int V = 6 + NL;         // 6 geometric sums + the feature sums
    constexpr int NP = (V + 1) / 2;   // after the permlane32 stage
    constexpr int NQ = (NP + 1) / 2;  // after the permlane16 stage: registers reduced by DPP rows
    constexpr int NL4 = (NL + 3) / 4;
    const int lane = threadIdx.x;
    const float pxq[2] = {wt.pfx, wt.pfx + 8.f}, pyq[2] = {wt.pfy, wt.pfy + 8.f};
    float Sr[4];  // the recurrence as in gsr_render_bwd.hip
#pragma unroll
    for (int q = 0; q < 4; q++) Sr[q] = 0.f;
    const int row = lane >> 4, col = lane & 15;
    const int vrow = row == 0 ? 0 : row == 1 ? 2 : row == 2 ? 1 : 3;
    const int vreg = row_sums_t_reg<NQ>(col);  // the register whose row sums this lane ends with
    const int vidx = (vreg >= 0 && 4 * vreg + vrow < V) ? 4 * vreg + vrow : -1;
    const lmask mb3 = __ballot((col & 8) != 0), mb2 = __ballot((col & 4) != 0);
    // values 0-4 carry the opacity; the conic, -1/2 and the screen scale are applied per
    // Gaussian by the preprocess backward (acc_raw), as in gsr_render_bwd.hip
    const bool vop = vidx >= 0 && vidx <= 4;
    // the channel of this lane's feature sum
    const int fch = vidx - 6;
    const bool vfeat = vidx >= 6 && fch >= 0 && fch < a.nch;

    // back to front from the tile's last contributor (as gsr_render_bwd.hip)
    const unsigned sth = st_sth(a.grid_x, a.grid_y);
    const unsigned st = ((tile / a.grid_x) >> sth) * a.gsx + (tile % a.grid_x) / GSR_ST_W;
    // the forward's survivor list when it stored one, else the super-tile list (as gsr_render_bwd.hip)
    const uint32_t sn = a.surv ? a.surv_n[tile] : SURV_NONE;
    const bool lst = sn != SURV_NONE;
    uint32_t li = lst ? sn : 0u;
    const uint2* const sl = a.surv + (size_t)tile * SURV_CAP;
    uint2 nv = lst ? sl[max((int)li - 1 - lane, 0)] : make_uint2(0u, 0u);
    TileList<false> tl;
    if (!lst)
        tl.init(a.ent, a.st_ranges[st], tile, a.grid_x, sth, nmax ? a.tile_emax[tile] : 0u, nmax ? a.tile_nmax[tile] : 0u);
    const uint32_t rbase = DET ? a.ranges[tile].x : 0u;
    __shared__ unsigned long long s_gexp[EXACT ? 32 : 1];  // exact mode: glibc_expf's table
    if (EXACT) gexp_table_init(s_gexp);
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
            tl.fill(sm.list);
            uint32_t ei = 0, p0 = 0;
            nb = tl.take(sm.list, id, ei, p0);
            if (nb == 0) break;
            p = p0 - (uint32_t)lane;
        }
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
        float4 f[NC4];
#pragma unroll
        for (int g = 0; g < NC4; g++) f[g] = ra;
        if ((uint32_t)lane < nb) {
            const Rec r = a.rec[id];
            if (!lst) qm = wt.reach(r, p, qlim);
            ra = EXACT ? r.a : make_float4(r.a.x, r.a.y, TILE_STAGE_AC * r.a.z, TILE_STAGE_B * r.a.w);
            rb = make_float4(EXACT ? r.b.x : TILE_STAGE_AC * r.b.x, r.b.y, 0.f, 0.f);
#pragma unroll
            for (int g = 0; g < NC4; g++) f[g] = a.feat[(size_t)id * a.fstride4 + g];
        }
        wave_lds_sync();
        sm.a[lane] = ra;
        sm.b[lane] = rb;
        sm.q[lane] = make_uint2((p << 4) | qm, id);
#pragma unroll
        for (int g = 0; g < NC4; g++) sm.f[g][lane] = f[g];
        wave_lds_sync();
        uint64_t todo = __ballot(qm != 0);
        while (todo) {
            const int k = sgpr_ff1(todo);
            todo = sgpr_clear_bit(todo, k);
            const float4 A = sm.a[k], B = sm.b[k];
            const uint2 Q2 = sm.q[k];
            float F[4 * NL4];
#pragma unroll
            for (int g = 0; g < NL4; g++) {
                const float4 v = sm.f[g][k];
                F[4 * g] = v.x;
                F[4 * g + 1] = v.y;
                F[4 * g + 2] = v.z;
                F[4 * g + 3] = v.w;
            }
            const uint32_t mp = (uint32_t)__builtin_amdgcn_readfirstlane((int)Q2.x);
            const uint32_t m = mp & 15u;
            const float ax = A.x, ay = A.y, ka = A.z, kb = A.w, kc = B.x, op = B.y;
            const uint32_t pos = mp >> 4;  // list position
            float M1 = 0.f, M2 = 0.f, S2 = 0.f, S3 = 0.f, S4 = 0.f, S5 = 0.f;
            float SF[NL];
#pragma unroll
            for (int c = 0; c < NL; c++) SF[c] = 0.f;
            bool any = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (!((m >> q) & 1u)) continue;
                const float dx = ax - pxq[q & 1], dy = ay - pyq[q >> 1];
                float power, G, alpha;
                if (EXACT) {
#pragma clang fp contract(off)
                    power = ref_power(ka, kb, kc, dx, dy);
                    G = glibc_expf(power, s_gexp);
                    alpha = fminf(0.99f, op * G);
                } else {
                    power = gauss_power(ka, kb, kc, dx, dy);
                    G = tile_exp2(power);
                    alpha = fminf(0.99f, op * G);
                }
                // (compare results are 0 on inactive lanes, and every lane is on: no exec masking)
                const lmask act = (m_ult(pos, last[q]) & ~m_gt0(power)) & ~m_lt(alpha, 1.0f / 255.0f);
                if (act == 0ull) continue;
                any = true;
                const float ae = sel(act, alpha, 0.f);
                const float Ge = sel(act, G, 0.f);
                const float inv = __builtin_amdgcn_rcpf(1.f - ae);
                const float Tn = T[q] * inv;
                const float dch = ae * Tn;
                float cdp = F[0] * dpl[q][0];
#pragma unroll
                for (int c = 1; c < NL; c++) cdp = __builtin_fmaf(F[c], dpl[q][c], cdp);
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
#pragma unroll
                for (int c = 0; c < NL; c++) SF[c] = __builtin_fmaf(dch, dpl[q][c], SF[c]);
                T[q] = Tn;
            }
            if (any) {
                float S[2 * NP];
                S[0] = M1;  // raw: the preprocess backward applies the conic (acc_raw)
                S[1] = M2;
                S[2] = S2;
                S[3] = S3;
                S[4] = S4;
                S[5] = S5;
#pragma unroll
                for (int c = 0; c < V - 6; c++) S[6 + c] = SF[c];
#pragma unroll
                for (int c = V; c < 2 * NP; c++) S[c] = 0.f;
                float Pp[2 * NQ];
#pragma unroll
                for (int t = 0; t < NP; t++) Pp[t] = swap32_sum(S[2 * t], S[2 * t + 1]);
#pragma unroll
                for (int t = NP; t < 2 * NQ; t++) Pp[t] = 0.f;
                float Qr[NQ];
#pragma unroll
                for (int t = 0; t < NQ; t++) Qr[t] = swap16_sum(Pp[2 * t], Pp[2 * t + 1]);
                float v = row_sums_t<NQ>(Qr, mb3, mb2, col);
                v = vop ? v * op : v;
                if (DET) {  // the groups run one after another: plain read-modify-write
                    float* prow = a.partial + (size_t)(rbase + pos) * a.pstride;
                    if (vidx >= 0 && vidx < 6) prow[vidx] += v;
                    else if (vfeat) prow[a.pc0 + 6 + fch] = v;
                } else if (v != 0.f) {
                    const uint32_t gid = Q2.y;
                    if (vidx >= 0 && vidx < 6) atomicAdd(a.acc + (size_t)gid * ACC_STRIDE + vidx, v);
                    else if (vfeat) atomicAdd(a.dL_dfeat + (size_t)gid * a.fstride + fch, v);
                }
            }
        }
    }
}

// The tile's state (T, the background term, dL/dout, the last contributors), then the walk.
// (Round 5 also measured a split into two launches, one walking the tiles with at most 10 live
// channels over those only: k_render_bwd_mc 0.60 -> 0.79 ms per view at cfg4,
// profiles/r5x_mc_live_ab.txt.)
template <int NC4, int NCH, bool DET, bool EXACT>
__device__ __forceinline__ void render_bwd_mc_tile(const RenderMcArgs& a, const unsigned tile, const uint32_t qallow) {
    WaveTile wt;
    wt.init(tile, a.grid_x, a.W, a.H);
    const int HW = a.H * a.W;
    __shared__ McBwdLds<NC4> sm;
    float T[4], Tb[4], dp[4][NCH];
    uint32_t last[4], qlim[4];
    uint32_t nmax = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const bool in = wt.inside(q, a.W, a.H);
        const int pix = in ? wt.pixel(q, a.W) : 0;
        const float Tf = in ? a.final_T[pix] : 0.f;
        last[q] = in ? a.n_contrib[pix] : 0u;
        float bd = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            dp[q][c] = (in && c < a.nch) ? a.dL_dout[c * HW + pix] : 0.f;
            bd = c < a.nch ? __builtin_fmaf(a.bg[c], dp[q][c], bd) : bd;
        }
        T[q] = Tf;
        Tb[q] = -Tf * bd;
        qlim[q] = ((qallow >> q) & 1u) ? wave_max_u32(last[q]) : 0u;
        nmax = qlim[q] > nmax ? qlim[q] : nmax;
    }
    mc_bwd_walk<NC4, NCH, DET, EXACT>(a, tile, wt, sm, T, Tb, dp, last, qlim, nmax);
}

template <int NC4, int NCH = 4 * NC4, bool EXACT = false>
__global__ void __launch_bounds__(64) k_render_fwd_mc(RenderMcArgs a) {
    unsigned tile;
    uint32_t qallow;
    zero_slice(a.zero, a.zero_n4);
    if (!tile_unit_fwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow)) return;
    render_fwd_mc_tile<NC4, NCH, EXACT>(a, tile, qallow);
}

#ifdef GSR_RENDER_STATS
// timing build (make times): per unit of each composite-backward launch, (start, end)
// s_memrealtime, (tile | qallow << 20 | launch << 28), the unit's largest n_contrib
// (tools/mc_bwd_times.py); launch 0 = the only or the few-channel launch, 1 = the other
constexpr int MCB_UNITS = 1 << 17;
__device__ unsigned long long g_mcb_times[2][4 * MCB_UNITS];
extern "C" int gsr_debug_mcb_times(unsigned long long* out, int n, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mcb_times), sizeof(unsigned long long) * 2 * 4 * (size_t)n) != hipSuccess)
        return -1;
    if (reset) {  // the next launches' units then leave no stale records (their block -> unit map varies)
        static unsigned long long zeros[2 * 4 * MCB_UNITS];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_mcb_times), zeros, sizeof(zeros)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

template <int NC4, int NCH = 4 * NC4, bool DET = false, bool EXACT = false>
__global__ void __launch_bounds__(64) k_render_bwd_mc(RenderMcArgs a) {
    unsigned tile;
    uint32_t qallow;
    if (!tile_unit_bwd(a.grid_x * a.grid_y, a.order, a.nheavy, tile, qallow, DET)) return;
#ifdef GSR_RENDER_STATS
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
    render_bwd_mc_tile<NC4, NCH, DET, EXACT>(a, tile, qallow);
#ifdef GSR_RENDER_STATS
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)MCB_UNITS) {
        unsigned long long* r = g_mcb_times[0] + 4 * (size_t)blockIdx.x;
        r[0] = t0;
        r[1] = __builtin_amdgcn_s_memrealtime();
        r[2] = tile | ((unsigned long long)qallow << 20);
        r[3] = a.tile_nmax[tile];
    }
#endif
}

template <bool EXACT>
static void launch_fwd_mc(const RenderMcArgs& a, const dim3 grid, hipStream_t s) {
    switch ((a.nch + 3) / 4) {
        case 1: hipLaunchKernelGGL((k_render_fwd_mc<1, 4, EXACT>), grid, dim3(64), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_render_fwd_mc<2, 8, EXACT>), grid, dim3(64), 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_render_fwd_mc<3, 12, EXACT>), grid, dim3(64), 0, s, a); break;
        default:
            if (a.nch == 14) hipLaunchKernelGGL((k_render_fwd_mc<4, 14, EXACT>), grid, dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_render_fwd_mc<4, 16, EXACT>), grid, dim3(64), 0, s, a);
            break;
    }
}

void launch_render_fwd_mc(const RenderMcArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0 || a.nch <= 0) return;
    const dim3 grid(tile_pass_blocks(ntile, FWD_TAIL_SPLIT));
    if (a.exact) launch_fwd_mc<true>(a, grid, s);
    else launch_fwd_mc<false>(a, grid, s);
}

template <bool DET, bool EXACT>
static void launch_bwd_mc(const RenderMcArgs& a, const dim3 grid, hipStream_t s) {
    switch ((a.nch + 3) / 4) {
        case 1: hipLaunchKernelGGL((k_render_bwd_mc<1, 4, DET, EXACT>), grid, dim3(64), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_render_bwd_mc<2, 8, DET, EXACT>), grid, dim3(64), 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_render_bwd_mc<3, 12, DET, EXACT>), grid, dim3(64), 0, s, a); break;
        default:
            if (a.nch == 14) hipLaunchKernelGGL((k_render_bwd_mc<4, 14, DET, EXACT>), grid, dim3(64), 0, s, a);
            else hipLaunchKernelGGL((k_render_bwd_mc<4, 16, DET, EXACT>), grid, dim3(64), 0, s, a);
            break;
    }
}

void launch_render_bwd_mc(const RenderMcArgs& a, hipStream_t s) {
    const unsigned ntile = a.grid_x * a.grid_y;
    if (ntile == 0 || a.nch <= 0) return;
    const dim3 grid(tile_pass_blocks_bal(ntile, 0u));
    if (a.exact) {
        if (a.partial) launch_bwd_mc<true, true>(a, grid, s);
        else launch_bwd_mc<false, true>(a, grid, s);
    } else {
        if (a.partial) launch_bwd_mc<true, false>(a, grid, s);
        else launch_bwd_mc<false, false>(a, grid, s);
    }
}

}  // namespace gsr
