/*
 * oracle/gsr_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (relightable3dgaussians-w_amd/) never links,
 * imports or calls it.
 *
 * What it is: a plain-C, single-threaded restatement of the reference's
 * differentiable Gaussian rasterizer
 *   /root/reference/submodules/diff-gaussian-rasterization/cuda_rasterizer/
 * and of the per-Gaussian relighting shade
 *   /root/reference/scene/NVDIFFREC/light.py, utils/sh_utils.py.
 * Every function cites the reference file:line it follows.  Floating point is
 * evaluated in the reference's source order with no FMA contraction
 * (-ffp-contract=off), glm's column-major matrix semantics restated exactly,
 * ndc2Pix in double, so the preprocess / binning outputs are the bit-exact
 * contract the HIP kernels are checked against.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - rasterizer: PARTIALLY PINNED.  The reference CUDA cannot be built or run
 *     here (no nvcc; hipify would be a port).  Pinned pieces: cov3D against the
 *     reference's own Python build_covariance_from_scaling_rotation, SH->RGB
 *     against the reference's eval_sh (same polynomial/constants as
 *     auxiliary.h:22-39), depth against GaussianModel.get_depth, cameras against
 *     getWorld2View2/getProjectionMatrix (fixtures in tests/golden/).  The
 *     backward formulas are additionally checked by float64 finite differences.
 *     EWA projection/compositing/sort order have no reference-side fixture:
 *     "parity unpinned" for those beyond this restatement.
 *   - shade: PINNED by golden vectors generated from the imported reference
 *     EnvironmentLight.shade (forward + autograd backward), EXCEPT the FG-LUT
 *     bilinear lookup (3rd-party nvdiffrast, not vendored): parity unpinned.
 *
 * Build: oracle/Makefile -> oracle/_build/liboracle.so (REAL=float) and
 *        oracle/_build/liboracle64.so (REAL=double, finite-difference checks).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef ORC_F64
typedef double REAL;
#define F(x) x
#define SQRT sqrt
#define EXP exp
#define CEIL ceil
#define FMIN fmin
#define FMAX fmax
#define FLOOR floor
#define POW pow
#else
typedef float REAL;
#define F(x) x##f
#define SQRT sqrtf
#define EXP expf
#define CEIL ceilf
#define FMIN fminf
#define FMAX fmaxf
#define FLOOR floorf
#define POW powf
#endif

/* ---- the Gaussian's exponent at a pixel: forward.cu:335,343 and backward.cu:494-498 --------
 * power = -0.5 (a dx^2 + c dy^2) - b dx dy,  G = exp(power).
 * Error-budget variants (oracle/Makefile; tools/error_budget.py) -- the canonical
 * build defines none of them:
 *   ORC_GPU_EXPONENT  the HIP tile passes' arithmetic (gsr_tile.hpp gauss_power / tile_exp2):
 *                     conic pre-scaled by log2(e), two fused multiply-adds, exp2.  It proves
 *                     (or refutes) that the GPU's per-pair decisions differ from this oracle's
 *                     only through this arithmetic.
 *   ORC_EXP_ULP=k     expf's result moved by a deterministic pseudo-random whole number of
 *                     ulps in [-k, k] (CUDA's expf is specified to 2 ulp, glibc's to < 1):
 *                     how far the reference's own libm choice moves its outputs.
 * (A third variant, liboracle_fma.so, is this source built with FMA contraction on, as nvcc
 * builds the reference by default: -fmad=true.) */
#if defined(ORC_GPU_EXPONENT) && !defined(ORC_F64)
static inline REAL orc_gauss(const REAL* co, REAL dx, REAL dy, REAL* power) {
    const float h = -0.5f * 1.44269504088896340736f, n = -1.44269504088896340736f;
    const float na = h * co[0], nb = n * co[1], nc = h * co[2];
    *power = fmaf(na * dx, dx, fmaf(nc * dy, dy, (nb * dx) * dy));  /* log2 units: same sign */
    return exp2f(*power);
}
#else
static inline REAL orc_gauss(const REAL* co, REAL dx, REAL dy, REAL* power) {
    *power = F(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
    REAL G = EXP(*power);
#if defined(ORC_EXP_ULP) && !defined(ORC_F64)
    {
        uint32_t u, k;
        memcpy(&u, power, 4);
        k = u * 2654435761u;
        k ^= k >> 15;
        k *= 2246822519u;
        k ^= k >> 13;
        int off = (int)(k % (2u * ORC_EXP_ULP + 1u)) - ORC_EXP_ULP;
        uint32_t g;
        memcpy(&g, &G, 4);
        if (G >= 1.17549435e-38f) g = (uint32_t)((int32_t)g + off); /* normal numbers only */
        memcpy(&G, &g, 4);
    }
#endif
    return G;
}
#endif

#define BLOCK_X 16
#define BLOCK_Y 16

/* auxiliary.h:22-39 */
static const REAL SH_C0 = F(0.28209479177387814);
static const REAL SH_C1 = F(0.4886025119029199);
static const REAL SH_C2[5] = {F(1.0925484305920792), F(-1.0925484305920792), F(0.31539156525252005),
                              F(-1.0925484305920792), F(0.5462742152960396)};
static const REAL SH_C3[7] = {F(-0.5900435899266435), F(2.890611442640554), F(-0.4570457994644658),
                              F(0.3731763325901154), F(-0.4570457994644658), F(1.445305721320277),
                              F(-0.5900435899266435)};

/* float -> int as the GPU converts (saturating, NaN -> 0); the reference relies on
 * the implicit conversions at forward.cu:235 (getRect's int max_radius) and :251. */
static int f2i(REAL v) {
    if (v != v) return 0;
    if (v >= (REAL)2147483647.0) return 2147483647;
    if (v <= (REAL)-2147483648.0) return (-2147483647 - 1);
    return (int)v;
}

/* ---- glm::mat3 restated: m[c][r] (column c, row r) -------------------------------- */
typedef struct { REAL m[3][3]; } mat3;

/* glm type_mat3x3.inl operator*(mat3, mat3): R[c][r] = A[0][r]B[c][0] + A[1][r]B[c][1] + A[2][r]B[c][2] */
static mat3 mmul(mat3 A, mat3 B) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return R;
}
static mat3 mtrans(mat3 A) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) R.m[c][r] = A.m[r][c];
    return R;
}
/* glm::mat3(x0,y0,z0, x1,y1,z1, x2,y2,z2): columns given in order */
static mat3 mcols(REAL a0, REAL a1, REAL a2, REAL b0, REAL b1, REAL b2, REAL c0, REAL c1, REAL c2) {
    mat3 R;
    R.m[0][0] = a0; R.m[0][1] = a1; R.m[0][2] = a2;
    R.m[1][0] = b0; R.m[1][1] = b1; R.m[1][2] = b2;
    R.m[2][0] = c0; R.m[2][1] = c1; R.m[2][2] = c2;
    return R;
}

/* auxiliary.h:58-66 */
static void transformPoint4x3(const REAL* p, const REAL* m, REAL* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
/* auxiliary.h:68-77 */
static void transformPoint4x4(const REAL* p, const REAL* m, REAL* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
/* auxiliary.h:41-44: evaluated in double, rounded to float on return */
static REAL ndc2Pix(REAL v, int S) { return (REAL)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

/* auxiliary.h:46-56 (note: p + r + 16 - 1 is evaluated left to right in float) */
static void getRect(const REAL* p, int max_radius, unsigned gx, unsigned gy, unsigned* rmin, unsigned* rmax) {
    int a, b;
    a = f2i((p[0] - (REAL)max_radius) / (REAL)BLOCK_X); a = a > 0 ? a : 0; rmin[0] = (unsigned)a < gx ? (unsigned)a : gx;
    a = f2i((p[1] - (REAL)max_radius) / (REAL)BLOCK_Y); a = a > 0 ? a : 0; rmin[1] = (unsigned)a < gy ? (unsigned)a : gy;
    b = f2i((p[0] + (REAL)max_radius + (REAL)BLOCK_X - (REAL)1) / (REAL)BLOCK_X); b = b > 0 ? b : 0;
    rmax[0] = (unsigned)b < gx ? (unsigned)b : gx;
    b = f2i((p[1] + (REAL)max_radius + (REAL)BLOCK_Y - (REAL)1) / (REAL)BLOCK_Y); b = b > 0 ? b : 0;
    rmax[1] = (unsigned)b < gy ? (unsigned)b : gy;
}

/* forward.cu:118-152 (quaternion used as given, not normalised: :127) */
static void computeCov3D(const REAL* scale, REAL mod, const REAL* rot, REAL* cov3D) {
    mat3 S = mcols(F(1.0), 0, 0, 0, F(1.0), 0, 0, 0, F(1.0));
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    REAL r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = mcols(F(1.0) - F(2.0) * (y * y + z * z), F(2.0) * (x * y - r * z), F(2.0) * (x * z + r * y),
                   F(2.0) * (x * y + r * z), F(1.0) - F(2.0) * (x * x + z * z), F(2.0) * (y * z - r * x),
                   F(2.0) * (x * z - r * y), F(2.0) * (y * z + r * x), F(1.0) - F(2.0) * (x * x + y * y));
    mat3 M = mmul(S, R);
    mat3 Sigma = mmul(mtrans(M), M);
    cov3D[0] = Sigma.m[0][0]; cov3D[1] = Sigma.m[0][1]; cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1]; cov3D[4] = Sigma.m[1][2]; cov3D[5] = Sigma.m[2][2];
}

/* forward.cu:74-113 */
static void computeCov2D(const REAL* mean, REAL focal_x, REAL focal_y, REAL tan_fovx, REAL tan_fovy,
                         const REAL* cov3D, const REAL* viewmatrix, REAL* out) {
    REAL t[3];
    transformPoint4x3(mean, viewmatrix, t);
    const REAL limx = F(1.3) * tan_fovx;
    const REAL limy = F(1.3) * tan_fovy;
    const REAL txtz = t[0] / t[2];
    const REAL tytz = t[1] / t[2];
    t[0] = FMIN(limx, FMAX(-limx, txtz)) * t[2];
    t[1] = FMIN(limy, FMAX(-limy, tytz)) * t[2];
    mat3 J = mcols(focal_x / t[2], F(0.0), -(focal_x * t[0]) / (t[2] * t[2]),
                   F(0.0), focal_y / t[2], -(focal_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
    const REAL* v = viewmatrix;
    mat3 W = mcols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 T = mmul(W, J);
    mat3 Vrk = mcols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 cov = mmul(mmul(mtrans(T), mtrans(Vrk)), T);
    cov.m[0][0] += F(0.3);
    cov.m[1][1] += F(0.3);
    out[0] = cov.m[0][0]; out[1] = cov.m[0][1]; out[2] = cov.m[1][1];
}

/* forward.cu:20-71 (glm vec3 ops restated per component, same association) */
static void computeColorFromSH(int idx, int deg, int max_coeffs, const REAL* means, const REAL* campos,
                               const REAL* shs, uint8_t* clamped, REAL* out) {
    const REAL* pos = means + 3 * idx;
    REAL dir[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    REAL len = SQRT(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    const REAL* sh = shs + (size_t)idx * max_coeffs * 3;
#define SHC(k, c) sh[3 * (k) + (c)]
    REAL res[3];
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * SHC(0, c);
    if (deg > 0) {
        REAL x = dir[0], y = dir[1], z = dir[2];
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - SH_C1 * y * SHC(1, c) + SH_C1 * z * SHC(2, c) - SH_C1 * x * SHC(3, c);
        if (deg > 1) {
            REAL xx = x * x, yy = y * y, zz = z * z;
            REAL xy = x * y, yz = y * z, xz = x * z;
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + SH_C2[0] * xy * SHC(4, c) + SH_C2[1] * yz * SHC(5, c) +
                         SH_C2[2] * (F(2.0) * zz - xx - yy) * SHC(6, c) + SH_C2[3] * xz * SHC(7, c) +
                         SH_C2[4] * (xx - yy) * SHC(8, c);
            if (deg > 2) {
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + SH_C3[0] * y * (F(3.0) * xx - yy) * SHC(9, c) +
                             SH_C3[1] * xy * z * SHC(10, c) +
                             SH_C3[2] * y * (F(4.0) * zz - xx - yy) * SHC(11, c) +
                             SH_C3[3] * z * (F(2.0) * zz - F(3.0) * xx - F(3.0) * yy) * SHC(12, c) +
                             SH_C3[4] * x * (F(4.0) * zz - xx - yy) * SHC(13, c) +
                             SH_C3[5] * z * (xx - yy) * SHC(14, c) +
                             SH_C3[6] * x * (xx - F(3.0) * yy) * SHC(15, c);
            }
        }
    }
#undef SHC
    for (int c = 0; c < 3; c++) {
        res[c] += F(0.5);
        clamped[3 * idx + c] = (res[c] < 0);
        out[c] = res[c] < 0 ? F(0.0) : res[c];
    }
}

/* forward.cu:155-256 preprocessCUDA + auxiliary.h:139-164 in_frustum.
 * Returns 0, or -1 if a point was culled although prefiltered is set (the
 * reference's device printf + __trap(), auxiliary.h:156-160). */
int orc_preprocess(int P, int D, int M, const REAL* orig_points, const REAL* scales, REAL scale_modifier,
                   const REAL* rotations, const REAL* opacities, const REAL* shs, const REAL* cov3D_precomp,
                   const REAL* colors_precomp, const REAL* viewmatrix, const REAL* projmatrix,
                   const REAL* cam_pos, int W, int H, REAL tan_fovx, REAL tan_fovy, int prefiltered,
                   int32_t* radii, REAL* points_xy, REAL* depths, REAL* cov3Ds, REAL* rgb,
                   REAL* conic_opacity, uint8_t* clamped, uint32_t* tiles_touched) {
    /* rasterizer_impl.cu:221-222 */
    const REAL focal_y = (REAL)H / (F(2.0) * tan_fovy);
    const REAL focal_x = (REAL)W / (F(2.0) * tan_fovx);
    const unsigned gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    int err = 0;
    for (int idx = 0; idx < P; idx++) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        const REAL* p_orig = orig_points + 3 * idx;
        REAL p_view[3];
        transformPoint4x3(p_orig, viewmatrix, p_view);
        if (p_view[2] <= F(0.2)) {
            if (prefiltered) err = -1;
            continue;
        }
        REAL p_hom[4];
        transformPoint4x4(p_orig, projmatrix, p_hom);
        REAL p_w = F(1.0) / (p_hom[3] + F(0.0000001));
        REAL p_proj[3] = {p_hom[0] * p_w, p_hom[1] * p_w, p_hom[2] * p_w};
        const REAL* cov3D;
        if (cov3D_precomp) {
            cov3D = cov3D_precomp + 6 * idx;
        } else {
            computeCov3D(scales + 3 * idx, scale_modifier, rotations + 4 * idx, cov3Ds + 6 * idx);
            cov3D = cov3Ds + 6 * idx;
        }
        REAL cov[3];
        computeCov2D(p_orig, focal_x, focal_y, tan_fovx, tan_fovy, cov3D, viewmatrix, cov);
        REAL det = (cov[0] * cov[2] - cov[1] * cov[1]);
        if (det == F(0.0)) continue;
        REAL det_inv = F(1.0) / det;
        REAL conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        REAL mid = F(0.5) * (cov[0] + cov[2]);
        REAL lambda1 = mid + SQRT(FMAX(F(0.1), mid * mid - det));
        REAL lambda2 = mid - SQRT(FMAX(F(0.1), mid * mid - det));
        REAL my_radius = CEIL(F(3.0) * SQRT(FMAX(lambda1, lambda2)));
        REAL point_image[2] = {ndc2Pix(p_proj[0], W), ndc2Pix(p_proj[1], H)};
        unsigned rmin[2], rmax[2];
        getRect(point_image, f2i(my_radius), gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (colors_precomp == NULL) computeColorFromSH(idx, D, M, orig_points, cam_pos, shs, clamped, rgb + 3 * idx);
        depths[idx] = p_view[2];
        radii[idx] = f2i(my_radius);
        points_xy[2 * idx + 0] = point_image[0];
        points_xy[2 * idx + 1] = point_image[1];
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = opacities[idx];
        tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
    }
    return err;
}

/* rasterizer_impl.cu:54-66 checkFrustum (present = p_view.z > 0.2) */
void orc_mark_visible(int P, const REAL* means3D, const REAL* viewmatrix, uint8_t* present) {
    for (int i = 0; i < P; i++) {
        REAL pv[3];
        transformPoint4x3(means3D + 3 * i, viewmatrix, pv);
        present[i] = !(pv[2] <= F(0.2));
    }
}

/* rasterizer_impl.cu:35-50 */
uint32_t orc_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

/* Stable LSD radix sort of (u64 key, u32 value) pairs on bits [0, end_bit): the CUB
 * DeviceRadixSort::SortPairs contract used at rasterizer_impl.cu:303-308. */
static void radix_sort_pairs(uint64_t* keys, uint32_t* vals, int64_t n, int end_bit) {
    if (n <= 1) return;
    uint64_t* k2 = (uint64_t*)malloc(sizeof(uint64_t) * n);
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * n);
    int64_t cnt[256];
    for (int shift = 0; shift < end_bit; shift += 8) {
        memset(cnt, 0, sizeof(cnt));
        uint64_t mask = (end_bit - shift >= 8) ? 0xFFull : ((1ull << (end_bit - shift)) - 1);
        for (int64_t i = 0; i < n; i++) cnt[(keys[i] >> shift) & mask]++;
        int64_t s = 0;
        for (int d = 0; d < 256; d++) { int64_t c = cnt[d]; cnt[d] = s; s += c; }
        for (int64_t i = 0; i < n; i++) {
            int64_t o = cnt[(keys[i] >> shift) & mask]++;
            k2[o] = keys[i]; v2[o] = vals[i];
        }
        memcpy(keys, k2, sizeof(uint64_t) * n);
        memcpy(vals, v2, sizeof(uint32_t) * n);
    }
    free(k2); free(v2);
}

/* rasterizer_impl.cu:274-318: inclusive scan of tiles_touched, duplicateWithKeys
 * (:70-111), SortPairs on [0, 32+getHigherMsb(tiles)), memset + identifyTileRanges
 * (:116-138).  keys/vals/ranges must hold R / R / 2*T entries.  Returns R. */
int64_t orc_num_rendered(int P, const uint32_t* tiles_touched) {
    uint32_t acc = 0; /* the reference scans in uint32 */
    for (int i = 0; i < P; i++) acc += tiles_touched[i];
    return (int64_t)acc;
}

int64_t orc_binning(int P, int W, int H, const REAL* points_xy, const REAL* depths, const int32_t* radii,
                    const uint32_t* tiles_touched, uint64_t* keys, uint32_t* vals, uint32_t* ranges) {
    const unsigned gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    uint32_t off = 0;
    for (int idx = 0; idx < P; idx++) {
        uint32_t o = off;
        off += tiles_touched[idx];
        if (radii[idx] > 0) {
            unsigned rmin[2], rmax[2];
            getRect(points_xy + 2 * idx, radii[idx], gx, gy, rmin, rmax);
            for (unsigned y = rmin[1]; y < rmax[1]; y++)
                for (unsigned x = rmin[0]; x < rmax[0]; x++) {
                    uint64_t key = (uint64_t)(y * gx + x);
                    key <<= 32;
                    uint32_t dbits;
                    float df = (float)depths[idx];
                    memcpy(&dbits, &df, 4);
                    key |= dbits;
                    keys[o] = key;
                    vals[o] = (uint32_t)idx;
                    o++;
                }
        }
    }
    int64_t R = off;
    int bit = (int)orc_higher_msb(gx * gy);
    radix_sort_pairs(keys, vals, R, 32 + bit);
    memset(ranges, 0, sizeof(uint32_t) * 2 * gx * gy);
    for (int64_t i = 0; i < R; i++) {
        uint32_t cur = (uint32_t)(keys[i] >> 32);
        if (i == 0) ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(keys[i - 1] >> 32);
            if (cur != prev) { ranges[2 * prev + 1] = (uint32_t)i; ranges[2 * cur] = (uint32_t)i; }
        }
        if (i == R - 1) ranges[2 * cur + 1] = (uint32_t)R;
    }
    return R;
}

/* forward.cu:261-374 renderCUDA<3>.  tile_list == NULL renders every tile; otherwise
 * only the listed tiles (pixels of other tiles are left untouched). */
void orc_render_fwd(int W, int H, const uint32_t* ranges, const uint32_t* point_list, const REAL* points_xy,
                    const REAL* features, const REAL* conic_opacity, const REAL* bg, REAL* out_color,
                    REAL* final_T, uint32_t* n_contrib, const int32_t* tile_list, int n_tiles) {
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    int nt = tile_list ? n_tiles : gx * gy;
    for (int ti = 0; ti < nt; ti++) {
        int tile = tile_list ? tile_list[ti] : ti;
        int bx = tile % gx, by = tile / gx;
        uint32_t rx = ranges[2 * tile], ry = ranges[2 * tile + 1];
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                int px = bx * BLOCK_X + tx, py = by * BLOCK_Y + ty;
                if (!(px < W && py < H)) continue;
                REAL pixf[2] = {(REAL)px, (REAL)py};
                REAL T = F(1.0);
                uint32_t contributor = 0, last_contributor = 0;
                REAL C[3] = {0, 0, 0};
                for (uint32_t j = rx; j < ry; j++) {
                    contributor++;
                    uint32_t g = point_list[j];
                    REAL d[2] = {points_xy[2 * g] - pixf[0], points_xy[2 * g + 1] - pixf[1]};
                    const REAL* co = conic_opacity + 4 * g;
                    REAL power;
                    const REAL G = orc_gauss(co, d[0], d[1], &power);
                    if (power > F(0.0)) continue;
                    REAL alpha = FMIN(F(0.99), co[3] * G);
                    if (alpha < F(1.0) / F(255.0)) continue;
                    REAL test_T = T * (1 - alpha);
                    if (test_T < F(0.0001)) break;
                    for (int ch = 0; ch < 3; ch++) C[ch] += features[3 * g + ch] * alpha * T;
                    T = test_T;
                    last_contributor = contributor;
                }
                int pix = W * py + px;
                final_T[pix] = T;
                n_contrib[pix] = last_contributor;
                for (int ch = 0; ch < 3; ch++) out_color[ch * H * W + pix] = C[ch] + T * bg[ch];
            }
    }
}

/* backward.cu:399-557 renderCUDA<3> (backward).  The reference's float atomicAdds are
 * accumulated here in double (a tighter estimate of the exact sum), then rounded once.
 * dL_dconic is the reference's [P,2,2] buffer (components 0,1,3 written). */
void orc_render_bwd(int P, int W, int H, const uint32_t* ranges, const uint32_t* point_list, const REAL* bg,
                    const REAL* points_xy, const REAL* conic_opacity, const REAL* colors, const REAL* final_Ts,
                    const uint32_t* n_contrib, const REAL* dL_dpixels, REAL* dL_dmean2D, REAL* dL_dconic,
                    REAL* dL_dopacity, REAL* dL_dcolors, const int32_t* tile_list, int n_tiles) {
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    double* acc = (double*)calloc((size_t)P * 9, sizeof(double)); /* m2x m2y cx cy cw op r g b */
    const REAL ddelx_dx = (REAL)(0.5 * W);
    const REAL ddely_dy = (REAL)(0.5 * H);
    int nt = tile_list ? n_tiles : gx * gy;
    for (int ti = 0; ti < nt; ti++) {
        int tile = tile_list ? tile_list[ti] : ti;
        int bx = tile % gx, by = tile / gx;
        uint32_t rx = ranges[2 * tile], ry = ranges[2 * tile + 1];
        for (int ty = 0; ty < BLOCK_Y; ty++)
            for (int tx = 0; tx < BLOCK_X; tx++) {
                int px = bx * BLOCK_X + tx, py = by * BLOCK_Y + ty;
                if (!(px < W && py < H)) continue;
                int pix = W * py + px;
                REAL pixf[2] = {(REAL)px, (REAL)py};
                const REAL T_final = final_Ts[pix];
                REAL T = T_final;
                uint32_t contributor = ry - rx;
                const uint32_t last_contributor = n_contrib[pix];
                REAL accum_rec[3] = {0, 0, 0}, dL_dpixel[3], last_color[3] = {0, 0, 0};
                for (int c = 0; c < 3; c++) dL_dpixel[c] = dL_dpixels[c * H * W + pix];
                REAL last_alpha = 0;
                for (uint32_t k = 0; k < ry - rx; k++) {
                    contributor--;
                    if (contributor >= last_contributor) continue;
                    uint32_t g = point_list[ry - k - 1];
                    REAL d[2] = {points_xy[2 * g] - pixf[0], points_xy[2 * g + 1] - pixf[1]};
                    const REAL* co = conic_opacity + 4 * g;
                    REAL power;
                    REAL G = orc_gauss(co, d[0], d[1], &power);
                    if (power > F(0.0)) continue;
                    REAL alpha = FMIN(F(0.99), co[3] * G);
                    if (alpha < F(1.0) / F(255.0)) continue;
                    T = T / (F(1.0) - alpha);
                    REAL dchannel_dcolor = alpha * T;
                    REAL dL_dalpha = F(0.0);
                    for (int ch = 0; ch < 3; ch++) {
                        REAL c = colors[3 * g + ch];
                        accum_rec[ch] = last_alpha * last_color[ch] + (F(1.0) - last_alpha) * accum_rec[ch];
                        last_color[ch] = c;
                        REAL dL_dchannel = dL_dpixel[ch];
                        dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                        acc[9 * (size_t)g + 6 + ch] += (double)(dchannel_dcolor * dL_dchannel);
                    }
                    dL_dalpha *= T;
                    last_alpha = alpha;
                    REAL bg_dot_dpixel = 0;
                    for (int i = 0; i < 3; i++) bg_dot_dpixel += bg[i] * dL_dpixel[i];
                    dL_dalpha += (-T_final / (F(1.0) - alpha)) * bg_dot_dpixel;
                    REAL dL_dG = co[3] * dL_dalpha;
                    REAL gdx = G * d[0];
                    REAL gdy = G * d[1];
                    REAL dG_ddelx = -gdx * co[0] - gdy * co[1];
                    REAL dG_ddely = -gdy * co[2] - gdx * co[1];
                    double* a = acc + 9 * (size_t)g;
                    a[0] += (double)(dL_dG * dG_ddelx * ddelx_dx);
                    a[1] += (double)(dL_dG * dG_ddely * ddely_dy);
                    a[2] += (double)(F(-0.5) * gdx * d[0] * dL_dG);
                    a[3] += (double)(F(-0.5) * gdx * d[1] * dL_dG);
                    a[4] += (double)(F(-0.5) * gdy * d[1] * dL_dG);
                    a[5] += (double)(G * dL_dalpha);
                }
            }
    }
    for (int g = 0; g < P; g++) {
        const double* a = acc + 9 * (size_t)g;
        dL_dmean2D[3 * g + 0] = (REAL)a[0];
        dL_dmean2D[3 * g + 1] = (REAL)a[1];
        dL_dmean2D[3 * g + 2] = 0;
        dL_dconic[4 * g + 0] = (REAL)a[2];
        dL_dconic[4 * g + 1] = (REAL)a[3];
        dL_dconic[4 * g + 2] = 0;
        dL_dconic[4 * g + 3] = (REAL)a[4];
        dL_dopacity[g] = (REAL)a[5];
        for (int c = 0; c < 3; c++) dL_dcolors[3 * g + c] = (REAL)a[6 + c];
    }
    free(acc);
}

/* auxiliary.h:107-117 */
static void dnormvdv3(const REAL* v, const REAL* dv, REAL* o) {
    REAL sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    REAL invsum32 = F(1.0) / SQRT(sum2 * sum2 * sum2);
    o[0] = ((+sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    o[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    o[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* backward.cu:20-139 computeColorFromSH (backward) */
static void shBackward(int idx, int deg, int max_coeffs, const REAL* means, const REAL* campos, const REAL* shs,
                       const uint8_t* clamped, const REAL* dL_dcolor, REAL* dL_dmeans, REAL* dL_dshs) {
    const REAL* pos = means + 3 * idx;
    REAL dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    REAL len = SQRT(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    REAL dir[3] = {dir_orig[0] / len, dir_orig[1] / len, dir_orig[2] / len};
    const REAL* sh = shs + (size_t)idx * max_coeffs * 3;
    REAL* dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
#define SHC(k, c) sh[3 * (k) + (c)]
    REAL g[3];
    for (int c = 0; c < 3; c++) g[c] = dL_dcolor[3 * idx + c] * (clamped[3 * idx + c] ? 0 : 1);
    REAL dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
    REAL x = dir[0], y = dir[1], z = dir[2];
    for (int c = 0; c < 3; c++) dsh[c] = SH_C0 * g[c];
    if (deg > 0) {
        REAL b1 = -SH_C1 * y, b2 = SH_C1 * z, b3 = -SH_C1 * x;
        for (int c = 0; c < 3; c++) {
            dsh[3 + c] = b1 * g[c]; dsh[6 + c] = b2 * g[c]; dsh[9 + c] = b3 * g[c];
            dx[c] = -SH_C1 * SHC(3, c);
            dy[c] = -SH_C1 * SHC(1, c);
            dz[c] = SH_C1 * SHC(2, c);
        }
        if (deg > 1) {
            REAL xx = x * x, yy = y * y, zz = z * z;
            REAL xy = x * y, yz = y * z, xz = x * z;
            REAL b4 = SH_C2[0] * xy, b5 = SH_C2[1] * yz, b6 = SH_C2[2] * (F(2.0) * zz - xx - yy);
            REAL b7 = SH_C2[3] * xz, b8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; c++) {
                dsh[12 + c] = b4 * g[c]; dsh[15 + c] = b5 * g[c]; dsh[18 + c] = b6 * g[c];
                dsh[21 + c] = b7 * g[c]; dsh[24 + c] = b8 * g[c];
                dx[c] += SH_C2[0] * y * SHC(4, c) + SH_C2[2] * F(2.0) * -x * SHC(6, c) + SH_C2[3] * z * SHC(7, c) +
                         SH_C2[4] * F(2.0) * x * SHC(8, c);
                dy[c] += SH_C2[0] * x * SHC(4, c) + SH_C2[1] * z * SHC(5, c) + SH_C2[2] * F(2.0) * -y * SHC(6, c) +
                         SH_C2[4] * F(2.0) * -y * SHC(8, c);
                dz[c] += SH_C2[1] * y * SHC(5, c) + SH_C2[2] * F(2.0) * F(2.0) * z * SHC(6, c) + SH_C2[3] * x * SHC(7, c);
            }
            if (deg > 2) {
                REAL b9 = SH_C3[0] * y * (F(3.0) * xx - yy);
                REAL b10 = SH_C3[1] * xy * z;
                REAL b11 = SH_C3[2] * y * (F(4.0) * zz - xx - yy);
                REAL b12 = SH_C3[3] * z * (F(2.0) * zz - F(3.0) * xx - F(3.0) * yy);
                REAL b13 = SH_C3[4] * x * (F(4.0) * zz - xx - yy);
                REAL b14 = SH_C3[5] * z * (xx - yy);
                REAL b15 = SH_C3[6] * x * (xx - F(3.0) * yy);
                for (int c = 0; c < 3; c++) {
                    dsh[27 + c] = b9 * g[c]; dsh[30 + c] = b10 * g[c]; dsh[33 + c] = b11 * g[c];
                    dsh[36 + c] = b12 * g[c]; dsh[39 + c] = b13 * g[c]; dsh[42 + c] = b14 * g[c];
                    dsh[45 + c] = b15 * g[c];
                    dx[c] += (SH_C3[0] * SHC(9, c) * F(3.0) * F(2.0) * xy + SH_C3[1] * SHC(10, c) * yz +
                              SH_C3[2] * SHC(11, c) * F(-2.0) * xy + SH_C3[3] * SHC(12, c) * F(-3.0) * F(2.0) * xz +
                              SH_C3[4] * SHC(13, c) * (F(-3.0) * xx + F(4.0) * zz - yy) +
                              SH_C3[5] * SHC(14, c) * F(2.0) * xz + SH_C3[6] * SHC(15, c) * F(3.0) * (xx - yy));
                    dy[c] += (SH_C3[0] * SHC(9, c) * F(3.0) * (xx - yy) + SH_C3[1] * SHC(10, c) * xz +
                              SH_C3[2] * SHC(11, c) * (F(-3.0) * yy + F(4.0) * zz - xx) +
                              SH_C3[3] * SHC(12, c) * F(-3.0) * F(2.0) * yz + SH_C3[4] * SHC(13, c) * F(-2.0) * xy +
                              SH_C3[5] * SHC(14, c) * F(-2.0) * yz + SH_C3[6] * SHC(15, c) * F(-3.0) * F(2.0) * xy);
                    dz[c] += (SH_C3[1] * SHC(10, c) * xy + SH_C3[2] * SHC(11, c) * F(4.0) * F(2.0) * yz +
                              SH_C3[3] * SHC(12, c) * F(3.0) * (F(2.0) * zz - xx - yy) +
                              SH_C3[4] * SHC(13, c) * F(4.0) * F(2.0) * xz + SH_C3[5] * SHC(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SHC
    REAL dL_ddir[3] = {dx[0] * g[0] + dx[1] * g[1] + dx[2] * g[2], dy[0] * g[0] + dy[1] * g[1] + dy[2] * g[2],
                       dz[0] * g[0] + dz[1] * g[1] + dz[2] * g[2]};
    REAL dm[3];
    dnormvdv3(dir_orig, dL_ddir, dm);
    for (int c = 0; c < 3; c++) dL_dmeans[3 * idx + c] += dm[c];
}

/* backward.cu:144-274 computeCov2DCUDA */
static void cov2DBackward(int idx, const REAL* means, const REAL* cov3D, REAL h_x, REAL h_y, REAL tan_fovx,
                          REAL tan_fovy, const REAL* view_matrix, const REAL* dL_dconics, REAL* dL_dmeans,
                          REAL* dL_dcov) {
    const REAL* mean = means + 3 * idx;
    REAL dc[3] = {dL_dconics[4 * idx], dL_dconics[4 * idx + 1], dL_dconics[4 * idx + 3]};
    REAL t[3];
    transformPoint4x3(mean, view_matrix, t);
    const REAL limx = F(1.3) * tan_fovx;
    const REAL limy = F(1.3) * tan_fovy;
    const REAL txtz = t[0] / t[2];
    const REAL tytz = t[1] / t[2];
    t[0] = FMIN(limx, FMAX(-limx, txtz)) * t[2];
    t[1] = FMIN(limy, FMAX(-limy, tytz)) * t[2];
    const REAL x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const REAL y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    mat3 J = mcols(h_x / t[2], F(0.0), -(h_x * t[0]) / (t[2] * t[2]), F(0.0), h_y / t[2],
                   -(h_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
    const REAL* v = view_matrix;
    mat3 W = mcols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 Vrk = mcols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 T = mmul(W, J);
    mat3 cov2D = mmul(mmul(mtrans(T), mtrans(Vrk)), T);
    REAL a = cov2D.m[0][0] += F(0.3);
    REAL b = cov2D.m[0][1];
    REAL c = cov2D.m[1][1] += F(0.3);
    REAL denom = a * c - b * b;
    REAL dL_da = 0, dL_db = 0, dL_dc = 0;
    REAL denom2inv = F(1.0) / ((denom * denom) + F(0.0000001));
    REAL* dcov = dL_dcov + 6 * idx;
#define TT(i, j) T.m[i][j]
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dc[0] + 2 * b * c * dc[1] + (denom - a * c) * dc[2]);
        dL_dc = denom2inv * (-a * a * dc[2] + 2 * a * b * dc[1] + (denom - a * c) * dc[0]);
        dL_db = denom2inv * 2 * (b * c * dc[0] - (denom + 2 * b * b) * dc[1] + a * b * dc[2]);
        dcov[0] = (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc);
        dcov[3] = (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc);
        dcov[5] = (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc);
        dcov[1] = 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 1) * dL_dc;
        dcov[2] = 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 2) * dL_dc;
        dcov[4] = 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                  2 * TT(1, 1) * TT(1, 2) * dL_dc;
    } else {
        for (int i = 0; i < 6; i++) dcov[i] = 0;
    }
#define VV(i, j) Vrk.m[i][j]
    REAL dL_dT00 = 2 * (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_da +
                   (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_db;
    REAL dL_dT01 = 2 * (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_da +
                   (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_db;
    REAL dL_dT02 = 2 * (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_da +
                   (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_db;
    REAL dL_dT10 = 2 * (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_dc +
                   (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_db;
    REAL dL_dT11 = 2 * (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_dc +
                   (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_db;
    REAL dL_dT12 = 2 * (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_dc +
                   (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_db;
#undef VV
#undef TT
#define WW(i, j) W.m[i][j]
    REAL dL_dJ00 = WW(0, 0) * dL_dT00 + WW(0, 1) * dL_dT01 + WW(0, 2) * dL_dT02;
    REAL dL_dJ02 = WW(2, 0) * dL_dT00 + WW(2, 1) * dL_dT01 + WW(2, 2) * dL_dT02;
    REAL dL_dJ11 = WW(1, 0) * dL_dT10 + WW(1, 1) * dL_dT11 + WW(1, 2) * dL_dT12;
    REAL dL_dJ12 = WW(2, 0) * dL_dT10 + WW(2, 1) * dL_dT11 + WW(2, 2) * dL_dT12;
#undef WW
    REAL tz = F(1.0) / t[2];
    REAL tz2 = tz * tz;
    REAL tz3 = tz2 * tz;
    REAL dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    REAL dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    REAL dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t[0]) * tz3 * dL_dJ02 +
                  (2 * h_y * t[1]) * tz3 * dL_dJ12;
    /* auxiliary.h:89-97 transformVec4x3Transpose; assigned, not accumulated (:273) */
    dL_dmeans[3 * idx + 0] = v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz;
    dL_dmeans[3 * idx + 1] = v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz;
    dL_dmeans[3 * idx + 2] = v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz;
}

/* backward.cu:278-341 computeCov3D (backward) */
static void cov3DBackward(int idx, const REAL* scale, REAL mod, const REAL* rot, const REAL* dL_dcov3Ds,
                          REAL* dL_dscales, REAL* dL_drots) {
    REAL r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = mcols(F(1.0) - F(2.0) * (y * y + z * z), F(2.0) * (x * y - r * z), F(2.0) * (x * z + r * y),
                   F(2.0) * (x * y + r * z), F(1.0) - F(2.0) * (x * x + z * z), F(2.0) * (y * z - r * x),
                   F(2.0) * (x * z - r * y), F(2.0) * (y * z + r * x), F(1.0) - F(2.0) * (x * x + y * y));
    mat3 S = mcols(F(1.0), 0, 0, 0, F(1.0), 0, 0, 0, F(1.0));
    REAL s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    mat3 M = mmul(S, R);
    const REAL* dc = dL_dcov3Ds + 6 * idx;
    mat3 dL_dSigma = mcols(dc[0], F(0.5) * dc[1], F(0.5) * dc[2], F(0.5) * dc[1], dc[3], F(0.5) * dc[4],
                           F(0.5) * dc[2], F(0.5) * dc[4], dc[5]);
    mat3 M2;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M2.m[i][j] = F(2.0) * M.m[i][j];
    mat3 dL_dM = mmul(M2, dL_dSigma);
    mat3 Rt = mtrans(R);
    mat3 dMt = mtrans(dL_dM);
    REAL* ds = dL_dscales + 3 * idx;
    for (int k = 0; k < 3; k++)
        ds[k] = Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1] + Rt.m[k][2] * dMt.m[k][2];
    for (int k = 0; k < 3; k++)
        for (int j = 0; j < 3; j++) dMt.m[k][j] *= s[k];
#define D(i, j) dMt.m[i][j]
    REAL* dq = dL_drots + 4 * idx;
    dq[0] = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    dq[1] = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) -
            4 * x * (D(2, 2) + D(1, 1));
    dq[2] = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) -
            4 * y * (D(2, 2) + D(0, 0));
    dq[3] = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) -
            4 * z * (D(1, 1) + D(0, 0));
#undef D
}

/* rasterizer_impl.cu:379-432 + backward.cu:559-622: computeCov2DCUDA then
 * preprocessCUDA (backward.cu:346-396).  cov3Ds: the forward's cov3D (or the
 * caller's cov3D_precomp).  Outputs must be zero-initialised by the caller
 * (rasterize_points.cu:139-147 torch::zeros). */
void orc_preprocess_bwd(int P, int D, int M, const REAL* means3D, const int32_t* radii, const REAL* shs,
                        const uint8_t* clamped, const REAL* scales, const REAL* rotations, REAL scale_modifier,
                        const REAL* cov3Ds, const REAL* viewmatrix, const REAL* projmatrix, int W, int H,
                        REAL tan_fovx, REAL tan_fovy, const REAL* campos, const REAL* dL_dmean2D,
                        const REAL* dL_dconic, const REAL* dL_dcolor, REAL* dL_dmean3D, REAL* dL_dcov3D,
                        REAL* dL_dsh, REAL* dL_dscale, REAL* dL_drot) {
    const REAL focal_y = (REAL)H / (F(2.0) * tan_fovy);
    const REAL focal_x = (REAL)W / (F(2.0) * tan_fovx);
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        cov2DBackward(idx, means3D, cov3Ds + 6 * idx, focal_x, focal_y, tan_fovx, tan_fovy, viewmatrix, dL_dconic,
                      dL_dmean3D, dL_dcov3D);
    }
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const REAL* m = means3D + 3 * idx;
        const REAL* proj = projmatrix;
        REAL m_hom[4];
        transformPoint4x4(m, proj, m_hom);
        REAL m_w = F(1.0) / (m_hom[3] + F(0.0000001));
        REAL mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * m_w * m_w;
        REAL mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * m_w * m_w;
        const REAL* g = dL_dmean2D + 3 * idx;
        REAL dm[3];
        dm[0] = (proj[0] * m_w - proj[3] * mul1) * g[0] + (proj[1] * m_w - proj[3] * mul2) * g[1];
        dm[1] = (proj[4] * m_w - proj[7] * mul1) * g[0] + (proj[5] * m_w - proj[7] * mul2) * g[1];
        dm[2] = (proj[8] * m_w - proj[11] * mul1) * g[0] + (proj[9] * m_w - proj[11] * mul2) * g[1];
        for (int c = 0; c < 3; c++) dL_dmean3D[3 * idx + c] += dm[c];
        if (shs) shBackward(idx, D, M, means3D, campos, shs, clamped, dL_dcolor, dL_dmean3D, dL_dsh);
        if (scales) cov3DBackward(idx, scales + 3 * idx, scale_modifier, rotations + 4 * idx, dL_dcov3D, dL_dscale, dL_drot);
    }
}

/* ==================================================================================
 * Relighting shade: scene/NVDIFFREC/light.py:131-193 EnvironmentLight.shade with
 * utils/sh_utils.py:81-151 eval_sh, :162-181 gauss_kernel, :184-187 gamma_correction,
 * scene/NVDIFFREC/util.py:21-31 dot/reflect/length/safe_normalize, and the
 * nvdiffrast dr.texture(filter_mode='linear', boundary_mode='clamp') lookup restated
 * (parity unpinned: nvdiffrast is not vendored).
 * ================================================================================== */

/* sh_utils.py:35-77 */
static const double SC0 = 0.28209479177387814, SC1 = 0.4886025119029199;
static const double SC2[5] = {1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
                              0.5462742152960396};
static const double SC3[7] = {-0.5900435899266435, 2.890611442640554,   -0.4570457994644658, 0.3731763325901154,
                              -0.4570457994644658, 1.445305721320277, -0.5900435899266435};
static const double SC4[9] = {2.5033429417967046,  -1.7701307697799304, 0.9461746957575601,
                              -0.6690465435572892, 0.10578554691520431, -0.6690465435572892,
                              0.47308734787878004, -1.7701307697799304, 0.6258357354491761};
static const double SC5[11] = {-0.6563820568401703, 8.302649259524165,   -0.48923829943525043, 4.793536784973324,
                               -0.452946651195697,  0.1169503224534236,  -0.452946651195697,   2.3967683924866,
                               -0.48923829943525043, 2.075662314881041, -0.6563820568401701};

/* The 36 basis polynomials exactly as sh_utils.py:97-150 codes them (signs, and the
 * reference's own deg-5 forms: :138 has no y factor, :144 has "+ 15"), with
 * their gradients in (x, y, z).  Y[k] = constant * poly_k. */
static void sh_basis(int deg, REAL x, REAL y, REAL z, REAL* Y, REAL* dYx, REAL* dYy, REAL* dYz) {
    const REAL xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    REAL p[36], px[36], py[36], pz[36];
    REAL c[36];
    int n = (deg + 1) * (deg + 1);
    for (int k = 0; k < 36; k++) p[k] = px[k] = py[k] = pz[k] = 0;
    c[0] = (REAL)SC0; p[0] = 1;
    if (deg > 0) {
        c[1] = (REAL)SC1; p[1] = -y; py[1] = -1;
        c[2] = (REAL)SC1; p[2] = z; pz[2] = 1;
        c[3] = (REAL)SC1; p[3] = -x; px[3] = -1;
    }
    if (deg > 1) {
        for (int i = 0; i < 5; i++) c[4 + i] = (REAL)SC2[i];
        p[4] = xy; px[4] = y; py[4] = x;
        p[5] = yz; py[5] = z; pz[5] = y;
        p[6] = 2 * zz - xx - yy; px[6] = -2 * x; py[6] = -2 * y; pz[6] = 4 * z;
        p[7] = xz; px[7] = z; pz[7] = x;
        p[8] = xx - yy; px[8] = 2 * x; py[8] = -2 * y;
    }
    if (deg > 2) {
        for (int i = 0; i < 7; i++) c[9 + i] = (REAL)SC3[i];
        p[9] = y * (3 * xx - yy); px[9] = 6 * xy; py[9] = 3 * xx - 3 * yy;
        p[10] = xy * z; px[10] = yz; py[10] = xz; pz[10] = xy;
        p[11] = y * (4 * zz - xx - yy); px[11] = -2 * xy; py[11] = 4 * zz - xx - 3 * yy; pz[11] = 8 * yz;
        p[12] = z * (2 * zz - 3 * xx - 3 * yy); px[12] = -6 * xz; py[12] = -6 * yz; pz[12] = 6 * zz - 3 * xx - 3 * yy;
        p[13] = x * (4 * zz - xx - yy); px[13] = 4 * zz - 3 * xx - yy; py[13] = -2 * xy; pz[13] = 8 * xz;
        p[14] = z * (xx - yy); px[14] = 2 * xz; py[14] = -2 * yz; pz[14] = xx - yy;
        p[15] = x * (xx - 3 * yy); px[15] = 3 * xx - 3 * yy; py[15] = -6 * xy;
    }
    if (deg > 3) {
        for (int i = 0; i < 9; i++) c[16 + i] = (REAL)SC4[i];
        p[16] = xy * (xx - yy); px[16] = 3 * xx * y - yy * y; py[16] = xx * x - 3 * x * yy;
        p[17] = yz * (3 * xx - yy); px[17] = 6 * x * yz; py[17] = 3 * xx * z - 3 * yy * z; pz[17] = 3 * xx * y - yy * y;
        p[18] = xy * (7 * zz - 1); px[18] = y * (7 * zz - 1); py[18] = x * (7 * zz - 1); pz[18] = 14 * xy * z;
        p[19] = yz * (7 * zz - 3); py[19] = z * (7 * zz - 3); pz[19] = 21 * y * zz - 3 * y;
        p[20] = zz * (35 * zz - 30) + 3; pz[20] = 140 * zz * z - 60 * z;
        p[21] = xz * (7 * zz - 3); px[21] = z * (7 * zz - 3); pz[21] = 21 * x * zz - 3 * x;
        p[22] = (xx - yy) * (7 * zz - 1); px[22] = 2 * x * (7 * zz - 1); py[22] = -2 * y * (7 * zz - 1);
        pz[22] = 14 * z * (xx - yy);
        p[23] = xz * (xx - 3 * yy); px[23] = 3 * xx * z - 3 * yy * z; py[23] = -6 * xy * z; pz[23] = xx * x - 3 * x * yy;
        p[24] = xx * (xx - 3 * yy) - yy * (3 * xx - yy); px[24] = 4 * xx * x - 12 * x * yy; py[24] = -12 * xx * y + 4 * yy * y;
    }
    if (deg > 4) {
        for (int i = 0; i < 11; i++) c[25 + i] = (REAL)SC5[i];
        p[25] = 5 * xx * xx - 10 * yy * xx + yy * yy; px[25] = 20 * xx * x - 20 * x * yy; py[25] = -20 * xx * y + 4 * yy * y;
        p[26] = xy * z * (xx - yy); px[26] = 3 * xx * yz - yy * yz; py[26] = xx * xz - 3 * yy * xz; pz[26] = xx * xy - xy * yy;
        {
            REAL A = 9 * zz - 1, B = 3 * xx - yy;
            p[27] = y * A * B; px[27] = y * A * 6 * x; py[27] = A * (B - 2 * yy); pz[27] = y * B * 18 * z;
        }
        p[28] = xy * z * (3 * zz - 1); px[28] = yz * (3 * zz - 1); py[28] = xz * (3 * zz - 1); pz[28] = 9 * xy * zz - xy;
        p[29] = y * (zz * (-14 + 21 * zz) + 1); py[29] = zz * (-14 + 21 * zz) + 1; pz[29] = y * (84 * zz * z - 28 * z);
        p[30] = z * (zz * (63 * zz - 70) + 15); pz[30] = 315 * zz * zz - 210 * zz + 15;
        p[31] = x * (zz * (21 * zz - 14) + 15); px[31] = zz * (21 * zz - 14) + 15; pz[31] = x * (84 * zz * z - 28 * z);
        {
            REAL A = xx - yy, B = 3 * zz - 1;
            p[32] = z * A * B; px[32] = z * 2 * x * B; py[32] = -z * 2 * y * B; pz[32] = A * (B + 6 * zz);
        }
        {
            REAL A = xx - 3 * yy, B = 9 * zz - 1;
            p[33] = x * A * B; px[33] = B * (A + 2 * xx); py[33] = -6 * xy * B; pz[33] = x * A * 18 * z;
        }
        p[34] = z * (xx * (xx - 6 * yy) + yy * yy); px[34] = z * (4 * xx * x - 12 * x * yy);
        py[34] = z * (-12 * xx * y + 4 * yy * y); pz[34] = xx * (xx - 6 * yy) + yy * yy;
        p[35] = x * (xx * (xx - 10 * yy) + 5 * yy * yy); px[35] = 5 * xx * xx - 30 * xx * yy + 5 * yy * yy;
        py[35] = -20 * xx * xy + 20 * xy * yy;
    }
    for (int k = 0; k < n; k++) {
        Y[k] = c[k] * p[k];
        if (dYx) { dYx[k] = c[k] * px[k]; dYy[k] = c[k] * py[k]; dYz[k] = c[k] * pz[k]; }
    }
}

/* sh_utils.py:81-151 for one direction: out[c] = sum_k Y_k * sh[k*3 + c] */
void orc_eval_sh(int deg, int N, const REAL* sh /* N x K x 3, K >= (deg+1)^2 */, int K, const REAL* dirs, REAL* out) {
    REAL Y[36];
    int n = (deg + 1) * (deg + 1);
    for (int i = 0; i < N; i++) {
        sh_basis(deg, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], Y, NULL, NULL, NULL);
        for (int c = 0; c < 3; c++) {
            REAL r = 0;
            for (int k = 0; k < n; k++) r += Y[k] * sh[((size_t)i * K + k) * 3 + c];
            out[3 * i + c] = r;
        }
    }
}

/* nvdiffrast dr.texture, 2D (third-party, not vendored; called at light.py:170 with
 * filter 'linear' / boundary 'clamp' and at util.py:117 with the default 'wrap').
 * Restated from nvdiffrast's published 2D semantics -- parity unpinned beyond its call
 * sites: texel space u*w - 0.5 (wrap first takes u - floor(u)); clamp clamps the texel
 * coordinate to [0, w-1] before the floor and then uses the same texel twice on the edge
 * (zero uv gradient); wrap takes indices modulo the size; zero drops taps outside;
 * nearest reads texel floor(u*w).  tex [tnb][th][tw][C], uv [nb][npix][2].
 * filter: 0 nearest, 1 linear; boundary: 0 wrap, 1 clamp, 2 zero. */
static int tex_nearest(REAL u, REAL v, int w, int h, int boundary) {
    if (boundary == 0) { u = u - FLOOR(u); v = v - FLOOR(v); }
    int iu = (int)FLOOR(u * (REAL)w), iv = (int)FLOOR(v * (REAL)h);
    if (boundary != 2) {
        iu = iu < 0 ? 0 : (iu > w - 1 ? w - 1 : iu);
        iv = iv < 0 ? 0 : (iv > h - 1 ? h - 1 : iv);
    }
    return (iu < 0 || iu >= w || iv < 0 || iv >= h) ? -1 : iv * w + iu;
}

static void tex_linear(REAL u, REAL v, int w, int h, int boundary, int* idx, REAL* fu, REAL* fv) {
    if (boundary == 0) { u = u - FLOOR(u); v = v - FLOOR(v); }
    u = u * (REAL)w - F(0.5);
    v = v * (REAL)h - F(0.5);
    int cu = 0, cv = 0;
    if (boundary == 1) {
        u = FMIN(FMAX(u, F(0.0)), (REAL)(w - 1));
        v = FMIN(FMAX(v, F(0.0)), (REAL)(h - 1));
        cu = (u == F(0.0) || u == (REAL)(w - 1));
        cv = (v == F(0.0) || v == (REAL)(h - 1));
    }
    int iu0 = (int)FLOOR(u), iv0 = (int)FLOOR(v);
    int iu1 = iu0 + (cu ? 0 : 1), iv1 = iv0 + (cv ? 0 : 1);
    *fu = u - (REAL)iu0;
    *fv = v - (REAL)iv0;
    if (boundary == 0) {
        if (iu0 < 0) iu0 += w;
        if (iv0 < 0) iv0 += h;
        if (iu1 >= w) iu1 -= w;
        if (iv1 >= h) iv1 -= h;
    }
    int us[2] = {iu0, iu1}, vs[2] = {iv0, iv1};
    for (int k = 0; k < 4; k++) {
        int a = us[k & 1], b = vs[k >> 1];
        idx[k] = (a < 0 || a >= w || b < 0 || b >= h) ? -1 : b * w + a;
    }
}

void orc_texture2d_fwd(int nb, int npix, int tnb, int th, int tw, int C, const REAL* tex, const REAL* uv, int filter,
                       int boundary, REAL* out) {
    for (int i = 0; i < nb * npix; i++) {
        const REAL* t = tex + (size_t)(tnb == 1 ? 0 : i / npix) * th * tw * C;
        REAL u = uv[2 * i], v = uv[2 * i + 1];
        if (filter == 0) {
            int k = tex_nearest(u, v, tw, th, boundary);
            for (int c = 0; c < C; c++) out[(size_t)i * C + c] = k < 0 ? F(0.0) : t[(size_t)k * C + c];
            continue;
        }
        int idx[4];
        REAL fu, fv;
        tex_linear(u, v, tw, th, boundary, idx, &fu, &fv);
        for (int c = 0; c < C; c++) {
            REAL a[4];
            for (int k = 0; k < 4; k++) a[k] = idx[k] < 0 ? F(0.0) : t[(size_t)idx[k] * C + c];
            REAL x0 = a[0] + fu * (a[1] - a[0]), x1 = a[2] + fu * (a[3] - a[2]);
            out[(size_t)i * C + c] = x0 + fv * (x1 - x0);
        }
    }
}

/* d_uv [nb][npix][2] (written), d_tex (accumulated; may be NULL) */
void orc_texture2d_bwd(int nb, int npix, int tnb, int th, int tw, int C, const REAL* tex, const REAL* uv, int filter,
                       int boundary, const REAL* dout, REAL* d_uv, REAL* d_tex) {
    for (int i = 0; i < nb * npix; i++) {
        size_t layer = (size_t)(tnb == 1 ? 0 : i / npix) * th * tw * C;
        const REAL* t = tex + layer;
        const REAL* g = dout + (size_t)i * C;
        REAL u = uv[2 * i], v = uv[2 * i + 1];
        if (filter == 0) {
            int k = tex_nearest(u, v, tw, th, boundary);
            if (d_tex && k >= 0)
                for (int c = 0; c < C; c++) d_tex[layer + (size_t)k * C + c] += g[c];
            d_uv[2 * i] = d_uv[2 * i + 1] = F(0.0);
            continue;
        }
        int idx[4];
        REAL fu, fv;
        tex_linear(u, v, tw, th, boundary, idx, &fu, &fv);
        REAL gu = F(0.0), gv = F(0.0);
        for (int c = 0; c < C; c++) {
            REAL a[4];
            for (int k = 0; k < 4; k++) a[k] = idx[k] < 0 ? F(0.0) : t[(size_t)idx[k] * C + c];
            gu += g[c] * ((a[1] - a[0]) * (1 - fv) + (a[3] - a[2]) * fv);
            gv += g[c] * ((a[2] - a[0]) * (1 - fu) + (a[3] - a[1]) * fu);
            if (d_tex) {
                REAL wt[4] = {(1 - fu) * (1 - fv), fu * (1 - fv), (1 - fu) * fv, fu * fv};
                for (int k = 0; k < 4; k++)
                    if (idx[k] >= 0) d_tex[layer + (size_t)idx[k] * C + c] += g[c] * wt[k];
            }
        }
        d_uv[2 * i] = gu * (REAL)tw;
        d_uv[2 * i + 1] = gv * (REAL)th;
    }
}

/* util.py:523-526 gamma_correction and its derivative (clamp mask inclusive, as torch) */
static REAL gamma_f(REAL x) { REAL c = x < 0 ? 0 : (x > 1 ? 1 : x); return POW(c + F(1e-4), (REAL)(1.0 / 2.2)); }
static REAL gamma_d(REAL x) {
    if (x < 0 || x > 1) return 0;
    return (REAL)(1.0 / 2.2) * POW(x + F(1e-4), (REAL)(1.0 / 2.2 - 1.0));
}

/* nvdiffrast texture, filter 'linear', boundary 'clamp', texel centres at (i+0.5)/256:
 * u (NdotV) indexes columns, v (roughness) indexes rows of lut[256][256][2]. */
static void lut_lookup(const REAL* lut, REAL u, REAL v, REAL* out, REAL* du, REAL* dv) {
    const int Wt = 256, Ht = 256;
    REAL x = u * (REAL)Wt - F(0.5), y = v * (REAL)Ht - F(0.5);
    REAL fx0 = FLOOR(x), fy0 = FLOOR(y);
    int x0 = f2i(fx0), y0 = f2i(fy0);
    REAL fx = x - fx0, fy = y - fy0;
    int x1 = x0 + 1, y1 = y0 + 1;
    x0 = x0 < 0 ? 0 : (x0 > Wt - 1 ? Wt - 1 : x0);
    x1 = x1 < 0 ? 0 : (x1 > Wt - 1 ? Wt - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > Ht - 1 ? Ht - 1 : y0);
    y1 = y1 < 0 ? 0 : (y1 > Ht - 1 ? Ht - 1 : y1);
    for (int c = 0; c < 2; c++) {
        REAL t00 = lut[((size_t)y0 * Wt + x0) * 2 + c], t10 = lut[((size_t)y0 * Wt + x1) * 2 + c];
        REAL t01 = lut[((size_t)y1 * Wt + x0) * 2 + c], t11 = lut[((size_t)y1 * Wt + x1) * 2 + c];
        REAL a = t00 + (t10 - t00) * fx, b = t01 + (t11 - t01) * fx;
        out[c] = a + (b - a) * fy;
        if (du) {
            du[c] = (REAL)Wt * ((t10 - t00) * (1 - fy) + (t11 - t01) * fy);
            dv[c] = (REAL)Ht * (b - a);
        }
    }
}

/* light.py:131-193.  N foreground Gaussians; km may be NULL (F0 = 0.04, light.py:176-177).
 * base is [(deg+1)^2][3]; lut is [256][256][2]. */
void orc_shade_fwd(int N, int deg, const REAL* pos, const REAL* nrm, const REAL* albedo, const REAL* view_pos,
                   const REAL* kr, const REAL* km, const REAL* base, const REAL* lut, int specular, REAL* rgb,
                   REAL* diffuse, REAL* spec) {
    const REAL C1 = (REAL)0.429043, C2 = (REAL)0.511664, C3 = (REAL)0.743125, C4 = (REAL)0.886227, C5 = (REAL)0.247708;
    int K = (deg + 1) * (deg + 1);
    REAL Y[36];
    for (int i = 0; i < N; i++) {
        const REAL *p = pos + 3 * i, *n = nrm + 3 * i, *a = albedo + 3 * i, *vp = view_pos + 3 * i;
        REAL x = n[0], y = n[1], z = n[2];
        REAL dh[3];
        for (int c = 0; c < 3; c++) {
            const REAL* b = base;
            REAL irr = C1 * b[24 + c] * (x * x - y * y) + C3 * b[18 + c] * (z * z) + C4 * b[c] - C5 * b[18 + c] +
                       (REAL)(2 * 0.429043) * b[12 + c] * x * y + (REAL)(2 * 0.429043) * b[21 + c] * x * z +
                       (REAL)(2 * 0.429043) * b[15 + c] * y * z + (REAL)(2 * 0.511664) * b[9 + c] * x +
                       (REAL)(2 * 0.511664) * b[3 + c] * y + (REAL)(2 * 0.511664) * b[6 + c] * z;
            irr = irr < F(1e-4) ? F(1e-4) : irr;
            dh[c] = a[c] * irr;
            diffuse[3 * i + c] = gamma_f(dh[c]);
        }
        if (!specular) {
            for (int c = 0; c < 3; c++) { rgb[3 * i + c] = diffuse[3 * i + c]; spec[3 * i + c] = 0; }
            continue;
        }
        REAL wo[3] = {vp[0] - p[0], vp[1] - p[1], vp[2] - p[2]};
        REAL l2 = wo[0] * wo[0] + wo[1] * wo[1] + wo[2] * wo[2];
        REAL len = SQRT(l2 < F(1e-20) ? F(1e-20) : l2);
        for (int c = 0; c < 3; c++) wo[c] = wo[c] / len;
        REAL dwn = wo[0] * n[0] + wo[1] * n[1] + wo[2] * n[2];
        REAL rv[3];
        for (int c = 0; c < 3; c++) rv[c] = 2 * dwn * n[c] - wo[c];
        REAL rl2 = rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2];
        REAL rlen = SQRT(rl2 < F(1e-20) ? F(1e-20) : rl2);
        REAL r[3] = {rv[0] / rlen, rv[1] / rlen, rv[2] / rlen};
        REAL NdotV = dwn < F(1e-4) ? F(1e-4) : dwn;
        REAL fg[2];
        lut_lookup(lut, NdotV, kr[i], fg, NULL, NULL);
        sh_basis(deg, r[0], r[1], r[2], Y, NULL, NULL, NULL);
        REAL F0c = F(0.04);
        for (int c = 0; c < 3; c++) {
            REAL si = 0;
            for (int l = 0, k = 0; l <= deg; l++) {
                REAL gw = EXP((REAL)(-l * (l + 1)) * (F(0.3) * kr[i]));
                for (int m = 0; m < 2 * l + 1; m++, k++) si += Y[k] * (gw * base[3 * k + c]);
            }
            (void)K;
            si = si < F(1e-4) ? F(1e-4) : si;
            REAL F0 = km ? (F(1.0) - km[i]) * F0c + a[c] * km[i] : F0c;
            REAL refl = F0 * fg[0] + fg[1];
            REAL sh_hdr = si * refl;
            REAL shaded = km ? (1 - km[i]) * dh[c] + sh_hdr : dh[c] + sh_hdr;
            rgb[3 * i + c] = gamma_f(shaded);
            spec[3 * i + c] = gamma_f(sh_hdr);
        }
    }
}

/* Autograd-equivalent backward of orc_shade_fwd (torch clamp/pow/sqrt rules).
 * Gradient outputs are overwritten (d_base accumulated over N, in double). */
void orc_shade_bwd(int N, int deg, const REAL* pos, const REAL* nrm, const REAL* albedo, const REAL* view_pos,
                   const REAL* kr, const REAL* km, const REAL* base, const REAL* lut, int specular,
                   const REAL* g_rgb, const REAL* g_diff, const REAL* g_spec, REAL* d_pos, REAL* d_nrm,
                   REAL* d_albedo, REAL* d_view_pos, REAL* d_kr, REAL* d_km, REAL* d_base) {
    const REAL C1 = (REAL)0.429043, C2 = (REAL)0.511664, C3 = (REAL)0.743125, C4 = (REAL)0.886227, C5 = (REAL)0.247708;
    const REAL C1x2 = (REAL)(2 * 0.429043), C2x2 = (REAL)(2 * 0.511664);
    int K = (deg + 1) * (deg + 1);
    double* db = (double*)calloc((size_t)K * 3, sizeof(double));
    REAL Y[36], Yx[36], Yy[36], Yz[36];
    for (int i = 0; i < N; i++) {
        const REAL *p = pos + 3 * i, *n = nrm + 3 * i, *a = albedo + 3 * i, *vp = view_pos + 3 * i;
        REAL x = n[0], y = n[1], z = n[2];
        REAL irr_raw[3], irr[3], dh[3];
        for (int c = 0; c < 3; c++) {
            const REAL* b = base;
            irr_raw[c] = C1 * b[24 + c] * (x * x - y * y) + C3 * b[18 + c] * (z * z) + C4 * b[c] - C5 * b[18 + c] +
                         C1x2 * b[12 + c] * x * y + C1x2 * b[21 + c] * x * z + C1x2 * b[15 + c] * y * z +
                         C2x2 * b[9 + c] * x + C2x2 * b[3 + c] * y + C2x2 * b[6 + c] * z;
            irr[c] = irr_raw[c] < F(1e-4) ? F(1e-4) : irr_raw[c];
            dh[c] = a[c] * irr[c];
        }
        REAL g_dh[3], g_a[3] = {0, 0, 0}, g_n[3] = {0, 0, 0}, g_p[3] = {0, 0, 0}, g_vp[3] = {0, 0, 0};
        REAL g_kr = 0, g_km = 0;
        for (int c = 0; c < 3; c++) g_dh[c] = g_diff[3 * i + c] * gamma_d(dh[c]);
        if (!specular) {
            for (int c = 0; c < 3; c++) g_dh[c] += g_rgb[3 * i + c] * gamma_d(dh[c]);
        } else {
            REAL wv[3] = {vp[0] - p[0], vp[1] - p[1], vp[2] - p[2]};
            REAL l2 = wv[0] * wv[0] + wv[1] * wv[1] + wv[2] * wv[2];
            int lclamp = l2 < F(1e-20);
            REAL len = SQRT(lclamp ? F(1e-20) : l2);
            REAL wo[3] = {wv[0] / len, wv[1] / len, wv[2] / len};
            REAL dwn = wo[0] * n[0] + wo[1] * n[1] + wo[2] * n[2];
            REAL rv[3];
            for (int c = 0; c < 3; c++) rv[c] = 2 * dwn * n[c] - wo[c];
            REAL rl2 = rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2];
            int rclamp = rl2 < F(1e-20);
            REAL rlen = SQRT(rclamp ? F(1e-20) : rl2);
            REAL r[3] = {rv[0] / rlen, rv[1] / rlen, rv[2] / rlen};
            REAL NdotV = dwn < F(1e-4) ? F(1e-4) : dwn;
            REAL fg[2], fgu[2], fgv[2];
            lut_lookup(lut, NdotV, kr[i], fg, fgu, fgv);
            sh_basis(deg, r[0], r[1], r[2], Y, Yx, Yy, Yz);
            REAL gw[6];
            for (int l = 0; l <= deg; l++) gw[l] = EXP((REAL)(-l * (l + 1)) * (F(0.3) * kr[i]));
            REAL g_fg0 = 0, g_fg1 = 0, g_r[3] = {0, 0, 0};
            REAL g_gw[6] = {0, 0, 0, 0, 0, 0};
            for (int c = 0; c < 3; c++) {
                REAL si_raw = 0;
                for (int l = 0, k = 0; l <= deg; l++)
                    for (int m = 0; m < 2 * l + 1; m++, k++) si_raw += Y[k] * (gw[l] * base[3 * k + c]);
                REAL si = si_raw < F(1e-4) ? F(1e-4) : si_raw;
                REAL F0 = km ? (F(1.0) - km[i]) * F(0.04) + a[c] * km[i] : F(0.04);
                REAL refl = F0 * fg[0] + fg[1];
                REAL sh_hdr = si * refl;
                REAL shaded = km ? (1 - km[i]) * dh[c] + sh_hdr : dh[c] + sh_hdr;
                REAL g_sh = g_rgb[3 * i + c] * gamma_d(shaded);
                REAL g_hdr = g_sh + g_spec[3 * i + c] * gamma_d(sh_hdr);
                if (km) { g_dh[c] += (1 - km[i]) * g_sh; g_km += -dh[c] * g_sh; }
                else g_dh[c] += g_sh;
                REAL g_si = si_raw >= F(1e-4) ? g_hdr * refl : 0;
                REAL g_refl = g_hdr * si;
                REAL g_F0 = g_refl * fg[0];
                g_fg0 += g_refl * F0;
                g_fg1 += g_refl;
                if (km) { g_km += (a[c] - F(0.04)) * g_F0; g_a[c] += km[i] * g_F0; }
                for (int l = 0, k = 0; l <= deg; l++)
                    for (int m = 0; m < 2 * l + 1; m++, k++) {
                        db[3 * k + c] += (double)(Y[k] * gw[l] * g_si);
                        g_gw[l] += Y[k] * base[3 * k + c] * g_si;
                        REAL s = gw[l] * base[3 * k + c] * g_si;
                        g_r[0] += Yx[k] * s; g_r[1] += Yy[k] * s; g_r[2] += Yz[k] * s;
                    }
            }
            for (int l = 0; l <= deg; l++) g_kr += g_gw[l] * gw[l] * ((REAL)(-l * (l + 1)) * F(0.3));
            REAL g_ndv = g_fg0 * fgu[0] + g_fg1 * fgu[1];
            g_kr += g_fg0 * fgv[0] + g_fg1 * fgv[1];
            /* r = safe_normalize(rv) */
            REAL g_rv[3];
            REAL rdg = r[0] * g_r[0] + r[1] * g_r[1] + r[2] * g_r[2];
            for (int c = 0; c < 3; c++) g_rv[c] = rclamp ? g_r[c] / rlen : (g_r[c] - r[c] * rdg) / rlen;
            /* rv = 2 dwn n - wo */
            REAL g_dwn = 2 * (n[0] * g_rv[0] + n[1] * g_rv[1] + n[2] * g_rv[2]);
            if (dwn >= F(1e-4)) g_dwn += g_ndv;
            REAL g_wo[3];
            for (int c = 0; c < 3; c++) {
                g_n[c] += 2 * dwn * g_rv[c] + g_dwn * wo[c];
                g_wo[c] = -g_rv[c] + g_dwn * n[c];
            }
            REAL wdg = wo[0] * g_wo[0] + wo[1] * g_wo[1] + wo[2] * g_wo[2];
            for (int c = 0; c < 3; c++) {
                REAL gwv = lclamp ? g_wo[c] / len : (g_wo[c] - wo[c] * wdg) / len;
                g_vp[c] += gwv;
                g_p[c] -= gwv;
            }
        }
        /* diffuse: dh = a * irr */
        for (int c = 0; c < 3; c++) {
            g_a[c] += g_dh[c] * irr[c];
            REAL gi = irr_raw[c] >= F(1e-4) ? g_dh[c] * a[c] : 0;
            const REAL* b = base;
            db[24 + c] += (double)(gi * C1 * (x * x - y * y));
            db[18 + c] += (double)(gi * (C3 * z * z - C5));
            db[c] += (double)(gi * C4);
            db[12 + c] += (double)(gi * C1x2 * x * y);
            db[21 + c] += (double)(gi * C1x2 * x * z);
            db[15 + c] += (double)(gi * C1x2 * y * z);
            db[9 + c] += (double)(gi * C2x2 * x);
            db[3 + c] += (double)(gi * C2x2 * y);
            db[6 + c] += (double)(gi * C2x2 * z);
            g_n[0] += gi * (C1 * b[24 + c] * 2 * x + C1x2 * b[12 + c] * y + C1x2 * b[21 + c] * z + C2x2 * b[9 + c]);
            g_n[1] += gi * (-C1 * b[24 + c] * 2 * y + C1x2 * b[12 + c] * x + C1x2 * b[15 + c] * z + C2x2 * b[3 + c]);
            g_n[2] += gi * (C3 * b[18 + c] * 2 * z + C1x2 * b[21 + c] * x + C1x2 * b[15 + c] * y + C2x2 * b[6 + c]);
        }
        for (int c = 0; c < 3; c++) {
            d_pos[3 * i + c] = g_p[c];
            d_nrm[3 * i + c] = g_n[c];
            d_albedo[3 * i + c] = g_a[c];
            d_view_pos[3 * i + c] = g_vp[c];
        }
        d_kr[i] = g_kr;
        if (d_km) d_km[i] = g_km;
    }
    for (int k = 0; k < K * 3; k++) d_base[k] = (REAL)db[k];
    free(db);
}

/* ---------------- simple-knn distCUDA2 (submodules/simple-knn/simple_knn.cu:119-220) --------
 * Sequential restatement of SimpleKNN::knn: bounds seeded with 0 (cub Reduce init, :190-200),
 * 10-bit Morton codes (:53-71), stable sort by code, 1024-point boxes (:79-113), +-3
 * neighbour rejection bound and the box scan in index order (:144-181).  Float arithmetic
 * only; sums of squares as fma(z, z, fma(y, y, x * x)) -- the contraction nvcc applies to
 * `x*x + y*y + z*z` (parity w.r.t. nvcc's contraction choice is unpinned).  Test
 * infrastructure only. */
#define KNN_BOX 1024
static float knn_sq3(float x, float y, float z) { return fmaf(z, z, fmaf(y, y, x * x)); }
static uint32_t knn_prep(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
static uint32_t knn_f2u(float f) {
    if (!(f > 0.f)) return 0u;
    if (f >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
static float knn_box_dist(const float* mn, const float* mx, const float* p) {
    float d[3] = {0.f, 0.f, 0.f};
    for (int k = 0; k < 3; k++)
        if (p[k] < mn[k] || p[k] > mx[k]) d[k] = fminf(fabsf(p[k] - mn[k]), fabsf(p[k] - mx[k]));
    return knn_sq3(d[0], d[1], d[2]);
}
static void knn_update(const float* ref, const float* p, float* best) {
    float d = knn_sq3(p[0] - ref[0], p[1] - ref[1], p[2] - ref[2]);
    for (int j = 0; j < 3; j++)
        if (best[j] > d) {
            float t = best[j];
            best[j] = d;
            d = t;
        }
}
void orc_knn(int P, const float* pts, float* dists) {
    if (P <= 0) return;
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < P; i++)
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], pts[3 * i + k]);
            mx[k] = fmaxf(mx[k], pts[3 * i + k]);
        }
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * P);
    uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * P);
    for (int i = 0; i < P; i++) {
        uint32_t c[3];
        for (int k = 0; k < 3; k++) c[k] = knn_prep(knn_f2u(((pts[3 * i + k] - mn[k]) / (mx[k] - mn[k])) * 1023.f));
        keys[i] = c[0] | (c[1] << 1) | (c[2] << 2);
        ids[i] = (uint32_t)i;
    }
    radix_sort_pairs(keys, ids, P, 30);
    float* sp = (float*)malloc(sizeof(float) * 3 * P);
    for (int i = 0; i < P; i++)
        for (int k = 0; k < 3; k++) sp[3 * i + k] = pts[3 * ids[i] + k];
    const int nbox = (P + KNN_BOX - 1) / KNN_BOX;
    float* bmn = (float*)malloc(sizeof(float) * 3 * nbox);
    float* bmx = (float*)malloc(sizeof(float) * 3 * nbox);
    for (int b = 0; b < nbox; b++) {
        for (int k = 0; k < 3; k++) {
            bmn[3 * b + k] = 3.402823466e+38f;
            bmx[3 * b + k] = -3.402823466e+38f;
        }
        for (int i = b * KNN_BOX; i < P && i < (b + 1) * KNN_BOX; i++)
            for (int k = 0; k < 3; k++) {
                bmn[3 * b + k] = fminf(bmn[3 * b + k], sp[3 * i + k]);
                bmx[3 * b + k] = fmaxf(bmx[3 * b + k], sp[3 * i + k]);
            }
    }
    for (int idx = 0; idx < P; idx++) {
        const float* point = sp + 3 * idx;
        float best[3] = {3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f};
        for (int i = (idx - 3 > 0 ? idx - 3 : 0); i <= (P - 1 < idx + 3 ? P - 1 : idx + 3); i++)
            if (i != idx) knn_update(point, sp + 3 * i, best);
        const float reject = best[2];
        best[0] = best[1] = best[2] = 3.402823466e+38f;
        for (int b = 0; b < nbox; b++) {
            const float dist = knn_box_dist(bmn + 3 * b, bmx + 3 * b, point);
            if (dist > reject || dist > best[2]) continue;
            for (int i = b * KNN_BOX; i < P && i < (b + 1) * KNN_BOX; i++)
                if (i != idx) knn_update(point, sp + 3 * i, best);
        }
        dists[ids[idx]] = (best[0] + best[1] + best[2]) / 3.0f;
    }
    free(keys);
    free(ids);
    free(sp);
    free(bmn);
    free(bmx);
}
