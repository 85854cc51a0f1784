// gsr_shade.hpp -- fused per-Gaussian relighting shade (scene/NVDIFFREC/light.py:131-193).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace gsr {

struct ShadeArgs {
    int N, deg;
    const float* pos;
    const float* normal;
    const float* albedo;
    const float* view_pos;
    const float* kr;
    const float* km;  // nullable
    const float* base;
    const float* lut;
    int specular;
    // Row addressing (the fused relit features op, gsr_relit_features): Gaussian i of the
    // shaded set is row rows[i] of pos and of the rgb/diffuse/specular outputs and their
    // gradients (i when rows is null); those outputs/gradients have io_stride floats per
    // row; view_pos advances vp_stride floats per Gaussian (0: one shared camera centre).
    const int* rows = nullptr;
    int io_stride = 3;
    int vp_stride = 3;
    // Whole-row mode (gsr_relit_features, io_stride == RELIT_STRIDE, rgb/diffuse/specular at
    // row offsets 0/3/6): also the row's depth (viewmatrix column 2, device), 0.5 n + 0.5, alpha
    // 1 and the padding, so every 64-B feature row is written by one kernel in full.
    const float* viewmatrix = nullptr;
};

struct ShadeGrads {
    const float* g_rgb;
    const float* g_diffuse;
    const float* g_specular;
    float* d_pos;
    float* d_normal;
    float* d_albedo;
    float* d_view_pos;
    float* d_kr;
    float* d_km;
    float* d_base;
    unsigned acc;  // ACC_ALBEDO / ACC_ROUGH / ACC_METAL: add into d_albedo / d_kr / d_km
};

// Fused relit features (gsr_shade.hip k_relit_fwd / k_relit_bwd).
constexpr int RELIT_STRIDE = 16;  // feature row: rgb, diffuse, specular, depth, normal01, alpha, 0, 0
struct RelitArgs {
    int P;
    const float* xyz;       // [P,3]
    const float* rotation;  // [P,4]
    const float* scaling;   // [P,3]
    const int* fg_rank;     // [P]: rank among the foreground Gaussians, -1 for sky
    int sky_deg;            // -1: fix_sky (sky colour 1)
    const float* sky_sh;    // [(sky_deg+1)^2][3]
    const float* campos;    // [3]
    const float* viewmatrix;  // world_view_transform, row-major [4,4]
    float* features;        // [P][RELIT_STRIDE]
};
struct RelitGrads {
    const float* dL_dfeatures;  // [P][RELIT_STRIDE]
    float* d_xyz;               // [P,3]
    float* d_rotation;          // [P,4]
    float* d_sky_sh;            // [(sky_deg+1)^2][3] or null
    float* workspace;           // relit_workspace_bytes
    unsigned acc;               // ACC_MEAN3D / ACC_ROT: add into d_xyz / d_rotation
};
size_t relit_workspace_bytes(int P, int sky_deg);
// the relit features of all P in one launch (a: the foreground shade's arguments, whole-row
// mode; a.N = N_fg, its rows are the Gaussians themselves)
void launch_relit_fwd(const RelitArgs& ra, const ShadeArgs& a, hipStream_t s);
// the relit features' backward over all P in one launch (+ the fixed-order d_base and d_sky_sh
// reductions): ws_base holds shade_workspace_bytes(P, deg)
void launch_relit_bwd(const RelitArgs& ra, const RelitGrads& rg, const ShadeArgs& a, const ShadeGrads& g,
                      void* ws_base, hipStream_t s);

constexpr int SHADE_THREADS = 256;
size_t shade_workspace_bytes(int N, int deg);
void launch_shade_fwd(const ShadeArgs& a, float* rgb, float* diffuse, float* specular, hipStream_t s);
void launch_shade_bwd(const ShadeArgs& a, const ShadeGrads& g, void* workspace, hipStream_t s);

}  // namespace gsr
