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
};

constexpr int SHADE_THREADS = 256;
size_t shade_workspace_bytes(int N, int deg);
void launch_shade_fwd(const ShadeArgs& a, float* rgb, float* diffuse, float* specular, hipStream_t s);
void launch_shade_bwd(const ShadeArgs& a, const ShadeGrads& g, void* workspace, hipStream_t s);

}  // namespace gsr
