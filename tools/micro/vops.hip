// Microbenchmark: issue cost of wave64 VALU instruction kinds on gfx950 (tools only).
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

__global__ void k_fma(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    float a = 1.0001f, b = 0.5f;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_readlane(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_readlane_b32 %0, %4, 5\n v_readlane_b32 %1, %5, 7\n v_readlane_b32 %2, %6, 9\n v_readlane_b32 %3, %7, 11" : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3) : "v"(x0), "v"(x1), "v"(x2), "v"(x3));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 + s1 + s2 + s3;
}
__global__ void k_dpp(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %2, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %3, %3, %3 row_ror:4 row_mask:0xf bank_mask:0xf" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_swap(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_cnd(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %2, vcc\n v_cndmask_b32 %0, %0, %3, vcc" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "vcc");)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_dep(float* out, int iters) {  // one dependent chain
    float x0 = threadIdx.x;
    float a = 1.0001f, b = 0.5f;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2\n v_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    const int iters = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[] = {"v_fma_f32", "v_readlane", "v_add_dpp", "v_permlane32_swap", "cmp+3cndmask", "dep fma chain"};
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;
        for (int which = 0; which < 6; which++) {
            float ms = 0;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(e0);
                switch (which) {
                    case 0: hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 1: hipLaunchKernelGGL(k_readlane, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 2: hipLaunchKernelGGL(k_dpp, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 3: hipLaunchKernelGGL(k_swap, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 4: hipLaunchKernelGGL(k_cnd, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 5: hipLaunchKernelGGL(k_dep, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double per_simd = (double)wps * iters * 32;  // wave-instructions per SIMD
            printf("waves/SIMD %d  %-18s %.3f ms  %.2f ns/instr/SIMD\n", wps, names[which], ms,
                   ms * 1e6 / per_simd);
        }
    }
    return 0;
}
