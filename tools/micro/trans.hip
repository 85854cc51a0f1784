// Microbenchmark (tools only): wave64 issue cost on gfx950 of the tile passes' instruction
// mix -- v_fma_f32, v_pk_fma_f32, v_pk_mul_f32, v_exp_f32, v_rcp_f32, and exp/rcp interleaved
// with independent FMAs (does the transcendental unit co-issue with the FMA pipe?).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float float2v __attribute__((ext_vector_type(2)));
#define REP8(x) x x x x x x x x

template <int K>
__global__ void k_op(float* out, int iters) {
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
          x7 = x0 + 7;
    float2v p0 = {x0, x1}, p1 = {x2, x3}, p2 = {x4, x5}, p3 = {x6, x7};
    const float a = 0.999f, b = 1e-3f;
    const float2v av = {a, a}, bv = {b, b};
    for (int i = 0; i < iters; i++) {
        if constexpr (K == 0) {
            REP8(asm volatile("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b));)
        } else if constexpr (K == 1) {
            REP8(asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(av), "v"(bv));)
        } else if constexpr (K == 2) {
            REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(av));)
        } else if constexpr (K == 3) {
            REP8(asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));)
        } else if constexpr (K == 4) {
            REP8(asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));)
        } else if constexpr (K == 5) {  // 1 exp + 3 independent fma
            REP8(asm volatile("v_exp_f32 %0, %0\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b));)
        } else if constexpr (K == 6) {  // v_cndmask_b32_e64 with an SGPR-pair mask
            REP8(asm volatile("v_cmp_lt_f32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %2, %2, %3, s[40:41]\n v_cndmask_b32_e64 %3, %3, %2, s[40:41]\n v_cndmask_b32_e64 %0, %0, %3, s[40:41]" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : : "s40", "s41");)
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + p0.x + p1.y + p2.x + p3.y;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    const int iters = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_exp_f32", "v_rcp_f32", "exp+3fma",
                           "cmp+3cndmask_e64"};
    for (int wps : {2, 4, 8}) {
        const int blocks = 256 * wps;
        for (int which = 0; which < 7; which++) {
            float ms = 0;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(e0);
                switch (which) {
                    case 0: hipLaunchKernelGGL(k_op<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 1: hipLaunchKernelGGL(k_op<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 2: hipLaunchKernelGGL(k_op<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 3: hipLaunchKernelGGL(k_op<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 4: hipLaunchKernelGGL(k_op<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 5: hipLaunchKernelGGL(k_op<5>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 6: hipLaunchKernelGGL(k_op<6>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double per_simd = (double)wps * iters * 32;  // wave-instructions per SIMD
            printf("waves/SIMD %d  %-18s %.3f ms  %.3f ns/instr/SIMD\n", wps, names[which], ms, ms * 1e6 / per_simd);
        }
    }
    return 0;
}
