// Microbenchmark: wave64 v_fma_f32 vs v_pk_fma_f32 throughput on gfx950 (tools only).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float float2v __attribute__((ext_vector_type(2)));

__global__ void k_fma(float* out, int iters, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x2) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x3) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x4) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x5) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x6) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x7) : "v"(a), "v"(b));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

__global__ void k_pkfma(float* out, int iters, float a, float b) {
    float2v x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
            x7 = x0 + 7;
    float2v av = {a, a}, bv = {b, b};
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x2) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x3) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x4) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x5) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x6) : "v"(av), "v"(bv));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x7) : "v"(av), "v"(bv));
        }
    }
    float2v s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

__global__ void k_exp(float* out, int iters, float a, float b) {
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1e-3f, x2 = x0 + 2e-3f, x3 = x0 + 3e-3f;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            asm volatile("v_exp_f32 %0, %0" : "+v"(x0));
            asm volatile("v_exp_f32 %0, %0" : "+v"(x1));
            asm volatile("v_exp_f32 %0, %0" : "+v"(x2));
            asm volatile("v_exp_f32 %0, %0" : "+v"(x3));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

int main() {
    float* out;
    hipMalloc(&out, 1 << 26);
    const int iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int waves_per_simd : {1, 2, 4, 8}) {
        const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 4 waves, one per SIMD
        for (int which = 0; which < 3; which++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (which == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
                if (which == 1) hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
                if (which == 2) hipLaunchKernelGGL(k_exp, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double instr = (double)blocks * 4 * iters * 64;  // wave-instructions
                if (rep == 1)
                    printf("waves/SIMD %d %-6s %.3f ms  %.2f ns per wave-instr per SIMD (%.2f cyc @2.4GHz)\n",
                           waves_per_simd, which == 0 ? "fma" : which == 1 ? "pkfma" : "exp", ms,
                           ms * 1e6 / (instr / 1024), ms * 1e6 / (instr / 1024) * 2.4);
            }
        }
    }
    return 0;
}
