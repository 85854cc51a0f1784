// Microbenchmark: issue cost of compares and selects on gfx950 (tools only).
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(x) x x x x x x x x

__global__ void k_cmp_vcc(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1;
    unsigned long long m = 0;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cmp_gt_f32 vcc, %1, %2\n v_cmp_gt_f32 vcc, %2, %1\n v_cmp_lt_f32 vcc, %1, %2\n v_cmp_lt_f32 vcc, %2, %1" : "=r"(m) : "v"(x0), "v"(x1) : "vcc");)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + (float)m;
}
__global__ void k_cmp_sgpr(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1;
    unsigned long long m0, m1, m2, m3;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cmp_gt_f32_e64 %0, %4, %5\n v_cmp_gt_f32_e64 %1, %5, %4\n v_cmp_lt_f32_e64 %2, %4, %5\n v_cmp_lt_f32_e64 %3, %5, %4" : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(x0), "v"(x1));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + (float)(m0 + m1 + m2 + m3);
}
__global__ void k_cnd_vcc(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 7.f;
    asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(x0), "v"(x3) : "vcc");
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_cnd_sgpr(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 7.f;
    unsigned long long m;
    asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x0), "v"(x3));
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y), "s"(m));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_max(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 7.f;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_max_f32 %0, %0, %4\n v_max_f32 %1, %1, %4\n v_max_f32 %2, %2, %4\n v_max_f32 %3, %3, %4" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_cmp_cnd_dep(float* out, int iters) {  // cmp -> cndmask pairs on different vcc-free SGPRs
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 7.f;
    unsigned long long m0, m1;
    for (int i = 0; i < iters; i++) {
        REP8(asm volatile("v_cmp_gt_f32_e64 %4, %0, %6\n v_cmp_gt_f32_e64 %5, %1, %6\n v_cndmask_b32_e64 %2, %2, %6, %4\n v_cndmask_b32_e64 %3, %3, %6, %5" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=s"(m0), "=s"(m1) : "v"(y));)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    const int iters = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[] = {"v_cmp -> vcc", "v_cmp_e64 -> sgpr", "v_cndmask vcc", "v_cndmask_e64 sgpr", "v_max_f32",
                           "cmp_e64+cndmask_e64"};
    for (int wps : {1, 4, 8}) {
        const int blocks = 256 * wps;
        for (int which = 0; which < 6; which++) {
            float ms = 0;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(e0);
                switch (which) {
                    case 0: hipLaunchKernelGGL(k_cmp_vcc, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 1: hipLaunchKernelGGL(k_cmp_sgpr, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 2: hipLaunchKernelGGL(k_cnd_vcc, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 3: hipLaunchKernelGGL(k_cnd_sgpr, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 4: hipLaunchKernelGGL(k_max, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 5: hipLaunchKernelGGL(k_cmp_cnd_dep, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double per_simd = (double)wps * iters * 32;
            printf("waves/SIMD %d  %-22s %.3f ms  %.2f ns/instr/SIMD\n", wps, names[which], ms, ms * 1e6 / per_simd);
        }
    }
    return 0;
}
