// Microbenchmark (tools only): does a wave64 VALU instruction issue faster on gfx950 when
// its exec mask leaves a 32-lane half (or more) empty?  Independent v_fma_f32 streams and
// v_exp_f32 streams under several exec masks, 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

template <int MODE>
__global__ void k_fma(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    const float a = 1.0001f, b = 0.5f;
    const unsigned long long m = MODE == 0 ? ~0ull : MODE == 1 ? 0x00000000FFFFFFFFull : MODE == 2 ? 0x000000000000FFFFull
                                 : MODE == 3 ? 0x5555555555555555ull : MODE == 4 ? 0x0000FFFF0000FFFFull : 0x1ull;
    for (int i = 0; i < iters; i++) {
        asm volatile(
            "s_mov_b64 s[40:41], exec\n"
            "s_mov_b64 exec, %6\n"
            REP8("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5\n")
            "s_mov_b64 exec, s[40:41]\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
            : "v"(a), "v"(b), "s"(m)
            : "s40", "s41");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

template <int MODE>
__global__ void k_exp(float* out, int iters) {
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1e-3f, x2 = x0 + 2e-3f, x3 = x0 + 3e-3f;
    const unsigned long long m = MODE == 0 ? ~0ull : MODE == 1 ? 0x00000000FFFFFFFFull : MODE == 2 ? 0x000000000000FFFFull
                                 : MODE == 3 ? 0x5555555555555555ull : MODE == 4 ? 0x0000FFFF0000FFFFull : 0x1ull;
    for (int i = 0; i < iters; i++) {
        asm volatile(
            "s_mov_b64 s[40:41], exec\n"
            "s_mov_b64 exec, %4\n"
            REP8("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n")
            "s_mov_b64 exec, s[40:41]\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
            : "s"(m)
            : "s40", "s41");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

typedef void (*kfn)(float*, int);

int main() {
    float* out;
    (void)hipMalloc(&out, 1 << 26);
    const int iters = 1024;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* modes[] = {"exec all 64", "exec low 32", "exec low 16", "exec even lanes", "exec 0-15,32-47", "exec lane 0"};
    kfn fma[] = {k_fma<0>, k_fma<1>, k_fma<2>, k_fma<3>, k_fma<4>, k_fma<5>};
    kfn ex[] = {k_exp<0>, k_exp<1>, k_exp<2>, k_exp<3>, k_exp<4>, k_exp<5>};
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;
        for (int kind = 0; kind < 2; kind++) {
            for (int mode = 0; mode < 6; mode++) {
                float ms = 0;
                for (int rep = 0; rep < 3; rep++) {
                    (void)hipEventRecord(e0);
                    hipLaunchKernelGGL(kind ? ex[mode] : fma[mode], dim3(blocks), dim3(256), 0, 0, out, iters);
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    (void)hipEventElapsedTime(&ms, e0, e1);
                }
                const double per_simd = (double)wps * iters * 32;  // wave-instructions per SIMD
                printf("waves/SIMD %d  %-6s %-18s %.3f ms  %.3f ns/instr/SIMD\n", wps, kind ? "v_exp" : "v_fma",
                       modes[mode], ms, ms * 1e6 / per_simd);
            }
        }
    }
    return 0;
}
