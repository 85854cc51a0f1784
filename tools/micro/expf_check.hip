// gsr_tile.hpp glibc_expf and ref_power on the GPU against the host libm / float arithmetic:
//   hipcc --offload-arch=gfx950 -O3 -I relightable3dgaussians-w_amd/csrc tools/micro/expf_check.hip -o /tmp/expf_check
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include "gsr_tile.hpp"
using namespace gsr;
__global__ void k_expf(const float* x, float* y, long long n) {
    __shared__ unsigned long long tab[32];
    gexp_table_init(tab);
    __syncthreads();
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        y[i] = glibc_expf(x[i], tab);
}
__global__ void k_power(const float* a, float* out, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        out[i] = ref_power(a[5 * i], a[5 * i + 1], a[5 * i + 2], a[5 * i + 3], a[5 * i + 4]);
}
int main() {
    const long long n = 1 << 26;
    std::vector<float> x(n), y(n);
    unsigned s = 12345;
    for (long long i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        x[i] = -12.0f * (float)(s >> 8) / 16777216.0f;
    }
    float *dx, *dy;
    hipMalloc(&dx, n * 4);
    hipMalloc(&dy, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_expf, dim3(4096), dim3(256), 0, 0, dx, dy, n);
    hipMemcpy(y.data(), dy, n * 4, hipMemcpyDeviceToHost);
    long long bad = 0;
    for (long long i = 0; i < n; i++) {
        const float r = expf(x[i]);
        if (memcmp(&r, &y[i], 4)) { if (bad < 5) printf("expf %a host %a gpu %a\n", x[i], r, y[i]); bad++; }
    }
    printf("expf: %lld / %lld differ\n", bad, n);
    // ref_power on random conics and offsets
    std::vector<float> a(5 * n), p(n);
    for (long long i = 0; i < 5 * n; i++) {
        s = s * 1664525u + 1013904223u;
        a[i] = (float)(s >> 8) / 16777216.0f * ((i % 5) >= 3 ? 40.0f : 0.5f) - ((i % 5) >= 3 ? 20.0f : (i % 5 == 1 ? 0.25f : 0.f));
    }
    float* da;
    hipMalloc(&da, 5 * n * 4);
    hipMemcpy(da, a.data(), 5 * n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_power, dim3(4096), dim3(256), 0, 0, da, dy, n);
    hipMemcpy(p.data(), dy, n * 4, hipMemcpyDeviceToHost);
    bad = 0;
    for (long long i = 0; i < n; i++) {
        volatile float A = a[5 * i], B = a[5 * i + 1], Cc = a[5 * i + 2], X = a[5 * i + 3], Y = a[5 * i + 4];
        volatile float t1 = A * X; volatile float t2 = t1 * X; volatile float t3 = Cc * Y; volatile float t4 = t3 * Y;
        volatile float t5 = t2 + t4; volatile float t6 = -0.5f * t5; volatile float t7 = B * X; volatile float t8 = t7 * Y;
        const float r = t6 - t8;
        if (memcmp(&r, &p[i], 4)) { if (bad < 5) printf("power host %a gpu %a\n", r, p[i]); bad++; }
    }
    printf("ref_power: %lld / %lld differ\n", bad, n);
    return 0;
}
