// sort_probe.cpp -- the depth sort (gsr::depth_sort, libgsr.so) on its own against std::stable_sort:
// random float depth keys with a share of culled keys (0xFFFFFFFF), the rect payload moving along
// (8-B and packed 4-B), P_v, every sorted id and payload word compared.  Diagnostic tool, not the product.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/sort_probe.cpp -I relightable3dgaussians-w_amd/csrc \
//       -L relightable3dgaussians-w_amd/lib -lgsr -Wl,-rpath,'$ORIGIN/../relightable3dgaussians-w_amd/lib' \
//       -o tools/sort_probe && tools/sort_probe 1000 100000 1500000
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "gsr_kernels.hpp"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

static int run(long long P, unsigned seed, bool pack, int reps) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> depth(0.2f, 80.f);
    std::vector<uint32_t> keys(P);
    std::vector<uint2> rect(P);
    for (long long i = 0; i < P; i++) {
        const bool culled = (rng() % 10) == 0;
        float z = depth(rng);
        if (rng() % 7 == 0) z = 5.0f;  // ties: stability shows
        uint32_t k;
        memcpy(&k, &z, 4);
        keys[i] = culled ? 0xFFFFFFFFu : k;
        const uint32_t x0 = rng() % 200, y0 = rng() % 200;
        rect[i] = make_uint2(x0 | ((x0 + 1 + rng() % 50) << 16), y0 | ((y0 + 1 + rng() % 50) << 16));
    }
    std::vector<uint32_t> order(P);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
    const long long pv_ref = std::count_if(keys.begin(), keys.end(), [](uint32_t k) { return k != 0xFFFFFFFFu; });

    uint32_t *dk, *k0, *v0, *k1, *v1;
    uint2 *dr, *a0, *a1;
    void* tmp;
    unsigned long long* pv;
    CK(hipMalloc(&dk, 4 * P));
    CK(hipMalloc(&k0, 4 * P));
    CK(hipMalloc(&v0, 4 * P));
    CK(hipMalloc(&k1, 4 * P));
    CK(hipMalloc(&v1, 4 * P));
    CK(hipMalloc(&dr, 8 * P));
    CK(hipMalloc(&a0, 8 * P));
    CK(hipMalloc(&a1, 8 * P));
    const size_t tb = gsr::depth_sort_temp_bytes(P);
    CK(hipMalloc(&tmp, tb));
    CK(hipMalloc(&pv, 8));
    CK(hipMemcpy(dk, keys.data(), 4 * P, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, rect.data(), 8 * P, hipMemcpyHostToDevice));
    int bad = 0;
    for (int r = 0; r < reps; r++) {
        CK(hipMemset(tmp, 0xAB, tb));  // the scratch starts as garbage
        CK(hipMemset(pv, 0xFF, 8));
        const int flip = gsr::depth_sort(P, dk, k0, v0, k1, v1, dr, a0, a1, tmp, pv, nullptr, nullptr, 0, pack);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> gk(P), gv(P);
        std::vector<uint2> ga(P);
        CK(hipMemcpy(gk.data(), flip ? k1 : k0, 4 * P, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gv.data(), flip ? v1 : v0, 4 * P, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ga.data(), flip ? a1 : a0, 8 * P, hipMemcpyDeviceToHost));
        unsigned long long gpv = 0;
        CK(hipMemcpy(&gpv, pv, 8, hipMemcpyDeviceToHost));
        long long nbad = 0, first = -1;
        for (long long i = 0; i < P; i++) {
            const uint32_t id = order[i];
            bool ok = gv[i] == id;  // (the last pass does not store the sorted keys)
            if (pack) ok = ok && reinterpret_cast<uint32_t*>(ga.data())[i] == gsr::pack_rect(rect[id]);
            else ok = ok && ga[i].x == rect[id].x && ga[i].y == rect[id].y;
            if (!ok) {
                if (first < 0) first = i;
                nbad++;
            }
        }
        printf("P=%lld pack=%d rep=%d: %lld wrong (first at %lld), P_v %llu (want %lld)\n", P, (int)pack, r, nbad,
               first, gpv, pv_ref);
        if (nbad || (long long)gpv != pv_ref) {
            bad = 1;
            if (first >= 0)
                printf("  at %lld: got id %u, want id %u (key %08x)\n", first, gv[first], order[first],
                       keys[order[first]]);
        }
    }
    hipFree(dk); hipFree(k0); hipFree(v0); hipFree(k1); hipFree(v1); hipFree(dr); hipFree(a0); hipFree(a1);
    hipFree(tmp); hipFree(pv);
    return bad;
}

int main(int argc, char** argv) {
    int bad = 0;
    for (int i = 1; i < argc; i++) {
        const long long P = atoll(argv[i]);
        bad |= run(P, 1234u + i, false, 2);
        bad |= run(P, 99u + i, true, 2);
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad;
}
