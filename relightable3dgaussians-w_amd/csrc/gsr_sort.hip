// gsr_sort.hip -- stable LSD radix sort of (u32 key, u32 value) pairs, wave64-native.
//
// Replaces cub::DeviceRadixSort::SortPairs (rasterizer_impl.cu:303-308).  The binning
// stage sorts (a) the visible Gaussians by their 32-bit depth key and (b) the
// (tile, gaussian) instances by tile id only -- never the reference's 64-bit keys -- so
// the instance sort needs ceil(log2(T)/8) = 2 passes instead of 6.  Stability of every
// pass gives the reference's total order (tile, depth, gaussian index).
//
// One pass = 3 launches (reduce-then-scan):
//   k_radix_hist    per-tile digit histogram (per-wave LDS counters)
//   k_digit_scan    one workgroup per digit: exclusive scan of that digit's per-tile
//                   counts (contiguous in the digit-major table) + the digit's total
//   k_radix_scatter per-tile stable ranking: each wave ranks its contiguous keys
//                   with 8 ballots per 64-key row (peer masks, leader lane bumps the
//                   per-wave LDS counter), waves combine through LDS, the tile is
//                   reordered in LDS and written out in digit runs (coalesced).
#include "gsr_block.hpp"
#include "gsr_kernels.hpp"
#include "gsr_tile.hpp"

namespace gsr {

constexpr int WAVE_ITEMS = SORT_TILE / 4;  // contiguous keys per wave

// The depth sort's digit width: 4 passes of 8 bits (3 passes of 11 + 11 + 10 bits measured
// slower, profiles/r4r_ab_depth_sort.txt).
constexpr int DEPTH_BITS = 8;

template <int BITS>
__device__ __forceinline__ uint64_t peer_mask(uint32_t d, bool valid) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return valid ? m : 0ull;
}

template <int BITS>
__global__ void __launch_bounds__(SORT_THREADS) k_radix_hist(long long n, const uint32_t* keys, int shift,
                                                               uint32_t mask, uint32_t* hist, int nb) {
    constexpr int NB = 1 << BITS;
    // per-wave LDS sub-histograms (ds_add_u32), keys read 16 B per lane
    __shared__ uint32_t cnt[4][NB];
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4 * NB; i += SORT_THREADS) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const unsigned blk = xcd_remap(blockIdx.x, nb);  // neighbouring tiles' digit runs merge in one L2
    const long long tile_base = (long long)blk * SORT_TILE;
    uint32_t* wc = cnt[wave];
    if (tile_base + SORT_TILE <= n) {
        const uint4* k4 = reinterpret_cast<const uint4*>(keys + tile_base);
#pragma unroll
        for (int r = 0; r < SORT_ITEMS / 4; r++) {
            const uint4 v = k4[r * SORT_THREADS + threadIdx.x];
            atomicAdd(&wc[(v.x >> shift) & mask], 1u);
            atomicAdd(&wc[(v.y >> shift) & mask], 1u);
            atomicAdd(&wc[(v.z >> shift) & mask], 1u);
            atomicAdd(&wc[(v.w >> shift) & mask], 1u);
        }
    } else {
        for (long long i = tile_base + threadIdx.x; i < n; i += SORT_THREADS) atomicAdd(&wc[(keys[i] >> shift) & mask], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < NB; d += SORT_THREADS)
        hist[(long long)d * nb + blk] = cnt[0][d] + cnt[1][d] + cnt[2][d] + cnt[3][d];
}

// hist[d][0..nb) -> exclusive prefix within digit d; digit_tot[d] = the digit's total
// One row in place: each thread owns a contiguous chunk (all its loads in flight at once),
// one block scan of the chunk sums, then the chunk prefixes (one pass instead of one block
// scan per 256 columns: the depth sort's first table has ~6k columns per row at 1.5M keys).
__device__ __forceinline__ void digit_row_scan(uint32_t* h, int ncol, uint32_t* total, uint32_t* sh) {
    constexpr int CH = 32;  // columns per thread per round (8192 per round)
    uint32_t carry = 0;
    for (int c0 = 0; c0 < ncol; c0 += CH * SORT_THREADS) {
        const int b = c0 + threadIdx.x * CH;
        uint32_t v[CH], sum = 0;
#pragma unroll
        for (int k = 0; k < CH; k++) {
            v[k] = b + k < ncol ? h[b + k] : 0u;
            sum += v[k];
        }
        uint32_t tot;
        uint32_t run = carry + block256_exclusive_scan(sum, sh, &tot);
#pragma unroll
        for (int k = 0; k < CH; k++) {
            if (b + k < ncol) h[b + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// Workgroups past the ndig digits zero-fill a slice of `zero` (the depth sort carries the
// backward's gradient accumulators this way: the digit scans are latency-bound launches, and a
// separate memset before the backward's tile pass cost 13 us + a 6 us launch gap).
constexpr int ZERO_F4_PER_THREAD = 8;
__global__ void __launch_bounds__(SORT_THREADS) k_digit_scan(uint32_t* hist, int nb, uint32_t* digit_tot,
                                                             float4* zero = nullptr, long long zero_n4 = 0,
                                                             int ndig = 0x7fffffff) {
    if ((int)blockIdx.x >= ndig) {  // zero-fill workgroups (only the depth sort sets ndig)
        const long long b = (long long)(blockIdx.x - ndig) * SORT_THREADS * ZERO_F4_PER_THREAD + threadIdx.x;
#pragma unroll
        for (int k = 0; k < ZERO_F4_PER_THREAD; k++) {
            const long long i = b + (long long)k * SORT_THREADS;
            if (i < zero_n4) zero[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        return;
    }
    __shared__ uint32_t sh[4];
    digit_row_scan(hist + (long long)blockIdx.x * nb, nb, digit_tot + blockIdx.x, sh);
}

// Exclusive scan over the NB digits of a workgroup, DPT = NB / 256 consecutive digits per
// thread: the values v[0..DPT) of digits threadIdx.x * DPT + j -> their exclusive prefixes.
template <int DPT>
__device__ __forceinline__ void digits_exclusive_scan(uint32_t (&v)[DPT], uint32_t* sh) {
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < DPT; j++) sum += v[j];
    uint32_t run = block256_exclusive_scan(sum, sh, (uint32_t*)nullptr);
#pragma unroll
    for (int j = 0; j < DPT; j++) {
        const uint32_t x = v[j];
        v[j] = run;
        run += x;
    }
}

// AUX: a side payload (the Gaussians' tile rects) moves with every pair, so that the
// depth-sorted order never has to gather it at random afterwards.  PACK: 0 = an 8-byte rect
// (four 16-bit tile bounds) in and out; 1 = 8 bytes in, packed to 4 (four 8-bit bounds,
// pack_rect) on its way into LDS; 2 = 4 bytes in and out.  A grid of at most 255 x 255 tiles (4080
// x 4080 pixels) sorts its rects packed: 12 instead of 16 bytes move per key and pass.
// The offsets table has ocol columns (0: nb) and block blk's column is blk * ostride (the
// preprocess-made first table of the depth sort has 8 columns per 2048-key block).
// (Counting the NEXT pass's histogram here with global atomics per key, instead of the
// separate k_radix_hist, measured 5-15x slower: ~1.5M L2 atomics per pass.)
template <int PACK> struct AuxT { using in = uint2; using out = uint2; };
template <> struct AuxT<1> { using in = uint2; using out = uint32_t; };
template <> struct AuxT<2> { using in = uint32_t; using out = uint32_t; };
__device__ __forceinline__ uint2 aux_cvt(uint2 r, uint2*) { return r; }
__device__ __forceinline__ uint32_t aux_cvt(uint2 r, uint32_t*) { return pack_rect(r); }
__device__ __forceinline__ uint32_t aux_cvt(uint32_t r, uint32_t*) { return r; }

// KOUT false: the sorted keys are not stored (the depth sort's last pass: nothing reads them)
template <bool AUX, int BITS = 8, int PACK = 0, bool KOUT = true>
__global__ void __launch_bounds__(SORT_THREADS) k_radix_scatter(long long n, const uint32_t* keys_in,
                                                                  const uint32_t* vals_in, int shift, uint32_t mask,
                                                                  const uint32_t* offsets, const uint32_t* digit_tot,
                                                                  int nb, uint32_t* keys_out, uint32_t* vals_out,
                                                                  const typename AuxT<PACK>::in* aux_in,
                                                                  typename AuxT<PACK>::out* aux_out, int ocol = 0,
                                                                  int ostride = 1,
                                                                  unsigned long long* pv_out = nullptr) {
    constexpr int NB = 1 << BITS, DPT = NB / SORT_THREADS;
    static_assert(DPT >= 1, "at least one digit per thread");
    using AO = typename AuxT<PACK>::out;
    __shared__ uint32_t s_keys[SORT_TILE];
    __shared__ uint32_t s_vals[SORT_TILE];
    __shared__ AO s_aux[AUX ? SORT_TILE : 1];
    __shared__ uint32_t wh[4][NB];
    __shared__ uint32_t dstart[NB];
    __shared__ uint32_t goff[NB];
    __shared__ uint32_t scan_sh[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * NB; i += SORT_THREADS) (&wh[0][0])[i] = 0;
    __syncthreads();
    const unsigned blk = xcd_remap(blockIdx.x, nb);  // neighbouring tiles' digit runs merge in one L2
    const long long tile_base = (long long)blk * SORT_TILE;
    const long long base = tile_base + wave * WAVE_ITEMS;
    uint32_t key[SORT_ITEMS], val[SORT_ITEMS], rank[SORT_ITEMS];
    // the rects stay as loaded in registers (PACK 1 packs them on their way into LDS: packing at
    // the load would wait for each load before the ranking starts)
    using AI = typename AuxT<PACK>::in;
    AI aux[AUX ? SORT_ITEMS : 1];
    // the leader lanes' read-modify-writes of the per-wave counters: volatile, so a lane never
    // reuses a value another lane has since bumped; typed as LDS, so they are ds_ instructions
    // and not flat ones (a volatile generic pointer compiles to flat_load/flat_store)
    volatile __attribute__((address_space(3))) uint32_t* wc =
        (volatile __attribute__((address_space(3))) uint32_t*)(wh[wave]);
    const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    // all loads first (SORT_ITEMS per lane in flight), then the ranking
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++) {
        const long long i = base + k * 64 + lane;
        key[k] = i < n ? keys_in[i] : 0u;
        val[k] = i < n ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
        if constexpr (AUX) aux[k] = i < n ? aux_in[i] : AI{};
    }
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++) {
        const long long i = base + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (key[k] >> shift) & mask;
        const uint64_t m = peer_mask<BITS>(d, valid);
        const int leader = valid ? (int)(__ffsll((unsigned long long)m) - 1) : lane;
        uint32_t old = 0;
        if (valid && lane == leader) {
            old = wc[d];
            wc[d] = old + (uint32_t)__popcll(m);
        }
        old = __shfl(old, leader, 64);
        rank[k] = old + (uint32_t)__popcll(m & lt);
    }
    __syncthreads();
    {
        // digits d = threadIdx.x * DPT + j: the tile's digit starts and each wave's run start,
        // and the digits' global bases (exclusive scan of the digit totals)
        uint32_t c[4][DPT], st[DPT], gb[DPT];
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            const int d = threadIdx.x * DPT + j;
#pragma unroll
            for (int w = 0; w < 4; w++) c[w][j] = wh[w][d];
            st[j] = c[0][j] + c[1][j] + c[2][j] + c[3][j];
            gb[j] = digit_tot[d];
        }
        digits_exclusive_scan<DPT>(st, scan_sh);
        digits_exclusive_scan<DPT>(gb, scan_sh);
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            const int d = threadIdx.x * DPT + j;
            wh[0][d] = st[j];
            wh[1][d] = st[j] + c[0][j];
            wh[2][d] = st[j] + c[0][j] + c[1][j];
            wh[3][d] = st[j] + c[0][j] + c[1][j] + c[2][j];
            dstart[d] = st[j];
            // the depth sort's top pass: culled keys (0xFFFFFFFF) are exactly its largest digit
            // (mask), so that digit's start is the visible count P_v
            if (pv_out && blockIdx.x == 0 && (uint32_t)d == mask) *pv_out = gb[j];
            goff[d] = gb[j] + offsets[(long long)d * (ocol ? ocol : nb) + (long long)blk * ostride];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++) {
        const long long i = base + k * 64 + lane;
        if (i < n) {
            const uint32_t d = (key[k] >> shift) & mask;
            const uint32_t p = wh[wave][d] + rank[k];
            s_keys[p] = key[k];
            s_vals[p] = val[k];
            if constexpr (AUX) s_aux[p] = aux_cvt(aux[k], (AO*)nullptr);
        }
    }
    __syncthreads();
    const long long count = (n - tile_base) < SORT_TILE ? (n - tile_base) : SORT_TILE;
#pragma unroll
    for (int k = 0; k < SORT_ITEMS; k++) {
        const int p = k * SORT_THREADS + threadIdx.x;
        if (p < count) {
            const uint32_t kk = s_keys[p];
            const uint32_t d = (kk >> shift) & mask;
            const uint32_t g = goff[d] + (uint32_t)(p - dstart[d]);
            if constexpr (KOUT) keys_out[g] = kk;
            vals_out[g] = s_vals[p];
            if constexpr (AUX) aux_out[g] = s_aux[p];
        }
    }
}

void launch_digit_scan(int ndigits, uint32_t* table, int nb, uint32_t* digit_tot, hipStream_t s) {
    hipLaunchKernelGGL(k_digit_scan, dim3(ndigits), dim3(SORT_THREADS), 0, s, table, nb, digit_tot);
}

size_t radix_sort_temp_bytes(long long n) {
    const long long nb = sort_blocks(n);
    const long long h = 256 * nb;
    return (size_t)(4 * (h + 256) + 256);
}

int radix_sort_pairs_from(long long n, const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys,
                          uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, int end_bit, void* temp,
                          hipStream_t s, const uint2* aux_in, uint2* aux, uint2* aux_alt) {
    if (n <= 0 || end_bit <= 0) return -1;
    const int nb = sort_blocks(n);
    uint32_t* hist = reinterpret_cast<uint32_t*>(temp);
    uint32_t* digit_tot = hist + 256LL * nb;
    const uint32_t* kin = keys_in;
    const uint32_t* vin = vals_in;
    uint32_t* out_k[2] = {keys, keys_alt};
    uint32_t* out_v[2] = {vals, vals_alt};
    const uint2* ain = aux_in;
    uint2* out_a[2] = {aux, aux_alt};
    int cur = 0;
    for (int shift = 0; shift < end_bit; shift += 8) {
        const int nbits = (end_bit - shift) < 8 ? (end_bit - shift) : 8;
        const uint32_t mask = (1u << nbits) - 1u;
        hipLaunchKernelGGL(k_radix_hist<8>, dim3(nb), dim3(SORT_THREADS), 0, s, n, kin, shift, mask, hist, nb);
        hipLaunchKernelGGL(k_digit_scan, dim3(256), dim3(SORT_THREADS), 0, s, hist, nb, digit_tot);
        if (ain) {
            hipLaunchKernelGGL(k_radix_scatter<true>, dim3(nb), dim3(SORT_THREADS), 0, s, n, kin, vin, shift, mask,
                               hist, digit_tot, nb, out_k[cur], out_v[cur], ain, out_a[cur]);
            ain = out_a[cur];
        } else {
            hipLaunchKernelGGL(k_radix_scatter<false>, dim3(nb), dim3(SORT_THREADS), 0, s, n, kin, vin, shift, mask,
                               hist, digit_tot, nb, out_k[cur], out_v[cur], nullptr, nullptr);
        }
        kin = out_k[cur];
        vin = out_v[cur];
        cur ^= 1;
    }
    return cur ^ 1;  // the buffer pair written last
}

size_t depth_sort_temp_bytes(long long P) {
    const size_t nb = (size_t)sort_blocks(P), NB = (size_t)1 << DEPTH_BITS;
    return 4 * (NB * nb + NB) + 256;
}

int depth_sort(long long P, const uint32_t* keys_in, uint32_t* keys, uint32_t* vals, uint32_t* keys_alt,
               uint32_t* vals_alt, const uint2* aux_in, uint2* aux, uint2* aux_alt, void* temp,
               unsigned long long* pv_out, hipStream_t s, void* zero, size_t zero_bytes, bool pack) {
    if (P <= 0) return -1;
    constexpr int BITS = DEPTH_BITS, NB = 1 << BITS, NPASS = (32 + BITS - 1) / BITS;
    const int nb = sort_blocks(P);
    uint32_t* hist = reinterpret_cast<uint32_t*>(temp);
    uint32_t* digit_tot = hist + (long long)NB * nb;
    const uint32_t* kin = keys_in;
    const uint32_t* vin = nullptr;  // values 0..P-1
    uint32_t* out_k[2] = {keys, keys_alt};
    uint32_t* out_v[2] = {vals, vals_alt};
    const uint2* ain = aux_in;
    uint2* out_a[2] = {aux, aux_alt};
    int cur = 0;
    for (int pass = 0; pass < NPASS; pass++) {
        const int shift = BITS * pass;
        const int nbits = 32 - shift < BITS ? 32 - shift : BITS;
        const uint32_t mask = (nbits >= 32) ? 0xFFFFFFFFu : ((1u << nbits) - 1u);
        hipLaunchKernelGGL(k_radix_hist<BITS>, dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, shift, mask, hist, nb);
        // a share of the zero-fill (16-B multiples) rides in each pass's digit scan
        const long long n4 = (long long)(zero ? zero_bytes / 16 : 0);
        const long long q0 = n4 * pass / NPASS, q1 = n4 * (pass + 1) / NPASS;
        const long long per_blk = (long long)SORT_THREADS * ZERO_F4_PER_THREAD;
        const unsigned zb = (unsigned)((q1 - q0 + per_blk - 1) / per_blk);
        hipLaunchKernelGGL(k_digit_scan, dim3(NB + zb), dim3(SORT_THREADS), 0, s, hist, nb, digit_tot,
                           zb ? reinterpret_cast<float4*>(zero) + q0 : (float4*)nullptr, q1 - q0, NB);
        const bool lastp = pass == NPASS - 1;
        unsigned long long* pv = lastp ? pv_out : (unsigned long long*)nullptr;
        if (!pack && lastp)
            hipLaunchKernelGGL((k_radix_scatter<true, BITS, 0, false>), dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, vin,
                               shift, mask, hist, digit_tot, nb, out_k[cur], out_v[cur], ain, out_a[cur], 0, 1, pv);
        else if (!pack)
            hipLaunchKernelGGL((k_radix_scatter<true, BITS, 0>), dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, vin, shift,
                               mask, hist, digit_tot, nb, out_k[cur], out_v[cur], ain, out_a[cur], 0, 1, pv);
        else if (pass == 0)  // the packed rects (4 B) in the first half of each 8-B buffer
            hipLaunchKernelGGL((k_radix_scatter<true, BITS, 1>), dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, vin, shift,
                               mask, hist, digit_tot, nb, out_k[cur], out_v[cur], ain,
                               reinterpret_cast<uint32_t*>(out_a[cur]), 0, 1, pv);
        else if (lastp)
            hipLaunchKernelGGL((k_radix_scatter<true, BITS, 2, false>), dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, vin,
                               shift, mask, hist, digit_tot, nb, out_k[cur], out_v[cur],
                               reinterpret_cast<const uint32_t*>(ain), reinterpret_cast<uint32_t*>(out_a[cur]), 0, 1, pv);
        else
            hipLaunchKernelGGL((k_radix_scatter<true, BITS, 2>), dim3(nb), dim3(SORT_THREADS), 0, s, P, kin, vin, shift,
                               mask, hist, digit_tot, nb, out_k[cur], out_v[cur], reinterpret_cast<const uint32_t*>(ain),
                               reinterpret_cast<uint32_t*>(out_a[cur]), 0, 1, pv);
        ain = out_a[cur];
        kin = out_k[cur];
        vin = out_v[cur];
        cur ^= 1;
    }
    return cur ^ 1;
}

int radix_sort_pairs(long long n, uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                     int end_bit, void* temp, hipStream_t s) {
    if (n <= 1 || end_bit <= 0) return 0;
    // first pass reads (keys, vals) and writes the alt pair, then they alternate
    return radix_sort_pairs_from(n, keys, vals, keys_alt, vals_alt, keys, vals, end_bit, temp, s) ^ 1;
}

}  // namespace gsr
