// gsr_capi.cpp -- C ABI (include/gsr.h): buffer layout and stage orchestration of the
// forward / backward rasterizer (rasterizer_impl.cu:198-433 re-designed):
//
//   forward:  preprocess (+ P_v, R, S totals) -> depth sort of all P -> ONE D2H sync
//             -> depth sort of the P_v visible Gaussians (32-bit keys, 4 passes)
//             -> depth-order exclusive scan of tiles_touched -> instance emission
//             -> stable tile-id sort of the R instances (ceil(log2 T / 8) passes)
//             -> tile ranges -> LDS-staged tile compositing
//   backward: zero the per-Gaussian accumulator -> tile replay -> fused per-Gaussian
//             cov2D / projection / SH / cov3D backward writing all nine outputs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#ifdef GSR_WITH_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

#include "gsr_kernels.hpp"
#include "gsr_shade.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace

int gsr_fail_hip(hipError_t e, int line) {
    return fail(GSR_E_HIP, "HIP error %d (%s) at gsr_capi.cpp:%d", (int)e, hipGetErrorString(e), line);
}

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

struct Carver {
    size_t o = 0;
    size_t take(size_t bytes) {
        const size_t r = o;
        o = align_up(o + bytes, 256);
        return r;
    }
};

struct GeomLayout {
    size_t tot_dev, blk_tot, radii, tiles, st_count, depth_key, rect, rec, acc, shjac, vis_key, vis_val, vis_key_alt, vis_val_alt, rect_s, rect_s_alt,
        offsets, scan_tmp, sort_tmp, total;
};
struct ImgLayout {
    size_t final_T, n_contrib, ranges, tile_nmax, tile_emax, tile_cost, row_cost, order_fwd, order_bwd, nheavy, surv_n,
        surv, total;
};
// The binning buffer: a header (S), the super-tile ranges and entries at offsets independent of
// S (all the backward needs), then the forward's binning scratch.
struct BinLayout {
    size_t header, st_ranges, ent, st_keys, st_vals, st_keys_alt, st_vals_alt, sort_tmp, st_bin_tmp, total;
};

GeomLayout geom_layout(long long P) {
    Carver c;
    GeomLayout L;
    L.tot_dev = c.take(8 * 4);                                // P_v, R, S, error flag
    L.blk_tot = c.take(16 * (size_t)gsr::pre_blocks(P));      // per preprocess workgroup
    L.radii = c.take(4 * P);
    L.tiles = c.take(4 * P);
    L.st_count = c.take(4 * P);
    L.depth_key = c.take(4 * P);
    L.rect = c.take(8 * P);
    L.rec = c.take(sizeof(gsr::Rec) * P);
    L.acc = c.take(4 * gsr::ACC_STRIDE * P);
    L.shjac = c.take(4 * (size_t)gsr::SHJAC_ROWS * P);  // SH path: the forward's Jacobian for the backward
    L.vis_key = c.take(4 * P);
    L.vis_val = c.take(4 * P);
    L.vis_key_alt = c.take(4 * P);
    L.vis_val_alt = c.take(4 * P);
    L.rect_s = c.take(8 * P);
    L.rect_s_alt = c.take(8 * P);
    L.offsets = c.take(4 * P);
    L.scan_tmp = c.take(24 * (size_t)gsr::scan_blocks(P) + 16);
    L.sort_tmp = c.take(gsr::depth_sort_temp_bytes(P));
    L.total = c.o + 256;
    return L;
}

unsigned tiles_x(int W) { return (unsigned)((W + GSR_BLOCK_X - 1) / GSR_BLOCK_X); }
unsigned tiles_y(int H) { return (unsigned)((H + GSR_BLOCK_Y - 1) / GSR_BLOCK_Y); }

constexpr int FWD_NHEAVY = 40;  // the forward's band table within the image buffer's nheavy words
static_assert(FWD_NHEAVY == 8 + 32, "the backward (table at 8) reads the forward's band costs 32 words on (gsr_tile.hpp BWD_ROT_COST)");

// surv: reserve the survivor lists (the forward stores them: surv_on()).  They sit last, so every
// other offset (and the lists' own) is the same either way: a backward over a buffer made without
// them finds every tile's count SURV_NONE (the forward's order sets it) and never reads the lists.
ImgLayout img_layout(int W, int H, bool surv) {
    Carver c;
    ImgLayout L;
    const size_t N = (size_t)W * H;
    const size_t T = (size_t)tiles_x(W) * tiles_y(H);
    L.final_T = c.take(4 * N);
    L.n_contrib = c.take(4 * N);
    L.ranges = c.take(8 * T);  // the reference's tile ranges: filled only by the list materialisation
    L.tile_nmax = c.take(4 * T);
    L.tile_emax = c.take(4 * T);
    L.tile_cost = c.take(4 * T);  // the backward's cost estimate: (survivor, quadrant) evaluations
    L.row_cost = c.take(4 * (size_t)tiles_y(H));  // the same per tile row (the backward's balanced bands)
    L.order_fwd = c.take(4 * T);
    L.order_bwd = c.take(4 * T);
    // two band tables of 40 words, the backward's at 8 and the forward's at 40 (FWD_NHEAVY), each
    // (relative to its start): heavy counts [0..8), balanced bounds [8..17), band costs [24..32)
    L.nheavy = c.take(4 * 80);
    L.surv_n = c.take(4 * T);
    // the forward's survivor lists for the backward (RenderFwdArgs::surv): 8 B x SURV_CAP per tile,
    // written only as far as each tile's survivors reach (cfg2: ~1.4 KB of the 8 KB)
    L.surv = c.take(surv ? 8 * (size_t)gsr::SURV_CAP * T : 0);
    L.total = c.o + 256;
    return L;
}

unsigned st_x(int W) { return (tiles_x(W) + GSR_ST_W - 1) / GSR_ST_W; }
unsigned st_h(int W, int H) { return gsr::st_sth(tiles_x(W), tiles_y(H)); }  // log2 super-tile height
unsigned st_y(int W, int H) {
    const unsigned sth = st_h(W, H);
    return (tiles_y(H) + (1u << sth) - 1) >> sth;
}

// capS: the entry capacity (0: the fixed part only, as the backward computes it)
BinLayout bin_layout(long long capS, int W, int H, long long Pv) {
    Carver c;
    BinLayout L;
    const size_t NS = (size_t)st_x(W) * st_y(W, H);
    const bool fused = gsr::st_bin_supported((int)NS);
    L.header = c.take(16);
    L.st_ranges = c.take(8 * NS);
    L.ent = c.take(8 * (capS + 64));  // + slack: the tile passes' list loads read up to one entry past a range
    // emit + sort path for very large images (NS > 1365 super-tiles)
    L.st_keys = c.take(fused ? 0 : 4 * capS);
    L.st_vals = c.take(fused ? 0 : 4 * capS);
    L.st_keys_alt = c.take(fused ? 0 : 4 * capS);
    L.st_vals_alt = c.take(fused ? 0 : 4 * capS);
    L.sort_tmp = c.take(fused ? 0 : gsr::radix_sort_temp_bytes(capS));
    L.st_bin_tmp = c.take(fused ? gsr::st_bin_temp_bytes(Pv, (int)NS) : 0);
    L.total = c.o + 256;
    return L;
}

// rasterizer_impl.cu:35-50
uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

template <typename T>
T* at(void* base, size_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

char* align_base(void* p) { return reinterpret_cast<char*>(align_up(reinterpret_cast<size_t>(p), 256)); }

// Host-mapped, coherent: the depth sort's first histogram launch stores the frame totals
// in p[0..3], each tagged with the call's sequence number (gsr_sort.hip frame_totals).
struct PinnedHost {
    unsigned long long* p = nullptr;
    unsigned long long* p_dev = nullptr;  // its device address
    unsigned long long seq = 0;
    ~PinnedHost() {
        if (p) (void)hipHostFree(p);
    }
};
thread_local PinnedHost g_pinned;
// the previous forward's counts on this thread: the next call with the same P and image
// size sizes its binning buffer from them before the host synchronisation
struct BinHint {
    int P = -1, W = 0, H = 0;
    long long R = 0, S = 0;
};
thread_local BinHint g_hint;

// Geometry buffers whose gradient accumulators the forward zeroed (in the depth sort's digit
// scans) and no backward has used yet: the backward skips its zero-fill for them.  A second
// backward over the same forward, or a geometry buffer made by gsr_forward_reuse, zero-fills.
std::mutex g_zeroed_mu;
std::unordered_set<const void*> g_zeroed;
void zeroed_set(const void* geom, bool on) {
    std::lock_guard<std::mutex> lk(g_zeroed_mu);
    if (on) {
        // forwards without a backward (inference) leave entries behind: bounded, since a
        // forgotten entry only costs a backward its zero-fill
        if (g_zeroed.size() >= 4096) g_zeroed.clear();
        g_zeroed.insert(geom);
    } else {
        g_zeroed.erase(geom);
    }
}
bool zeroed_take(const void* geom) {
    std::lock_guard<std::mutex> lk(g_zeroed_mu);
    return g_zeroed.erase(geom) > 0;
}

// Deterministic backward (gsr_set_deterministic / GSR_DETERMINISTIC=1): per-instance partial
// rows summed in a fixed order (gsr_det.hip) instead of the tile passes' atomics.
std::atomic<int> g_det{-1};
bool det_on() {
    int v = g_det.load();
    if (v < 0) {
        const char* e = getenv("GSR_DETERMINISTIC");
        v = (e && e[0] && e[0] != '0') ? 1 : 0;
        g_det.store(v);
    }
    return v != 0;
}
// The forward's survivor lists for the backward (gsr_set_survivor_lists / GSR_SURV_LISTS=0 to
// turn off; on by default in builds with SURV_CAP > 0)
std::atomic<int> g_surv{-1};
bool surv_on() {
    int v = g_surv.load();
    if (v < 0) {
        const char* e = getenv("GSR_SURV_LISTS");
        v = (e && e[0] == '0') ? 0 : 1;
        g_surv.store(v);
    }
    return gsr::SURV_CAP > 0 && v != 0;
}
// Exact blend mode (gsr_set_exact_blend / GSR_EXACT_BLEND=1; gsr_tile.hpp "exact mode"): the tile
// passes evaluate every pair with the reference's float arithmetic bit for bit.  Each forward records
// its mode against its image buffer, so its backward (and a geometry-cache forward over the same
// buffers) replays the same arithmetic whatever the switch says by then.
std::atomic<int> g_exact{-1};
bool exact_on() {
    int v = g_exact.load();
    if (v < 0) {
        const char* e = getenv("GSR_EXACT_BLEND");
        v = (e && e[0] && e[0] != '0') ? 1 : 0;
        g_exact.store(v);
    }
    return v != 0;
}
std::mutex g_exact_mu;
std::unordered_set<const void*> g_exact_imgs;
void exact_set(const void* img, bool on) {
    std::lock_guard<std::mutex> lk(g_exact_mu);
    if (on) {
        if (g_exact_imgs.size() >= 65536) g_exact_imgs.clear();  // (far beyond any live set of buffers)
        g_exact_imgs.insert(img);
    } else {
        g_exact_imgs.erase(img);
    }
}
bool exact_get(const void* img) {
    std::lock_guard<std::mutex> lk(g_exact_mu);
    return g_exact_imgs.count(img) > 0;
}
// grow-only device scratch of one thread (the deterministic rows, the debug checks); the
// calls that use it synchronise their stream before returning, so it is free again
struct Scratch {
    void* p = nullptr;
    size_t n = 0;
    ~Scratch() {
        if (p) (void)hipFree(p);
    }
    void* get(size_t bytes) {
        if (bytes > n) {
            if (p) (void)hipFree(p);
            p = nullptr;
            n = 0;
            if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
            n = bytes;
        }
        return p;
    }
};
thread_local Scratch g_scratch;   // deterministic rows
thread_local Scratch g_scratch2;  // list materialisation, debug checks

// Wait until the device has stored the four totals of call `seq` (frame_totals: each word is
// value << 16 | seq mod 2^16) and unpack them into out[0..3].  Spins on the coherent
// host-mapped words; every 256 polls the stream is queried, so a failed or finished stream
// ends the wait (a finished stream must have stored them: the words are read once more after
// the query, since they may have landed between the last read and the query).
int wait_totals(const unsigned long long* p, unsigned long long seq, hipStream_t s, unsigned long long* out) {
    const unsigned long long tag = seq & 0xFFFFull;
    auto read = [&]() {
        bool ok = true;
        for (int k = 0; k < 4; k++) {
            const unsigned long long w = __atomic_load_n(p + k, __ATOMIC_ACQUIRE);
            ok = ok && (w & 0xFFFFull) == tag;
            out[k] = w >> 16;
        }
        return ok;
    };
    for (unsigned it = 1;; it++) {
        if (read()) return 0;
        if ((it & 255u) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipSuccess && q != hipErrorNotReady) return gsr_fail_hip(q, __LINE__);
            if (q == hipSuccess) {
                if (read()) return 0;
                return gsr_fail_hip(hipErrorUnknown, __LINE__);  // the stream is done and stored no totals
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

#define HIP_OK(x)                                              \
    do {                                                       \
        hipError_t _e = (x);                                   \
        if (_e != hipSuccess) return gsr_fail_hip(_e, __LINE__); \
    } while (0)

// ---- stage profiling: hipEvents recorded on the call's stream around each stage ----------
enum Stage {
    ST_PREPROCESS, ST_COMPACT, ST_DEPTH_SORT, ST_OFFSETS, ST_DUPLICATE, ST_TILE_SORT, ST_RANGES, ST_RENDER_FWD,
    ST_BWD_ZERO, ST_RENDER_BWD, ST_PREPROCESS_BWD, ST_SHADE_FWD, ST_SHADE_BWD, ST_RENDER_FWD_MC, ST_RENDER_BWD_MC,
    ST_COUNT
};
// render_fwd_mc / render_bwd_mc: the multi-channel composite's tile-pass launches alone (inside
// render_fwd / render_bwd, which also hold the backward's tile order), for the training leg's
// live launch times (bench.py)
const char* kStageNames[ST_COUNT] = {"preprocess",  "compact",      "depth_sort",     "offsets_scan", "st_emit",
                                     "st_sort",     "tile_order",       "render_fwd",     "bwd_zero",     "render_bwd",
                                     "preprocess_bwd", "shade_fwd", "shade_bwd", "render_fwd_mc", "render_bwd_mc"};
// Forward calls run on the Python thread and backward calls on autograd's device thread,
// so the pending list and the event pool are guarded by one mutex.
struct Prof {
    std::mutex mu;
    bool on = false;
    unsigned mask = ~0u;  // stages timed while on (gsr_profile_stages)
    std::vector<hipEvent_t> pool;
    struct Rec { hipEvent_t a, b; int stage; };
    std::vector<Rec> pending;
    double ms[ST_COUNT] = {0};
    long long n[ST_COUNT] = {0};
    hipEvent_t get() {
        std::lock_guard<std::mutex> lk(mu);
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
};
Prof g_prof;

// roctx ranges: with GSR_ROCTX=1 in the environment, every stage is also a named
// range ("gsr:<stage>") for external rocprofv3 --marker-trace timelines of the reference's own
// train.py on this path.  Builds without rocprofiler-sdk (make ROCTX=0) have no ranges.
static bool roctx_on() {
#ifdef GSR_WITH_ROCTX
    static const bool on = [] {
        const char* e = getenv("GSR_ROCTX");
        return e && e[0] && e[0] != '0';
    }();
    return on;
#else
    return false;
#endif
}
extern const char* kStageNames[];
struct StageTimer {
    hipEvent_t a = nullptr;
    int stage;
    hipStream_t s;
    bool rx = false;
    StageTimer(int st, hipStream_t ss) : stage(st), s(ss) {
        if (roctx_on()) {
            static const std::vector<std::string> names = [] {
                std::vector<std::string> v;
                for (int i = 0; i < ST_COUNT; i++) v.push_back(std::string("gsr:") + kStageNames[i]);
                return v;
            }();
#ifdef GSR_WITH_ROCTX
            roctxRangePushA(names[st].c_str());
            rx = true;
#endif
        }
        if (g_prof.on && ((g_prof.mask >> st) & 1u)) { a = g_prof.get(); (void)hipEventRecord(a, s); }
    }
    ~StageTimer() {
#ifdef GSR_WITH_ROCTX
        if (rx) roctxRangePop();
#endif
        if (a) {
            hipEvent_t b = g_prof.get();
            (void)hipEventRecord(b, s);
            std::lock_guard<std::mutex> lk(g_prof.mu);
            g_prof.pending.push_back({a, b, stage});
        }
    }
};
#define GSR_STAGE(st) StageTimer _timer_##st(st, s)


const char* debug_code_name(unsigned c) {
    static const char* names[] = {"ok", "tile range outside [0, R)", "listed id >= P", "listed Gaussian is culled",
                                  "tile outside the listed Gaussian's rect", "list not in (depth, index) order",
                                  "Gaussian not listed exactly area(rect) times", "range lengths do not sum to R",
                                  "n_contrib exceeds the tile's list"};
    return c < sizeof(names) / sizeof(names[0]) ? names[c] : "unknown";
}

// The reference's point_list [R] and tile ranges [T] from a forward's super-tile lists
// (synchronous: reads S from the binning buffer's header).  out_pl / out_ranges: device
// buffers of R and T entries; scratch from g_scratch2 beyond `keep` bytes.
int materialize_lists(long long R, int W, int H, const char* bin, uint32_t* out_pl, uint2* out_ranges, hipStream_t s) {
    const BinLayout bl = bin_layout(0, W, H, 0);
    unsigned long long S = 0;
    HIP_OK(hipMemcpyAsync(&S, bin + bl.header, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    const unsigned gx = tiles_x(W), gy = tiles_y(H), gsx = st_x(W);
    const int NS = (int)(st_x(W) * st_y(W, H)), T = (int)(gx * gy);
    void* tmp = g_scratch2.get(gsr::materialize_temp_bytes((long long)S, NS, T));
    if (!tmp) return fail(GSR_E_ALLOC, "list materialisation: scratch allocation failed");
    gsr::launch_materialize((long long)S, NS, reinterpret_cast<const uint2*>(bin + bl.st_ranges),
                            reinterpret_cast<const uint2*>(bin + bl.ent), gx, gy, gsx, tmp, out_pl, out_ranges, R, s);
    GSR_LAUNCH_CHECK();
    HIP_OK(hipStreamSynchronize(s));
    return GSR_OK;
}

// GSR_DEBUG: verify the forward's tile lists (materialised) and n_contrib (gsr_det.hip),
// synchronously
int debug_check_forward(int P, long long R, unsigned gx, unsigned gy, int W, int H, const int* radii, const uint2* rect,
                        const uint32_t* depth_key, const char* bin, const uint32_t* n_contrib, hipStream_t s) {
    const size_t T = (size_t)gx * gy;
    const size_t off_pl = 256 + 4 * (size_t)P, off_rg = off_pl + ((4 * (size_t)R + 255) & ~(size_t)255);
    const size_t bytes = off_rg + 8 * T + 256;
    // the report, counters and lists in g_scratch; materialisation scratch in g_scratch2
    char* sc = reinterpret_cast<char*>(g_scratch.get(bytes));
    if (!sc) return fail(GSR_E_ALLOC, "GSR_DEBUG: scratch allocation failed");
    uint32_t* pl = reinterpret_cast<uint32_t*>(sc + off_pl);
    uint2* ranges = reinterpret_cast<uint2*>(sc + off_rg);
    if (R > 0 && bin) {
        const int rc = materialize_lists(R, W, H, bin, pl, ranges, s);
        if (rc != GSR_OK) return rc;
    } else {
        HIP_OK(hipMemsetAsync(ranges, 0, 8 * T, s));
    }
    HIP_OK(hipMemsetAsync(sc, 0, off_pl, s));
    auto* rep = reinterpret_cast<gsr::DebugReport*>(sc);
    gsr::launch_check_lists(P, R, gx, gy, W, H, radii, rect, depth_key, ranges, pl, n_contrib,
                            reinterpret_cast<uint32_t*>(sc + 256), reinterpret_cast<unsigned long long*>(sc + 64), rep, s);
    GSR_LAUNCH_CHECK();
    gsr::DebugReport h{};
    HIP_OK(hipMemcpyAsync(&h, rep, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (h.code)
        return fail(GSR_E_DEVICE_CHECK, "GSR_DEBUG check failed: %s (%u, %u, %u)", debug_code_name(h.code), h.a, h.b, h.c);
    return GSR_OK;
}
}  // namespace

namespace {
// Multi-channel composite (gsr_render_mc.hip): nch feature channels per Gaussian, rows of
// fstride floats (a multiple of 4); composited in groups of MC_GROUP channels.
struct McSpec {
    int nch, fstride;
    const float* features;
    const float* bg;     // [nch]
    float* out;          // forward: [nch][H][W]
    const float* dL_dout;  // backward: [nch][H][W]
    float* dL_dfeat;       // backward: [P][fstride]
};
constexpr int MC_GROUP = 16;

gsr::RenderMcArgs mc_args(int W, int H, unsigned gx, unsigned gy, unsigned gsx, const uint2* st_ranges, const uint2* ent,
                          const gsr::Rec* rec, const uint32_t* order, const uint32_t* nheavy, uint32_t* tile_nmax,
                          uint32_t* tile_emax, const McSpec& mc, int c0) {
    gsr::RenderMcArgs m{};
    m.W = W; m.H = H; m.grid_x = gx; m.grid_y = gy;
    m.st_ranges = st_ranges; m.ent = ent; m.gsx = gsx; m.rec = rec;
    m.tile_nmax = tile_nmax; m.tile_emax = tile_emax;
    m.feat = reinterpret_cast<const float4*>(mc.features + c0);
    m.fstride4 = mc.fstride / 4;
    m.fstride = mc.fstride;
    m.nch = std::min(MC_GROUP, mc.nch - c0);
    m.bg = mc.bg + c0;
    m.order = order;
    m.nheavy = nheavy;
    return m;
}
}  // namespace

extern "C" {

const char* gsr_last_error(void) { return g_err.c_str(); }

const char* gsr_version(void) { return "gsr 0.1 gfx950"; }

int gsr_set_deterministic(int on) {
    g_det.store(on ? 1 : 0);
    return GSR_OK;
}

int gsr_get_deterministic(void) { return det_on() ? 1 : 0; }
int gsr_set_survivor_lists(int on) {
    g_surv.store(on ? 1 : 0);
    return GSR_OK;
}
int gsr_get_survivor_lists(void) { return surv_on() ? 1 : 0; }
int gsr_set_exact_blend(int on) {
    g_exact.store(on ? 1 : 0);
    return GSR_OK;
}
int gsr_get_exact_blend(void) { return exact_on() ? 1 : 0; }
// the backward's heavy-tile threshold (log2 of the estimate; < 0: the build's BWD_HEAVY_BITS)
static std::atomic<int> g_bwd_heavy_bits{-1};
int gsr_set_backward_heavy_bits(int bits) {
    if (bits > 32) return fail(GSR_E_ARG, "gsr_set_backward_heavy_bits: bits %d > 32", bits);
    g_bwd_heavy_bits.store(bits < 0 ? -1 : bits);
    return GSR_OK;
}

int gsr_check_buffers(int P, int R, int width, int height, const int* radii, void* geom_buffer, void* binning_buffer,
                      void* img_buffer, void* stream_) {
    if (P < 0 || R < 0 || width <= 0 || height <= 0 || !radii || !geom_buffer || !img_buffer || (R > 0 && !binning_buffer))
        return fail(GSR_E_ARG, "gsr_check_buffers: bad arguments");
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(width, height, false);
    char* geom = align_base(geom_buffer);
    char* img = align_base(img_buffer);
    char* bin = binning_buffer ? align_base(binning_buffer) : nullptr;
    return debug_check_forward(P, R, tiles_x(width), tiles_y(height), width, height, radii, at<uint2>(geom, gl.rect),
                               at<uint32_t>(geom, gl.depth_key), bin, at<uint32_t>(img, il.n_contrib),
                               reinterpret_cast<hipStream_t>(stream_));
}

int gsr_materialize_lists(int R, int width, int height, void* binning_buffer, unsigned* point_list, unsigned* ranges,
                          void* stream_) {
    if (R < 0 || width <= 0 || height <= 0 || !ranges || (R > 0 && (!binning_buffer || !point_list)))
        return fail(GSR_E_ARG, "gsr_materialize_lists: bad arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    if (R == 0) {
        HIP_OK(hipMemsetAsync(ranges, 0, 8 * (size_t)tiles_x(width) * tiles_y(height), s));
        return GSR_OK;
    }
    return materialize_lists(R, width, height, align_base(binning_buffer), point_list, reinterpret_cast<uint2*>(ranges), s);
}

int gsr_debug_build(void) {
#ifdef GSR_DEBUG
    return 1;
#else
    return 0;
#endif
}

int gsr_profile_enable(int on) {
    g_prof.on = on != 0;
    return GSR_OK;
}

int gsr_profile_stages(unsigned mask) {
    g_prof.mask = mask;
    return GSR_OK;
}

int gsr_profile_stage_count(void) { return ST_COUNT; }

const char* gsr_profile_stage_name(int i) { return (i >= 0 && i < ST_COUNT) ? kStageNames[i] : ""; }

int gsr_profile_read(double* ms, long long* counts, int n, int reset) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    for (auto& r : g_prof.pending) {
        HIP_OK(hipEventSynchronize(r.b));
        float t = 0.f;
        HIP_OK(hipEventElapsedTime(&t, r.a, r.b));
        g_prof.ms[r.stage] += t;
        g_prof.n[r.stage] += 1;
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < n && i < ST_COUNT; i++) {
        if (ms) ms[i] = g_prof.ms[i];
        if (counts) counts[i] = g_prof.n[i];
    }
    if (reset)
        for (int i = 0; i < ST_COUNT; i++) { g_prof.ms[i] = 0; g_prof.n[i] = 0; }
    return GSR_OK;
}

int gsr_get_layout(int P, long long R, int width, int height, gsr_layout* out) {
    if (!out || P < 0 || R < 0 || width < 0 || height < 0) return fail(GSR_E_ARG, "gsr_get_layout: bad arguments");
    const GeomLayout g = geom_layout(P);
    const ImgLayout im = img_layout(width, height, surv_on());
    const BinLayout b = bin_layout(0, width, height, 0);
    (void)R;
    out->geom_bytes = g.total;
    out->img_bytes = im.total;
    out->bin_bytes = b.total;
    out->geom_radii = g.radii;
    out->geom_tiles = g.tiles;
    out->geom_depth_key = g.depth_key;
    out->geom_rect = g.rect;
    out->geom_rec = g.rec;
    out->geom_acc = g.acc;
    out->img_final_T = im.final_T;
    out->img_n_contrib = im.n_contrib;
    out->img_ranges = im.ranges;
    out->img_tile_nmax = im.tile_nmax;
    out->img_tile_emax = im.tile_emax;
    out->bin_st_ranges = b.st_ranges;
    out->bin_entries = b.ent;
    out->img_tile_cost = im.tile_cost;
    out->img_row_cost = im.row_cost;
    out->img_order_bwd = im.order_bwd;
    out->img_nheavy = im.nheavy;
    out->img_surv_n = im.surv_n;
    out->img_surv = im.surv;
    out->surv_cap = gsr::SURV_CAP;
    return GSR_OK;
}

static int forward_impl(gsr_resize_fn geometry_buffer, void* geometry_ctx, gsr_resize_fn binning_buffer,
                        void* binning_ctx, gsr_resize_fn image_buffer, void* image_ctx, int P, int D, int M,
                        const float* background, int width, int height, const float* means3D, const float* shs,
                        const float* colors_precomp, const float* opacities, const float* scales, float scale_modifier,
                        const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                        const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered,
                        float* out_color, int* radii, void* stream_, int* num_rendered, const McSpec* mc) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    if (num_rendered) *num_rendered = 0;
    if (P < 0 || width <= 0 || height <= 0) return fail(GSR_E_ARG, "gsr_forward: bad sizes P=%d W=%d H=%d", P, width, height);
    if (!geometry_buffer || !binning_buffer || !image_buffer) return fail(GSR_E_ARG, "gsr_forward: missing buffer callbacks");
    if (!colors_precomp && !shs && P > 0 && !mc)
        return fail(GSR_E_ARG, "For non-RGB, provide precomputed Gaussian colors!");
    if (!cov3D_precomp && (!scales || !rotations) && P > 0)
        return fail(GSR_E_ARG, "gsr_forward: need scales+rotations or cov3D_precomp");
    if (tiles_x(width) > 65535u || tiles_y(height) > 65535u ||
        (unsigned long long)st_x(width) * st_y(width, height) >= (1ull << gsr::ST_KEY_BITS))
        return fail(GSR_E_ARG, "gsr_forward: image too large");

    // rasterizer_impl.cu:221-222 (host float arithmetic == device float arithmetic)
    const float focal_y = height / (2.0f * tan_fovy);
    const float focal_x = width / (2.0f * tan_fovx);
    const GeomLayout gl = geom_layout(P);
    const bool surv = surv_on();
    const ImgLayout il = img_layout(width, height, surv);
    char* geom = reinterpret_cast<char*>(geometry_buffer(geometry_ctx, gl.total));
    char* img = reinterpret_cast<char*>(image_buffer(image_ctx, il.total));
    if (!geom || !img) return fail(GSR_E_ALLOC, "gsr_forward: buffer allocation failed");
    geom = align_base(geom);
    img = align_base(img);
    const bool exact = exact_on();
    exact_set(img, exact);
    const unsigned gx = tiles_x(width), gy = tiles_y(height);
    const int T = (int)(gx * gy);
    if (!radii) radii = at<int>(geom, gl.radii);
    if (P == 0) {  // the reference renders nothing (rasterize_points.cu:84-86): zero image
        if (out_color) HIP_OK(hipMemsetAsync(out_color, 0, sizeof(float) * 3 * (size_t)width * height, s));
        return GSR_OK;
    }

    unsigned long long* tot_dev = at<unsigned long long>(geom, gl.tot_dev);

    gsr::PreprocessArgs pa{};
    pa.P = P; pa.D = D; pa.M = M;
    pa.means3D = means3D; pa.scales = scales; pa.scale_modifier = scale_modifier; pa.rotations = rotations;
    pa.opacities = opacities; pa.shs = shs; pa.cov3D_precomp = cov3D_precomp; pa.colors_precomp = colors_precomp;
    pa.viewmatrix = viewmatrix; pa.projmatrix = projmatrix; pa.campos = cam_pos;
    pa.W = width; pa.H = height; pa.tan_fovx = tan_fovx; pa.tan_fovy = tan_fovy;
    pa.focal_x = focal_x; pa.focal_y = focal_y; pa.grid_x = gx; pa.grid_y = gy; pa.prefiltered = prefiltered;
    pa.radii = radii;
    pa.tiles = at<uint32_t>(geom, gl.tiles);
    pa.st_count = at<uint32_t>(geom, gl.st_count);
    pa.depth_key = at<uint32_t>(geom, gl.depth_key);
    pa.rect = at<uint2>(geom, gl.rect);
    pa.rec = at<gsr::Rec>(geom, gl.rec);
    pa.shjac = (shs && !colors_precomp) ? at<float>(geom, gl.shjac) : nullptr;
    pa.blk_tot = at<uint4>(geom, gl.blk_tot);
    {
        GSR_STAGE(ST_PREPROCESS);
        gsr::launch_preprocess(pa, s);
    }
    GSR_LAUNCH_CHECK();

    // The forward's one host synchronisation (the reference's, rasterizer_impl.cu:281) reads
    // P_v, R and S: one workgroup sums the preprocess's per-workgroup totals into host-mapped
    // words tagged with this call's sequence number, and the host polls them (a D2H copy or an
    // event on the stream each left a 6-19 us bubble between kernels).
    //  * Speculative (an earlier call had the same P and image size): the binning buffer is
    //    sized from that call's counts with headroom; the binning and the forward tile pass
    //    are launched BEFORE the host waits (the kernels read P_v on the device, drop entries
    //    beyond the capacity and clamp the tile ranges to it), and the totals ride in an extra
    //    workgroup of the super-tile scatter.  A capacity overflow (rare: R grew by > 25 %)
    //    redoes the binning and the tile pass at the exact size.
    //  * Otherwise (first call, or images too large for the fused binning) the totals run
    //    right after the preprocess, the host waits while the depth sort runs, and sizes the
    //    binning buffer exactly.
    if (!g_pinned.p) {
        HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&g_pinned.p), 8 * 8, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&g_pinned.p_dev), g_pinned.p, 0));
        memset(g_pinned.p, 0, 8 * 8);
    }
    const unsigned long long seq = ++g_pinned.seq;
    const gsr::FrameTotals ft{pa.blk_tot, gsr::pre_blocks(P), g_pinned.p_dev, seq};
    const unsigned gsx = st_x(width), gsy = st_y(width, height);
    const int NS = (int)(gsx * gsy);
    const bool fused_bin = gsr::st_bin_supported(NS);
    const bool speculate = fused_bin && g_hint.P == P && g_hint.W == width && g_hint.H == height;
    if (!speculate) gsr::launch_frame_totals(ft, s);

    // Depth sort of all P Gaussians: culled ones carry key 0xFFFFFFFF and sort last, so the
    // first P_v sorted entries are the visible Gaussians in the reference's (depth, index)
    // order -- no separate visibility compaction.  Its last pass stores P_v to tot_dev.
    const bool rect_packed = gsr::rect_packable(gx, gy);  // 4-B rects through the sort and the binning
    uint32_t* vis_key = at<uint32_t>(geom, gl.vis_key);
    uint32_t* vis_val = at<uint32_t>(geom, gl.vis_val);
    int flip;
    {
        GSR_STAGE(ST_DEPTH_SORT);
        flip = gsr::depth_sort(P, pa.depth_key, vis_key, vis_val, at<uint32_t>(geom, gl.vis_key_alt),
                               at<uint32_t>(geom, gl.vis_val_alt), pa.rect, at<uint2>(geom, gl.rect_s),
                               at<uint2>(geom, gl.rect_s_alt), at<void>(geom, gl.sort_tmp), tot_dev, s,
                               nullptr, 0, rect_packed);
    }
    GSR_LAUNCH_CHECK();

    unsigned long long Pv = 0, R64 = 0, S64 = 0;
    auto read_totals = [&]() -> int {
        unsigned long long t[4];
        const int rc = wait_totals(g_pinned.p, seq, s, t);
        if (rc != GSR_OK) return rc;
        Pv = t[0];
        R64 = t[1];
        S64 = t[2];
        const unsigned long long errv = t[3];
        if (errv) return fail(GSR_E_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
        if (R64 > 0x7fffffffull) return fail(GSR_E_OVERFLOW, "gsr_forward: %llu instances overflow int", R64);
        return GSR_OK;
    };
    const uint32_t* sorted_ids = flip ? at<uint32_t>(geom, gl.vis_val_alt) : vis_val;
    const void* rect_sorted = flip ? at<void>(geom, gl.rect_s_alt) : at<void>(geom, gl.rect_s);
    char* bin = nullptr;
    BinLayout bl{};
    // binning into a buffer of entry capacity capS; dev: read P_v on the device (and run the
    // frame totals in the scatter)
    auto bin_pass = [&](long long capS, bool dev) -> int {
        bl = bin_layout(capS, width, height, dev ? P : (long long)Pv);
        bin = reinterpret_cast<char*>(binning_buffer(binning_ctx, bl.total));
        if (!bin) return fail(GSR_E_ALLOC, "gsr_forward: binning allocation failed");
        bin = align_base(bin);
        uint2* ent = at<uint2>(bin, bl.ent);
        uint2* st_ranges = at<uint2>(bin, bl.st_ranges);
        unsigned long long* header = at<unsigned long long>(bin, bl.header);
        // the forward's dispatch order (a tile's cost: its super-tile's entry count); zeroes
        // the tile maxima and summed cost the tile pass raises
        gsr::TileOrderArgs ord{};
        ord.ntile = (unsigned)T; ord.gx = gx; ord.gsx = gsx; ord.order = at<uint32_t>(img, il.order_fwd);
        ord.nheavy = at<uint32_t>(img, il.nheavy) + FWD_NHEAVY; ord.heavy_bits = gsr::FWD_HEAVY_BITS;
        ord.balance = 0;  // equal bands (tile_unit_fwd)
        ord.zero_a = at<uint32_t>(img, il.tile_nmax); ord.zero_b = at<uint32_t>(img, il.tile_emax);
        ord.zero_c = at<uint32_t>(img, il.tile_cost);
        ord.zero_rows = at<uint32_t>(img, il.row_cost); ord.nrows = gy;
        ord.unset = at<uint32_t>(img, il.surv_n);  // no list unless this forward stores one
        if (fused_bin) {  // the order runs in extra workgroups of the binning's scatter
            GSR_STAGE(ST_DUPLICATE);
            gsr::launch_st_bin(dev ? P : (int)Pv, dev ? tot_dev : nullptr, sorted_ids, rect_sorted, rect_packed, gsx, st_h(width, height), NS,
                               at<void>(bin, bl.st_bin_tmp), ent, st_ranges, header, (uint32_t)capS, s,
                               dev ? &ft : nullptr, &ord);
            GSR_LAUNCH_CHECK();
            return GSR_OK;
        } else {
            uint32_t* stk = at<uint32_t>(bin, bl.st_keys);
            uint32_t* stv = at<uint32_t>(bin, bl.st_vals);
            uint32_t* offsets = at<uint32_t>(geom, gl.offsets);
            {
                GSR_STAGE(ST_OFFSETS);
                gsr::launch_exclusive_scan_u32((long long)Pv, pa.st_count, sorted_ids, offsets,
                                               at<uint32_t>(geom, gl.scan_tmp), nullptr, s);
            }
            {
                GSR_STAGE(ST_DUPLICATE);
                gsr::launch_st_emit((int)Pv, sorted_ids, offsets, pa.rect, gsx, st_h(width, height), stk, stv, s);
            }
            int flip2;
            {
                GSR_STAGE(ST_TILE_SORT);
                flip2 = gsr::radix_sort_pairs(capS, stk, stv, at<uint32_t>(bin, bl.st_keys_alt),
                                              at<uint32_t>(bin, bl.st_vals_alt), (int)higher_msb((uint32_t)NS),
                                              at<void>(bin, bl.sort_tmp), s);
            }
            gsr::launch_seg_ranges(capS, NS, flip2 ? at<uint32_t>(bin, bl.st_keys_alt) : stk,
                                   flip2 ? at<uint32_t>(bin, bl.st_vals_alt) : stv, st_ranges, ent, header, s);
        }
        GSR_LAUNCH_CHECK();
        {
            GSR_STAGE(ST_RANGES);
            ord.st_ranges = st_ranges;
            gsr::launch_tile_order_args(ord, s);
        }
        GSR_LAUNCH_CHECK();
        return GSR_OK;
    };
    gsr::RenderFwdArgs ra{};
    ra.W = width; ra.H = height; ra.grid_x = gx; ra.grid_y = gy;
    ra.gsx = gsx; ra.rec = pa.rec; ra.bg = background;
    ra.out_color = out_color; ra.final_T = at<float>(img, il.final_T); ra.n_contrib = at<uint32_t>(img, il.n_contrib);
    ra.order = at<uint32_t>(img, il.order_fwd);
    ra.nheavy = at<uint32_t>(img, il.nheavy) + FWD_NHEAVY;
    ra.tile_nmax = at<uint32_t>(img, il.tile_nmax);
    ra.tile_emax = at<uint32_t>(img, il.tile_emax);
    ra.tile_cost = at<uint32_t>(img, il.tile_cost);
    ra.row_cost = at<uint32_t>(img, il.row_cost);
    ra.exact = exact ? 1 : 0;
    if (surv && !mc) {  // the single-channel backward walks the forward's survivor lists
        ra.surv = at<uint2>(img, il.surv);
        ra.surv_n = at<uint32_t>(img, il.surv_n);
    }
    // the forward tile pass over the binning in `bin`; its workgroups also zero the backward's
    // accumulator lines (zero_slice; the depth sort's digit scans did it up to round 3)
    ra.zero = reinterpret_cast<float4*>(at<float>(geom, gl.acc));
    ra.zero_n4 = (long long)gsr::ACC_STRIDE * P / 4;
    auto render_pass = [&]() -> int {
        ra.st_ranges = at<uint2>(bin, bl.st_ranges);
        ra.ent = at<uint2>(bin, bl.ent);
        GSR_STAGE(ST_RENDER_FWD);
        if (!mc) {
            gsr::launch_render_fwd(ra, s);
        } else {
            GSR_STAGE(ST_RENDER_FWD_MC);
            for (int c0 = 0; c0 < mc->nch; c0 += MC_GROUP) {
                gsr::RenderMcArgs ma = mc_args(ra.W, ra.H, gx, gy, gsx, ra.st_ranges, ra.ent, pa.rec, ra.order,
                                               ra.nheavy, ra.tile_nmax, ra.tile_emax, *mc, c0);
                ma.tile_cost = ra.tile_cost;
                ma.row_cost = ra.row_cost;
                ma.exact = ra.exact;
                ma.out = mc->out + (size_t)c0 * width * height;
                if (c0 == 0) {  // the other groups would write the same values
                    ma.final_T = ra.final_T;
                    ma.n_contrib = ra.n_contrib;
                    ma.zero = ra.zero;
                    ma.zero_n4 = ra.zero_n4;
                    if (surv) {  // the survivors (the same for every group)
                        ma.surv = at<uint2>(img, il.surv);
                        ma.surv_n = at<uint32_t>(img, il.surv_n);
                    }
                } else {
                    ma.tile_nmax = nullptr;
                }
                gsr::launch_render_fwd_mc(ma, s);
            }
        }
        GSR_LAUNCH_CHECK();
        zeroed_set(geom, true);  // the backward's accumulators are zero from here on
        return GSR_OK;
    };
    int rc;
    if (speculate) {
        const long long capS = g_hint.S + g_hint.S / 4 + 4096;
        if ((rc = bin_pass(capS, true)) != GSR_OK) return rc;
        if ((rc = render_pass()) != GSR_OK) return rc;
        if ((rc = read_totals()) != GSR_OK) return rc;
        if ((long long)S64 > capS) {  // overflow: redo at the exact size
            if ((rc = bin_pass((long long)S64, false)) != GSR_OK) return rc;
            if ((rc = render_pass()) != GSR_OK) return rc;
        }
    } else {
        if ((rc = read_totals()) != GSR_OK) return rc;
        if ((rc = bin_pass((long long)S64, false)) != GSR_OK) return rc;
        if ((rc = render_pass()) != GSR_OK) return rc;
    }
    const long long R = (long long)R64;
    g_hint.P = P;
    g_hint.W = width;
    g_hint.H = height;
    g_hint.R = R;
    g_hint.S = (long long)S64;
#ifdef GSR_DEBUG
    {
        const int rc_dbg = debug_check_forward(P, R, gx, gy, width, height, radii, pa.rect, pa.depth_key, bin,
                                               ra.n_contrib, s);
        if (rc_dbg != GSR_OK) return rc_dbg;
    }
#endif
    if (num_rendered) *num_rendered = (int)R;
    return GSR_OK;
}

int gsr_forward(gsr_resize_fn geometry_buffer, void* geometry_ctx, gsr_resize_fn binning_buffer, void* binning_ctx,
                gsr_resize_fn image_buffer, void* image_ctx, int P, int D, int M, const float* background, int width,
                int height, const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier, const float* rotations,
                const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix, const float* cam_pos,
                float tan_fovx, float tan_fovy, int prefiltered, float* out_color, int* radii, void* stream_,
                int* num_rendered) {
    return forward_impl(geometry_buffer, geometry_ctx, binning_buffer, binning_ctx, image_buffer, image_ctx, P, D, M,
                        background, width, height, means3D, shs, colors_precomp, opacities, scales, scale_modifier,
                        rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                        out_color, radii, stream_, num_rendered, nullptr);
}

static int check_mc(const char* fn, int nch, int fstride, const float* features) {
    if (nch <= 0 || fstride < nch || (fstride & 3) != 0)
        return fail(GSR_E_ARG, "%s: need 0 < nch <= feature_stride, feature_stride a multiple of 4 (nch=%d stride=%d)",
                    fn, nch, fstride);
    if ((reinterpret_cast<uintptr_t>(features) & 15u) != 0) return fail(GSR_E_ARG, "%s: features must be 16-B aligned", fn);
    return GSR_OK;
}

int gsr_forward_channels(gsr_resize_fn geometry_buffer, void* geometry_ctx, gsr_resize_fn binning_buffer,
                         void* binning_ctx, gsr_resize_fn image_buffer, void* image_ctx, int P, int nch,
                         int feature_stride, const float* features, const float* background, int width, int height,
                         const float* means3D, const float* opacities, const float* scales, float scale_modifier,
                         const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                         const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                         int prefiltered, float* out, int* radii, void* stream_, int* num_rendered) {
    if (num_rendered) *num_rendered = 0;
    if (P > 0 || features) {
        const int e = check_mc("gsr_forward_channels", nch, feature_stride, features);
        if (e != GSR_OK) return e;
    }
    if (!background || !out) return fail(GSR_E_ARG, "gsr_forward_channels: missing background or output");
    McSpec mc{nch, feature_stride, features, background, out, nullptr, nullptr};
    if (P == 0) {  // background everywhere (the reference's P == 0 forward renders nothing)
        hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
        HIP_OK(hipMemsetAsync(out, 0, sizeof(float) * (size_t)nch * width * height, s));
        return GSR_OK;
    }
    return forward_impl(geometry_buffer, geometry_ctx, binning_buffer, binning_ctx, image_buffer, image_ctx, P, 0, 0,
                        background, width, height, means3D, nullptr, nullptr, opacities, scales, scale_modifier,
                        rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                        nullptr, radii, stream_, num_rendered, &mc);
}

int gsr_forward_reuse(gsr_resize_fn geometry_buffer, void* geometry_ctx, const void* src_geom_buffer,
                      const int* src_radii, void* binning_buffer, void* image_buffer, int P, int R,
                      const float* background, int width, int height, const float* colors_precomp, float* out_color,
                      int* radii, void* stream_) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    if (P < 0 || R < 0 || width <= 0 || height <= 0) return fail(GSR_E_ARG, "gsr_forward_reuse: bad sizes");
    if (P == 0) return GSR_OK;
    if (!geometry_buffer || !src_geom_buffer || !src_radii || !image_buffer || !colors_precomp || !radii ||
        !binning_buffer)
        return fail(GSR_E_ARG, "gsr_forward_reuse: missing buffers");
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(width, height, false);
    const BinLayout bl = bin_layout(0, width, height, 0);
    char* geom = reinterpret_cast<char*>(geometry_buffer(geometry_ctx, gl.total));
    if (!geom) return fail(GSR_E_ALLOC, "gsr_forward_reuse: buffer allocation failed");
    geom = align_base(geom);
    zeroed_set(geom, false);  // its accumulators are not zeroed here: the backward zero-fills
    const char* src = align_base(const_cast<void*>(src_geom_buffer));
    char* img = align_base(image_buffer);
    char* bin = binning_buffer ? align_base(binning_buffer) : nullptr;
    {
        GSR_STAGE(ST_PREPROCESS);
        gsr::launch_recolor(P, src_radii, reinterpret_cast<const gsr::Rec*>(src + gl.rec), colors_precomp,
                            at<gsr::Rec>(geom, gl.rec), radii, s);
    }
    // the deterministic backward's gather reads this call's rects and depth keys; copied
    // always (12 B per Gaussian), so deterministic mode may be switched on between a cached
    // forward and its backward
    HIP_OK(hipMemcpyAsync(geom + gl.depth_key, src + gl.depth_key, 4 * (size_t)P, hipMemcpyDeviceToDevice, s));
    HIP_OK(hipMemcpyAsync(geom + gl.rect, src + gl.rect, 8 * (size_t)P, hipMemcpyDeviceToDevice, s));
    GSR_LAUNCH_CHECK();
    const unsigned gx = tiles_x(width), gy = tiles_y(height);
    gsr::RenderFwdArgs ra{};  // with R == 0 every super-tile list is empty: background everywhere
    ra.W = width; ra.H = height; ra.grid_x = gx; ra.grid_y = gy;
    ra.gsx = st_x(width);
    ra.st_ranges = bin ? at<uint2>(bin, bl.st_ranges) : nullptr;
    ra.ent = bin ? at<uint2>(bin, bl.ent) : nullptr;
    ra.rec = at<gsr::Rec>(geom, gl.rec); ra.bg = background;
    ra.out_color = out_color; ra.final_T = at<float>(img, il.final_T); ra.n_contrib = at<uint32_t>(img, il.n_contrib);
    ra.order = at<uint32_t>(img, il.order_fwd);
    ra.nheavy = at<uint32_t>(img, il.nheavy) + FWD_NHEAVY;
    ra.tile_nmax = at<uint32_t>(img, il.tile_nmax);  // re-maxed with identical values
    ra.tile_emax = at<uint32_t>(img, il.tile_emax);
    ra.tile_cost = nullptr;  // already summed by the cached call's forward
    ra.exact = exact_get(img) ? 1 : 0;  // the cached call's arithmetic
    // no survivor lists: the cached call's stay (its survivors are this call's -- they depend on the
    // geometry only -- and its buffer holds lists only if that forward stored them)
    if (!bin) return fail(GSR_E_ARG, "gsr_forward_reuse: missing binning buffer");
    {
        GSR_STAGE(ST_RENDER_FWD);
        gsr::launch_render_fwd(ra, s);  // the cached call's dispatch order is still valid
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

static int backward_impl(int P, int D, int M, int R, const float* background, int width, int height,
                         const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                         float scale_modifier, const float* rotations, const float* cov3D_precomp,
                         const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                         float tan_fovy, const int* radii, void* geom_buffer, void* binning_buffer, void* img_buffer,
                         const float* dL_dpix, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                         float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                         float* dL_drot, void* stream_, const McSpec* mc, unsigned acc_mask = 0) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    if (P < 0 || R < 0 || width <= 0 || height <= 0) return fail(GSR_E_ARG, "gsr_backward: bad sizes");
    if (P == 0) return GSR_OK;
    if (!geom_buffer || !img_buffer || (R > 0 && !binning_buffer)) return fail(GSR_E_ARG, "gsr_backward: missing buffers");
    const float focal_y = height / (2.0f * tan_fovy);
    const float focal_x = width / (2.0f * tan_fovx);
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(width, height, true);  // (the lists are read only where stored)
    const BinLayout bl = bin_layout(0, width, height, 0);
    char* geom = align_base(geom_buffer);
    char* img = align_base(img_buffer);
    char* bin = binning_buffer ? align_base(binning_buffer) : nullptr;
    const unsigned gx = tiles_x(width), gy = tiles_y(height);
    if (!radii) radii = at<int>(geom, gl.radii);
    float* acc = at<float>(geom, gl.acc);
    const bool acc_zero = zeroed_take(geom);  // zeroed by this buffer's forward, unused since
    if (!acc_zero || mc) {
        GSR_STAGE(ST_BWD_ZERO);
        if (!acc_zero) HIP_OK(hipMemsetAsync(acc, 0, sizeof(float) * gsr::ACC_STRIDE * (size_t)P, s));
        if (mc) HIP_OK(hipMemsetAsync(mc->dL_dfeat, 0, sizeof(float) * (size_t)mc->fstride * P, s));
    }

    // deterministic mode: one partial row per instance (indexed by the materialised lists),
    // summed per Gaussian in tile order
    const bool det = det_on() && R > 0;
    const int pstride = mc ? ((6 + mc->nch + 3) & ~3) : gsr::DET_ROW3;
    float* partial = nullptr;
    unsigned* det_missing = nullptr;
    uint32_t* det_pl = nullptr;
    uint2* det_ranges = nullptr;
    if (det) {
        const size_t pbytes = 4 * (size_t)pstride * (size_t)R, T = (size_t)gx * gy;
        const size_t off_pl = align_up(256 + pbytes, 256), off_rg = align_up(off_pl + 4 * (size_t)R, 256);
        char* sc = reinterpret_cast<char*>(g_scratch.get(off_rg + 8 * T));
        if (!sc) return fail(GSR_E_ALLOC, "gsr_backward: deterministic-mode scratch allocation failed");
        det_missing = reinterpret_cast<unsigned*>(sc);
        partial = reinterpret_cast<float*>(sc + 256);
        det_pl = reinterpret_cast<uint32_t*>(sc + off_pl);
        det_ranges = reinterpret_cast<uint2*>(sc + off_rg);
        HIP_OK(hipMemsetAsync(sc, 0, 256 + pbytes, s));
        const int rc = materialize_lists(R, width, height, bin, det_pl, det_ranges, s);
        if (rc != GSR_OK) return rc;
    }
    if (R > 0) {
        gsr::RenderBwdArgs ra{};
        ra.W = width; ra.H = height; ra.grid_x = gx; ra.grid_y = gy;
        ra.st_ranges = at<uint2>(bin, bl.st_ranges);
        ra.ent = at<uint2>(bin, bl.ent);
        ra.gsx = st_x(width);
        ra.tile_emax = at<uint32_t>(img, il.tile_emax);
        ra.tile_nmax = at<uint32_t>(img, il.tile_nmax);
        ra.ranges = det_ranges;
        ra.rec = at<gsr::Rec>(geom, gl.rec);
        ra.colors = colors_precomp;
        ra.bg = background;
        ra.final_T = at<float>(img, il.final_T);
        ra.n_contrib = at<uint32_t>(img, il.n_contrib);
        ra.dL_dpix = dL_dpix;
        ra.acc = acc;
        ra.order = at<uint32_t>(img, il.order_bwd);
        ra.nheavy = at<uint32_t>(img, il.nheavy) + 8;
        ra.partial = partial;
        ra.exact = exact_get(img) ? 1 : 0;  // the forward's arithmetic
        ra.surv = at<uint2>(img, il.surv);
        ra.surv_n = at<uint32_t>(img, il.surv_n);
        {
            GSR_STAGE(ST_RANGES);  // "tile_order": the backward's dispatch order
            gsr::launch_tile_order(gx * gy, nullptr, at<uint32_t>(img, il.tile_cost), at<uint32_t>(img, il.order_bwd),
                                   at<uint32_t>(img, il.nheavy) + 8,
                                   det ? 32 : (g_bwd_heavy_bits.load() >= 0 ? g_bwd_heavy_bits.load() : gsr::BWD_HEAVY_BITS),
                                   s,  // det: one writer per row
                                   at<uint32_t>(img, il.row_cost), gy);
        }
        {
            GSR_STAGE(ST_RENDER_BWD);  // the tile pass alone (roofline.avg_launch_ms in bench.py)
            if (!mc) {
                gsr::launch_render_bwd(ra, s);
            } else {
                GSR_STAGE(ST_RENDER_BWD_MC);
                for (int c0 = 0; c0 < mc->nch; c0 += MC_GROUP) {
                    gsr::RenderMcArgs ma = mc_args(width, height, gx, gy, ra.gsx, ra.st_ranges, ra.ent, ra.rec, ra.order,
                                                   ra.nheavy, at<uint32_t>(img, il.tile_nmax),
                                                   at<uint32_t>(img, il.tile_emax), *mc, c0);
                    ma.ranges = det_ranges;
                    ma.surv = const_cast<uint2*>(ra.surv);
                    ma.surv_n = const_cast<uint32_t*>(ra.surv_n);
                    ma.final_T = const_cast<float*>(ra.final_T);
                    ma.n_contrib = const_cast<uint32_t*>(ra.n_contrib);
                    ma.dL_dout = mc->dL_dout + (size_t)c0 * width * height;
                    ma.acc = acc;
                    ma.dL_dfeat = mc->dL_dfeat + c0;
                    ma.partial = partial;
                    ma.pstride = pstride;
                    ma.pc0 = c0;
                    ma.exact = ra.exact;
                    gsr::launch_render_bwd_mc(ma, s);
                }
            }
        }
        GSR_LAUNCH_CHECK();
        if (det) {
            gsr::DetGatherArgs da{};
            da.P = P; da.gx = gx; da.gy = gy;
            da.radii = radii;
            da.rect = at<uint2>(geom, gl.rect);
            da.depth_key = at<uint32_t>(geom, gl.depth_key);
            da.ranges = det_ranges;
            da.point_list = det_pl;
            da.partial = partial;
            da.mode = mc ? 1 : 0;
            da.pstride = pstride;
            da.nch = mc ? mc->nch : 0;
            da.fstride = mc ? mc->fstride : 0;
            da.acc = acc;
            da.dL_dfeat = mc ? mc->dL_dfeat : nullptr;
            da.missing = det_missing;
            gsr::launch_det_gather(da, s);
            GSR_LAUNCH_CHECK();
            unsigned miss = 0;
            HIP_OK(hipMemcpyAsync(&miss, det_missing, 4, hipMemcpyDeviceToHost, s));
            HIP_OK(hipStreamSynchronize(s));  // the scratch is free again when this call returns
            if (miss) return fail(GSR_E_DEVICE_CHECK, "gsr_backward (deterministic): %u instances not found in their tile lists", miss);
        }
    }
    gsr::PreprocessBwdArgs pb{};
    pb.P = P; pb.D = D; pb.M = M;
    pb.means3D = means3D; pb.radii = radii; pb.shs = shs; pb.scales = scales; pb.rotations = rotations;
    pb.scale_modifier = scale_modifier; pb.cov3D_precomp = cov3D_precomp;
    pb.viewmatrix = viewmatrix; pb.projmatrix = projmatrix; pb.campos = campos;
    pb.tan_fovx = tan_fovx; pb.tan_fovy = tan_fovy; pb.focal_x = focal_x; pb.focal_y = focal_y;
    pb.acc = acc;
    pb.acc_raw = 1;  // the tile passes' raw sums (gsr_render_bwd.hip)
    pb.W = width;
    pb.H = height;
    pb.shjac = at<float>(geom, gl.shjac);
    pb.dL_dmean2D = dL_dmean2D; pb.dL_dconic = dL_dconic; pb.dL_dopacity = dL_dopacity; pb.dL_dcolor = dL_dcolor;
    pb.dL_dmean3D = dL_dmean3D; pb.dL_dcov3D = dL_dcov3D; pb.dL_dsh = M > 0 ? dL_dsh : nullptr;
    pb.dL_dscale = dL_dscale; pb.dL_drot = dL_drot;
    pb.acc_mask = acc_mask;
    if ((dL_dscale == nullptr) != (dL_drot == nullptr)) return fail(GSR_E_ARG, "gsr_backward: dL_dscale/dL_drot must both be given");
    {
        GSR_STAGE(ST_PREPROCESS_BWD);
        gsr::launch_preprocess_bwd(pb, s);
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height, const float* means3D,
                 const float* shs, const float* colors_precomp, const float* scales, float scale_modifier,
                 const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                 void* geom_buffer, void* binning_buffer, void* img_buffer, const float* dL_dpix, float* dL_dmean2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                 float* dL_dsh, float* dL_dscale, float* dL_drot, void* stream_) {
    // dL_dcolor / dL_dcov3D may be NULL: not stored (the SH and scale/rotation gradients keep
    // them in registers; an autograd caller passes NULL for inputs that need no gradient)
    return backward_impl(P, D, M, R, background, width, height, means3D, shs, colors_precomp, scales, scale_modifier,
                         rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                         geom_buffer, binning_buffer, img_buffer, dL_dpix, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor,
                         dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot, stream_, nullptr);
}

int gsr_backward_channels(int P, int nch, int feature_stride, const float* features, int R, const float* background,
                          int width, int height, const float* means3D, const float* scales, float scale_modifier,
                          const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                          const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                          const int* radii, void* geom_buffer, void* binning_buffer, void* img_buffer,
                          const float* dL_dout, float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                          float* dL_dfeatures, float* dL_dmean3D, float* dL_dcov3D, float* dL_dscale, float* dL_drot,
                          unsigned accumulate, void* stream_) {
    if (P == 0) return GSR_OK;
    const int e = check_mc("gsr_backward_channels", nch, feature_stride, features);
    if (e != GSR_OK) return e;
    if (!background || !dL_dout || !dL_dfeatures) return fail(GSR_E_ARG, "gsr_backward_channels: missing buffers");
    McSpec mc{nch, feature_stride, features, background, nullptr, dL_dout, dL_dfeatures};
    return backward_impl(P, 0, 0, R, background, width, height, means3D, nullptr, nullptr, scales, scale_modifier,
                         rotations, cov3D_precomp, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, radii,
                         geom_buffer, binning_buffer, img_buffer, nullptr, dL_dmean2D, dL_dconic, dL_dopacity, nullptr,
                         dL_dmean3D, dL_dcov3D, nullptr, dL_dscale, dL_drot, stream_, &mc,
                         accumulate & (gsr::ACC_MEAN3D | gsr::ACC_SCALE | gsr::ACC_ROT | gsr::ACC_OPACITY));
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                     void* stream_) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_E_ARG, "gsr_mark_visible: bad P");
    gsr::launch_mark_visible(P, means3D, viewmatrix, reinterpret_cast<bool*>(present),
                             reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

size_t gsr_knn_workspace_bytes(int P) { return gsr::knn_workspace_bytes(P); }

int gsr_knn_mean_dist(int P, const float* points, float* mean_dists, void* workspace, void* stream_) {
    if (P < 0) return fail(GSR_E_ARG, "gsr_knn_mean_dist: bad P");
    if (P == 0) return GSR_OK;
    if (!points || !mean_dists || !workspace) return fail(GSR_E_ARG, "gsr_knn_mean_dist: missing buffers");
    gsr::launch_knn(P, points, mean_dists, workspace, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

size_t gsr_shade_workspace_bytes(int N, int deg) { return gsr::shade_workspace_bytes(N, deg); }

int gsr_shade_forward(int N, int deg, const float* pos, const float* normal, const float* albedo,
                      const float* view_pos, const float* kr, const float* km, const float* base,
                      const float* fg_lut, int specular, float* rgb, float* diffuse, float* specular_out,
                      void* stream_) {
    if (N < 0 || deg < 2 || deg > 5) return fail(GSR_E_ARG, "gsr_shade_forward: bad N=%d deg=%d (2..5: the diffuse term reads base[0..8])", N, deg);
    if (N == 0) return GSR_OK;
    gsr::ShadeArgs a{N, deg, pos, normal, albedo, view_pos, kr, km, base, fg_lut, specular};
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    {
        GSR_STAGE(ST_SHADE_FWD);
        gsr::launch_shade_fwd(a, rgb, diffuse, specular_out, s);
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_shade_backward(int N, int deg, const float* pos, const float* normal, const float* albedo,
                       const float* view_pos, const float* kr, const float* km, const float* base,
                       const float* fg_lut, int specular, const float* g_rgb, const float* g_diffuse,
                       const float* g_specular, float* d_pos, float* d_normal, float* d_albedo, float* d_view_pos,
                       float* d_kr, float* d_km, float* d_base, void* workspace, void* stream_) {
    if (N < 0 || deg < 2 || deg > 5) return fail(GSR_E_ARG, "gsr_shade_backward: bad N=%d deg=%d (2..5)", N, deg);
    gsr::ShadeArgs a{N, deg, pos, normal, albedo, view_pos, kr, km, base, fg_lut, specular};
    gsr::ShadeGrads g{g_rgb, g_diffuse, g_specular, d_pos, d_normal, d_albedo, d_view_pos, d_kr, d_km, d_base};
    if (d_base && !workspace && N > 0) return fail(GSR_E_ARG, "gsr_shade_backward: workspace required for d_base");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    {
        GSR_STAGE(ST_SHADE_BWD);
        gsr::launch_shade_bwd(a, g, workspace, s);
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

// ---- fused relit features ----------------------------------------------
namespace {
struct RelitWs {
    size_t shade_ws, relit_ws, total;
};
RelitWs relit_ws_layout(int P, int N_fg, int deg, int sky_deg) {
    RelitWs w{};
    size_t t = 0;
    auto take = [&](size_t b) { const size_t o = t; t += (b + 255) & ~(size_t)255; return o; };
    w.shade_ws = take(gsr::shade_workspace_bytes(P, deg));  // d_base partials per 256 Gaussians of all P
    w.relit_ws = take(gsr::relit_workspace_bytes(P, sky_deg));
    w.total = t + 256;
    return w;
}
}  // namespace

size_t gsr_relit_workspace_bytes(int P, int N_fg, int deg, int sky_deg) {
    return relit_ws_layout(P, N_fg, deg, sky_deg).total;
}

int gsr_relit_features(int P, int N_fg, const float* xyz, const float* rotation, const float* scaling,
                       const int* fg_rank, const int* fg_rows, const float* albedo, const float* roughness,
                       const float* metalness, int deg, const float* base, const float* fg_lut, int specular,
                       int sky_deg, const float* sky_sh, const float* campos, const float* viewmatrix,
                       float* features, void* workspace, void* stream_) {
    if (P < 0 || N_fg < 0 || N_fg > P || deg < 2 || deg > 5 || sky_deg < -1 || sky_deg > 3)
        return fail(GSR_E_ARG, "gsr_relit_features: bad sizes P=%d N_fg=%d deg=%d sky_deg=%d", P, N_fg, deg, sky_deg);
    if (P == 0) return GSR_OK;
    if (!xyz || !rotation || !scaling || !fg_rank || !features || !workspace || !campos || !viewmatrix ||
        (N_fg > 0 && (!fg_rows || !albedo || !base || !fg_lut || (specular && !roughness))) ||
        (sky_deg >= 0 && !sky_sh))
        return fail(GSR_E_ARG, "gsr_relit_features: missing inputs");
    if ((reinterpret_cast<uintptr_t>(features) & 15u) != 0)
        return fail(GSR_E_ARG, "gsr_relit_features: features must be 16-B aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    const RelitWs wl = relit_ws_layout(P, N_fg, deg, sky_deg);
    char* ws = align_base(workspace);
    gsr::RelitArgs ra{P, xyz, rotation, scaling, fg_rank, sky_deg, sky_sh, campos, viewmatrix, features};
    {
        GSR_STAGE(ST_SHADE_FWD);
        // one pass over all P: geometry, sky rows, and the foreground shade in place
        // (gsr_shade.hip k_relit_fwd; the shade's rows are the Gaussians themselves)
        gsr::ShadeArgs a{N_fg, deg, xyz, nullptr, albedo, campos, roughness, metalness, base, fg_lut, specular};
        a.io_stride = gsr::RELIT_STRIDE;
        a.vp_stride = 0;
        a.viewmatrix = viewmatrix;
        gsr::launch_relit_fwd(ra, a, s);
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_relit_features_backward(int P, int N_fg, const float* xyz, const float* rotation, const float* scaling,
                                const int* fg_rank, const int* fg_rows, const float* albedo, const float* roughness,
                                const float* metalness, int deg, const float* base, const float* fg_lut, int specular,
                                int sky_deg, const float* sky_sh, const float* campos, const float* viewmatrix,
                                const float* dL_dfeatures, float* d_xyz, float* d_rotation, float* d_albedo,
                                float* d_roughness, float* d_metalness, float* d_base, float* d_sky_sh,
                                void* workspace, unsigned accumulate, void* stream_) {
    if (P < 0 || N_fg < 0 || N_fg > P || deg < 2 || deg > 5 || sky_deg < -1 || sky_deg > 3)
        return fail(GSR_E_ARG, "gsr_relit_features_backward: bad sizes");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream_);
    if (P == 0) {
        if (d_base) HIP_OK(hipMemsetAsync(d_base, 0, sizeof(float) * 3 * (deg + 1) * (deg + 1), s));
        if (d_sky_sh && sky_deg >= 0) HIP_OK(hipMemsetAsync(d_sky_sh, 0, sizeof(float) * 3 * (sky_deg + 1) * (sky_deg + 1), s));
        return GSR_OK;
    }
    if (!dL_dfeatures || !d_xyz || !d_rotation || !workspace) return fail(GSR_E_ARG, "gsr_relit_features_backward: missing buffers");
    const RelitWs wl = relit_ws_layout(P, N_fg, deg, sky_deg);
    char* ws = align_base(workspace);
    gsr::RelitArgs ra{P, xyz, rotation, scaling, fg_rank, sky_deg, sky_sh, campos, viewmatrix, nullptr};
    {
        GSR_STAGE(ST_SHADE_BWD);
        // one pass over all P (gsr_shade.hip k_relit_bwd): the foreground shade backward on the
        // recomputed normal, then the preparation's chain; d_base / d_sky_sh by fixed-order
        // reductions of its per-workgroup partials
        gsr::ShadeArgs a{N_fg, deg, xyz, nullptr, albedo, campos, roughness, metalness, base, fg_lut, specular};
        a.io_stride = gsr::RELIT_STRIDE;
        a.vp_stride = 0;
        gsr::ShadeGrads g{dL_dfeatures, dL_dfeatures + 3, specular ? dL_dfeatures + 6 : nullptr, nullptr, nullptr,
                          N_fg > 0 ? d_albedo : nullptr, nullptr, (specular && N_fg > 0) ? d_roughness : nullptr,
                          (specular && N_fg > 0) ? d_metalness : nullptr, d_base};
        g.acc = accumulate & (gsr::ACC_ALBEDO | gsr::ACC_ROUGH | gsr::ACC_METAL);
        gsr::RelitGrads rg{dL_dfeatures, d_xyz, d_rotation, d_sky_sh, at<float>(ws, wl.relit_ws),
                           accumulate & (gsr::ACC_MEAN3D | gsr::ACC_ROT)};
        gsr::launch_relit_bwd(ra, rg, a, g, at<void>(ws, wl.shade_ws), s);
    }
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_relit_epilogue(int width, int height, const float* cam12, const float* n01, const float* depth,
                       const float* alpha, const float* sky_mask, int normal_view, float* normal, float* normal_ref,
                       void* stream_) {
    if (width <= 0 || height <= 0) return fail(GSR_E_ARG, "gsr_relit_epilogue: bad size");
    if (!cam12 || !n01 || !depth || !alpha || !sky_mask || !normal || !normal_ref)
        return fail(GSR_E_ARG, "gsr_relit_epilogue: missing buffers");
    gsr::launch_epilogue_fwd(width, height, cam12, n01, depth, alpha, sky_mask, normal_view, normal, normal_ref,
                             reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_relit_epilogue_backward(int width, int height, const float* cam12, const float* depth, const float* alpha,
                                const float* sky_mask, int normal_view, const float* g_normal,
                                const float* g_normal_ref, float* d_n01, float* d_depth, void* stream_) {
    if (width <= 0 || height <= 0) return fail(GSR_E_ARG, "gsr_relit_epilogue_backward: bad size");
    if (!cam12 || !depth || !alpha || !sky_mask) return fail(GSR_E_ARG, "gsr_relit_epilogue_backward: missing buffers");
    gsr::launch_epilogue_bwd(width, height, cam12, depth, alpha, sky_mask, normal_view, g_normal, g_normal_ref, d_n01,
                             d_depth, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_texture2d_forward(int nb, int npix, int tex_nb, int tex_h, int tex_w, int C, const float* tex,
                          const float* uv, int filter, int boundary, float* out, void* stream_) {
    if (nb < 0 || npix < 0 || tex_h <= 0 || tex_w <= 0 || C <= 0 || (tex_nb != 1 && tex_nb != nb))
        return fail(GSR_E_ARG, "gsr_texture2d_forward: bad sizes");
    if (filter < 0 || filter > 1 || boundary < 0 || boundary > 2)
        return fail(GSR_E_ARG, "gsr_texture2d_forward: bad filter/boundary mode");
    if ((long long)nb * npix > 0x7fffffffLL) return fail(GSR_E_OVERFLOW, "gsr_texture2d_forward: too many lookups");
    if (nb * npix > 0 && (!tex || !uv || !out)) return fail(GSR_E_ARG, "gsr_texture2d_forward: missing buffers");
    gsr::launch_texture_fwd(nb, npix, tex_nb, tex_h, tex_w, C, tex, uv, filter, boundary, out,
                            reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_texture2d_backward(int nb, int npix, int tex_nb, int tex_h, int tex_w, int C, const float* tex,
                           const float* uv, int filter, int boundary, const float* dout, float* d_uv, float* d_tex,
                           void* stream_) {
    if (nb < 0 || npix < 0 || tex_h <= 0 || tex_w <= 0 || C <= 0 || (tex_nb != 1 && tex_nb != nb))
        return fail(GSR_E_ARG, "gsr_texture2d_backward: bad sizes");
    if (filter < 0 || filter > 1 || boundary < 0 || boundary > 2)
        return fail(GSR_E_ARG, "gsr_texture2d_backward: bad filter/boundary mode");
    if ((long long)nb * npix > 0x7fffffffLL) return fail(GSR_E_OVERFLOW, "gsr_texture2d_backward: too many lookups");
    if (nb * npix > 0 && (!tex || !uv || !dout)) return fail(GSR_E_ARG, "gsr_texture2d_backward: missing buffers");
    gsr::launch_texture_bwd(nb, npix, tex_nb, tex_h, tex_w, C, tex, uv, filter, boundary, dout, d_uv, d_tex,
                            reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_adam_step(long long n, int nseg, const long long* seg_end, const double* seg_lr, double beta1, double beta2,
                  double eps, int step, float grad_scale, float* param, const float* grad, float* exp_avg,
                  float* exp_avg_sq, void* stream_) {
    return gsr_adam_step_range(n, 0, n, nseg, seg_end, seg_lr, beta1, beta2, eps, step, grad_scale, param, grad,
                               exp_avg, exp_avg_sq, stream_);
}

int gsr_adam_step_range(long long n, long long lo, long long hi, int nseg, const long long* seg_end,
                        const double* seg_lr, double beta1, double beta2, double eps, int step, float grad_scale,
                        float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* stream_) {
    if (n < 0 || nseg < 1 || nseg > gsr::ADAM_MAX_SEGS || step < 1)
        return fail(GSR_E_ARG, "gsr_adam_step: bad sizes n=%lld nseg=%d step=%d", n, nseg, step);
    if (lo < 0 || hi > n || lo > hi || (lo & 3))
        return fail(GSR_E_ARG, "gsr_adam_step_range: bad range [%lld, %lld) of %lld (lo must be a multiple of 4)", lo,
                    hi, n);
    if (n == 0 || lo == hi) return GSR_OK;
    if (!seg_end || !seg_lr || !param || !grad || !exp_avg || !exp_avg_sq)
        return fail(GSR_E_ARG, "gsr_adam_step: missing buffers");
    for (const void* q : {(const void*)param, (const void*)grad, (const void*)exp_avg, (const void*)exp_avg_sq})
        if (reinterpret_cast<uintptr_t>(q) & 15u) return fail(GSR_E_ARG, "gsr_adam_step: buffers must be 16-B aligned");
    if (seg_end[nseg - 1] != n) return fail(GSR_E_ARG, "gsr_adam_step: last segment must end at n");
    gsr::AdamSegs s;
    memset(&s, 0, sizeof(s));
    s.n = nseg;
    // torch: bias_correction1 = 1 - beta1 ** step, step_size = lr / bias_correction1,
    // bias_correction2_sqrt = (1 - beta2 ** step) ** 0.5 (Python floats, i.e. double)
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    long long prev = 0;
    for (int k = 0; k < nseg; k++) {
        if (seg_end[k] < prev) return fail(GSR_E_ARG, "gsr_adam_step: segment ends must ascend");
        prev = s.end[k] = seg_end[k];
        s.step_size[k] = (float)(seg_lr[k] / bc1);
    }
    s.bc2_sqrt = (float)sqrt(bc2);
    // the scalars as torch passes them (Python floats, cast to the fp32 op math)
    s.one_minus_b1 = (float)(1.0 - beta1);
    s.b2 = (float)beta2;
    s.one_minus_b2 = (float)(1.0 - beta2);
    s.eps = (float)eps;
    s.grad_scale = grad_scale;
    gsr::launch_adam(lo, hi, s, param, grad, exp_avg, exp_avg_sq, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

long long gsr_ssim_partials(int C, int height, int width) {
    if (C <= 0 || height <= 0 || width <= 0) return 0;
    const dim3 g = gsr::ssim_grid(C, height, width);
    return (long long)g.x * g.y * g.z;
}

static bool ssim_window(const float* window, gsr::SsimWindow& w) {
    if (!window) return false;
    for (int k = 0; k < 11; k++) w.w[k] = window[k];
    return true;
}

int gsr_ssim_forward(int C, int height, int width, const float* img1, const float* img2, const float* mask,
                     long long mask_cstride, const float* window, float* block_sums, float* dmaps, void* stream_) {
    if (C <= 0 || C > 65535 || height <= 0 || width <= 0) return fail(GSR_E_ARG, "gsr_ssim_forward: bad sizes");
    gsr::SsimWindow w;
    if (!img1 || !img2 || !block_sums || !ssim_window(window, w)) return fail(GSR_E_ARG, "gsr_ssim_forward: missing buffers");
    gsr::launch_ssim_fwd(C, height, width, img1, img2, mask, mask_cstride, w, 0.01f * 0.01f, 0.03f * 0.03f, block_sums,
                         dmaps, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_ssim_backward(int C, int height, int width, const float* img1, const float* img2, const float* dmaps,
                      const float* gscale, const float* window, float* dimg1, int accumulate, void* stream_) {
    if (C <= 0 || C > 65535 || height <= 0 || width <= 0) return fail(GSR_E_ARG, "gsr_ssim_backward: bad sizes");
    gsr::SsimWindow w;
    if (!img1 || !img2 || !dmaps || !gscale || !dimg1 || !ssim_window(window, w))
        return fail(GSR_E_ARG, "gsr_ssim_backward: missing buffers");
    gsr::launch_ssim_bwd(C, height, width, img1, img2, dmaps, gscale, w, dimg1, accumulate ? 1 : 0,
                         reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_ssim_l1_backward(int C, int height, int width, const float* img1, const float* img2, const float* dmaps,
                         const float* gscale, const float* window, const float* occ, const float* l1_coef,
                         float* dimg1, void* stream_) {
    if (C <= 0 || C > 65535 || height <= 0 || width <= 0) return fail(GSR_E_ARG, "gsr_ssim_l1_backward: bad sizes");
    gsr::SsimWindow w;
    if (!img1 || !img2 || !dmaps || !gscale || !occ || !l1_coef || !dimg1 || !ssim_window(window, w))
        return fail(GSR_E_ARG, "gsr_ssim_l1_backward: missing buffers");
    gsr::launch_ssim_bwd(C, height, width, img1, img2, dmaps, gscale, w, dimg1, 0, reinterpret_cast<hipStream_t>(stream_),
                         occ, l1_coef);
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_objective(int n_loss_partials, const float* loss_partials, long long n_ssim_partials,
                       const float* ssim_partials, int npix, double lambda_dssim, double lambda_sky,
                       double lambda_normal, float* loss, float* coef, void* stream_) {
    if (n_loss_partials <= 0 || n_ssim_partials <= 0 || n_ssim_partials > 0x7fffffffLL || npix <= 0)
        return fail(GSR_E_ARG, "gsr_view_objective: bad sizes");
    if (!loss_partials || !ssim_partials || !loss || !coef) return fail(GSR_E_ARG, "gsr_view_objective: missing buffers");
    gsr::launch_view_objective(n_loss_partials, loss_partials, (int)n_ssim_partials, ssim_partials, npix, lambda_dssim,
                               lambda_sky, lambda_normal, loss, coef, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_loss_partials(int npix) { return npix > 0 ? gsr::view_loss_blocks(npix) : 0; }

int gsr_view_loss_forward(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                          const float* nrm, const float* nref, const float* sky, const float* occ, float* partials,
                          void* stream_) {
    if (npix <= 0) return fail(GSR_E_ARG, "gsr_view_loss_forward: bad size");
    if (!img || !gt || !diff || !spec || !nrm || !nref || !sky || !occ || !partials)
        return fail(GSR_E_ARG, "gsr_view_loss_forward: missing buffers");
    gsr::launch_view_loss_fwd(npix, img, gt, diff, spec, nrm, nref, sky, occ, partials,
                              reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_loss_backward(int npix, const float* img, const float* gt, const float* diff, const float* spec,
                           const float* nrm, const float* nref, const float* sky, const float* occ, const float* coef,
                           float* d_img, float* d_diff, float* d_spec, float* d_nrm, float* d_nref, void* stream_) {
    if (npix <= 0) return fail(GSR_E_ARG, "gsr_view_loss_backward: bad size");
    if (!img || !gt || !diff || !spec || !nrm || !nref || !sky || !occ || !coef)
        return fail(GSR_E_ARG, "gsr_view_loss_backward: missing buffers");
    gsr::launch_view_loss_bwd(npix, img, gt, diff, spec, nrm, nref, sky, occ, coef, d_img, d_diff, d_spec, d_nrm,
                              d_nref, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

/* ---- training-step bookkeeping (csrc/gsr_trainaux.hip) ---- */
static int view_ptrs_int(int V, const int* const* src, gsr::ViewPtrs<int>& dst) {
    for (int v = 0; v < gsr::REG_MAXV; v++) dst.p[v] = nullptr;
    for (int v = 0; v < V; v++) {
        if (!src[v]) return 0;
        dst.p[v] = src[v];
    }
    return 1;
}

int gsr_view_regularisers_partials(int P) { return P <= 0 ? 0 : gsr::view_regs_blocks(P); }

int gsr_view_regularisers_forward(int P, int V, const float* xyz, const float* scaling, const int* const* radii,
                                  const unsigned char* is_sky, const float* depth_cols, float* partials,
                                  void* stream_) {
    if (P <= 0 || V <= 0 || V > gsr::REG_MAXV)
        return fail(GSR_E_ARG, "gsr_view_regularisers_forward: bad P=%d V=%d (1..%d views)", P, V, gsr::REG_MAXV);
    if (!xyz || !scaling || !radii || !is_sky || !depth_cols || !partials)
        return fail(GSR_E_ARG, "gsr_view_regularisers_forward: missing buffers");
    gsr::ViewPtrs<int> rp;
    if (!view_ptrs_int(V, radii, rp)) return fail(GSR_E_ARG, "gsr_view_regularisers_forward: missing radii");
    gsr::launch_view_regs_fwd(P, V, xyz, scaling, rp, is_sky, depth_cols, partials,
                              reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_regularisers_backward(int P, int V, const float* scaling, const int* const* radii,
                                   const unsigned char* is_sky, const float* depth_cols, const float* grad_sums,
                                   float* d_xyz, float* d_scaling, unsigned accumulate, void* stream_) {
    if (P <= 0 || V <= 0 || V > gsr::REG_MAXV)
        return fail(GSR_E_ARG, "gsr_view_regularisers_backward: bad P=%d V=%d (1..%d views)", P, V, gsr::REG_MAXV);
    if (!scaling || !radii || !is_sky || !depth_cols || !grad_sums)
        return fail(GSR_E_ARG, "gsr_view_regularisers_backward: missing buffers");
    gsr::ViewPtrs<int> rp;
    if (!view_ptrs_int(V, radii, rp)) return fail(GSR_E_ARG, "gsr_view_regularisers_backward: missing radii");
    gsr::launch_view_regs_bwd(P, V, scaling, rp, is_sky, depth_cols, grad_sums, d_xyz, d_scaling,
                              accumulate & (gsr::ACC_MEAN3D | gsr::ACC_SCALE), reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_densify_stats(int P, int V, const float* const* grad_means2D, const int* const* radii, float* accum,
                      float* denom, float* max_radii, void* stream_) {
    if (P < 0 || V <= 0 || V > gsr::REG_MAXV)
        return fail(GSR_E_ARG, "gsr_densify_stats: bad P=%d V=%d (1..%d views)", P, V, gsr::REG_MAXV);
    if (P == 0) return GSR_OK;
    const bool sums = accum || denom;
    if (!radii || !max_radii || (sums && (!accum || !denom || !grad_means2D)))
        return fail(GSR_E_ARG, "gsr_densify_stats: missing buffers");
    gsr::ViewPtrs<int> rp;
    gsr::ViewPtrs<float> gp;
    if (!view_ptrs_int(V, radii, rp)) return fail(GSR_E_ARG, "gsr_densify_stats: missing radii");
    for (int v = 0; v < gsr::REG_MAXV; v++) gp.p[v] = nullptr;
    for (int v = 0; sums && v < V; v++) {
        if (!grad_means2D[v]) return fail(GSR_E_ARG, "gsr_densify_stats: missing means2D gradient");
        gp.p[v] = grad_means2D[v];
    }
    gsr::launch_densify_stats(P, V, gp, rp, accum, denom, max_radii, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_sh_basis(int N, int deg, const float* dirs, float* out, void* stream_) {
    if (N < 0 || deg < 0 || deg > 4) return fail(GSR_E_ARG, "gsr_sh_basis: bad N=%d deg=%d (0..4)", N, deg);
    if (N == 0) return GSR_OK;
    if (!dirs || !out) return fail(GSR_E_ARG, "gsr_sh_basis: missing buffers");
    gsr::launch_sh_basis(N, deg, dirs, out, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_sky_xyz_partials(int N) { return N <= 0 ? 0 : gsr::sky_blocks(N); }

int gsr_sky_xyz_forward(int N, const float* angles, const float* radius, const float* center, float* xyz,
                        void* stream_) {
    if (N < 0) return fail(GSR_E_ARG, "gsr_sky_xyz_forward: bad N");
    if (N == 0) return GSR_OK;
    if (!angles || !radius || !center || !xyz) return fail(GSR_E_ARG, "gsr_sky_xyz_forward: missing buffers");
    gsr::launch_sky_xyz_fwd(N, angles, radius, center, xyz, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_sky_xyz_backward(int N, const float* angles, const float* radius, const float* grad_xyz, float* d_angles,
                         float* d_radius_partials, void* stream_) {
    if (N < 0) return fail(GSR_E_ARG, "gsr_sky_xyz_backward: bad N");
    if (N == 0) return GSR_OK;
    if (!angles || !radius || !grad_xyz || !d_angles || !d_radius_partials)
        return fail(GSR_E_ARG, "gsr_sky_xyz_backward: missing buffers");
    gsr::launch_sky_xyz_bwd(N, angles, radius, grad_xyz, d_angles, d_radius_partials,
                            reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

/* ---- the model's activations (csrc/gsr_trainaux.hip) ---- */
static int act_args(int P, int n_fg, int n_sky, const int* src, const float* xyz_fg, const float* angles,
                    const float* radius, const float* center, const float* scale_raw, const float* rot_raw,
                    const float* op_raw, const float* alb_raw, const float* rough_raw, const float* metal_raw,
                    gsr::ActArgs& a) {
    if (P < 0 || n_fg < 0 || n_sky < 0 || n_fg + n_sky != P) return 0;
    if (P && (!scale_raw || !rot_raw || !op_raw)) return 0;
    if (n_fg && (!xyz_fg || !alb_raw || !rough_raw || !metal_raw)) return 0;
    if (n_sky && (!angles || !radius || !center)) return 0;
    a = gsr::ActArgs{P, n_fg, n_sky, src, xyz_fg, angles, radius, center, scale_raw, rot_raw, op_raw, alb_raw, rough_raw,
                     metal_raw};
    return 1;
}

int gsr_activations_partials(int P, int n_fg) {
    gsr::ActArgs a{};
    a.P = P;
    a.Nfg = n_fg;
    return (P <= 0 && n_fg <= 0) ? 0 : gsr::activation_blocks(a);
}

int gsr_activations_forward(int P, int n_fg, int n_sky, const int* src, const float* xyz_fg, const float* angles,
                            const float* radius, const float* center, const float* scale_raw, const float* rot_raw,
                            const float* op_raw, const float* alb_raw, const float* rough_raw, const float* metal_raw,
                            float* xyz, float* scale, float* rot, float* op, float* alb, float* rough, float* metal,
                            void* stream_) {
    gsr::ActArgs a;
    if (!act_args(P, n_fg, n_sky, src, xyz_fg, angles, radius, center, scale_raw, rot_raw, op_raw, alb_raw, rough_raw,
                  metal_raw, a))
        return fail(GSR_E_ARG, "gsr_activations_forward: bad sizes (P=%d fg=%d sky=%d) or missing inputs", P, n_fg, n_sky);
    if (P + n_fg == 0) return GSR_OK;
    if ((P && (!xyz || !scale || !rot || !op)) || (n_fg && (!alb || !rough || !metal)))
        return fail(GSR_E_ARG, "gsr_activations_forward: missing outputs");
    gsr::launch_activations_fwd(a, gsr::ActOutW{xyz, scale, rot, op, alb, rough, metal},
                                reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_activations_backward(int P, int n_fg, int n_sky, const int* src, const float* xyz_fg, const float* angles,
                             const float* radius, const float* center, const float* scale_raw, const float* rot_raw,
                             const float* op_raw, const float* alb_raw, const float* rough_raw, const float* metal_raw,
                             const float* scale, const float* rot, const float* op, const float* alb,
                             const float* rough, const float* metal, const float* g_xyz, const float* g_scale,
                             const float* g_rot, const float* g_op, const float* g_alb, const float* g_rough,
                             const float* g_metal, float* d_xyz_fg, float* d_angles, float* d_radius,
                             float* radius_partials, float* d_scale_raw, float* d_rot_raw, float* d_op_raw,
                             float* d_alb_raw, float* d_rough_raw, float* d_metal_raw, void* stream_) {
    gsr::ActArgs a;
    if (!act_args(P, n_fg, n_sky, src, xyz_fg, angles, radius, center, scale_raw, rot_raw, op_raw, alb_raw, rough_raw,
                  metal_raw, a))
        return fail(GSR_E_ARG, "gsr_activations_backward: bad sizes (P=%d fg=%d sky=%d) or missing inputs", P, n_fg, n_sky);
    if (P + n_fg == 0) return GSR_OK;
    if ((P && (!scale || !rot || !op || !d_scale_raw || !d_rot_raw || !d_op_raw)) ||
        (n_fg && (!alb || !rough || !metal || !d_xyz_fg || !d_alb_raw || !d_rough_raw || !d_metal_raw)) ||
        (n_sky && (!d_angles || !d_radius || !radius_partials)))
        return fail(GSR_E_ARG, "gsr_activations_backward: missing buffers");
    const gsr::ActOut o{nullptr, scale, rot, op, alb, rough, metal};
    const gsr::ActOut g{g_xyz, g_scale, g_rot, g_op, g_alb, g_rough, g_metal};
    const gsr::ActGrad d{d_xyz_fg, d_angles, n_sky ? radius_partials : nullptr, d_scale_raw, d_rot_raw, d_op_raw,
                         d_alb_raw, d_rough_raw, d_metal_raw};
    gsr::launch_activations_bwd(a, o, g, d, n_sky ? d_radius : nullptr, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_regularisers_tail_forward(int V, int n_samples, const float* sums, const float* basis, const float* env_sh,
                                       float lambda_env, float lambda_scale, float lambda_depth, float gamma,
                                       int depth_on, float* total, void* stream_) {
    if (V <= 0 || V > 8 || n_samples <= 0 || n_samples > 32)
        return fail(GSR_E_ARG, "gsr_view_regularisers_tail_forward: bad V=%d samples=%d (1..8, 1..32)", V, n_samples);
    if (!sums || !basis || !env_sh || !total) return fail(GSR_E_ARG, "gsr_view_regularisers_tail_forward: missing buffers");
    const gsr::RegsTail t{V, n_samples, depth_on ? 1 : 0, lambda_env, lambda_scale, lambda_depth, gamma, sums, basis, env_sh};
    gsr::launch_regs_tail_fwd(t, total, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

int gsr_view_regularisers_tail_backward(int V, int n_samples, const float* sums, const float* basis,
                                        const float* env_sh, float lambda_env, float lambda_scale, float lambda_depth,
                                        float gamma, int depth_on, const float* grad_total, float* d_sums,
                                        float* d_env_sh, void* stream_) {
    if (V <= 0 || V > 8 || n_samples <= 0 || n_samples > 32)
        return fail(GSR_E_ARG, "gsr_view_regularisers_tail_backward: bad V=%d samples=%d (1..8, 1..32)", V, n_samples);
    if (!sums || !basis || !env_sh || !grad_total || !d_sums || !d_env_sh)
        return fail(GSR_E_ARG, "gsr_view_regularisers_tail_backward: missing buffers");
    const gsr::RegsTail t{V, n_samples, depth_on ? 1 : 0, lambda_env, lambda_scale, lambda_depth, gamma, sums, basis, env_sh};
    gsr::launch_regs_tail_bwd(t, grad_total, d_sums, d_env_sh, reinterpret_cast<hipStream_t>(stream_));
    GSR_LAUNCH_CHECK();
    return GSR_OK;
}

}  // extern "C"
