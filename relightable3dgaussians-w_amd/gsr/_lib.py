"""ctypes binding of libgsr.so (C ABI: include/gsr.h).

The product path: every call lands in hand-written HIP for gfx950.  There is no CPU or
PyTorch fallback -- if the library or a GPU is missing, calls raise.
"""
import contextlib
import ctypes as C
import os
import subprocess
import threading

import torch

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GSR_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libgsr.so")
CSRC = os.path.join(PKG_DIR, "csrc")

RESIZE_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_size_t)

_lib = None
_lock = threading.Lock()


class Layout(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in (
        "geom_bytes", "img_bytes", "bin_bytes", "geom_radii", "geom_tiles", "geom_depth_key", "geom_rect",
        "geom_rec", "geom_acc", "img_final_T", "img_n_contrib", "img_ranges", "img_tile_nmax", "img_tile_emax",
        "bin_st_ranges", "bin_entries", "img_tile_cost", "img_row_cost", "img_order_bwd", "img_nheavy",
        "img_surv_n", "img_surv", "surv_cap")]


DEBUG_LIB_PATH = os.path.join(PKG_DIR, "lib", "debug", "libgsr.so")


def build(jobs=8, arch="gfx950"):
    """Compile libgsr.so in-tree (hipcc --offload-arch=gfx950), and the GSR_DEBUG
    invariant-checking variant lib/debug/libgsr.so (selected with GSR_LIB_PATH)."""
    subprocess.check_call(["make", "-s", "-C", CSRC, f"-j{jobs}", f"ARCH={arch}"])
    subprocess.check_call(["make", "-s", "-C", CSRC, f"-j{jobs}", f"ARCH={arch}", "debug"])


def _declare(lib):
    vp, i, f, sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
    lib.gsr_forward.argtypes = [RESIZE_FN, vp, RESIZE_FN, vp, RESIZE_FN, vp, i, i, i, vp, i, i, vp, vp, vp, vp, vp, f,
                                vp, vp, vp, vp, vp, f, f, i, vp, vp, vp, C.POINTER(C.c_int)]
    lib.gsr_backward.argtypes = [i, i, i, i, vp, i, i, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, f, f, vp, vp, vp, vp,
                                 vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.gsr_mark_visible.argtypes = [i, vp, vp, vp, vp, vp]
    lib.gsr_knn_workspace_bytes.argtypes = [i]
    lib.gsr_knn_workspace_bytes.restype = sz
    lib.gsr_knn_mean_dist.argtypes = [i, vp, vp, vp, vp]
    lib.gsr_forward_reuse.argtypes = [RESIZE_FN, vp, vp, vp, vp, vp, i, i, vp, i, i, vp, vp, vp, vp]
    lib.gsr_forward_channels.argtypes = [RESIZE_FN, vp, RESIZE_FN, vp, RESIZE_FN, vp, i, i, i, vp, vp, i, i, vp, vp, vp,
                                         f, vp, vp, vp, vp, vp, f, f, i, vp, vp, vp, C.POINTER(C.c_int)]
    lib.gsr_backward_channels.argtypes = [i, i, i, vp, i, vp, i, i, vp, vp, f, vp, vp, vp, vp, vp, f, f, vp, vp, vp, vp,
                                          vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_uint, vp]
    lib.gsr_relit_workspace_bytes.argtypes = [i, i, i, i]
    lib.gsr_relit_workspace_bytes.restype = sz
    lib.gsr_relit_features.argtypes = [i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, vp, i, i, vp, vp, vp, vp, vp, vp]
    lib.gsr_relit_features_backward.argtypes = [i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, vp, i, i, vp, vp, vp, vp,
                                                vp, vp, vp, vp, vp, vp, vp, vp, C.c_uint, vp]
    lib.gsr_relit_epilogue.argtypes = [i, i, vp, vp, vp, vp, vp, i, vp, vp, vp]
    lib.gsr_relit_epilogue_backward.argtypes = [i, i, vp, vp, vp, vp, i, vp, vp, vp, vp, vp]
    lib.gsr_texture2d_forward.argtypes = [i, i, i, i, i, i, vp, vp, i, i, vp, vp]
    lib.gsr_texture2d_backward.argtypes = [i, i, i, i, i, i, vp, vp, i, i, vp, vp, vp, vp]
    lib.gsr_shade_forward.argtypes = [i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, vp, vp, vp]
    lib.gsr_shade_backward.argtypes = [i, i, vp, vp, vp, vp, vp, vp, vp, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                       vp, vp, vp]
    lib.gsr_adam_step.argtypes = [C.c_longlong, i, C.POINTER(C.c_longlong), C.POINTER(C.c_double), C.c_double, C.c_double,
                                  C.c_double, i, f, vp, vp, vp, vp, vp]
    lib.gsr_adam_step_range.argtypes = [C.c_longlong, C.c_longlong, C.c_longlong, i, C.POINTER(C.c_longlong),
                                        C.POINTER(C.c_double), C.c_double, C.c_double, C.c_double, i, f, vp, vp, vp,
                                        vp, vp]
    lib.gsr_view_loss_partials.argtypes = [i]
    lib.gsr_view_loss_forward.argtypes = [i] + [vp] * 9 + [vp]
    lib.gsr_view_loss_backward.argtypes = [i] + [vp] * 9 + [vp] * 5 + [vp]
    pa = C.POINTER(C.c_void_p)  # host array of device pointers, one per view
    lib.gsr_view_regularisers_partials.argtypes = [i]
    lib.gsr_view_regularisers_forward.argtypes = [i, i, vp, vp, pa, vp, vp, vp, vp]
    lib.gsr_view_regularisers_backward.argtypes = [i, i, vp, pa, vp, vp, vp, vp, vp, C.c_uint, vp]
    lib.gsr_densify_stats.argtypes = [i, i, pa, pa, vp, vp, vp, vp]
    lib.gsr_sh_basis.argtypes = [i, i, vp, vp, vp]
    lib.gsr_view_regularisers_tail_forward.argtypes = [i, i, vp, vp, vp, f, f, f, f, i, vp, vp]
    lib.gsr_view_regularisers_tail_backward.argtypes = [i, i, vp, vp, vp, f, f, f, f, i, vp, vp, vp, vp]
    lib.gsr_sky_xyz_partials.argtypes = [i]
    lib.gsr_sky_xyz_forward.argtypes = [i, vp, vp, vp, vp, vp]
    lib.gsr_sky_xyz_backward.argtypes = [i, vp, vp, vp, vp, vp, vp]
    lib.gsr_activations_partials.argtypes = [i, i]
    lib.gsr_activations_forward.argtypes = [i, i, i] + [vp] * 18 + [vp]
    lib.gsr_activations_backward.argtypes = [i, i, i] + [vp] * 34 + [vp]
    lib.gsr_ssim_partials.argtypes = [i, i, i]
    lib.gsr_ssim_partials.restype = C.c_longlong
    lib.gsr_ssim_forward.argtypes = [i, i, i, vp, vp, vp, C.c_longlong, C.POINTER(C.c_float), vp, vp, vp]
    lib.gsr_ssim_backward.argtypes = [i, i, i, vp, vp, vp, vp, C.POINTER(C.c_float), vp, i, vp]
    lib.gsr_ssim_l1_backward.argtypes = [i, i, i, vp, vp, vp, vp, C.POINTER(C.c_float), vp, vp, vp, vp]
    lib.gsr_view_objective.argtypes = [i, vp, C.c_longlong, vp, i, C.c_double, C.c_double, C.c_double, vp, vp, vp]
    lib.gsr_shade_workspace_bytes.argtypes = [i, i]
    lib.gsr_shade_workspace_bytes.restype = sz
    lib.gsr_get_layout.argtypes = [i, C.c_longlong, i, i, C.POINTER(Layout)]
    lib.gsr_profile_enable.argtypes = [i]
    lib.gsr_profile_stages.argtypes = [C.c_uint]
    lib.gsr_profile_stage_count.restype = i
    lib.gsr_profile_stage_name.argtypes = [i]
    lib.gsr_profile_stage_name.restype = C.c_char_p
    lib.gsr_profile_read.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_longlong), i, i]
    lib.gsr_set_deterministic.argtypes = [i]
    lib.gsr_set_survivor_lists.argtypes = [i]
    lib.gsr_set_exact_blend.argtypes = [i]
    lib.gsr_set_backward_heavy_bits.argtypes = [i]
    lib.gsr_check_buffers.argtypes = [i, i, i, i, vp, vp, vp, vp, vp]
    lib.gsr_materialize_lists.argtypes = [i, i, i, vp, vp, vp, vp]
    lib.gsr_last_error.restype = C.c_char_p
    lib.gsr_version.restype = C.c_char_p
    for fn in ("gsr_forward", "gsr_forward_reuse", "gsr_knn_mean_dist", "gsr_backward", "gsr_mark_visible", "gsr_shade_forward",
               "gsr_shade_backward", "gsr_forward_channels", "gsr_backward_channels",
               "gsr_relit_features", "gsr_relit_features_backward", "gsr_relit_epilogue",
               "gsr_relit_epilogue_backward", "gsr_adam_step", "gsr_adam_step_range", "gsr_ssim_forward", "gsr_ssim_backward",
               "gsr_ssim_l1_backward",
               "gsr_view_loss_forward", "gsr_view_loss_backward", "gsr_view_objective", "gsr_view_regularisers_forward",
               "gsr_view_regularisers_backward", "gsr_view_regularisers_tail_forward",
               "gsr_view_regularisers_tail_backward", "gsr_densify_stats", "gsr_sh_basis", "gsr_sky_xyz_forward",
               "gsr_sky_xyz_backward", "gsr_activations_forward", "gsr_activations_backward",
               "gsr_texture2d_forward", "gsr_texture2d_backward", "gsr_get_layout", "gsr_set_deterministic",
               "gsr_get_deterministic", "gsr_set_survivor_lists", "gsr_get_survivor_lists", "gsr_set_exact_blend", "gsr_get_exact_blend", "gsr_set_backward_heavy_bits", "gsr_debug_build", "gsr_check_buffers", "gsr_materialize_lists"):
        getattr(lib, fn).restype = C.c_int


def lib():
    """Load (never silently substitute) libgsr.so."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"libgsr.so not built ({LIB_PATH}); run __graft_entry__.build() "
                                       "or `make -C relightable3dgaussians-w_amd/csrc`")
                L = C.CDLL(LIB_PATH)
                _declare(L)
                _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().gsr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def require_gpu_tensor(t, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a GPU (HIP) tensor; this rasterizer has no CPU path")


def fptr(t):
    """Device pointer of a float32 tensor, or None for an empty tensor (= 'absent', as the
    reference's data<float>() of an empty tensor)."""
    if t is None or t.numel() == 0:
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"expected float32 tensor, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError("internal: pointer of a non-contiguous tensor")
    return t.data_ptr()


def ptr_array(ts):
    """A host array of the device pointers of ``ts`` (contiguous tensors), for the C ABI's
    per-view pointer-table arguments."""
    for t in ts:
        if not t.is_contiguous():
            raise RuntimeError("internal: pointer of a non-contiguous tensor")
    return (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def stream_of(device):
    return torch.cuda.current_stream(device).cuda_stream


def set_deterministic(on=True):
    """Deterministic backward (gsr_set_deterministic): fixed-order gradient sums instead of
    the tile passes' float atomics; bit-reproducible, slower (a debugging mode)."""
    check(lib().gsr_set_deterministic(int(bool(on))), "gsr_set_deterministic")


def deterministic():
    return bool(lib().gsr_get_deterministic())


def set_survivor_lists(on=True):
    """Survivor lists (gsr_set_survivor_lists): the backward walks the forward's per-tile
    survivors instead of re-filtering the super-tile lists (default on; identical results)."""
    check(lib().gsr_set_survivor_lists(int(bool(on))), "gsr_set_survivor_lists")


def survivor_lists():
    return bool(lib().gsr_get_survivor_lists())


def set_exact_blend(on=True):
    """Exact blend mode (gsr_set_exact_blend): the tile passes evaluate every (pixel, Gaussian)
    pair with the reference's float arithmetic bit for bit (forward colours, transmittance and
    n_contrib equal the canonical oracle's; slower).  Takes effect at the next forward; its
    backward replays that forward's mode."""
    check(lib().gsr_set_exact_blend(int(bool(on))), "gsr_set_exact_blend")


def exact_blend():
    return bool(lib().gsr_get_exact_blend())


@contextlib.contextmanager
def exact_blend_mode(on=True):
    """with _lib.exact_blend_mode(): ... -- exact blend mode inside the block, restored after."""
    before = exact_blend()
    set_exact_blend(on)
    try:
        yield
    finally:
        set_exact_blend(before)


def set_backward_heavy_bits(bits=-1):
    """The backward's heavy-tile split threshold, log2 of the estimated cost
    (gsr_set_backward_heavy_bits; -1: the build's default)."""
    check(lib().gsr_set_backward_heavy_bits(int(bits)), "gsr_set_backward_heavy_bits")


def debug_build():
    """True when the loaded library is the GSR_DEBUG build (lib/debug/libgsr.so)."""
    return bool(lib().gsr_debug_build())


def check_buffers(P, R, W, H, radii, geom, binb, img):
    """Verify a forward's tile lists and n_contrib against its preprocess (gsr_check_buffers);
    raises RuntimeError naming the first violated invariant."""
    check(lib().gsr_check_buffers(int(P), int(R), int(W), int(H), radii.data_ptr(), geom.data_ptr(),
                                  binb.data_ptr() if binb.numel() else None, img.data_ptr(),
                                  stream_of(radii.device)), "gsr_check_buffers")


def materialize_lists(R, W, H, binb):
    """The reference's point_list (int32 [R]) and tile ranges (int32 [T, 2]) of a forward, written
    from its binning buffer's super-tile lists (gsr_materialize_lists; synchronous)."""
    dev = binb.device
    T = ((W + 15) // 16) * ((H + 15) // 16)
    pl = torch.empty(max(int(R), 1), dtype=torch.int32, device=dev)
    rg = torch.empty((T, 2), dtype=torch.int32, device=dev)
    check(lib().gsr_materialize_lists(int(R), int(W), int(H), binb.data_ptr() if binb.numel() else None,
                                      pl.data_ptr(), rg.data_ptr(), stream_of(dev)), "gsr_materialize_lists")
    return pl[:int(R)], rg


def profile_enable(on=True):
    lib().gsr_profile_enable(int(bool(on)))


def profile_stages(names=None):
    """Time only the named stages while profiling is on (None: all)."""
    L = lib()
    if names is None:
        mask = 0xFFFFFFFF
    else:
        all_names = [L.gsr_profile_stage_name(k).decode() for k in range(L.gsr_profile_stage_count())]
        mask = 0
        for n in names:
            mask |= 1 << all_names.index(n)
    check(L.gsr_profile_stages(mask), "gsr_profile_stages")


def profile_read(reset=True):
    """{stage: (total_ms, launches)} accumulated since the last reset (waits for the events)."""
    L = lib()
    n = L.gsr_profile_stage_count()
    ms = (C.c_double * n)()
    cnt = (C.c_longlong * n)()
    check(L.gsr_profile_read(ms, cnt, n, int(bool(reset))), "gsr_profile_read")
    return {L.gsr_profile_stage_name(k).decode(): (ms[k], cnt[k]) for k in range(n)}


def layout(P, R, W, H):
    L = Layout()
    check(lib().gsr_get_layout(int(P), int(R), int(W), int(H), C.byref(L)), "gsr_get_layout")
    return L


class BufferSet:
    """Owns the three growable byte buffers of one forward call (the reference's
    geomBuffer / binningBuffer / imgBuffer torch.uint8 tensors, rasterize_points.cu:70-77)."""

    def __init__(self, device):
        self.device = device
        self.bufs = [torch.empty(0, dtype=torch.uint8, device=device) for _ in range(3)]


_live = {}
_next = [1]


def _resize(ctx, n):
    key = int(ctx)
    bs = _live[key >> 2]
    t = torch.empty(int(n), dtype=torch.uint8, device=bs.device)
    bs.bufs[key & 3] = t
    return t.data_ptr()


RESIZE = RESIZE_FN(_resize)


class ResizeContexts:
    def __init__(self, bs):
        with _lock:
            self.id = _next[0]
            _next[0] += 1
        _live[self.id] = bs
        self.ctx = [C.c_void_p((self.id << 2) | k) for k in range(3)]

    def close(self):
        _live.pop(self.id, None)
