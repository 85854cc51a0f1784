"""CPU checks of the drop-in boundary: libgsr.so loads and exports every symbol that
include/gsr.h declares; the Python package imports and refuses CPU tensors (no fallback)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gsr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsr_[a-z_]+)\s*\(", src)) - {"gsr_resize_fn"})


def test_header_declares_the_reference_entry_points():
    syms = declared_symbols()
    for s in ("gsr_forward", "gsr_backward", "gsr_mark_visible", "gsr_shade_forward", "gsr_shade_backward"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gsr import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert _lib.lib().gsr_version().decode().startswith("gsr")


def test_layout_query_is_consistent():
    from gsr import _lib
    L = _lib.layout(1000, 12345, 1920, 1080)
    assert L.geom_bytes > 1000 * (48 + 64) and L.bin_bytes >= 8 * 255 and L.img_bytes >= 1920 * 1080 * 8
    for off in (L.geom_rec, L.geom_acc, L.img_ranges, L.bin_st_ranges, L.bin_entries):
        assert off % 256 == 0
    # the backward's order buffers and the survivor lists (appended fields): disjoint, in order,
    # inside the image buffer; the lists (the last region) are reserved only while they are on
    T, gy = 120 * 68, 68
    spans = [(L.img_tile_cost, 4 * T), (L.img_row_cost, 4 * gy), (L.img_order_bwd, 4 * T), (L.img_nheavy, 4 * 80),
             (L.img_surv_n, 4 * T), (L.img_surv, 8 * L.surv_cap * T)]
    for (a, n), (b, _) in zip(spans, spans[1:]):
        assert a + n <= b
    before = _lib.survivor_lists()
    try:
        _lib.set_survivor_lists(True)
        on = _lib.layout(1000, 12345, 1920, 1080)
        assert on.img_surv + 8 * on.surv_cap * T <= on.img_bytes
        _lib.set_survivor_lists(False)
        off = _lib.layout(1000, 12345, 1920, 1080)
        assert off.img_surv == on.img_surv and off.img_surv_n == on.img_surv_n  # the same offsets
        assert off.img_surv <= off.img_bytes < on.img_bytes - 8 * on.surv_cap * T + 4096
    finally:
        _lib.set_survivor_lists(before)


def test_cpu_tensors_are_rejected():
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    e = torch.empty(0)
    with pytest.raises(RuntimeError, match="GPU"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(10, 3), e, e, e, e, 1.0, e, torch.eye(4), torch.eye(4), 1.0,
                               1.0, 8, 8, e, 0, torch.zeros(3), False)
    assert hasattr(dgr, "GaussianRasterizationSettings") and hasattr(dgr, "_RasterizeGaussians")
    assert dgr.GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered")


def test_refalgo_baseline_loads_and_exports():
    """The reference-structure GPU baseline bench.py times (baseline/) is built and loadable."""
    from baseline import refalgo
    L = refalgo.lib()
    for s in refalgo.SYMBOLS:
        assert hasattr(L, s), s


def test_every_entry_point_with_parameters_has_ctypes_argtypes():
    """A pointer passed without argtypes is truncated to a C int: every header function that
    takes parameters must be declared in gsr._lib."""
    import re

    from gsr import _lib
    L = _lib.lib()
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "gsr.h")).read(), flags=re.S)
    for name, params in re.findall(r"\b(gsr_[a-z_0-9]+)\(([^)]*)\)\s*;", hdr):
        if params.strip() in ("", "void"):
            continue
        assert getattr(L, name).argtypes is not None, name


def test_debug_build_and_deterministic_toggle():
    """lib/debug/libgsr.so (GSR_DEBUG) exports the same ABI and reports itself; the product
    library does not.  The deterministic-backward toggle is host state (no GPU needed)."""
    from gsr import _lib
    if not os.path.exists(_lib.DEBUG_LIB_PATH):
        _lib.build()
    D = ctypes.CDLL(_lib.DEBUG_LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(D, s)]
    assert not missing, missing
    assert D.gsr_debug_build() == 1
    assert _lib.lib().gsr_debug_build() == 0
    before = _lib.deterministic()
    try:
        _lib.set_deterministic(True)
        assert _lib.deterministic()
        _lib.set_deterministic(False)
        assert not _lib.deterministic()
    finally:
        _lib.set_deterministic(before)
