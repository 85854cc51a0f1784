#!/usr/bin/env python
"""Times the fused SSIM kernels alone (gsr_ssim_forward / gsr_ssim_backward through the C ABI
at 3x1080x1920 with an occluder mask, HIP events over 100 back-to-back launches each; tools
only, GPU box).

    GSR_LIB_PATH=... python tools/bench_ssim.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402


def main():
    import ctypes as C

    from gsr import _lib, train
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Cn, H, W = 3, 1080, 1920
    a = torch.rand(Cn, H, W, device=dev, generator=g)
    b = torch.rand(Cn, H, W, device=dev, generator=g)
    m = (torch.rand(1, H, W, device=dev, generator=g) > 0.1).float()
    L = _lib.lib()
    win = (C.c_float * 11)(*train.gaussian_1d(11).tolist())
    parts = torch.empty(int(L.gsr_ssim_partials(Cn, H, W)) * 2, device=dev)
    dmaps = torch.empty(3, Cn, H, W, device=dev)
    gs = torch.ones(1, device=dev)
    d = torch.empty_like(a)
    st = _lib.stream_of(dev)
    fwd = lambda: L.gsr_ssim_forward(Cn, H, W, a.data_ptr(), b.data_ptr(), m.data_ptr(), 0, win, parts.data_ptr(),
                                     dmaps.data_ptr(), st)
    bwd = lambda: L.gsr_ssim_backward(Cn, H, W, a.data_ptr(), b.data_ptr(), dmaps.data_ptr(), gs.data_ptr(), win,
                                      d.data_ptr(), 0, st)
    for _ in range(5):
        fwd()
        bwd()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    n = 100
    ev[0].record()
    for _ in range(n):
        fwd()
    ev[1].record()
    for _ in range(n):
        bwd()
    ev[2].record()
    torch.cuda.synchronize()
    print(f"k_ssim_fwd {1000 * ev[0].elapsed_time(ev[1]) / n:.1f} us, k_ssim_bwd {1000 * ev[1].elapsed_time(ev[2]) / n:.1f} us"
          f" (sum {float(parts[0::2].sum()):.3f})")


if __name__ == "__main__":
    main()
