#!/usr/bin/env python
"""Per-unit timing of the composite backward tile pass (timing build: make -C csrc times)
over cfg4's training views: per launch, the units that walked (end > start + a few us)
against the ones that exited early, their durations, and the launch's makespan.

    python3 tools/mc_bwd_times.py [iterations=2]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
os.environ.setdefault("GSR_LIB_PATH", os.path.join(PKG, "lib", "times", "libgsr.so"))
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

UNITS = 1 << 17


def main():
    from gsr import _lib, train
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda", 0)
    scene, views, gts = train.synthetic_relit_scene(1_363_637, 4, 1920, 1080, 1400.0, dev, seed=0)
    scene.iteration = train.REG_NORMAL_FROM_ITER
    L = _lib.lib()
    L.gsr_debug_mcb_times.argtypes = [C.c_void_p, C.c_int, C.c_int]
    scratch = np.zeros((2, UNITS, 4), np.uint64)  # (kept alive across the call)
    L.gsr_debug_mcb_times(scratch.ctypes.data, UNITS, 1)  # start clean
    for it in range(iters):
        # one view per step, so the records hold that view's launches only
        train.train_step(scene, views, [it % 4], gts)
        torch.cuda.synchronize()
        buf = np.zeros((2, UNITS, 4), np.uint64)
        assert L.gsr_debug_mcb_times(buf.ctypes.data, UNITS, 1) == 0
        dump = os.environ.get("GSR_STATS_DUMP")
        if dump:  # raw records for offline analysis (row = the launch's blockIdx)
            np.save(f"{dump}_{it}.npy", buf)
        for launch in range(2):
            t = buf[launch].astype(np.int64)
            ok = t[:, 1] > 0
            if not ok.any():
                continue
            t = t[ok]
            d = (t[:, 1] - t[:, 0]) / 100.0  # s_memrealtime: 100 MHz -> us
            span = (t[:, 1].max() - t[:, 0].min()) / 100.0
            walked = d > 3.0
            q = np.percentile(d[walked], [50, 90, 99, 100]) if walked.any() else [0, 0, 0, 0]
            top = np.argsort(-d)[:5]
            print(f"iter {it} launch {launch}: {ok.sum()} units, {walked.sum()} walked, makespan {span:.1f} us, "
                  f"walked durations p50/p90/p99/max {q[0]:.1f}/{q[1]:.1f}/{q[2]:.1f}/{q[3]:.1f} us, "
                  f"sum {d[walked].sum() / 1e3:.1f} ms; longest units (tile, qallow, nmax, us): "
                  + ", ".join(f"({int(t[i, 2]) & 0xFFFFF}, {(int(t[i, 2]) >> 20) & 0xF}, {int(t[i, 3])}, {d[i]:.0f})"
                              for i in top))


if __name__ == "__main__":
    main()
