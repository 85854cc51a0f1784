#!/usr/bin/env python
"""Host-side cost of cfg4's train_step (tools only; GPU box): wall time per iteration with the
two streams bench.py uses, the CPU time the process spends per iteration, and where it goes
(cProfile over a few iterations, top functions by own time).

    python tools/train_host.py [iters]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402


def main():
    from gsr import train
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    scene, views, gts = train.synthetic_relit_scene(1_363_637, 4, 1920, 1080, 1400.0, dev, seed=0)
    scene.iteration = train.REG_NORMAL_FROM_ITER
    ids = list(range(4))
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    step = lambda: train.train_step(scene, views, ids, gts, streams=streams)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0, c0 = time.perf_counter(), time.process_time()
    for _ in range(iters):
        step()
    t1, c1 = time.perf_counter(), time.process_time()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{iters} iterations: issue {1e3 * (t1 - t0) / iters:.3f} ms/iter wall, {1e3 * (c1 - c0) / iters:.3f} ms/iter "
          f"CPU; with the final sync {1e3 * (t2 - t0) / iters:.3f} ms/iter")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
