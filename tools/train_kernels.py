#!/usr/bin/env python
"""cfg4's training iteration on ONE stream (the views back to back), for a rocprofv3 kernel
trace whose per-kernel durations are not inflated by the two-stream overlap bench.py uses
(tools only; GPU box):

    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -- python3 tools/train_kernels.py [iters]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402


def main():
    from gsr import train
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    scene, views, gts = train.synthetic_relit_scene(1_363_637, 4, 1920, 1080, 1400.0, dev, seed=0)
    scene.iteration = train.REG_NORMAL_FROM_ITER
    ids = list(range(4))
    for _ in range(3):
        train.train_step(scene, views, ids, gts)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        train.train_step(scene, views, ids, gts)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"one stream: {ev[0].elapsed_time(ev[1]) / iters:.3f} ms per iteration over {iters}")


if __name__ == "__main__":
    main()
