"""simple_knn._C -- the extension module of submodules/simple-knn (ext.cpp:15-17) over the C
ABI of libgsr.so: `distCUDA2(points[P,3]) -> [P]`, the mean squared distance of every point
to its 3 nearest other points (spatial.cu:14-26), bit-identical to the reference's
Morton/box algorithm.  GPU tensors only; there is no CPU path."""
import os
import sys

import torch

_here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _here not in sys.path:
    sys.path.insert(0, _here)

from gsr import _lib  # noqa: E402


def distCUDA2(points):
    _lib.require_gpu_tensor(points, "points")
    if points.ndimension() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    pts = points.float().contiguous()
    P = pts.size(0)
    means = torch.zeros(P, dtype=torch.float32, device=pts.device)
    if P == 0:
        return means
    L = _lib.lib()
    ws = torch.empty(int(L.gsr_knn_workspace_bytes(P)), dtype=torch.uint8, device=pts.device)
    _lib.check(L.gsr_knn_mean_dist(P, pts.data_ptr(), means.data_ptr(), ws.data_ptr(), _lib.stream_of(pts.device)),
               "distCUDA2")
    return means
