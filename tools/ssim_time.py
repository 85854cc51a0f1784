"""Time the fused SSIM forward/backward alone at 1080p (tools only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]
import torch  # noqa: E402

from gsr import train  # noqa: E402

a = torch.rand(3, 1080, 1920, device="cuda", requires_grad=True)
b = torch.rand(3, 1080, 1920, device="cuda")
m = (torch.rand(1, 1080, 1920, device="cuda") > 0.1).float()
for _ in range(3):
    train.ssim(a, b, m).backward()
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
fw = bw = 0.0
n = 20
for _ in range(n):
    e[0].record()
    v = train.ssim(a, b, m)
    e[1].record()
    v.backward()
    e[2].record()
    torch.cuda.synchronize()
    fw += e[0].elapsed_time(e[1])
    bw += e[1].elapsed_time(e[2])
print(f"ssim fwd {fw / n * 1e3:.1f} us (incl. count/where), bwd {bw / n * 1e3:.1f} us")
