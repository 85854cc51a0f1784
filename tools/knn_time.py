import sys, time, torch
sys.path[:0] = ["/root/repo", "/root/repo/relightable3dgaussians-w_amd"]
from simple_knn._C import distCUDA2
for P in (200_000, 1_500_000):
    x = torch.randn(P, 3, device="cuda") * 4
    distCUDA2(x); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3): d = distCUDA2(x)
    torch.cuda.synchronize()
    print(P, "points:", round((time.perf_counter() - t) / 3 * 1e3, 2), "ms", float(d.mean()))
