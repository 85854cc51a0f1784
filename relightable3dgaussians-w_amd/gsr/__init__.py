"""gsr: host-side runtime of the MI355X-native Gaussian rasterizer + relighting shade.

The product path is libgsr.so (hand-written HIP for gfx950, C ABI declared in
include/gsr.h) driven from Python through ctypes; PyTorch only provides device memory,
the current stream and torch.distributed.
"""
