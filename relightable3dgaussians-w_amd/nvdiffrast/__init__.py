"""Drop-in `nvdiffrast` package for MI355X: the part of NVlabs nvdiffrast the reference
imports (`import nvdiffrast.torch as dr`, scene/NVDIFFREC/light.py:4, util.py:13) backed by
libgsr.so.  nvdiffrast is CUDA-only and not importable on ROCm; without this package the
reference's gaussian_renderer/__init__.py cannot even import its EnvironmentLight."""
