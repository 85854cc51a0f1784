"""Drop-in `simple_knn` package (submodules/simple-knn) for MI355X: `simple_knn._C.distCUDA2`
backed by libgsr.so (gsr_knn_mean_dist, hand-written gfx950 HIP)."""
