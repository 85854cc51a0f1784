export TMPDIR=/tmp
for v in base exp; do
  L=relightable3dgaussians-w_amd/lib/libgsr.so; [ $v = exp ] && L=relightable3dgaussians-w_amd/lib/exp/libgsr.so
  GSR_LIB_PATH=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$v -- python3 bench.py --steps 10 --warmup 3 --no-minibatch --no-refalgo --no-cpu-baseline --no-train > gpurun_out/tl_$v.log 2>&1 || exit 1
  echo $v; python3 tools/timeline.py gpurun_out/tl_$v | grep -E "seg_lists|window"
done
