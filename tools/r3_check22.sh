#!/bin/bash
# round 3: shade backward without SLP packing and with its d_base partials before the SH-gradient
# phase (159 VGPRs, 3 waves per SIMD); tests, then cfg3 and cfg4 A/B against the HEAD build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/relightable3dgaussians-w_amd/lib
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 env GSR_LIB_PATH=${TEST_LIB:-$L/libgsr.so} python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shade.py \
  tests/test_gpu_relit.py tests/test_gpu_render_golden.py tests/test_gpu_trainaux.py tests/test_gpu_train.py \
  > gpurun_out/r3_t22.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_t22.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r3_t22.log | head -20; exit $rc; }
for v in ${VARIANTS:-new old new old}; do
  lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 5 > gpurun_out/r3_c3_$v.log 2>&1 || exit 1
  GSR_LIB_PATH=$lib timeout -k 10 300 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_c4_$v.log 2>&1 || exit 1
  python - <<PY
import json
a=json.loads(open('gpurun_out/r3_c3_$v.log').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/r3_c4_$v.log').read().strip().splitlines()[-1])
print('$v', 'cfg3', a['value'], a['ms_per_step'], 'cfg4', b['value'], b['ms_per_step'])
PY
done
