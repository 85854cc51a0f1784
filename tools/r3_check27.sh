#!/bin/bash
# round 3: 64-B accumulator lines: kernel trace at cfg2 (base, a16, a16b = the preprocess
# backward's ninth value read by a 16-B load), then cfg4 and cfg5 A/B (base vs a16)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
L=relightable3dgaussians-w_amd/lib
bash tools/kt_variants.sh '--steps 20 --warmup 5 --no-cpu-baseline --no-refalgo --no-train --no-minibatch' base a16 a16b || exit 1
cd "$R"
for v in base a16 base a16; do lib=$R/$L/$v/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 300 python bench.py --config cfg4 --steps 20 --warmup 5 > gpurun_out/r3_c4_$v.log 2>&1 || exit 1
  GSR_LIB_PATH=$lib timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 3 --no-cpu-baseline --no-refalgo --no-train --no-minibatch > gpurun_out/r3_c5_$v.log 2>&1 || exit 1
  python - <<PY
import json
a=json.loads(open('gpurun_out/r3_c4_$v.log').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/r3_c5_$v.log').read().strip().splitlines()[-1])
print('$v', 'cfg4', a['value'], a['ms_per_step'], 'cfg5', b['value'], b['ms_per_step'])
PY
done
