#!/bin/bash
# A/B timing of libgsr builds: tools/variants.sh name[=path/to/libgsr.so] ...  (no path: the in-tree lib)
set -o pipefail
mkdir -p gpurun_out
for spec in "${@:-base}"; do
  v=${spec%%=*}; L=${spec#*=}; [ "$L" = "$spec" ] && L=relightable3dgaussians-w_amd/lib/libgsr.so
  GSR_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-refalgo --no-train --steps ${STEPS:-20} --warmup 5 $BENCH_ARGS \
    > gpurun_out/v_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/v_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], (d.get('single_call') or {}).get('median_ms'), d.get('stage_ms'))"
done
