#!/bin/bash
# alternate default-bench runs of several libgsr builds (lib/<v>/libgsr.so, "new" = lib/libgsr.so):
# value (4 views / 3 streams), single call, live render_bwd, and the clustered / relit / train
# legs when they ran.  BENCH_ARGS replaces the default "--no-relit --no-train" (EXTRA is appended).
R="${GRAFT_REPO_ROOT:-/root/repo}"; L=$R/relightable3dgaussians-w_amd/lib
TAG=$1; shift; i=0
for v in "$@"; do i=$((i+1)); lib=$L/$v/libgsr.so; [ $v = new ] && lib=$L/libgsr.so
  GSR_LIB_PATH=$lib timeout -k 10 400 python3 $R/bench.py --no-cpu-baseline --no-refalgo ${BENCH_ARGS---no-relit --no-train} $EXTRA > $R/gpurun_out/${TAG}_${v}_$i.log 2>&1 || { echo "$v failed"; exit 1; }
  python3 - $R/gpurun_out/${TAG}_${v}_$i.log $v <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
c=d.get("clustered",{}); rl=d.get("relit",{}); tr=d.get("train",{})
out=[sys.argv[2], "value", d["value"], "single", d["single_call"]["median_ms"], "bwd_live", d["roofline"]["avg_launch_ms"],
     "| cfg2c", c.get("value"), c.get("single_call",{}).get("median_ms")]
for k, v in rl.items():
    if isinstance(v, dict) and "value" in v: out += ["|", k, v["value"]]
if tr: out += ["| train", tr.get("value"), "bwd_mc", tr.get("roofline",{}).get("avg_launch_ms")]
print(*out)
PY
done
