cd ${GRAFT_REPO_ROOT:-/root/repo}
for r in 1 2; do for s in def 3 4; do
  a=""; [ $s = def ] || a="--streams $s"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-refalgo $a > gpurun_out/st_${s}_$r.log 2>&1 || { echo "$s failed"; exit 1; }
  python3 - gpurun_out/st_${s}_$r.log $s <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
rl=d.get("relit",{}); tr=d.get("train",{}); c=d.get("clustered",{})
print(sys.argv[2], "value", d["value"], "single", d["single_call"]["median_ms"], "cfg2c", c.get("value"), "train", tr.get("value"), "cfg3", rl.get("cfg3",{}).get("value"), "cfg5r", rl.get("cfg5_relit",{}).get("value"))
PY
done; done
