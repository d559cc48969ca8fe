set -e
# A/B of two library builds on the same box: bash tools/ab_lib.sh <libA.so> <libB.so> [bench args]
mkdir -p gpurun_out/ab
A=$1; B=$2; shift 2
for i in 1 2 3; do
  for L in $A $B; do
    SWMI355_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab/$(basename $L)_$i.json 2>/dev/null
  done
done
python3 - <<'PY'
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[f.split("/")[-1].rsplit("_", 1)[0]].append(d["kernel_ms_per_launch"])
for k, v in r.items():
    print(k, v)
PY
