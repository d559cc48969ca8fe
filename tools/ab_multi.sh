set -e
# A/B/C.. of library builds on one box, interleaved: bash tools/ab_multi.sh "libA libB ..." [bench args]
mkdir -p gpurun_out/ab
LIBS=$1; shift
for i in 1 2 3; do
  for L in $LIBS; do
    SWMI355_LIB=concurrentproject_amd/$L.so timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab/${L}__$i.json 2>/dev/null
  done
done
python3 - <<'PY'
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*__*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[f.split("/")[-1].rsplit("__", 1)[0]].append(d["kernel_ms_per_launch"])
for k, v in r.items():
    print(k, v)
PY
