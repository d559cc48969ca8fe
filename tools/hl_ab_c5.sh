set -e
# C5 (ring mode): whole-chunk LDS links vs half-chunk links (option f3rhl), 3 alternations on one box
mkdir -p gpurun_out/hlr
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flow3.py 2>&1 | tail -3
for i in 1 2 3; do for h in 0 1; do
  timeout -k 10 120 python bench.py --workload slab --no-cpu-baseline --steps 3 --warmup 1 --opt f3rhl=$h > gpurun_out/hlr/c5_${h}_$i.json 2>/dev/null
done; done
python3 - <<'PY'
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/hlr/c5_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[f.split("/")[-1].rsplit("_", 1)[0]].append((d["ms_per_step"], d.get("kernel_ms_per_launch")))
for k, v in r.items(): print(k, v)
PY
