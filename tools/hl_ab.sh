set -e
mkdir -p gpurun_out/hl
timeout -k 10 120 python tools/hl_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flow3.py 2>&1 | tail -3
for i in 1 2 3; do for h in 0 1; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 10 --warmup 2 --opt f3hl=$h > gpurun_out/hl/c2_${h}_$i.json 2>/dev/null
done; done
python3 - <<'PY'
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/hl/c2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[f.split("/")[-1].rsplit("_", 1)[0]].append((d["ms_per_step"], d.get("kernel_ms_per_launch")))
for k, v in r.items(): print(k, v)
PY
