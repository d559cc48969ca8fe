#!/bin/bash
# A/B runner (GPU box): alternates bench.py variants REPS times on one box and prints the
# kernel ms of each run per variant, so box-to-box noise cancels.  Replaces the round-2..4
# one-off ab_*.sh / hl_ab*.sh / c5_grid_sweep.sh scripts.
#   bash tools/ab.sh REPS "label=bench args" "label=bench args" ...
#       e.g. bash tools/ab.sh 3 "hl1=--no-extra --opt f3hl=1" "hl0=--no-extra --opt f3hl=0"
#            bash tools/ab.sh 2 "c5=--workload slab --steps 3" "wgs3=--workload slab --steps 3 --opt f2_wgs=3"
#   bash tools/ab.sh REPS --libs libA.so libB.so ... -- [bench args]   (library builds, SWMI355_LIB)
# Every run has its own time limit; the first failing run ends the script.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
reps=$1; shift
out=gpurun_out/ab; rm -rf $out; mkdir -p $out
run() {  # label, env, args...
  local label=$1 env=$2; shift 2
  env $env timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > $out/${label}_$i.json 2> $out/${label}_$i.err \
    || { tail -5 $out/${label}_$i.err; exit 1; }
}
for i in $(seq 1 $reps); do
  if [ "$1" = "--libs" ]; then
    libs=(); shift_n=1
    for x in "${@:2}"; do shift_n=$((shift_n + 1)); [ "$x" = "--" ] && break; libs+=("$x"); done
    for L in "${libs[@]}"; do
      run "$(basename $L .so)" "SWMI355_LIB=$L" "${@:$((shift_n + 1))}"
    done
  else
    for v in "$@"; do
      run "${v%%=*}" "" ${v#*=}
    done
  fi
done
python3 - <<'PY'
import collections, glob, json
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[f.split("/")[-1].rsplit("_", 1)[0]].append((d["ms_per_step"], d.get("kernel_ms_per_launch"), d.get("parity")))
for k, v in r.items():
    print(k, v)
PY
