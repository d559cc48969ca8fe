#!/bin/bash
# One parameterised GPU-box runner (replaces the per-call tools/gpu_r3*.sh scripts).
# Every step has its own time limit; the first failing step ends the run.
#   bash tools/gpu_run.sh STEP [STEP ...]
# STEP:
#   tests[:FILES]       pytest -m gpu (FILES: comma-separated test files, default all)
#   sweep:CASES[@OPTS]  tools/sweep.py --cases CASES (OPTS: k=v+k=v engine options)
#   trace:N:C[@OPTS]    tools/trace_flow.py N C 1 N 5 2 (W2 single pair) with options
#   bench[:ARGS]        bench.py ARGS (words joined by +), JSON line to gpurun_out/bench_<n>.json
#   prof:WHICH          tools/prof_round.sh WHICH (c2 c3 c5 c5p8 ...; words joined by +)
#   harness             the reference's TestFileWithGPU against the library
#   smoke               __graft_entry__.smoke()
#   ab:REPS:V1:V2...    tools/ab.sh REPS V1 V2 ... (V = label=bench args, words joined by +)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=0
for st in "$@"; do
  n=$((n + 1))
  kind=${st%%:*}
  rest=${st#*:}
  [ "$rest" = "$st" ] && rest=""
  echo "== step $n: $st  ($(date +%T))"
  case $kind in
    tests)
      files=${rest:-tests}
      timeout -k 10 900 python -u -m pytest ${files//,/ } -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/tests_$n.log 2>&1 || { tail -30 gpurun_out/tests_$n.log; exit 1; }
      tail -3 gpurun_out/tests_$n.log ;;
    sweep)
      cases=${rest%%@*}; opts=${rest#*@}; [ "$opts" = "$rest" ] && opts=""
      oargs=""; for o in ${opts//+/ }; do oargs="$oargs --opt $o"; done
      timeout -k 10 300 python tools/sweep.py --reps 5 --cases "$cases" $oargs | tee gpurun_out/sweep_$n.jsonl ;;
    trace)
      nc=${rest%%@*}; opts=${rest#*@}; [ "$opts" = "$rest" ] && opts=""
      N=${nc%%:*}; C=${nc#*:}
      oargs=""; for o in ${opts//+/ }; do k=${o%%=*}; v=${o#*=}; oargs="$oargs $k=$v"; done
      TRACE_OPTS="$oargs" timeout -k 10 200 python tools/trace_flow.py "$N" "$C" 1 "$N" 5 2 > gpurun_out/trace_$n.txt 2>&1 \
        || { tail -20 gpurun_out/trace_$n.txt; exit 1; }
      head -1 gpurun_out/trace_$n.txt ;;
    bench)
      timeout -k 10 400 python bench.py ${rest//+/ } > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err \
        || { tail -20 gpurun_out/bench_$n.err; exit 1; }
      cut -c1-400 gpurun_out/bench_$n.json ;;
    prof)
      bash tools/prof_round.sh ${rest//+/ } ;;
    harness)
      timeout -k 10 300 python -u -m pytest tests/test_harness.py -m gpu -x -q --timeout 250 --timeout-method thread \
        > gpurun_out/harness_$n.log 2>&1 || { tail -20 gpurun_out/harness_$n.log; exit 1; }
      tail -2 gpurun_out/harness_$n.log ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$n.log 2>&1 \
        || { tail -20 gpurun_out/smoke_$n.log; exit 1; }
      tail -2 gpurun_out/smoke_$n.log ;;
    ab)
      reps=${rest%%:*}; vs=${rest#*:}
      IFS=':' read -ra V <<< "$vs"
      args=(); for v in "${V[@]}"; do args+=("${v//+/ }"); done
      bash tools/ab.sh "$reps" "${args[@]}" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
