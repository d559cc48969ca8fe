#!/bin/bash
# Round-end evidence in one GPU call: the -m gpu suite and smoke, the round's rocprof kernel-trace
# and counter passes, the counter summaries stamped for this build (profiles/pmc_*.json on the box),
# then the bench lines that read them.  Afterwards, in the build container:
#   python tools/pmc_summary.py gpurun_out/prof rNN && cp gpurun_out/lines/bench_*.json -> profiles/rNN_bench_*.json
# usage: bash tools/final_round.sh rNN   (one call fits only when the box is quick; otherwise split it:
# tests + smoke + prof c2 c3 c3a c2a | prof c5 c5a c5p8 | pmc_summary here | bench_lines.sh)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof gpurun_out/lines
bash tools/gpu_run.sh tests smoke
round=${1:-r06}
bash tools/prof_round.sh c2 c3 c3a c5 c5p8 c2a c5a
timeout -k 10 120 python tools/pmc_summary.py gpurun_out/prof "$round" > gpurun_out/pmc_summary.log 2>&1
bash tools/bench_lines.sh
echo "final_round done"
