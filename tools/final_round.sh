#!/bin/bash
# Round-end evidence in one GPU call: the -m gpu suite and smoke, the round's rocprof kernel-trace
# and counter passes, the counter summaries stamped for this build (profiles/pmc_*.json on the box),
# then the bench lines that read them.  Afterwards, in the build container:
#   python tools/pmc_summary.py gpurun_out/prof r05 && cp gpurun_out/lines/bench_*.json -> profiles/r05_bench_*.json
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof gpurun_out/lines
bash tools/gpu_run.sh tests smoke
bash tools/prof_round.sh c2 c3 c5 c5p8 c2a c5a
timeout -k 10 120 python tools/pmc_summary.py gpurun_out/prof r05 > gpurun_out/pmc_summary.log 2>&1
bash tools/bench_lines.sh
echo "final_round done"
