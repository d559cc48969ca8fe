#!/bin/bash
# Round-6 final evidence, part A (GPU box): the -m gpu suite, smoke, then the rocprof kernel-trace and
# counter passes of C2, C3 and their affine forms (tools/prof_round.sh).  Part B: tools/final_r06b.sh.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof gpurun_out/lines
bash tools/gpu_run.sh tests smoke
bash tools/prof_round.sh c2 c3 c3a c2a
echo "final_r06a done"
