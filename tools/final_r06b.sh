#!/bin/bash
# Round-6 final evidence, part B (GPU box): the counter passes of C5, C5 affine and slab 0 of 8.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/prof_round.sh c5 c5a c5p8
echo "final_r06b done"
