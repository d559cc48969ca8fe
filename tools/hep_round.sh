#!/bin/bash
# The seven-letter and byte-batch paths on the GPU box (tools only): the -m gpu suite, then
# tools/bench_hep.py (single pairs) and the C2 bench line without extras.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hep
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/hep/tests.log 2>&1
rc=$?; tail -3 gpurun_out/hep/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/hep/tests.log; exit $rc; }
timeout -k 10 300 python tools/bench_hep.py > gpurun_out/hep/bench_hep.jsonl && cat gpurun_out/hep/bench_hep.jsonl
