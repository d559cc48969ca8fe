#!/bin/bash
# The seven-letter and byte-batch paths on the GPU box (tools only): their tests, the -m gpu suite,
# then tools/bench_hep.py (single pairs, C2 and C5 shapes).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hep
timeout -k 10 600 python -u -m pytest tests/test_hepta.py -x -v --timeout 300 --timeout-method thread > gpurun_out/hep/t1.log 2>&1
rc=$?; tail -4 gpurun_out/hep/t1.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/hep/t1.log; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hep/tests.log 2>&1
rc=$?; tail -3 gpurun_out/hep/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/hep/tests.log; exit $rc; }
timeout -k 10 300 python tools/bench_hep.py > gpurun_out/hep/bench_hep.jsonl && cat gpurun_out/hep/bench_hep.jsonl
timeout -k 10 400 python tools/bench_hep.py --n 1048576 --reps 2 --params "1,-1,1,1" > gpurun_out/hep/bench_hep_c5.jsonl && cat gpurun_out/hep/bench_hep_c5.jsonl
