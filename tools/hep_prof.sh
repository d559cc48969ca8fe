#!/bin/bash
# rocprofv3 kernel-trace stats and one SQ counter pass for the seven-letter kernels (tools only):
# tools/bench_hep.py at C2 size (both constant sets) and at C5 size (the reference's constants).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hepprof
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hepprof/kt2 -o c2 -- \
  python tools/bench_hep.py --reps 3 --params "1,-1,1,1;2,-3,5,2" > gpurun_out/hepprof/kt2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hepprof/kt5 -o c5 -- \
  python tools/bench_hep.py --n 1048576 --reps 1 --params "1,-1,1,1" > gpurun_out/hepprof/kt5.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/hepprof/sq2 -o c2 -- \
  python tools/bench_hep.py --reps 1 --params "1,-1,1,1" > gpurun_out/hepprof/sq2.log 2>&1 || exit 1
find gpurun_out/hepprof -name "*stats*.csv" -o -name "*counter_collection*.csv" | sort
