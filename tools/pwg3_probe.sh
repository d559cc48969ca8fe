#!/bin/bash
# Counters and kernel stats of the int32 batch kernel (flow3 three-column ring step, a pair per
# workgroup: sw_flow3r3p_kernel) on C3, for the issue-bound analysis in DESIGN.md (tools only).
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pwg3
A="--workload batch --steps 3 --warmup 1 --no-cpu-baseline --mode 5 --opt f2pwg=1 --opt f3pwg=1"
timeout -k 10 200 python bench.py $A > gpurun_out/pwg3/bench.json
cut -c1-600 gpurun_out/pwg3/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pwg3/kt -o p -- python bench.py $A > gpurun_out/pwg3/kt.log 2>&1
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/pwg3/sq -o p -- python bench.py $A > gpurun_out/pwg3/sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pwg3/sq2 -o p -- python bench.py $A > gpurun_out/pwg3/sq2.log 2>&1
echo done
