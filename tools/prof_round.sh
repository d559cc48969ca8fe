set -e
# Round profiles: bench lines, rocprofv3 kernel-trace stats and the counter passes
# (one counter group per run, nothing else traced: MI355X_MICROARCH.md, rocprofv3
# PMC slots) for C2 (pair), C3 (batch) and C5 (slab workload, 1 GPU):
#   FETCH_SIZE | WRITE_SIZE | SQ (8 slots) | GRBM
# then python tools/pmc_summary.py gpurun_out/prof <round> (in the build container).
# usage (on the GPU box): bash tools/prof_round.sh [c2 c3 c5 c5p8]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
which="${*:-c2 c3 c5}"
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
for w in $which; do
  case $w in
    c2) args="--steps 10 --warmup 2"; pargs="--workload pair --steps 5 --warmup 1";;
    c3) args="--workload batch --steps 5 --warmup 1"; pargs="--workload batch --steps 3 --warmup 1";;
    c5) args="--workload slab --steps 3 --warmup 1 --cpu-seconds 10"; pargs="--workload slab --steps 2 --warmup 1";;
    c5p8) args="--workload slab --slab-of 8 --steps 3 --warmup 1 --no-cpu-baseline"; pargs="--workload slab --slab-of 8 --steps 2 --warmup 1";;
    c2a) args="--workload pair --params 2,-3,5,2 --steps 10 --warmup 2 --no-cpu-baseline"; pargs="--workload pair --params 2,-3,5,2 --steps 5 --warmup 1";;
    c3a) args="--workload batch --params 2,-3,5,2 --steps 5 --warmup 1 --no-cpu-baseline"; pargs="--workload batch --params 2,-3,5,2 --steps 3 --warmup 1";;
    c5a) args="--workload slab --params 2,-3,5,2 --steps 3 --warmup 1 --no-cpu-baseline"; pargs="--workload slab --params 2,-3,5,2 --steps 2 --warmup 1";;
  esac
  timeout -k 10 240 python bench.py $args > gpurun_out/prof/bench_$w.json 2> gpurun_out/prof/bench_$w.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/kt_$w.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/fetch_$w.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/write_$w.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/prof/sq_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/sq_$w.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/prof/grbm_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/grbm_$w.log 2>&1
done
