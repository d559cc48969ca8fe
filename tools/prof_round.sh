set -e
# Round profiles: bench lines, rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE
# passes (one counter set per run) for C2 (pair), C3 (batch) and C5 (slab workload, 1 GPU).
# usage (on the GPU box): bash tools/prof_round.sh [c2 c3 c5]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
which="${*:-c2 c3 c5}"
for w in $which; do
  case $w in
    c2) args="--steps 10 --warmup 2"; pargs="--steps 5 --warmup 1";;
    c3) args="--workload batch --steps 5 --warmup 1"; pargs="--workload batch --steps 3 --warmup 1";;
    c5) args="--workload slab --steps 3 --warmup 1 --cpu-seconds 10"; pargs="--workload slab --steps 2 --warmup 1";;
  esac
  timeout -k 10 240 python bench.py $args > gpurun_out/prof/bench_$w.json 2> gpurun_out/prof/bench_$w.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/kt_$w.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/fetch_$w.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_$w -o $w -- python bench.py $pargs --no-cpu-baseline > gpurun_out/prof/write_$w.log 2>&1
done
