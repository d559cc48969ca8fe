# C5 (N = 2^20, ring mode) with one and two columns per lane (GPU box)
set -e
mkdir -p gpurun_out
for v in 1 2; do
  timeout -k 10 200 python bench.py --workload slab --no-cpu-baseline --steps 3 --warmup 1 --opt f2w=$v >> gpurun_out/c5_ab.jsonl 2>> gpurun_out/c5_ab.err
done
