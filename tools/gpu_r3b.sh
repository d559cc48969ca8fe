set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
for i in 1 2; do timeout -k 10 200 python bench.py --workload batch --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/c3_lines.jsonl 2>> gpurun_out/c3.err; done
AB_VARIANTS="sp4 sp8 sp12" bash tools/ab_f2w2.sh
