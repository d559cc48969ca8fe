# W2 (two columns per lane) parity + C2 A/B against W = 1 (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flow2_w2.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w2_tests.log 2>&1
for v in 1 2 1 2; do
  timeout -k 10 120 python bench.py --workload pair --no-cpu-baseline --steps 20 --opt f2w=$v >> gpurun_out/c2_ab.jsonl 2>> gpurun_out/c2_ab.err
done
