set -e
mkdir -p gpurun_out/pr
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ring.py > gpurun_out/pr/ring.txt 2>&1
timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/pr/bench_c5.txt 2>&1
