set -e
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_c2.json 2>&1
timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_c5.json 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ring.py tests/test_slab.py -k "not c5_golden" > gpurun_out/t1.log 2>&1
