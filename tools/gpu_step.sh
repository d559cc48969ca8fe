set -e
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --workload batch --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3.json 2>&1
timeout -k 10 120 python bench.py --workload batch --steps 5 --warmup 1 --no-cpu-baseline --opt linear=0 > gpurun_out/b_c3_aff.json 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_db.py -k "duo or c3 or c4 or db or search" > gpurun_out/t1.log 2>&1
