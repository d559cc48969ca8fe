set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_slab.py tests/test_gpu_parity.py tests/test_db.py tests/test_harness.py > gpurun_out/t1.log 2>&1
