set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/t2.log 2>&1
bash tools/prof_round.sh c2 c3 c5
