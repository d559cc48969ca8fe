set -e
mkdir -p gpurun_out/pr
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_ring.py tests/test_slab.py > gpurun_out/pr/par.txt 2>&1
rm -rf gpurun_out/ab; mkdir -p gpurun_out/ab
bash tools/ab_multi.sh "lib_base lib_lin3" --workload pair --steps 20 --warmup 3 --no-extra > gpurun_out/ab/pair.txt 2>&1
rm -f gpurun_out/ab/*.json
bash tools/ab_multi.sh "lib_base lib_lin3" --workload slab --steps 2 --warmup 1 --no-extra > gpurun_out/ab/slab.txt 2>&1
