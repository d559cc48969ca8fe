set -e
mkdir -p gpurun_out/pr
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_ring.py tests/test_slab.py > gpurun_out/pr/par.txt 2>&1
timeout -k 10 120 python bench.py --workload pair --steps 20 --warmup 3 > gpurun_out/pr/bench_c2.txt 2>&1
rm -rf gpurun_out/ab; mkdir -p gpurun_out/ab
bash tools/ab_multi.sh "lib_base libswmi355_aff2" --workload pair --steps 20 --warmup 3 --no-extra --opt linear=0 > gpurun_out/ab/aff.txt 2>&1
