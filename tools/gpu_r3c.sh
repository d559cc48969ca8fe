# W2 compiler-max build vs the previous library: parity of the flow2 tests, C2 A/B with traces, C5 line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flow2_w2.py tests/test_gpu_parity.py tests/test_ring.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_c.log 2>&1
AB_VARIANTS="prev" bash tools/ab_f2w2.sh
timeout -k 10 240 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_new.json 2> gpurun_out/c5_new.err
SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_prev.so timeout -k 10 240 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_prev.json 2> gpurun_out/c5_prev.err
