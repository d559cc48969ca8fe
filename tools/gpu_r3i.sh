# balanced ring rounds (up to 5 workgroups per CU): ring/slab parity, C5, slab 0 of 8 (GPU box)
set -e
mkdir -p gpurun_out/slab
timeout -k 10 600 python -u -m pytest tests/test_ring.py tests/test_slab.py tests/test_flow2_w2.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ring_tests.log 2>&1
timeout -k 10 240 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_bal.json 2> gpurun_out/c5_bal.err

for k in 8 4 2; do
  timeout -k 10 240 python bench.py --workload slab --slab-of $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/slab/bal_slab0_of$k.json 2> gpurun_out/slab/bal_slab0_of$k.err
done
