set -e
# C5 grid shapes: ring-mode blocks and workgroups per CU (bench.py --workload slab, 1 GPU)
mkdir -p gpurun_out/c5
run() { timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/c5/$(echo "$@" | tr ' =' '__').json 2>/dev/null; }
run --opt blocks=0
run --opt blocks=833
run --opt blocks=694
run --opt f2_wgs=3
run --opt blocks=1024 --opt ring_rows=8192
