set -e
# C5 grid shapes: ring-mode workgroups per CU, ring rows (bench.py --workload slab, 1 GPU)
mkdir -p gpurun_out/c5
run() { timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/c5/$(echo "x$@" | tr ' =' '__').json 2>/dev/null; }
run
run --opt f2_wgs=3
run --opt f2_wgs=2
run --opt ring_rows=8192
run --opt ring_rows=2048
