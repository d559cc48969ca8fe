# the aligned-loop build: GPU suite, smoke, default bench line, C3 and C5 lines (GPU box)
set -e
bash tools/gpu_check.sh
timeout -k 10 240 python bench.py --workload batch --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_al.json 2> gpurun_out/c3_al.err
timeout -k 10 240 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_al.json 2> gpurun_out/c5_al.err
