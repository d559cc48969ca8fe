# The round's bench lines for C2 (default auto line), C3 (batch), C5 (slab workload, one GPU), slab 0 of
# C5's 8-way split, and C2 / C3 / C5 with the affine constants (c2a, c3a, c5a),
# taken after tools/pmc_summary.py has stamped profiles/pmc_*.json for this build, so every line's
# roofline carries the counter-derived `achieved` / `frac` (GPU box).
set -e
mkdir -p gpurun_out/lines
timeout -k 10 240 python bench.py --steps 10 --warmup 2 > gpurun_out/lines/bench_c2.json 2> gpurun_out/lines/bench_c2.err
timeout -k 10 240 python bench.py --workload batch --steps 5 --warmup 1 > gpurun_out/lines/bench_c3.json 2> gpurun_out/lines/bench_c3.err
timeout -k 10 240 python bench.py --workload slab --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/lines/bench_c5.json 2> gpurun_out/lines/bench_c5.err
timeout -k 10 240 python bench.py --workload slab --slab-of 8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lines/bench_c5p8.json 2> gpurun_out/lines/bench_c5p8.err
timeout -k 10 240 python bench.py --workload pair --params 2,-3,5,2 --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/lines/bench_c2a.json 2> gpurun_out/lines/bench_c2a.err
timeout -k 10 240 python bench.py --workload slab --params 2,-3,5,2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lines/bench_c5a.json 2> gpurun_out/lines/bench_c5a.err
timeout -k 10 240 python bench.py --workload batch --params 2,-3,5,2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/lines/bench_c3a.json 2> gpurun_out/lines/bench_c3a.err
