# slab 0 of 8 alone (the f-1 per-rank cost): chunk size and edge kind (GPU box)
set -e
mkdir -p gpurun_out/slab
for o in "C=64" "C=32" "C=32 --opt ring=0" "C=64 --opt ring=0"; do
  n=$(echo $o | tr ' =' '__')
  timeout -k 10 240 python bench.py --workload slab --slab-of 8 --steps 3 --warmup 1 --no-cpu-baseline --opt $o > gpurun_out/slab/s8_$n.json 2> gpurun_out/slab/s8_$n.err
done
