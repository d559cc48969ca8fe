# per-rank cost of the f-1 column slabs on the W2 build: slab 0 of a 2/4/8-way split alone (GPU box)
set -e
mkdir -p gpurun_out/slab
for k in 8 4 2; do
  timeout -k 10 240 python bench.py --workload slab --slab-of $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/slab/slab0_of$k.json 2> gpurun_out/slab/slab0_of$k.err
done
