set -e
mkdir -p gpurun_out/c5v
for L in "" g2 ss2 gp2 ""; do
  lib=$PWD/concurrentproject_amd/libswmi355${L:+_$L}.so
  SWMI355_LIB=$lib timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/c5v/${L:-def}.jsonl 2>/dev/null
done
