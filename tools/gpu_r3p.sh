set -e
# final bench lines, then the int32 strip kernel (pairwg, forced) rolled vs whole-chunk unroll on C3 (GPU box)
bash tools/bench_lines.sh
for L in "" su32; do
  lib=$PWD/concurrentproject_amd/libswmi355${L:+_$L}.so
  SWMI355_LIB=$lib timeout -k 10 120 python tools/sweep.py --reps 3 --opt mode=1 --cases batch:8192:8192:8:64:1024,batch:8192:8192:8:64:1024 > gpurun_out/abs_${L:-def}.log 2>&1
done
