# A/B of flow2 build variants on C2 with the W2 kernel (the automatic choice at the reference's
# constants): sweep median/min ms per library, interleaved, plus a W2 strip trace of each (GPU box).
#   AB_VARIANTS="sp4 sp8" bash tools/ab_f2w2.sh
set -e
mkdir -p gpurun_out
cases=${AB_CASES:-pair:65536:65536:1:32:1:5,pair:65536:65536:1:32:1:5,pair:65536:65536:1:32:1:5}
for v in default $AB_VARIANTS; do
  lib=$PWD/concurrentproject_amd/libswmi355${v/default/}.so
  [ "$v" = default ] || lib=$PWD/concurrentproject_amd/libswmi355_$v.so
  SWMI355_LIB=$lib timeout -k 10 120 python tools/sweep.py --reps 10 --cases $cases > gpurun_out/ab_$v.log 2>&1
  SWMI355_LIB=$lib timeout -k 10 100 python tools/trace_flow.py 65536 32 1 65536 5 2 > gpurun_out/tr_$v.txt 2>&1
done
