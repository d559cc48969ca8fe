set -e
# A/B of duo builds on the C3 batch at W = 8 and W = 4: bash tools/ab_duo.sh <variant>...
mkdir -p gpurun_out
for L in "" "$@"; do
  lib=$PWD/concurrentproject_amd/libswmi355${L:+_$L}.so
  SWMI355_LIB=$lib timeout -k 10 120 python tools/sweep.py --reps 5 --cases batch:8192:8192:8:64:1024,batch:8192:8192:4:64:1024,batch:8192:8192:8:64:1024,batch:8192:8192:4:64:1024 > gpurun_out/abd_${L:-def}.log 2>&1
done
