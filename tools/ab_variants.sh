set -e
# A/B of flow2 hand-off variants (libswmi355_<v>.so built by make variants) on C2, with a strip trace each,
# then C5 and the GPU tests on the default build
mkdir -p gpurun_out
C2=pair:65536:65536:1:32:1:5
for L in "" ${AB_VARIANTS:-ld0 q8 q2}; do
  lib=$PWD/concurrentproject_amd/libswmi355${L:+_$L}.so
  SWMI355_LIB=$lib timeout -k 10 120 python tools/sweep.py --reps 10 --cases $C2,$C2 > gpurun_out/ab_${L:-def}.log 2>&1
  SWMI355_LIB=$lib timeout -k 10 100 python tools/trace_flow.py 65536 32 1 65536 5 > gpurun_out/tr_${L:-def}.txt 2>&1
done
if [ -z "$AB_QUICK" ]; then
  timeout -k 10 120 python tools/sweep.py --reps 3 --cases pair:1048576:1048576:1:32:1:5 > gpurun_out/ab_c5.log 2>&1
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
fi
