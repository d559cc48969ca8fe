# A/B of flow2 build variants on C2 (median/min ms over reps) plus a production-build strip trace each.
set -e
cases=${AB_CASES:-pair:65536:65536:1:32:1:5,pair:65536:65536:1:64:1:5,pair:65536:65536:1:32:1:5,pair:65536:65536:1:64:1:5}
timeout -k 10 120 python tools/sweep.py --reps 10 --cases $cases > gpurun_out/ab_default.log 2>&1
timeout -k 10 100 python tools/trace_flow.py 65536 32 1 65536 5 > gpurun_out/tr_default.txt 2>&1
for v in $AB_VARIANTS; do
  SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_$v.so timeout -k 10 120 python tools/sweep.py --reps 10 --cases $cases > gpurun_out/ab_$v.log 2>&1
  SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_$v.so timeout -k 10 100 python tools/trace_flow.py 65536 32 1 65536 5 > gpurun_out/tr_$v.txt 2>&1
done
