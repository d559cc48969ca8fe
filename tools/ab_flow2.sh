# A/B of flow2 build variants on C2 (kernel ms per launch), then a timeline of the default build.
set -e
cases=pair:65536:65536:1:32:1:5,pair:65536:65536:1:16:1:5,pair:65536:65536:1:64:1:5
timeout -k 10 120 python tools/sweep.py --cases $cases > gpurun_out/ab_default.log 2>&1
for v in $AB_VARIANTS; do
  SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_$v.so timeout -k 10 120 python tools/sweep.py --cases $cases > gpurun_out/ab_$v.log 2>&1
done
SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_timeline.so timeout -k 10 100 python tools/trace_flow.py 65536 32 1 65536 5 > gpurun_out/tr_f2_32.txt 2>&1
