set -e
cases=pair:65536:65536:1:16:1:4,pair:65536:65536:1:32:1:4,pair:65536:65536:1:32:1:2
timeout -k 10 120 python tools/sweep.py --cases $cases > gpurun_out/ab_default.log 2>&1
for v in s0 s2 g1 g1s0; do
  SWMI355_LIB=$PWD/concurrentproject_amd/libswmi355_$v.so timeout -k 10 120 python tools/sweep.py --cases pair:65536:65536:1:16:1:4,pair:65536:65536:1:32:1:4 > gpurun_out/ab_$v.log 2>&1
done
