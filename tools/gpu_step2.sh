set -e
rm -rf gpurun_out/ab gpurun_out/ab2
bash tools/ab_multi.sh "libswmi355 libswmi355_DW8" --workload batch --steps 5 --warmup 1
mv gpurun_out/ab gpurun_out/ab2
bash tools/ab_multi.sh "libswmi355 libswmi355_DW8" --workload batch --steps 5 --warmup 1 --W 4
