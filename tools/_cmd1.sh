set -e
bash tools/gpu_run.sh tests
bash tools/ab.sh 2 --libs ablib/lib_ring0.so ablib/lib_spin.so -- --no-extra --steps 20 --warmup 3
cp -r gpurun_out/ab gpurun_out/ab_c2
bash tools/ab.sh 1 --libs ablib/lib_ring0.so ablib/lib_spin.so -- --workload batch --steps 5 --warmup 1
cp -r gpurun_out/ab gpurun_out/ab_c3
bash tools/ab.sh 1 --libs ablib/lib_ring0.so ablib/lib_spin.so -- --workload slab --steps 3 --warmup 1
cp -r gpurun_out/ab gpurun_out/ab_c5
bash tools/ab.sh 1 --libs ablib/lib_ring0.so ablib/lib_spin.so -- --workload slab --slab-of 8 --steps 3 --warmup 1
