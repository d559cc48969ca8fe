set -e
mkdir -p gpurun_out/w
for w in 1 2 3 4; do
  timeout -k 10 120 python bench.py --workload slab --steps 3 --warmup 1 --no-cpu-baseline --opt f2_wgs=$w > gpurun_out/w/c5_$w.json 2>&1
done
bash tools/ab_lib.sh concurrentproject_amd/libswmi355_head.so concurrentproject_amd/libswmi355.so --workload pair --steps 10 --warmup 2
