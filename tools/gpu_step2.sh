set -e
mkdir -p gpurun_out/pr
timeout -k 10 100 python tools/probe_ring.py 400000 2 5 > gpurun_out/pr/a.txt 2>&1
timeout -k 10 100 python tools/probe_ring.py 1048576 2 5 > gpurun_out/pr/b.txt 2>&1
