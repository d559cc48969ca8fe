# strip timelines of the C2 pair: W = 1 and W = 2 (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 120 python tools/trace_flow.py 65536 32 1 65536 5 1 > gpurun_out/trace_w1.txt 2>&1
timeout -k 10 120 python tools/trace_flow.py 65536 32 1 65536 5 2 > gpurun_out/trace_w2.txt 2>&1
