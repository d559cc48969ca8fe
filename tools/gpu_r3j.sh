# C5 strip timeline (W2, ring mode): where the third round's groups end (GPU box)
set -e
mkdir -p gpurun_out
TRACE_DUMP=gpurun_out/trace_c5.npy timeout -k 10 200 python tools/trace_flow.py 1048576 64 1 1048576 5 2 > gpurun_out/trace_c5.txt 2>&1
