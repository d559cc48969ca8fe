set -e
TRACE_OPTS="ring=1" timeout -k 10 120 python tools/trace_flow.py 131072 64 1 131040 5 2 > gpurun_out/trace_s17.txt 2>&1
TRACE_OPTS="ring=1" timeout -k 10 120 python tools/trace_flow.py 262144 64 1 131040 5 2 > gpurun_out/trace_s18.txt 2>&1
TRACE_OPTS="ring=1" timeout -k 10 120 python tools/trace_flow.py 1048576 64 1 131040 5 2 > gpurun_out/trace_s20.txt 2>&1
