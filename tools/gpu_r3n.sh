# batch-size rule: parity (full GPU suite) and the automatic choice's times (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
cases=batch:8192:8192:8:64:512,batch:8192:8192:8:64:256,batch:8192:8192:8:64:128,batch:16384:16384:8:64:128,batch:65536:65536:8:64:16,batch:4096:4096:8:64:2048,batch:4096:4096:8:64:256,batch:32768:32768:8:64:64,batch:8192:8192:8:64:1024
timeout -k 10 280 python tools/sweep.py --reps 3 --cases $cases > gpurun_out/batch_auto.jsonl 2>&1
