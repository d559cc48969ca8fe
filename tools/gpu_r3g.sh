# PWG 4-B round buffer: parity, C3 on int32, slab per-rank costs (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pwg.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pwg_tests.log 2>&1
timeout -k 10 200 python tools/sweep.py --reps 5 --opt f2pwg=1 --cases batch:8192:8192:1:64:1024:5,batch:8192:8192:1:64:1024:5 > gpurun_out/c3_pwg4.jsonl 2>&1
bash tools/gpu_r3f.sh
