# PWG (flow2 pair per workgroup) parity + C3 int32 timing (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pwg.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pwg_tests.log 2>&1
o=gpurun_out/c3_pwg.jsonl
timeout -k 10 200 python tools/sweep.py --reps 5 --opt f2pwg=1 --cases batch:8192:8192:1:64:1024:5,batch:8192:8192:8:64:1024:1,batch:8192:8192:8:64:1024 > $o 2>&1
for w in 1 2; do
  timeout -k 10 200 python tools/sweep.py --reps 5 --opt f2pwg=1 --opt f2_wgs=$w --cases batch:8192:8192:1:64:1024:5 >> $o 2>&1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
