# C3 batch on the flow2 kernel (int32, W2 linear step) vs duo and pairwg (GPU box)
set -e
mkdir -p gpurun_out
o=gpurun_out/c3_flow2.jsonl
timeout -k 10 200 python tools/sweep.py --reps 3 --cases batch:8192:8192:8:64:1024,batch:8192:8192:8:64:1024:1,batch:8192:8192:1:32:1024:5,batch:8192:8192:1:64:1024:5 >> $o 2>&1
for w in 2 4; do
  timeout -k 10 200 python tools/sweep.py --reps 3 --opt f2stream=1 --opt f2_wgs=$w --cases batch:8192:8192:1:32:1024:5,batch:8192:8192:1:64:1024:5 >> $o 2>&1
done
