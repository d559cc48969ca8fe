# long pairs in a batch (64 x 32768, 256 x 16384): duo (u16, no f16 max3), pairwg, flow2 PWG, flow2 item claim (GPU box)
set -e
mkdir -p gpurun_out
o=gpurun_out/long_batch.jsonl
timeout -k 10 250 python tools/sweep.py --reps 3 --cases batch:32768:32768:8:64:64,batch:32768:32768:8:64:64:1,batch:16384:16384:8:64:256,batch:16384:16384:8:64:256:1 > $o 2>&1
timeout -k 10 250 python tools/sweep.py --reps 3 --opt f2pwg=1 --cases batch:32768:32768:1:64:64:5,batch:16384:16384:1:64:256:5 >> $o 2>&1
timeout -k 10 250 python tools/sweep.py --reps 3 --opt f2pwg=0 --opt f2stream=1 --opt f2_wgs=2 --cases batch:32768:32768:1:64:64:5,batch:16384:16384:1:64:256:5 >> $o 2>&1
