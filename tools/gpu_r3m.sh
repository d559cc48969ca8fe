# batch kernel choice vs batch size: duo (auto), flow2 PWG, flow2 item claim (streamed, 2 per CU) (GPU box)
set -e
mkdir -p gpurun_out
o=gpurun_out/batch_choice.jsonl
cases=batch:8192:8192:8:64:512,batch:8192:8192:8:64:256,batch:8192:8192:8:64:128,batch:16384:16384:8:64:128,batch:65536:65536:8:64:16,batch:4096:4096:8:64:2048,batch:4096:4096:8:64:256
timeout -k 10 280 python tools/sweep.py --reps 3 --cases $cases > $o 2>&1
c5=$(echo $cases | sed 's/:8:64:\([0-9]*\)/:1:64:\1:5/g')
timeout -k 10 280 python tools/sweep.py --reps 3 --opt f2pwg=1 --cases $c5 >> $o 2>&1
timeout -k 10 280 python tools/sweep.py --reps 3 --opt f2pwg=0 --opt f2stream=1 --opt f2_wgs=2 --cases $c5 >> $o 2>&1
