set -e
# Shader clock and package power while each workload runs (rocm-smi polled every ~0.5 s beside a
# long sweep): is the VALU-heavy batch kernel running at the boost clock or power-limited?
# usage (GPU box): bash tools/clock_probe.sh
mkdir -p gpurun_out/clk
for w in idle c2 c3 c5; do
  case $w in
    idle) cases="";;
    c2) cases="pair:65536:65536:1:32:1:5"; reps=6000;;
    c3) cases="batch:8192:8192:8:64:1024"; reps=3000;;
    c5) cases="pair:1048576:1048576:1:32:1:5"; reps=80;;
  esac
  if [ -n "$cases" ]; then
    timeout -k 10 150 python tools/sweep.py --reps $reps --cases $cases > gpurun_out/clk/sweep_$w.log 2>&1 &
    pid=$!
    sleep 6
  fi
  for i in 1 2 3 4 5 6; do
    timeout -k 5 20 rocm-smi --showclocks --showpower --json >> gpurun_out/clk/smi_$w.jsonl 2>/dev/null || true
    echo >> gpurun_out/clk/smi_$w.jsonl
    sleep 0.5
  done
  if [ -n "$cases" ]; then wait $pid; fi
done
