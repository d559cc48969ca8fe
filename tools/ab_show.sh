# summarise gpurun_out/ab_*.log and tr_*.txt written by tools/ab_flow2.sh
for f in gpurun_out/ab_*.log; do
  v=${f#gpurun_out/ab_}; v=${v%.log}
  echo "== $v"
  grep "^{" $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  ', d['case'], d.get('ms_med'), d.get('ms_min'), d.get('gcups'), d.get('score0'))"
  [ -f gpurun_out/tr_$v.txt ] && grep "^{" gpurun_out/tr_$v.txt | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('   trace', {k:d[k] for k in ('total_ms','lag_end_ns_ingroup','lag_end_ns_crossgroup','strip0_run_ns_per_step','slow_chunks_ingroup_mean','slow_chunks_crossgroup_mean')})"
done
