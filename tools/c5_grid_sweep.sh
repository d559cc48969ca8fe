set -e
# C5 ring mode: persistent grid size vs the last round's tail (2081 groups over G blocks run in
# ceil(2081 / G) rounds; G = 1024 leaves a 33-group third round running alone)
mkdir -p gpurun_out/grid
for cfg in "0 0" "694 3" "694 4" "521 3" "417 2" "1024 4"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --workload slab --no-cpu-baseline --steps 2 --warmup 1 --opt blocks=$1 --opt f2_wgs=$2 > gpurun_out/grid/c5_$1_$2.json 2> gpurun_out/grid/c5_$1_$2.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/grid/c5_$1_$2.json').read().strip().splitlines()[-1])
print('blocks $1 f2_wgs $2', d['ms_per_step'], d.get('kernel_ms_per_launch'), d['config'].get('blocks'), d.get('score', d.get('scores')))"
done
