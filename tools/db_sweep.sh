#!/bin/bash
# DB search plan sweep on the GPU box (tools only): the default plan against other columns per lane
# and duo scheduling options, DNA and protein, one JSON line per setting (opts joined by +).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dbs
out=gpurun_out/dbs/sweep.jsonl
: > $out
for al in dna protein; do
  for o in "" "W=2+C=32" "W=8" "duo_prio=0" "duo_roles=0" "duo_tab=0" "duo_lds=0"; do
    args=""; for kv in ${o//+/ }; do args="$args --opt $kv"; done
    echo "== $al $o ($(date +%T))"
    timeout -k 10 120 python tools/bench_db.py --alphabet $al --steps 5 $args > gpurun_out/dbs/one.json 2> gpurun_out/dbs/one.err
    rc=$?
    if [ $rc -eq 0 ]; then
      python -c "import json; d=json.load(open('gpurun_out/dbs/one.json')); d['opt']='$o'; print(json.dumps(d))" >> $out
      tail -1 $out | cut -c1-300
    elif [ $rc -eq 1 ]; then
      tail -1 gpurun_out/dbs/one.err
    else
      tail -5 gpurun_out/dbs/one.err; exit $rc
    fi
  done
done
