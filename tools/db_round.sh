#!/bin/bash
# Database search on the GPU box (tools only): the DB tests, then one query and 16 pipelined queries,
# DNA and protein.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/db
timeout -k 10 600 python -u -m pytest tests/test_db.py tests/test_hepta.py tests/test_duo_raw.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/db/t.log 2>&1
rc=$?; tail -3 gpurun_out/db/t.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/db/t.log; exit $rc; }
for al in dna protein; do
  timeout -k 10 300 python tools/bench_db.py --alphabet $al --queries 16 >> gpurun_out/db/bench_db.jsonl || exit 1
done
cat gpurun_out/db/bench_db.jsonl
