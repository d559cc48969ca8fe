#!/bin/bash
# Seven-letter tests after the alphabet-scan change, then the driver's bench command (tools only).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hep2
timeout -k 10 600 python -u -m pytest tests/test_hepta.py tests/test_duo_raw.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hep2/t.log 2>&1
rc=$?; tail -3 gpurun_out/hep2/t.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/hep2/t.log; exit $rc; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/hep2/bench.json 2> gpurun_out/hep2/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/hep2/bench.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/hep2/bench.json')); print(json.dumps(d['summary'])); print(json.dumps(d.get('byte_alphabets'))[:1500])"
