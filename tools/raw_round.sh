set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/raw
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/raw/tests.log 2>&1 || { tail -30 gpurun_out/raw/tests.log; exit 1; }
tail -2 gpurun_out/raw/tests.log
timeout -k 10 300 python tools/bench_raw.py --reps 7 > gpurun_out/raw/bench_raw.jsonl
cat gpurun_out/raw/bench_raw.jsonl
for al in dna protein; do for r in 1 0; do
  timeout -k 10 300 python tools/bench_db.py --alphabet $al --opt duo_raw=$r >> gpurun_out/raw/bench_db.jsonl
done; done
cat gpurun_out/raw/bench_db.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/raw/kt -o raw -- python tools/bench_raw.py --alpha protein,acgt --reps 3 > gpurun_out/raw/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/raw/sq -o raw -- python tools/bench_raw.py --alpha protein,acgt --reps 1 > gpurun_out/raw/sq.log 2>&1
echo done
