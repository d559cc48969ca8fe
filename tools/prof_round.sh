set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/prof/bench_c2.json 2> gpurun_out/prof/bench_c2.err
timeout -k 10 200 python bench.py --workload batch --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_c3.json 2> gpurun_out/prof/bench_c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt_c2 -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/kt_c2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt_c3 -o c3 -- python bench.py --workload batch --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/kt_c3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_c2 -o c2 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch_c2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_c2 -o c2 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write_c2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch_c3 -o c3 -- python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch_c3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write_c3 -o c3 -- python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write_c3.log 2>&1
