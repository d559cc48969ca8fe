# One GPU call: the GPU test suite (or the test files given), smoke(), and the default
# bench line.  Every GPU step has its own time limit; set -e stops at the first failure.
# usage (on the GPU box): bash tools/gpu_check.sh [pytest args...]
set -e
mkdir -p gpurun_out
tests="${*:-tests -m gpu}"
timeout -k 10 900 python -u -m pytest $tests -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
