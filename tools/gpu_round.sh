# One GPU call: the full GPU test suite, smoke(), then the round's profiles
# (tools/prof_round.sh: bench lines, kernel-trace stats, FETCH/WRITE/SQ/GRBM passes
# for C2, C3 and C5).  Every GPU step has its own time limit; set -e stops at the
# first failure.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
bash tools/prof_round.sh
