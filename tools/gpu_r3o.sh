set -e
# full duo unroll: GPU tests, C3 A/B against the 8-of-16 build, C3 profiles (GPU box)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
bash tools/ab_duo.sh du8
bash tools/prof_round.sh c3
