#!/bin/bash
# bin-mean split path: parity tests (CPU oracle), then the off-shape timings with kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or config3 or config5 or special or skewed or edge or range" > gpurun_out/split_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/split_tests.log | head -30; tail -5 gpurun_out/split_tests.log; exit 1; }
tail -1 gpurun_out/split_tests.log
bash tools/gpu/shapes.sh
