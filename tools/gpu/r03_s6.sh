#!/bin/bash
# GPU tests, then the per-call shim latency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/bench_shim_calls.py --calls 200 > gpurun_out/shim.log 2>&1 || { tail -5 gpurun_out/shim.log; exit 1; }
tail -1 gpurun_out/shim.log
