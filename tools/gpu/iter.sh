#!/bin/bash
# Iteration loop: GPU parity tests, then the bench and a bin-mean variant/phase timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
SPX_VARIANTS=${SPX_VARIANTS:-7,0} timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases.json 2>gpurun_out/phases.err || { tail -5 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.json
