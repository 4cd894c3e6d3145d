#!/bin/bash
# Quick iteration: GPU parity tests -> bench -> phase/variant timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases.json 2>gpurun_out/phases.err || { tail -5 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.json
