#!/bin/bash
# Gap-average iteration: GPU parity tests (gap + precursor) -> config-3 shard bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gap or precursor or smoke or shim" > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python tools/bench_gap_average.py --check 300 > gpurun_out/gap.log 2>&1 || { tail -5 gpurun_out/gap.log; exit 1; }
tail -1 gpurun_out/gap.log
