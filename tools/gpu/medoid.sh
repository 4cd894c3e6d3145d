#!/bin/bash
# Medoid large-path iteration: parity tests -> bench -> config-4 check + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 python tools/bench_medoid_large.py --check > gpurun_out/medoid_large.log 2>&1 || { tail -5 gpurun_out/medoid_large.log; exit 1; }
tail -1 gpurun_out/medoid_large.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_md -o run -- python3 tools/bench_medoid_large.py > gpurun_out/prof_md.log 2>&1 || { tail -5 gpurun_out/prof_md.log; exit 1; }
f=$(find gpurun_out/prof_md -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -14
