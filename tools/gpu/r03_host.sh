#!/bin/bash
# Round 3 host pipeline evidence: GPU tests -> tier 3 at configs[1] size (100k
# clusters, ~9 GB MGF per CLI) -> bench.py with extras (incl. tier 2 at configs[4]).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
df -h /tmp "$R" > gpurun_out/r03_env.txt 2>&1; free -g >> gpurun_out/r03_env.txt 2>&1; nproc >> gpurun_out/r03_env.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 900 python -u tools/bench_tiers.py --skip-t2 ${T3_ARGS} > gpurun_out/tiers.json 2> gpurun_out/tiers.err || { tail -20 gpurun_out/tiers.err; exit 1; }
cat gpurun_out/tiers.json
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
