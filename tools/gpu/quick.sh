#!/bin/bash
# Iteration loop: GPU parity tests (TESTS, default all) -> bench headline only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 600 python bench.py --no-extras --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernels'], 'bm frac', d['roofline']['frac'], 'md frac', d['roofline_medoid']['frac'])"
