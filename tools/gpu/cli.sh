#!/bin/bash
# CLI-level GPU session: sharded/native/dict CLI parity tests, then the host-inclusive tiers.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_sharded_cli.py tests/test_gpu_shims.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/cli_tests.log 2>&1
rc=$?
tail -3 gpurun_out/cli_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E  )" gpurun_out/cli_tests.log | head -30; exit 1; }
timeout -k 10 600 python -u tools/bench_tiers.py ${TIER_ARGS:-} > gpurun_out/tiers.json 2> gpurun_out/tiers.err || { tail -5 gpurun_out/tiers.err; exit 1; }
cat gpurun_out/tiers.json
