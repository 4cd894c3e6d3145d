#!/bin/bash
# r03: the hashed single-pass bin-mean kernel (ab_${TESTLIB:-hash}.so) through the bin-mean
# parity tests, then the headline A/B (r03_ab_head.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPX_LIB="$R/specpride_amd/lib/ab_${TESTLIB:-hash}.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or edge or special or skewed or config5 or config4 or range or kept or golden" > gpurun_out/ab_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/ab_tests.log | head -30; tail -5 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash tools/gpu/r03_ab_head.sh
