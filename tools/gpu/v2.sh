#!/bin/bash
# Round 6: the one-read fused pass -- its parity tests, then an A/B of the variant
# libraries on the configs[4] batch (digests must agree between variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread \
  -k "${TESTS:-fused or bin_mean or medoid}" > gpurun_out/${TAG:-v2}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG:-v2}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG:-v2}_tests.txt
VARIANTS="${VARIANTS:-pre_prune v2km8 v2km6 v2km4 pre_prune v2km8}" WHICH=${WHICH:-bm,md,fu} CLUSTERS=${CLUSTERS:-385000} REPS=${REPS:-5} bash tools/gpu/ab.sh
