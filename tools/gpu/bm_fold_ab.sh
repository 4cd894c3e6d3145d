#!/bin/bash
# Round 5: the bin-mean fold-by-slot register path -- bin-mean / fused parity tests on the
# in-tree build, then the A/B of the variant libraries on the configs[4] batch (digests
# must agree).  VARIANTS="old fold ..." (tools/build_variants.py), TAG=...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-bmfold}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py \
  -k "bin_mean or fused or config5 or config3_skewed_bin" > gpurun_out/${TAG}_tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
VARIANTS="${VARIANTS}" WHICH=${WHICH:-bm} CLUSTERS=${CLUSTERS:-385000} REPS=${REPS:-10} bash tools/gpu/ab.sh \
  | tee gpurun_out/${TAG}_ab.txt
