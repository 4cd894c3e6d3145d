#!/bin/bash
# Round 5: medoid register-kernel variants -- medoid / fused parity tests on the in-tree
# build, then the A/B of the variant libraries (digests must agree).  VARIANTS, TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-md}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py tests/test_gpu_shims.py \
  -k "medoid or fused or config5" > gpurun_out/${TAG}_tests.txt 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
VARIANTS="${VARIANTS}" WHICH=${WHICH:-md} CLUSTERS=${CLUSTERS:-385000} REPS=${REPS:-10} bash tools/gpu/ab.sh \
  | tee gpurun_out/${TAG}_ab.txt
