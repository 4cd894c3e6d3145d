#!/bin/bash
# Gap-average giant intake (round 6): gap GPU tests, then the A/B on skewed configs[3] and configs[4].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "gap" > gpurun_out/ga_intake_tests.txt 2>&1 || { tail -30 gpurun_out/ga_intake_tests.txt; exit 1; }
tail -3 gpurun_out/ga_intake_tests.txt
for round in 1 2; do
  VARIANTS="${AB:-ga_nointake ga_own64k ga_own16k}" WHICH=ga EXTRA="--shape skewed_config3" REPS=10 bash tools/gpu/ab.sh || exit 1
done
VARIANTS="${AB:-ga_nointake ga_own64k ga_own16k}" WHICH=ga EXTRA="--shape long_spectra_600" REPS=10 bash tools/gpu/ab.sh || exit 1
