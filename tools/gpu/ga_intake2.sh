#!/bin/bash
# gap tests, then the intake variants on skewed configs[3] (3 rounds: digests must agree), then a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "gap" > gpurun_out/ga_intake_tests.txt 2>&1 || { tail -30 gpurun_out/ga_intake_tests.txt; exit 1; }
tail -3 gpurun_out/ga_intake_tests.txt
for round in 1 2 3; do
  VARIANTS="ga_nointake ga_lo0 ga_lo32k" WHICH=ga EXTRA="--shape skewed_config3" REPS=10 bash tools/gpu/ab.sh || exit 1
done
mkdir -p gpurun_out/kt_ga3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_ga3 -o kt -- python $R/tools/profile_kernels.py --which ga --shape skewed_config3 --reps 3 > $R/gpurun_out/kt_ga3/run.log 2>&1
