#!/bin/bash
# Medoid intake (round 6): medoid GPU tests, then the A/B on skewed configs[3] and configs[4]-law 100k.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_streams.py -k "medoid or stream or fused or config3" > gpurun_out/md_intake_tests.txt 2>&1 || { tail -30 gpurun_out/md_intake_tests.txt; exit 1; }
tail -2 gpurun_out/md_intake_tests.txt
for round in 1 2 3; do
  VARIANTS="md_in0 md_in1" WHICH=md EXTRA="--shape skewed_config3" REPS=10 bash tools/gpu/ab.sh || exit 1
done
VARIANTS="md_in0 md_in1" WHICH=md CLUSTERS=100000 REPS=5 bash tools/gpu/ab.sh || exit 1
