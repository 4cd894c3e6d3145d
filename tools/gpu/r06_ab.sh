#!/bin/bash
# Round 6 A/B pass: parity tests of the touched kernels on the default build, then the
# medoid per-spectrum variants on configs[4] and the gap-average partial-record pass 5 on
# the skewed configs[3] batch (digests must agree between variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "${TESTS:-medoid or fused or empty or gap or config3}" > gpurun_out/r06ab_tests.txt 2>&1 || { tail -30 gpurun_out/r06ab_tests.txt; exit 1; }
tail -2 gpurun_out/r06ab_tests.txt
VARIANTS="${MDV:-mdold mdc mdc6 mde mdold mdc}" WHICH=md,fu CLUSTERS=385000 REPS=10 bash tools/gpu/ab.sh || exit 1
VARIANTS="${GAV:-gaold ganew gaold ganew}" WHICH=ga REPS=10 EXTRA="--shape skewed_config3" bash tools/gpu/ab.sh
