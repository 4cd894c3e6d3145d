#!/bin/bash
# A/B of the medoid Gram variants on configs[3] (+ oracle check of the large clusters), then
# the medoid GPU tests and the MFMA PMC record of the product build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:?set VARIANTS to the ab_<name>.so builds to compare}; do
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 300 python tools/bench_medoid_large.py --reps 5 --check > gpurun_out/gram_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/gram_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/gram_$v.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "medoid or config3" > gpurun_out/gram_tests.log 2>&1 || { tail -20 gpurun_out/gram_tests.log; exit 1; }
tail -1 gpurun_out/gram_tests.log
bash tools/gpu/mfma.sh
