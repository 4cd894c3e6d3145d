#!/bin/bash
# Config 4 (skewed sizes, MFMA Gram path): kernel stats + MFMA busy-cycle PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
rm -rf gpurun_out/mfma && mkdir -p gpurun_out/mfma
timeout -k 10 300 python tools/bench_medoid_large.py --reps 5 > gpurun_out/mfma/bench.log 2>&1 || { tail -5 gpurun_out/mfma/bench.log; exit 1; }
tail -1 gpurun_out/mfma/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/mfma/kt" -o kt --output-format csv -- python3 "$R/tools/bench_medoid_large.py" --reps 5 > gpurun_out/mfma/kt.log 2>&1 || { tail -5 gpurun_out/mfma/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex 'medoid_gram_(mfma|reg|lds)' -d "$R/gpurun_out/mfma/pmc" -o pmc --output-format csv -- python3 "$R/tools/bench_medoid_large.py" --reps 1 > gpurun_out/mfma/pmc.log 2>&1 || { tail -5 gpurun_out/mfma/pmc.log; exit 1; }
find gpurun_out/mfma -name "*.csv" | head
