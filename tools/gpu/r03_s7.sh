#!/bin/bash
# GPU tests, per-call shim latency, binning CLI stage times on a tier-3 file.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/r03_s6.sh || exit 1
timeout -k 10 600 python tools/tier3_stages.py --clusters 100000 > gpurun_out/t3stages.log 2>&1 || { tail -5 gpurun_out/t3stages.log; exit 1; }
tail -3 gpurun_out/t3stages.log
