#!/bin/bash
# The binning CLI's stage times on a tier-3 file, then tier 3 for all three CLIs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/tier3_stages.py --clusters 100000 > gpurun_out/t3stages.log 2>&1 || { tail -5 gpurun_out/t3stages.log; exit 1; }
tail -1 gpurun_out/t3stages.log
timeout -k 10 900 python tools/bench_tiers.py --skip-t2 > gpurun_out/tiers.log 2>&1 || { tail -5 gpurun_out/tiers.log; exit 1; }
tail -1 gpurun_out/tiers.log
