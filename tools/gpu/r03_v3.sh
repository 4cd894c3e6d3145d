#!/bin/bash
# r03 v3: bin-mean parity (kept-bin fold, segmented fold, split path) + off-shape
# shapes with kernel trace; the headline bench with a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/r03_seg.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/head_kt" -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-extras > gpurun_out/head_kt.log 2>&1 || { tail -5 gpurun_out/head_kt.log; exit 1; }
tail -1 gpurun_out/head_kt.log
echo done
