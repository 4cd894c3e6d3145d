#!/bin/bash
# Side benches of the other §8 rows, each with its CPU baseline (1 host core).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out/side
timeout -k 10 300 python tools/bench_gap_average.py --check 200 > gpurun_out/side/gap.log 2>&1 || { tail -5 gpurun_out/side/gap.log; exit 1; }
tail -1 gpurun_out/side/gap.log
timeout -k 10 300 python tools/bench_cosine.py > gpurun_out/side/cosine.log 2>&1 || { tail -5 gpurun_out/side/cosine.log; exit 1; }
tail -1 gpurun_out/side/cosine.log
timeout -k 10 300 python tools/bench_best_score.py > gpurun_out/side/best.log 2>&1 || { tail -5 gpurun_out/side/best.log; exit 1; }
tail -1 gpurun_out/side/best.log
