#!/bin/bash
# Per-call shim latency (tools/bench_shim_calls.py), then the same under a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_shim_calls.py --calls 200 > gpurun_out/shim.log 2>&1 || { tail -5 gpurun_out/shim.log; exit 1; }
tail -1 gpurun_out/shim.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/shim_kt" -o kt --output-format csv -- python3 tools/bench_shim_calls.py --calls 50 > gpurun_out/shim_kt.log 2>&1 || { tail -5 gpurun_out/shim_kt.log; exit 1; }
echo done
