#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"; mkdir -p gpurun_out/l2pmc; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/l2pmc/h" -o h --output-format csv -- python3 tools/run_shape.py skewed_config3 3 ga > gpurun_out/l2pmc/h.log 2>&1 || { tail -5 gpurun_out/l2pmc/h.log; exit 1; }
echo done
