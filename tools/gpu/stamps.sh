#!/bin/bash
# bin-mean parity tests, then kernel timing + phase stamps (diagnostic build) on a 100k batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/profile_kernels.py --which ${WHICH:-bm,md} --clusters 100000 > gpurun_out/prof_k.json 2>&1 || { tail -5 gpurun_out/prof_k.json; exit 1; }
tail -1 gpurun_out/prof_k.json
timeout -k 10 300 python tools/profile_kernels.py --which bm --stamps --clusters 100000 > gpurun_out/stamps.json 2>&1 || { tail -5 gpurun_out/stamps.json; exit 1; }
tail -1 gpurun_out/stamps.json
