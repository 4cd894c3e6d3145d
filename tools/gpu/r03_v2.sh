#!/bin/bash
# r03 v2: bin-mean parity + off-shape shapes with kernel trace (LDS-slot segmented
# fold), medoid parity + headline medoid, tier-2 host-inclusive rate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/r03_seg.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded_cli.py -m gpu -x -v --timeout 300 --timeout-method thread -k "medoid or xcorr or representative" > gpurun_out/md_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/md_tests.log | head -30; tail -5 gpurun_out/md_tests.log; exit 1; }
tail -1 gpurun_out/md_tests.log
timeout -k 10 300 python -c "import bench, json; o = {}; bench.medoid_shapes(None, o); print(json.dumps(o))" > gpurun_out/md_shapes.log 2>&1 || { tail -5 gpurun_out/md_shapes.log; exit 1; }
tail -1 gpurun_out/md_shapes.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/head_kt" -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-extras > gpurun_out/head_kt.log 2>&1 || { tail -5 gpurun_out/head_kt.log; exit 1; }
tail -1 gpurun_out/head_kt.log
timeout -k 10 400 python -c "import sys, bench, json; sys.argv = ['bench.py']; o = {}; bench.tier2(bench.parse(), o); print(json.dumps(o))" > gpurun_out/tier2.log 2>&1 || { tail -5 gpurun_out/tier2.log; exit 1; }
tail -1 gpurun_out/tier2.log
echo done
