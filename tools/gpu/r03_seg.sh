#!/bin/bash
# Round 3: bin-mean parity (segmented fold, split path, wide kernel), host copy rates,
# off-shape shapes with kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or edge or special or skewed or config5 or range or kept" > gpurun_out/bm_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/bm_tests.log | head -30; tail -5 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
timeout -k 10 300 python tools/bench_h2d.py > gpurun_out/h2d.json 2>&1 || { tail -5 gpurun_out/h2d.json; exit 1; }
cat gpurun_out/h2d.json
timeout -k 10 300 python -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_main.log 2>&1 || { tail -5 gpurun_out/shapes_main.log; exit 1; }
tail -1 gpurun_out/shapes_main.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/shapes_kt" -o kt --output-format csv -- python3 -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_kt.log 2>&1 || { tail -5 gpurun_out/shapes_kt.log; exit 1; }
echo done
