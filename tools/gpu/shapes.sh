#!/bin/bash
# bin-mean on the skewed configs[3] law and on >252-peak spectra (bench.py bin_mean_shapes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes.log 2>&1 || { tail -5 gpurun_out/shapes.log; exit 1; }
tail -1 gpurun_out/shapes.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/shapes_kt" -o kt --output-format csv -- python3 -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_kt.log 2>&1 || { tail -5 gpurun_out/shapes_kt.log; exit 1; }
f=$(find gpurun_out/shapes_kt -name "*kernel_stats.csv" | head -1)
cut -d, -f1-6 "$f" | head -12
