#!/bin/bash
# Round 3 bin-mean work: parity of the bin-mean paths (main library) -> reg-kernel
# A/B variants -> off-shape shapes with the old LDS kernel (ab_lds.so) and the wide
# kernel (main library), with kernel traces.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or edge or special or skewed or config5 or range" > gpurun_out/bm_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/bm_tests.log | head -30; tail -5 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
[ -n "$AB" ] && { VARIANTS="$AB" WHICH=bm CLUSTERS=385000 bash tools/gpu/ab.sh || exit 1; }
for lib in ${SHAPES:-ab_lds ""}; do
  [ "$lib" = main ] && lib=""
  tag=${lib:-main}
  SPX_LIB=${lib:+$R/specpride_amd/lib/$lib.so} timeout -k 10 300 python -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_$tag.log 2>&1 || { tail -5 gpurun_out/shapes_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/shapes_$tag.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/shapes_kt" -o kt --output-format csv -- python3 -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_kt.log 2>&1 || { tail -5 gpurun_out/shapes_kt.log; exit 1; }
f=$(find gpurun_out/shapes_kt -name "*kernel_stats.csv" | head -1)
cut -d, -f1-6 "$f" | awk "NR<=14"
