#!/bin/bash
# r03 v4: bin-mean parity, then the off-shape shapes under a kernel trace for the
# main library and each A/B variant in $VARIANTS (specpride_amd/lib/ab_<v>.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or edge or special or skewed or config5 or range or kept" > gpurun_out/bm_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/bm_tests.log | head -30; tail -5 gpurun_out/bm_tests.log; exit 1; }
tail -1 gpurun_out/bm_tests.log
for V in main ${VARIANTS}; do
  if [ "$V" = main ]; then unset SPX_LIB; else export SPX_LIB="$R/specpride_amd/lib/ab_$V.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_$V" -o kt --output-format csv -- python3 -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_$V.log 2>&1 || { tail -5 gpurun_out/shapes_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/shapes_$V.log | cut -c1-400)"
done
unset SPX_LIB
echo done
