#!/bin/bash
# Medoid A/B: VARIANTS (ab_*.so) on the 385k headline batch (WHICH=md) and on the
# 600-peak shape (bench.medoid_shapes), then the medoid GPU tests with the main library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  lib="$R/specpride_amd/lib/ab_$v.so"; [ "$v" = main ] && lib=""
  SPX_LIB=$lib timeout -k 10 200 python tools/profile_kernels.py --which md --clusters ${CLUSTERS:-385000} --reps 10 > gpurun_out/abmd_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abmd_$v.log; exit 1; }
  SPX_LIB=$lib timeout -k 10 300 python -c "import bench, json; o = {}; bench.medoid_shapes(None, o); print(json.dumps(o))" > gpurun_out/mdshape_$v.log 2>&1 || { echo "shape $v failed"; tail -5 gpurun_out/mdshape_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/abmd_$v.log) $(tail -1 gpurun_out/mdshape_$v.log)"
done
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "medoid or config3 or config5 or cli" > gpurun_out/md_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/md_tests.log | head -30; tail -5 gpurun_out/md_tests.log; exit 1; }
tail -1 gpurun_out/md_tests.log
