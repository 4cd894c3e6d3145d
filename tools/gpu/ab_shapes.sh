#!/bin/bash
# A/B of variant libraries (specpride_amd/lib/ab_<v>.so) on the off-shape batches with
# result digests: VARIANTS="a b" [MEDOID=1] bash tools/gpu/ab_shapes.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 180 python tools/ab_shapes.py ${MEDOID:+--medoid} > gpurun_out/abs_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abs_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/abs_$v.log)"
done
