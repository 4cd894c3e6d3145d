#!/bin/bash
# A/B the variant libraries specpride_amd/lib/ab_*.so (tools/build_variants.py) on
# one batch each: VARIANTS="a b c" WHICH=bm CLUSTERS=100000 [EXTRA="--shape long_spectra_600"] bash tools/gpu/ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 120 python tools/profile_kernels.py --which ${WHICH:-bm} --clusters ${CLUSTERS:-100000} --reps ${REPS:-10} ${EXTRA:-} > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/ab_$v.log)"
done
