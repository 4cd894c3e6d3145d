#!/bin/bash
# Phase stamps of several diagnostic builds (specpride_amd/lib/ab_<v>.so built with
# -DSPX_STAMPS by tools/build_variants.py): VARIANTS="stold stfold" K=bm CLUSTERS=100000
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  SPX_STAMPS_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 200 python tools/profile_kernels.py --which ${K:-bm} \
    --stamps --stamps-kernel ${K:-bm} --clusters ${CLUSTERS:-100000} --reps 2 > gpurun_out/stamps_$v.json 2>&1 \
    || { echo "variant $v failed"; tail -5 gpurun_out/stamps_$v.json; exit 1; }
  echo "$v $(grep '^{' gpurun_out/stamps_$v.json)"
done
