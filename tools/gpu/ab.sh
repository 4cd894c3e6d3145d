#!/bin/bash
# A/B of experimental engine builds (specpride_amd/lib/exp/*.so, SPX_LIB) on the
# bench batch: bin-mean variant timing per build, default build last.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
for so in specpride_amd/lib/exp/*.so; do
  echo "== $so"
  SPX_LIB="$R/$so" SPX_VARIANTS=${SPX_VARIANTS:-0} timeout -k 10 200 python tools/profile_phases.py 2>>gpurun_out/ab.err || exit 1
done
echo "== default"
SPX_VARIANTS=${SPX_VARIANTS:-0} timeout -k 10 200 python tools/profile_phases.py 2>>gpurun_out/ab.err
