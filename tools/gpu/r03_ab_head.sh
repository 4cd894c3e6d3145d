#!/bin/bash
# r03: headline A/B -- for the main library and each variant in $VARIANTS
# (specpride_amd/lib/ab_<v>.so): a kernel-trace of the headline bench and a
# FETCH_SIZE pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in main ${VARIANTS}; do
  if [ "$V" = main ]; then unset SPX_LIB; else export SPX_LIB="$R/specpride_amd/lib/ab_$V.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/hk_$V" -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/hk_$V.log 2>&1 || { tail -5 gpurun_out/hk_$V.log; exit 1; }
  echo "$V $(grep '^{' gpurun_out/hk_$V.log | cut -c1-120)"
  if [ -n "$PMC" ]; then
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/hp_$V" -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/hp_$V.log 2>&1 || { tail -5 gpurun_out/hp_$V.log; exit 1; }
  fi
done
unset SPX_LIB
echo done
