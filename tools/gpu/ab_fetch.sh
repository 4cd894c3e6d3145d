#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the bin-mean register kernel for each variant library in
# $VARIANTS (specpride_amd/lib/ab_<v>.so) on the configs[4] batch, one --pmc run each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'spx::bin_mean_reg_kernel' -d "$R/gpurun_out/abf_${v}_$c" -o f --output-format csv -- python3 "$R/tools/profile_kernels.py" --which bm --clusters ${CLUSTERS:-385000} --reps 2 > gpurun_out/abf_${v}_$c.log 2>&1 || { echo "variant $v $c failed"; tail -5 gpurun_out/abf_${v}_$c.log; exit 1; }
  done
  echo "$v $(python3 tools/kstat.py gpurun_out/abf_${v}_FETCH_SIZE gpurun_out/abf_${v}_WRITE_SIZE | tr '\n' ' ')"
done
