#!/bin/bash
# Off-shape PMC traffic: FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3
# --pmc run) and a kernel trace over tools/run_shape.py for the bin-mean shapes and
# the medoid 600-peak shape; per-call bytes of all spx:: kernels ->
# gpurun_out/shapes_pmc/pmc_traffic_shapes.json (profiles/ format read by bench.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/shapes_pmc && mkdir -p gpurun_out/shapes_pmc
export TMPDIR=/tmp
O=gpurun_out/shapes_pmc
# SHAPES_PMC (optional): a comma-separated subset, e.g. "skewed_config3 ga,long_spectra_600 ga"
if [ -n "$SHAPES_PMC" ]; then
  IFS=',' read -ra LIST <<< "$SHAPES_PMC"
else
  LIST=("skewed_config3 bm" "long_spectra_600 bm" "long_spectra_600 md" "skewed_config3 ga" "long_spectra_600 ga")
fi
for S in "${LIST[@]}"; do
  set -- $S
  N="$2_$1"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/$N/f" -o f --output-format csv -- python3 tools/run_shape.py $1 3 $2 > $O/$N.f.log 2>&1 || { tail -5 $O/$N.f.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/$N/w" -o w --output-format csv -- python3 tools/run_shape.py $1 3 $2 > $O/$N.w.log 2>&1 || { tail -5 $O/$N.w.log; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/$O/$N/kt" -o kt --output-format csv -- python3 tools/run_shape.py $1 3 $2 > $O/$N.kt.log 2>&1 || { tail -5 $O/$N.kt.log; exit 1; }
  echo "$N done"
done
python3 tools/shapes_traffic.py $O > $O/summary.txt && cat $O/summary.txt
