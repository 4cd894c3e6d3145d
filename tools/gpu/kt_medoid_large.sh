#!/bin/bash
# configs[3] medoid per-kernel split (rocprofv3 kernel trace) for variant libraries: VARIANTS="a b"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VARIANTS; do
  ( cd /tmp && SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ktml_$v" -o run --output-format csv \
      -- python3 "$R/tools/bench_medoid_large.py" --reps 5 > "$R/gpurun_out/ktml_$v.log" 2>&1 ) || { echo "variant $v failed"; tail -5 gpurun_out/ktml_$v.log; exit 1; }
  echo "== $v $(grep '^{' gpurun_out/ktml_$v.log)"
  f=$(find gpurun_out/ktml_$v -name '*kernel_stats.csv' | head -1)
  python3 tools/kstats.py "$f" 2>/dev/null | head -20 || head -20 "$f"
done
