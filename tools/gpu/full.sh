#!/usr/bin/env bash
# One GPU-box pass: parity tests, smoke, headline bench and a rocprofv3 kernel-trace summary.
# Usage (from this container):  gpurun --timeout 1000 -- 'bash tools/gpu/full.sh r03_v12'
# Every GPU step has its own time limit and the steps are chained with &&, so the first
# failure (fault, abort, timeout) ends the script. Results land under gpurun_out/.
set -euo pipefail
tag="${1:-run}"
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out"
mkdir -p "$out"
cd "$root"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/${tag}_gpu_tests.txt" 2>&1
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke(); print("SMOKE OK")' \
  > "$out/${tag}_smoke.txt" 2>&1
timeout -k 10 400 python bench.py > "$out/${tag}_bench.json" 2> "$out/${tag}_bench.err"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_${tag}" -o run --output-format csv \
  -- python3 "$root/bench.py" --steps 5 --warmup 2 --no-extras --no-cpu-baseline > "$out/${tag}_prof_bench.log" 2>&1
cd "$root"
if [ -z "${NO_PMC:-}" ]; then
  CLUSTERS=385000 bash tools/gpu/pmc.sh > "$out/${tag}_pmc.txt" 2>&1
fi
