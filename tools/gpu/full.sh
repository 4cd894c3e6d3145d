#!/bin/bash
# Round evidence: all GPU tests -> smoke -> bench (with extras) -> rocprofv3 kernel stats
# of the headline bench -> PMC passes on the bench configuration.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
[ -n "$NO_PMC" ] && exit 0
CLUSTERS=${PMC_CLUSTERS:-385000} bash tools/gpu/pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
echo pmc done
