#!/bin/bash
# Round-1 iteration: parity tests -> bench -> phase/variant timing -> config-3/4 side benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases.json 2>gpurun_out/phases.err || { tail -5 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.json
timeout -k 10 300 python tools/bench_gap_average.py --check 300 > gpurun_out/gap.log 2>&1 || { tail -5 gpurun_out/gap.log; exit 1; }
tail -1 gpurun_out/gap.log
timeout -k 10 400 python tools/bench_medoid_large.py > gpurun_out/medoid_large.log 2>&1 || { tail -5 gpurun_out/medoid_large.log; exit 1; }
tail -1 gpurun_out/medoid_large.log
echo done
