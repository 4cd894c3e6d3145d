#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace -> side benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || { grep -E "^(FAILED|E  )" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
timeout -k 10 300 python tools/bench_gap_average.py > gpurun_out/gap.log 2>&1 || { tail -5 gpurun_out/gap.log; exit 1; }
tail -1 gpurun_out/gap.log
timeout -k 10 300 python tools/bench_cosine.py > gpurun_out/cosine.log 2>&1 || { tail -5 gpurun_out/cosine.log; exit 1; }
tail -1 gpurun_out/cosine.log
timeout -k 10 400 python tools/bench_medoid_large.py > gpurun_out/medoid_large.log 2>&1 || { tail -5 gpurun_out/medoid_large.log; exit 1; }
tail -1 gpurun_out/medoid_large.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_side" -o side --output-format csv -- python3 "$R/tools/bench_gap_average.py" --reps 3 > gpurun_out/prof_side.log 2>&1 || { tail -5 gpurun_out/prof_side.log; exit 1; }
echo done
