#!/bin/bash
# Gap-average precursor radix select: gap/precursor GPU tests, the skewed and
# configs[4] gap-average timings and digests, a kernel trace of the skewed batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v \
  -k "gap or precursor or skewed" --timeout 300 --timeout-method thread > gpurun_out/s8_tests.log 2>&1 \
  || { grep -E "^(FAILED|E  )" gpurun_out/s8_tests.log | head -30; tail -5 gpurun_out/s8_tests.log; exit 1; }
tail -1 gpurun_out/s8_tests.log
timeout -k 10 300 python tools/ab_shapes.py --gap --shapes skewed_config3,long_spectra_600 > gpurun_out/s8_shapes.log 2>&1 || { tail -5 gpurun_out/s8_shapes.log; exit 1; }
tail -1 gpurun_out/s8_shapes.log
timeout -k 10 300 python tools/profile_kernels.py --clusters 385000 --which ga > gpurun_out/s8_ga.log 2>&1 || { tail -5 gpurun_out/s8_ga.log; exit 1; }
tail -1 gpurun_out/s8_ga.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s8_prof -o s8 -- python3 tools/run_gap_shape.py skewed_config3 > gpurun_out/s8_prof.log 2>&1 || { tail -5 gpurun_out/s8_prof.log; exit 1; }
echo done
