#!/bin/bash
# r03: bin-mean parity, then PMC passes (SQ issue/wait breakdown, LDS) over the
# skewed shape's kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bin_mean or edge or special or skewed or config5 or range or kept" > gpurun_out/bm_tests.log 2>&1 || { grep -E "^(FAILED|E  )" gpurun_out/bm_tests.log | head -30; tail -5 gpurun_out/bm_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/bm_tests.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_main" -o kt --output-format csv -- python3 -c "import bench, json; o = {}; bench.bin_mean_shapes(None, o); print(json.dumps(o))" > gpurun_out/shapes_main.log 2>&1 || { tail -5 gpurun_out/shapes_main.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS -d "$R/gpurun_out/pmc1" -o pmc --output-format csv -- python3 tools/run_shape.py skewed_config3 2 > gpurun_out/pmc1.log 2>&1 || { tail -5 gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$R/gpurun_out/pmc2" -o pmc --output-format csv -- python3 tools/run_shape.py skewed_config3 2 > gpurun_out/pmc2.log 2>&1 || { tail -5 gpurun_out/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc3" -o pmc --output-format csv -- python3 tools/run_shape.py skewed_config3 2 > gpurun_out/pmc3.log 2>&1 || { tail -5 gpurun_out/pmc3.log; exit 1; }
echo done
