#!/bin/bash
# Phase ablation + PMC counter passes (separate rocprofv3 --pmc runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases.json 2>gpurun_out/phases.err || { tail -5 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.json
K='spx::(bin_mean_lds_kernel|medoid_small_kernel)'
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/p1" -o p1 --output-format csv -- python "$R/tools/profile_phases.py" plain > gpurun_out/pmc/p1.log 2>&1 || { tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/p2" -o p2 --output-format csv -- python "$R/tools/profile_phases.py" plain > gpurun_out/pmc/p2.log 2>&1 || { tail -5 gpurun_out/pmc/p2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/p3" -o p3 --output-format csv -- python "$R/tools/profile_phases.py" plain > gpurun_out/pmc/p3.log 2>&1 || { tail -5 gpurun_out/pmc/p3.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head -20
