#!/bin/bash
# PMC counter passes (each its own rocprofv3 --pmc run, kernel-trace only) over
# tools/profile_kernels.py for the kernels matching K; summary via tools/pmc_summary.py.
#   K='spx::bin_mean_lds_kernel' CLUSTERS=100000 WHICH=bm bash tools/gpu/pmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
K=${K:-'spx::(bin_mean_reg_kernel|medoid_reg_kernel|gap_average_lds_kernel|bin_mean_medoid_kernel)'}
P="$R/tools/profile_kernels.py --which ${WHICH:-bm,md,ga,fu} --clusters ${CLUSTERS:-100000} --reps 2"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/$name" -o "$name" --output-format csv -- python3 $P > "gpurun_out/pmc/$name.log" 2>&1 || { tail -5 "gpurun_out/pmc/$name.log"; return 1; }
}
run a1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run a2 FETCH_SIZE &&
run a3 WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
run a4 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_ADD_F64 &&
run a5 TCC_HIT_sum TCC_MISS_sum &&
python3 tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc/pmc_traffic.json --peaks-from gpurun_out/pmc/a2.log > gpurun_out/pmc/summary.txt &&
cat gpurun_out/pmc/summary.txt
