#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per group, kernel-trace only) over
# tools/run_shape.py for the kernels matching K on one off-shape batch:
#   K='spx::bin_mean_wide_kernel' SHAPE=long_spectra_600 WHICH=bm bash tools/gpu/pmc_shape.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/pmc_${WHICH:-bm}_${SHAPE:-long_spectra_600}
rm -rf "$O" && mkdir -p "$O"
export TMPDIR=/tmp
K=${K:-'spx::bin_mean_wide_kernel'}
P="$R/tools/run_shape.py ${SHAPE:-long_spectra_600} 2 ${WHICH:-bm}"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/$O/$name" -o "$name" --output-format csv -- python3 $P > "$O/$name.log" 2>&1 || { tail -5 "$O/$name.log"; return 1; }
}
run a1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run a2 FETCH_SIZE &&
run a3 WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
run a4 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_ADD_F64 &&
python3 tools/pmc_summary.py "$O" > "$O/summary.txt" &&
cat "$O/summary.txt"
