#!/bin/bash
# PMC counter passes (separate rocprofv3 --pmc runs, kernel-trace only) for the
# headline kernels (both bin-mean variants) + the FETCH_SIZE calibration kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
K='spx::(bin_mean_list_kernel|bin_mean_lds_kernel|medoid_small_kernel)|calib_read'
run() {  # variant name counters...
  local var=$1 name=$2; shift 2
  SPX_BIN_KERNEL=$var timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/$name" -o "$name" --output-format csv -- python3 "$R/tools/profile_phases.py" plain > "gpurun_out/pmc/$name.log" 2>&1 || { tail -5 "gpurun_out/pmc/$name.log"; return 1; }
}
runc() {  # calibration pass
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/$name" -o "$name" --output-format csv -- python3 "$R/tools/calib/run_calib.py" > "gpurun_out/pmc/$name.log" 2>&1 || { tail -5 "gpurun_out/pmc/$name.log"; return 1; }
}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
run 0 a1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run 1 b1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run 0 a2 FETCH_SIZE &&
run 1 b2 FETCH_SIZE &&
run 0 a3 WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM &&
run 1 b3 WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM &&
runc c1 FETCH_SIZE &&
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt &&
cat gpurun_out/pmc/summary.txt &&
run 1 b4 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH &&
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt
