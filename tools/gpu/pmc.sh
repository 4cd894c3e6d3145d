#!/bin/bash
# Phase ablation + PMC counter passes (each its own rocprofv3 --pmc run,
# kernel-trace only) for the two headline kernels; then config-4 MFMA counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
K='spx::(bin_mean_lds_kernel|medoid_reg_kernel|medoid_gram_mfma_kernel)'
run() {  # name script counters...
  local name=$1 scr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmc/$name" -o "$name" --output-format csv -- python3 $scr > "gpurun_out/pmc/$name.log" 2>&1 || { tail -5 "gpurun_out/pmc/$name.log"; return 1; }
}
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases.json 2>gpurun_out/phases.err || { tail -5 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.json
P="$R/tools/profile_phases.py plain"
run a1 "$P" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run a2 "$P" FETCH_SIZE &&
run a3 "$P" WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM &&
run a4 "$P" SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH &&
run a5 "$P" TCC_HIT_sum TCC_MISS_sum &&
python3 tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc/pmc_traffic.json > gpurun_out/pmc/summary.txt &&
cat gpurun_out/pmc/summary.txt
