#!/bin/bash
# PMC passes over the configs[3] medoid large path (tools/bench_medoid_large.py) for the
# kernels matching K (default: leaves, fill, transpose, gram); summary via tools/pmc_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/pmcl && mkdir -p gpurun_out/pmcl
export TMPDIR=/tmp
K=${K:-'spx::medoid_(leaves|fill|transpose|gram_reg)_kernel'}
run() {  # name counters...
  local name=$1; shift
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmcl/$name" -o "$name" --output-format csv -- python3 "$R/tools/bench_medoid_large.py" --reps 2 > "$R/gpurun_out/pmcl/$name.log" 2>&1 ) || { tail -5 "gpurun_out/pmcl/$name.log"; return 1; }
}
run a1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run a2 FETCH_SIZE &&
run a3 WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS &&
python3 tools/pmc_summary.py gpurun_out/pmcl > gpurun_out/pmcl/summary.txt &&
cat gpurun_out/pmcl/summary.txt
