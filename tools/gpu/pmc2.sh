#!/bin/bash
# PMC counter passes (separate rocprofv3 --pmc runs, kernel-trace only) for the
# bin-mean variants (5 hash stream, 6 bitmap stream, 0 per-cluster) and the medoid.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
rm -rf gpurun_out/pmc2 && mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
K='spx::(bin_mean_stream|bin_mean_stream2|bin_mean_lds|medoid_reg)_kernel'
run() {  # variant name counters...
  local var=$1 name=$2; shift 2
  SPX_BIN_KERNEL=$var timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$R/gpurun_out/pmc2/$name" -o "$name" --output-format csv -- python3 "$R/tools/profile_phases.py" plain > "gpurun_out/pmc2/$name.log" 2>&1 || { tail -5 "gpurun_out/pmc2/$name.log"; return 1; }
}
for v in 5 6 0; do
  run $v v${v}a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
  run $v v${v}b FETCH_SIZE || exit 1
  run $v v${v}c WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT || exit 1
done
for v in 5 6 0; do echo "##### variant $v"; python3 tools/pmc_summary.py gpurun_out/pmc2 --only "v${v}" ; done > gpurun_out/pmc2/summary.txt
cat gpurun_out/pmc2/summary.txt
