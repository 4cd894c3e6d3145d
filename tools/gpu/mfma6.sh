#!/bin/bash
# Round 6: MFMA busy cycles of both MFMA paths, one --pmc pass each:
#   configs[3] large-cluster Gram (medoid_gram_reg_kernel, tools/bench_medoid_large.py);
#   configs[4] small-cluster P4 on the matrix cores past 32 spectra (medoid_reg_kernel, and
#   the fused pass bin_mean_medoid_kernel, tools/profile_kernels.py).
# busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) per dispatch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
rm -rf gpurun_out/mfma6 && mkdir -p gpurun_out/mfma6
C="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'medoid_gram_reg' -d "$R/gpurun_out/mfma6/c3" -o c3 --output-format csv -- python3 "$R/tools/bench_medoid_large.py" --reps 1 > gpurun_out/mfma6/c3.log 2>&1 || { tail -5 gpurun_out/mfma6/c3.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex 'spx::(medoid_reg_kernel|bin_mean_medoid_kernel)' -d "$R/gpurun_out/mfma6/c4" -o c4 --output-format csv -- python3 "$R/tools/profile_kernels.py" --which md,fu --clusters 385000 --reps 1 > gpurun_out/mfma6/c4.log 2>&1 || { tail -5 gpurun_out/mfma6/c4.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/mfma6 > gpurun_out/mfma6/summary.txt && cat gpurun_out/mfma6/summary.txt
