#!/bin/bash
# instruction-cache PMC pass (8 SQ-block counters) over tools/profile_kernels.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
O=gpurun_out/pmc_ic; rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
K=${K:-'spx::(bin_mean_reg_kernel|medoid_reg_kernel|gap_average_lds_kernel)'}
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-include-regex "$K" -d "$R/$O/i1" -o i1 --output-format csv -- python3 "$R/tools/profile_kernels.py" --which ${WHICH:-bm,md,ga} --clusters ${CLUSTERS:-100000} --reps 2 > $O/i1.log 2>&1 || { tail -5 $O/i1.log; exit 1; }
python3 tools/pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
