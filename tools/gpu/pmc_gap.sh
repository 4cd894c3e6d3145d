#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/pmc_gap; rm -rf $O && mkdir -p $O
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "gap_average_lds" -d $O/p$i -o p$i --output-format csv -- python3 tools/bench_gap_average.py --reps 1 --cpu-sample 0 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O
