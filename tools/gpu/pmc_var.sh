#!/bin/bash
# PMC passes for one bin-mean variant (SPX_BIN_KERNEL) and ablation mask (SPX_ABLATE).
# usage: tools/gpu/pmc_var.sh <variant> <ablate> <kernel-regex> <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
export TMPDIR=/tmp
V=$1; A=$2; K=$3; O=gpurun_out/$4
rm -rf "$O" && mkdir -p "$O"
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE"; do
  i=$((i+1))
  SPX_BIN_KERNEL=$V SPX_ABLATE=$A timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "$K" -d $O/p$i -o p$i --output-format csv -- python3 tools/profile_phases.py plain > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O
