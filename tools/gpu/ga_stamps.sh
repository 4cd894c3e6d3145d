#!/bin/bash
# Gap-average LDS kernel phase stamps (ab_ga_st.so: -DSPX_STAMPS -DSPX_STAMPS_GA -DSPX_GA_STAMP_MASK=0xFE)
# and the product library's timing on configs[4]-law batches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPX_STAMPS_LIB="$R/specpride_amd/lib/ab_ga_st.so" timeout -k 10 180 python tools/profile_kernels.py --which ga --clusters ${CLUSTERS:-100000} --reps 3 --stamps --stamps-kernel ga > gpurun_out/ga_stamps.log 2>&1 || { tail -5 gpurun_out/ga_stamps.log; exit 1; }
grep '^{' gpurun_out/ga_stamps.log
