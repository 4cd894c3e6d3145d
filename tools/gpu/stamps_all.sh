#!/bin/bash
# phase stamps (diagnostic build) for each kernel on a 100k batch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in ${KERNELS:-bm md ga}; do
  w=$k
  timeout -k 10 300 python tools/profile_kernels.py --which $w --stamps --stamps-kernel $k --clusters ${CLUSTERS:-100000} --reps 2 > gpurun_out/stamps_$k.json 2>&1 || { tail -5 gpurun_out/stamps_$k.json; exit 1; }
  echo "$k $(grep '^{' gpurun_out/stamps_$k.json)"
done
