#!/bin/bash
# A/B of specpride_amd/lib/ab_base.so vs ab_new.so on the binned cosine (tools/bench_cosine.py,
# 100k clusters) with result digests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-base new base new}; do
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 180 python tools/bench_cosine.py --clusters ${CLUSTERS:-100000} --cpu-sample 0 > gpurun_out/abc_$v.log 2>&1 || { tail -5 gpurun_out/abc_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/abc_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["binned_cosine_ms"], d["digest"], d["status_ok"])')"
done
