set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base new base new; do
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 120 python tools/profile_kernels.py --which md --clusters 100000 --reps 20 > gpurun_out/abm_$v.log 2>&1 || exit 1
  SPX_LIB="$R/specpride_amd/lib/ab_$v.so" timeout -k 10 180 python tools/bench_cosine.py --clusters 100000 --cpu-sample 0 > gpurun_out/abc_$v.log 2>&1 || exit 1
  echo "$v $(grep '^{' gpurun_out/abm_$v.log | cut -c60-200) | $(grep '^{' gpurun_out/abc_$v.log | cut -c1-250)"
done
