set -o pipefail
export TMPDIR=/tmp
for v in head n32; do
  SPX_LIB=$PWD/specpride_amd/lib/ab_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/kt_$v -o kt --output-format csv -- python3 tools/profile_kernels.py --which bm --clusters 100000 --reps 5 > gpurun_out/kt_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/kt_$v.log
done
