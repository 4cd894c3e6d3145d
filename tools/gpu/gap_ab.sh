export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gap or average" > gpurun_out/par.log 2>&1; echo rc=$? >> gpurun_out/par.log; tail -2 gpurun_out/par.log
grep -q "rc=0" gpurun_out/par.log || exit 1
for so in specpride_amd/lib/exp/*.so; do echo "== $so"; SPX_LIB=$PWD/$so timeout -k 10 200 python tools/bench_gap_average.py --cpu-sample 0 || exit 1; done
echo "== default"; timeout -k 10 200 python tools/bench_gap_average.py --cpu-sample 0 --check 2000
