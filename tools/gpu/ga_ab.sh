set -o pipefail
export TMPDIR=/tmp
WHICH=ga VARIANTS="head it0 it1" bash tools/gpu/ab.sh &&
CLUSTERS=125000 WHICH=ga VARIANTS="head it1" bash tools/gpu/ab.sh &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_shims.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gap or config2 or maracluster or zero" > gpurun_out/ga_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ga_tests.log; exit $rc
