set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python tools/profile_kernels.py --clusters 100000 --reps 10 > gpurun_out/pk100k.json 2>&1 && cat gpurun_out/pk100k.json &&
timeout -k 10 120 python tools/profile_kernels.py --clusters 125000 --seed 2 --which ga --reps 10 > gpurun_out/pk125k.json 2>&1 && cat gpurun_out/pk125k.json &&
CLUSTERS=100000 bash tools/gpu/pmc.sh
