"""Run the FETCH_SIZE calibration kernels on a 2 GiB buffer (> Infinity Cache),
3 launches per width.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC."""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libcalib.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "calib.hip")], check=True)
L = ctypes.CDLL(SO)
L.calib_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
nbytes = 2 << 30
a = torch.rand(nbytes // 8, dtype=torch.float64, device="cuda")
out = torch.zeros(1, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for width in (8, 16):
    for _ in range(3):
        assert L.calib_read(a.data_ptr(), nbytes, width, out.data_ptr(), st) == 0
torch.cuda.synchronize()
print("calibration bytes per launch:", nbytes, file=sys.stderr)
