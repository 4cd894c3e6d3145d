"""Run one bin-mean shape of bench.bin_mean_shapes a few times (profiling driver):
python tools/run_shape.py skewed_config3|long_spectra_600 [reps]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402

SHAPES = {"skewed_config3": dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000),
          "long_spectra_600": dict(n_clusters=20000, seed=6, n_template=600)}
t = make_clusters_torch(**SHAPES[sys.argv[1]])
batch = engine.DeviceBatch.from_device(t)
bm = engine.bin_mean(batch)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    engine.bin_mean(batch, out=bm)
torch.cuda.synchronize()
print("ok", int((bm.status[:batch.n_clusters] != 0).sum().item()))
