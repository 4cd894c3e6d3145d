"""Run one off-shape batch of bench.bin_mean_shapes / bench.medoid_shapes a few
times (profiling driver): python tools/run_shape.py skewed_config3|long_spectra_600
[reps] [bm|md|ga]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402

SHAPES = {"skewed_config3": dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000),
          "long_spectra_600": dict(n_clusters=20000, seed=6, n_template=600)}
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
which = sys.argv[3] if len(sys.argv) > 3 else "bm"
t = make_clusters_torch(**SHAPES[sys.argv[1]])
batch = engine.DeviceBatch.from_device(t)
if which == "md":
    md = engine.medoid(batch, check=True)
    for _ in range(reps):
        engine.medoid(batch, out=md, check=False)
    torch.cuda.synchronize()
    print("ok", int((md.rep[:batch.n_clusters] < 0).sum().item()))
elif which == "ga":
    ga = engine.gap_average(batch)
    for _ in range(reps):
        engine.gap_average(batch, out=ga)
    torch.cuda.synchronize()
    print("ok", int((ga.status[:batch.n_clusters] != 0).sum().item()))
else:
    bm = engine.bin_mean(batch)
    for _ in range(reps):
        engine.bin_mean(batch, out=bm)
    torch.cuda.synchronize()
    print("ok", int((bm.status[:batch.n_clusters] != 0).sum().item()))
