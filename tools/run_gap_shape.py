import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, numpy as np
from specpride_amd import engine
from specpride_amd.synthetic import make_clusters_torch
SH = {"skewed_config3": dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000),
      "long_spectra_600": dict(n_clusters=20000, seed=6, n_template=600)}
t = make_clusters_torch(**SH[sys.argv[1]]); b = engine.DeviceBatch.from_device(t)
g = engine.gap_average(b)
for _ in range(2): engine.gap_average(b, out=g)
torch.cuda.synchronize(); print("ok")
