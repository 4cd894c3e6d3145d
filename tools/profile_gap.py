"""Phase ablation timing of spx_gap_average on the config-3 shard (profiling aid).
SPX_ABLATE: 1 stop after extrema, 2 after bitmap+prefix, 4 after slot count/min/max,
8 after gap detection, 16 after group sums, 32 skip the precursor summary."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


b = engine.DeviceBatch.from_device(make_clusters_torch(125_000, seed=3, device="cuda"))
ga = engine.gap_average(b)
res = {}
for mask in (0, 1, 2, 4, 8, 16, 32, 1 | 32):
    os.environ["SPX_ABLATE"] = str(mask)
    res[f"gap_ablate{mask}_ms"] = timed(lambda: engine.gap_average(b, out=ga))
os.environ["SPX_ABLATE"] = "0"
print(json.dumps(res))
