"""Phase ablation timing of the two headline kernels (profiling aid, not a test).

Times spx_bin_mean and spx_medoid on the bench batch with SPX_ABLATE masks that
skip phases, so the cost of each phase is the difference.  Prints JSON.
bin-mean v5 (stream, default): 16 = no table updates, 2 = skip the drains (v3), 32 = no output stores;
v0: 1 = skip phase 3, 2 = skip phase 4.
medoid (small kernel): 16 = skip rows on, 64 = skip pairs, 32 = skip totals."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 100_000
    b = engine.DeviceBatch.from_device(make_clusters_torch(n, seed=0, device="cuda"))
    bm = engine.bin_mean(b)
    md = engine.medoid(b)
    res = {}
    torch.cuda.synchronize()
    # first int32 of each workspace = clusters deferred to the generic/large path
    res["bin_mean_deferred"] = int(b._ws["bin_mean"][:4].view(torch.int32).item())
    res["medoid_deferred"] = int(b._ws["medoid"][:4].view(torch.int32).item())
    for var in os.environ.get("SPX_VARIANTS", "6,5,0").split(","):
        os.environ["SPX_BIN_KERNEL"] = var
        masks = {"0": (0, 1, 2), "1": (0, 1, 2), "2": (0, 1, 2), "8": (0, 1, 2), "7": (0,), "9": (0,)}.get(
            var, (0, 2, 16, 32))
        for mask in masks:
            os.environ["SPX_ABLATE"] = str(mask)
            res[f"bin_mean_v{var}_ablate{mask}_ms"] = timed(lambda: engine.bin_mean(b, out=bm))
        os.environ["SPX_ABLATE"] = "0"
        torch.cuda.synchronize()
        b._ws["bin_mean"][:4].zero_()
        engine.bin_mean(b, out=bm)
        torch.cuda.synchronize()
        res[f"bin_mean_v{var}_deferred"] = int(b._ws["bin_mean"][:4].view(torch.int32).item())
    os.environ.pop("SPX_BIN_KERNEL", None)
    for mask in (0, 16, 64, 32, 1024, 4096):
        os.environ["SPX_ABLATE"] = str(mask)
        res[f"medoid_ablate{mask}_ms"] = timed(lambda: engine.medoid(b, out=md))
    os.environ["SPX_ABLATE"] = "0"
    print(json.dumps(res))




def plain(n=100_000, reps=3):
    """Just the two headline calls, for counter collection."""
    b = engine.DeviceBatch.from_device(make_clusters_torch(n, seed=0, device="cuda"))
    bm = engine.bin_mean(b)
    md = engine.medoid(b)
    for _ in range(reps):
        engine.bin_mean(b, out=bm)
        engine.medoid(b, out=md)
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "plain":
        plain()
    else:
        main()
