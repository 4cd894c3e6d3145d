#!/usr/bin/env python3
"""Off-shape A/B driver (profiling aid): bin-mean (and with --medoid the medoid) on the
bench.bin_mean_shapes batches, HIP-event time per call and an order-sensitive digest
of every result array, one JSON line.  Run once per variant library (SPX_LIB=...)."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402

SHAPES = {"skewed_config3": dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000),
          "long_spectra_600": dict(n_clusters=20000, seed=6, n_template=600)}


def digest(*arrays):
    h = hashlib.sha1()
    for a in arrays:
        h.update(np.ascontiguousarray(a.detach().cpu().numpy() if hasattr(a, "detach") else a).tobytes())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--medoid", action="store_true")
    ap.add_argument("--gap", action="store_true")
    ap.add_argument("--shapes", default="skewed_config3,long_spectra_600")
    a = ap.parse_args()
    res = {}
    for name in a.shapes.split(","):
        t = make_clusters_torch(**SHAPES[name])
        batch = engine.DeviceBatch.from_device(t)
        bm = engine.bin_mean(batch)
        torch.cuda.synchronize()
        C = batch.n_clusters
        ms = bench.time_launches(lambda: engine.bin_mean(batch, out=bm), a.reps, torch.cuda.current_stream())
        res[f"bm_{name}_ms"] = round(ms, 4)
        r = bm.to_host()  # compacted: the capacity layout's unused tail is not a result
        res[f"bm_{name}_digest"] = digest(*(r[k] for k in ("status", "out_off", "out_mz", "out_int", "prec", "charge")))
        del bm
        if a.medoid:
            md = engine.medoid(batch, check=True)
            torch.cuda.synchronize()
            ms = bench.time_launches(lambda: engine.medoid(batch, out=md, check=False), a.reps,
                                     torch.cuda.current_stream())
            res[f"md_{name}_ms"] = round(ms, 4)
            res[f"md_{name}_digest"] = digest(md.rep[:C])
            del md
        if a.gap:
            ga = engine.gap_average(batch)
            torch.cuda.synchronize()
            ms = bench.time_launches(lambda: engine.gap_average(batch, out=ga), a.reps, torch.cuda.current_stream())
            res[f"ga_{name}_ms"] = round(ms, 4)
            r = ga.to_host()
            res[f"ga_{name}_ok"] = int((r["status"] == 0).sum())
            res[f"ga_{name}_frac"] = round(bench.consensus_bytes(batch, int(r["out_off"][-1])) / (ms * 1e-3) / 8e12, 4)
            del ga
        del batch, t
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
