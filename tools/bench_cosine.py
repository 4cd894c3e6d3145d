#!/usr/bin/env python3
"""Binned-cosine evaluation (benchmark.py:10-38) on the
configs[1] batch: every cluster's bin-mean consensus scored against its members
with spx_binned_cosine, inputs resident in HBM, HIP-event timing.  Prints one
JSON line.  Algorithmic bytes: 16 B per member peak + 16 B per representative
peak + 8 B per spectrum (cosine out) + 20 B per cluster."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    b = engine.DeviceBatch.from_device(make_clusters_torch(args.clusters, seed=0))
    bm = engine.bin_mean(b)
    rep_off, rep_mz, rep_int = bm.compact()
    res = engine.binned_cosine(b, rep_off, rep_mz, rep_int)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.reps):
        engine.binned_cosine(b, rep_off, rep_mz, rep_int, out=res)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / args.reps
    nbytes = 16 * b.n_peaks + 16 * rep_mz.numel() + 8 * b.n_spectra + 20 * b.n_clusters
    st = res.status[:b.n_clusters]
    print(json.dumps({"workload": "configs[1] batch: cos_dist(bin-mean consensus, member) for every member",
                      "clusters": b.n_clusters, "member_peaks": b.n_peaks, "rep_peaks": int(rep_mz.numel()),
                      "binned_cosine_ms": round(ms, 4), "clusters_per_s": round(b.n_clusters / (ms * 1e-3), 1),
                      "algorithmic_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
                      "status_ok": int((st == 0).sum().item()),
                      "mean_avg_cos": round(float(res.avg[:b.n_clusters].mean().item()), 4)}), flush=True)


if __name__ == "__main__":
    main()
