#!/usr/bin/env python3
"""Binned-cosine evaluation (benchmark.py:10-38) on the
configs[1] batch: every cluster's bin-mean consensus scored against its members
with spx_binned_cosine, inputs resident in HBM, HIP-event timing.  Prints one
JSON line.  Algorithmic bytes: 16 B per member peak + 16 B per representative
peak + 8 B per spectrum (cosine out) + 20 B per cluster."""
import argparse
import json

import numpy as np
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=40, help="clusters timed on 1 host core (0: skip)")
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
    out = {"workload": "configs[1] batch: cos_dist(bin-mean consensus, member) for every member",
           "clusters": b.n_clusters, "member_peaks": b.n_peaks, "rep_peaks": int(rep_mz.numel()),
           "binned_cosine_ms": round(ms, 4), "clusters_per_s": round(b.n_clusters / (ms * 1e-3), 1),
           "algorithmic_GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
           "status_ok": int((st == 0).sum().item()),
           "mean_avg_cos": round(float(res.avg[:b.n_clusters].mean().item()), 4)}
    import hashlib  # order-sensitive digest of the results (A/B builds must agree)

    out["digest"] = hashlib.sha1(res.cos[:b.n_spectra].cpu().numpy().tobytes() +
                                 res.avg[:b.n_clusters].cpu().numpy().tobytes()).hexdigest()[:16]
    if args.cpu_sample > 0:
        # the reference's CPU path (dense sum-binning on ~400k edges per pair, benchmark.py:10-38),
        # restated in numpy (oracle/np_oracle.py), on 1 host core: the first clusters of the batch
        import time

        from oracle import np_oracle
        from specpride_amd.csr import SpectraCSR

        n = min(args.cpu_sample, b.n_clusters)
        co = b.t["cluster_off"][:n + 1].cpu().numpy()
        so = b.t["spec_off"][:co[-1] + 1].cpu().numpy()
        h = lambda k, m: b.t[k][:m].cpu().numpy()  # noqa: E731
        sub = SpectraCSR(co, so, h("mz", so[-1]), h("inten", so[-1]), h("prec_mz", co[-1]), h("charge", co[-1]),
                         h("rt", co[-1]))
        ro = rep_off[:n + 1].cpu().numpy()
        t0 = time.perf_counter()
        want = np_oracle.binned_cosine(sub, ro, rep_mz[:ro[-1]].cpu().numpy(), rep_int[:ro[-1]].cpu().numpy())
        dt = time.perf_counter() - t0
        got = res.avg[:n].cpu().numpy()
        out["cpu_baseline"] = {"value": round(n / dt, 2), "unit": "clusters/s", "cores": 1, "kind": "port",
                               "sample": f"first {n} clusters of the batch ({sub.n_spectra} member pairs), numpy "
                               f"benchmark.py restatement, {dt:.2f} s"}
        out["cpu_check_max_rel"] = float(np.max(np.abs(got - want[1]) / np.maximum(np.abs(want[1]), 1e-300)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
