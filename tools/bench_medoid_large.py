#!/usr/bin/env python3
"""Config 4 (BASELINE.json configs[3]): medoid on skewed cluster sizes -- 20k
clusters with n = min(5000, max(2, floor(2 U^(-1/1.1)))) plus 4 forced n = 5000
clusters -- timed with HIP events; run under ``rocprofv3 --kernel-trace --stats``
for the per-kernel split.  Prints one JSON line.

    python tools/bench_medoid_large.py [--clusters 20000] [--forced 4] [--reps 5] [--check]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=20000)
    ap.add_argument("--forced", type=int, default=4)
    ap.add_argument("--large", type=int, default=5000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--check", action="store_true", help="with totals, and print a digest of reps + totals")
    args = ap.parse_args()
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(args.clusters, seed=args.seed, skewed=True, forced_large=args.forced,
                            large_size=args.large)
    batch = engine.DeviceBatch.from_device(t)
    sizes = np.diff(batch.host_cluster_off)
    md = engine.medoid(batch, with_totals=args.check)
    torch.cuda.synchronize()
    rep = md.rep.cpu().numpy()
    if np.any(rep < 0):
        raise RuntimeError(f"unresolved clusters: {np.unique(rep[rep < 0])}")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.reps):
        engine.medoid(batch, out=md, check=False)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / args.reps
    # algorithmic Gram work of the large (n > 64) clusters: 2 * n(n+1)/2 * K_c with K_c <= peaks
    big = np.flatnonzero(sizes > 64)
    # 2 * n(n+1)/2 * K_c int ops per large cluster, K_c = its distinct
    # ceil(mz / 0.1) bins (the Gram's K); the MFMA kernel's time comes from rocprofv3
    mz = t["mz"].cpu().numpy()
    so = batch.host_spec_off
    gram_ops = 0
    for c in big:
        a, b = so[batch.host_cluster_off[c]], so[batch.host_cluster_off[c + 1]]
        k_c = len(np.unique(np.ceil(mz[a:b] / 0.1)))
        gram_ops += int(sizes[c]) * (int(sizes[c]) + 1) * k_c
    out = {"clusters": int(batch.n_clusters), "spectra": int(batch.n_spectra), "peaks": int(batch.n_peaks),
           "large_clusters": int(len(big)), "max_n": int(sizes.max()),
           "spectra_in_large": int(sizes[big].sum()), "medoid_ms": round(ms, 3),
           "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1), "gram_ops": gram_ops}
    if args.check:  # result digest: variants must agree (oracle parity: tests/test_gpu_configs.py)
        import hashlib

        h = hashlib.sha1(md.rep.cpu().numpy().tobytes())
        h.update(md.totals.cpu().numpy().tobytes())
        out["digest"] = h.hexdigest()[:16]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
