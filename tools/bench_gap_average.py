#!/usr/bin/env python3
"""Config 3 (BASELINE.json configs[2]): average_spectrum_clustering gap-average
consensus, one GPU's shard of the 1M-cluster / 8-GPU job (125k clusters of
U{2..50} spectra, ~200 peaks), inputs resident in HBM.  HIP-event timing of
spx_gap_average; run under ``rocprofv3 --kernel-trace --stats`` for the
per-kernel split.  Prints one JSON line.

    python tools/bench_gap_average.py [--clusters 125000] [--reps 10] [--check 200]

Algorithmic bytes per launch (gap-average): 16 B per input peak
(m/z + intensity), 28 B per spectrum (offset, precursor, charge, RT), 8 B per
cluster in, 16 B per output peak + 28 B per cluster out.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_PEAK_GBS = 8000.0


def gap_bytes(batch, kept):
    return 16 * batch.n_peaks + 28 * batch.n_spectra + 8 * batch.n_clusters + 16 * kept + 28 * batch.n_clusters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=125_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--check", type=int, default=0, help="compare the first N clusters with the numpy oracle")
    ap.add_argument("--cpu-sample", type=int, default=20000, help="clusters timed on 1 host core (0: skip)")
    args = ap.parse_args()
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(args.clusters, seed=args.seed)
    batch = engine.DeviceBatch.from_device(t)
    ga = engine.gap_average(batch)
    torch.cuda.synchronize()
    st = ga.status.cpu().numpy()
    kept = int(ga.count.sum().item())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(2):
        engine.gap_average(batch, out=ga)
    ev[0].record()
    for _ in range(args.reps):
        engine.gap_average(batch, out=ga)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / args.reps
    gbs = gap_bytes(batch, kept) / (ms * 1e-3) / 1e9
    out = {"workload": "configs[2] per-GPU shard: average_spectrum gap-average, U{2..50} spectra, ~200 peaks",
           "clusters": int(batch.n_clusters), "spectra": int(batch.n_spectra), "peaks": int(batch.n_peaks),
           "statuses": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
           "gap_average_ms": round(ms, 4), "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1),
           "algorithmic_bytes": gap_bytes(batch, kept), "achieved_GBs": round(gbs, 1),
           "frac_of_8TBs": round(gbs / HBM_PEAK_GBS, 4)}
    if args.check:
        from oracle import np_oracle
        from specpride_amd.csr import SpectraCSR

        csr = SpectraCSR.from_device(t)
        sub = csr.select(np.arange(min(args.check, batch.n_clusters)))
        want = np_oracle.gap_average(sub)
        got = engine.gap_average(engine.DeviceBatch.from_host(sub)).to_host()
        out.update(check_clusters=int(sub.n_clusters),
                   check_status=bool(np.array_equal(got["status"], want["status"])),
                   check_counts=bool(np.array_equal(got["out_off"], want["out_off"])))
    if args.cpu_sample > 0:
        # the reference's CPU path (argsort + cumsum groups per cluster), restated in
        # numpy (oracle/np_oracle.py), on 1 host core over a sample of the same law
        import time

        from oracle import np_oracle
        from specpride_amd.synthetic import make_clusters_np

        sample = make_clusters_np(args.cpu_sample, seed=args.seed + 7)
        t0 = time.perf_counter()
        np_oracle.gap_average(sample)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(args.cpu_sample / dt, 1), "unit": "clusters/s", "cores": 1,
                               "kind": "port", "sample": f"{args.cpu_sample} synthetic clusters, numpy "
                               f"average_spectrum restatement, {dt:.2f} s"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
