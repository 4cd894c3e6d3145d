#!/usr/bin/env python3
"""Per-call latency of the single-cluster shim APIs: a caller
that loops like the reference -- one combine_bin_mean per cluster (binning.py:291),
one average_spectrum per cluster (average_spectrum_clustering.py:158-165), one
distance per pair (most_similar_representative.py:91-93) -- pays one device round
trip per call.  Prints one JSON line of microseconds per call (median of the
timed calls, after warm-up).  GPU box only.

    python tools/bench_shim_calls.py [--calls 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from specpride_amd import average_spectrum_clustering as asc  # noqa: E402
from specpride_amd import most_similar_representative as msr  # noqa: E402
from specpride_amd.binning import RepresentativeSpectrumCreator  # noqa: E402
from specpride_amd.synthetic import make_clusters_np  # noqa: E402


def per_call(fn, args, warm=10):
    for a in args[:warm]:
        fn(*a)
    ts = []
    for a in args:
        t0 = time.perf_counter()
        fn(*a)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    csr = make_clusters_np(a.calls, seed=7)
    clusters = []
    for c in range(csr.n_clusters):
        spectra = []
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            lo, hi = csr.spec_off[s], csr.spec_off[s + 1]
            spectra.append({"m/z array": csr.mz[lo:hi], "intensity array": csr.inten[lo:hi],
                            "precursor mz": float(csr.prec_mz[s]), "precursor charge": int(csr.charge[s]),
                            "params": {"pepmass": (float(csr.prec_mz[s]), None), "charge": [int(csr.charge[s])],
                                       "rtinseconds": float(csr.rt[s])}})
        clusters.append(spectra)
    rsc = RepresentativeSpectrumCreator()
    res = {
        "combine_bin_mean_us": per_call(rsc.combine_bin_mean, [(cl,) for cl in clusters]),
        "average_spectrum_us": per_call(asc.average_spectrum, [(cl,) for cl in clusters]),
        "distance_us": per_call(msr.distance, [(cl[0], cl[1]) for cl in clusters]),
        "mean_spectra_per_cluster": float(np.mean(np.diff(csr.cluster_off))),
        "calls": a.calls,
    }
    # stage breakdown of one distance call (median over the calls)
    import torch

    from specpride_amd import engine
    from specpride_amd.csr import SpectraCSR
    st = {"pack": [], "from_host": [], "launch": [], "d2h": []}
    for cl in clusters:
        t0 = time.perf_counter()
        m1, m2 = cl[0]["m/z array"], cl[1]["m/z array"]
        csr = SpectraCSR.from_clusters([[{"m/z array": m1, "intensity array": np.zeros_like(m1)},
                                         {"m/z array": m2, "intensity array": np.zeros_like(m2)}]])
        t1 = time.perf_counter()
        b = engine.DeviceBatch.from_host(csr)
        t2 = time.perf_counter()
        d = engine.xcorr_distance(b, msr._pair01(b.device), 0.1)
        t3 = time.perf_counter()
        float(d.cpu().numpy()[0])
        t4 = time.perf_counter()
        for k, v in zip(st, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            st[k].append(v)
    res["distance_stages_us"] = {k: float(np.median(v) * 1e6) for k, v in st.items()}
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.current_stream().synchronize()
    res["empty_sync_us"] = (time.perf_counter() - t0) * 1e4
    print(json.dumps(res))


if __name__ == "__main__":
    main()
