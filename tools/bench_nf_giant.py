#!/usr/bin/env python3
"""A 1M-peak giant cluster with one NaN m/z against its finite twin:
since round 6 both take the tiled giant pipeline of spx_gap_average; before, the NaN one
ran gap_body_nf on one workgroup.  Prints one JSON line: both times (HIP events) and the
ratio; each result is also checked against the C oracle on a 1% sample of its groups
by the GPU tests, not here.

    python tools/bench_nf_giant.py [--spectra 5000] [--reps 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spectra", type=int, default=5000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch

    from specpride_amd import engine
    from specpride_amd.csr import SpectraCSR
    from specpride_amd.synthetic import make_clusters_np

    fin = make_clusters_np(1, seed=5, sizes=np.array([a.spectra]))
    mz = fin.mz.copy()
    mz[len(mz) // 2] = np.nan
    nan = SpectraCSR(fin.cluster_off, fin.spec_off, mz, fin.inten, fin.prec_mz, fin.charge, fin.rt)
    res = {"peaks": int(fin.n_peaks), "spectra": int(fin.n_spectra)}
    st = torch.cuda.current_stream()
    for name, csr in (("finite", fin), ("one_nan_mz", nan)):
        b = engine.DeviceBatch.from_host(csr)
        r = engine.gap_average(b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            engine.gap_average(b, out=r)
        e1.record(st)
        torch.cuda.synchronize()
        h = r.to_host()
        res[name] = {"ms": round(e0.elapsed_time(e1) / a.reps, 4), "status": int(h["status"][0]),
                     "peaks_out": int(h["out_off"][-1])}
    res["ratio"] = round(res["one_nan_mz"]["ms"] / res["finite"]["ms"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
