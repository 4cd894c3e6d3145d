#!/usr/bin/env python3
"""The two host-inclusive measurement tiers of SURVEY.md §8(d) (never `value`):

* tier 2 -- a packed host CSR (configs[1] law) -> H2D -> spx_bin_mean + spx_medoid
  -> compaction + D2H of the consensus peaks and representatives; and the same
  for each method alone (bin-mean, gap-average, medoid);
* tier 3 -- each CLI end to end on one synthetic clustered MGF of configs[1]'s size
  (100k clusters, ~2.6M spectra, ~9 GB of text): binning.py
  (binning.py:250-302), average_spectrum_clustering.py --encodedclusters
  (:168-210) and most_similar_representative.py (:22-115): MGF text in (native
  parser straight to the CSR) -> device -> MGF text out.

Prints one JSON line.  The reference's own CLI is timed on the same file shape by
tools/time_reference_cli.py in the build container (the reference never reaches the
GPU box); DESIGN.md §6 sets the two side by side.

    python tools/bench_tiers.py [--t2-clusters 20000] [--t3-clusters 100000] [--tmpdir DIR] [--skip-t2]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t2-clusters", type=int, default=20000)
    ap.add_argument("--t3-clusters", type=int, default=100000, help="configs[1] size")
    ap.add_argument("--tmpdir", default=None, help="where the tier-3 MGF files go")
    ap.add_argument("--skip-t2", action="store_true")
    ap.add_argument("--seed", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from specpride_amd import binning, engine
    from specpride_amd.synthetic import make_clusters_np

    out = {}
    # ---------------------------------------------------------------- tier 2
    if not args.skip_t2:
        csr = make_clusters_np(args.t2_clusters, seed=args.seed)
        for rep in range(2):  # the first pass warms the allocator and the code object
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b = engine.DeviceBatch.from_host(csr)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            bm = engine.bin_mean(b)
            md = engine.medoid(b)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            r = bm.to_host()
            rep_idx, _ = md.to_host()
            t3 = time.perf_counter()
        out["tier2"] = {"clusters": int(csr.n_clusters), "peaks": int(csr.n_peaks),
                        "h2d_s": round(t1 - t0, 4), "kernels_s": round(t2 - t1, 4), "d2h_s": round(t3 - t2, 4),
                        "clusters_per_s": round(csr.n_clusters / (t3 - t0), 1),
                        "h2d_GBs": round(16.0 * csr.n_peaks / (t1 - t0) / 1e9, 1),
                        "kept_peaks": int(r["out_off"][-1]), "reps_ok": bool((rep_idx >= 0).all())}
        per = {}
        for name, fn in (("bin_mean", lambda b: engine.bin_mean(b).to_host()),
                         ("gap_average", lambda b: engine.gap_average(b).to_host()),
                         ("medoid", lambda b: engine.medoid(b).to_host())):
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn(engine.DeviceBatch.from_host(csr))
                t1 = time.perf_counter()
            per[name] = {"s": round(t1 - t0, 4), "clusters_per_s": round(csr.n_clusters / (t1 - t0), 1)}
        out["tier2_per_method"] = per
    # ---------------------------------------------------------------- tier 3
    from specpride_amd import average_spectrum_clustering as asc
    from specpride_amd import most_similar_representative as msr
    from specpride_amd.synthetic import write_clustered_mgf as write_mgf

    clis = {"binning": lambda i, o: binning.main(["--mgf_file", i, "--out", o]),
            "average_spectrum_clustering": lambda i, o: asc.main([i, o, "--encodedclusters"]),
            "most_similar_representative": lambda i, o: msr.main(["-i", i, "-o", o])}
    with tempfile.TemporaryDirectory(dir=args.tmpdir) as td:
        warm_in, mgf_in, mgf_out = os.path.join(td, "w.mgf"), os.path.join(td, "in.mgf"), os.path.join(td, "out.mgf")
        write_mgf(warm_in, 200, args.seed + 2)
        t0 = time.perf_counter()
        S, P = write_mgf(mgf_in, args.t3_clusters, args.seed + 1)
        tw = time.perf_counter() - t0
        size = os.path.getsize(mgf_in)
        t3 = {"clusters": args.t3_clusters, "spectra": S, "peaks": P, "mgf_GB": round(size / 1e9, 2),
              "input_write_s": round(tw, 2)}
        for name, cli in clis.items():
            with contextlib.redirect_stdout(io.StringIO()):
                cli(warm_in, mgf_out)  # code objects, allocator, staging pool
                t0 = time.perf_counter()
                cli(mgf_in, mgf_out)
                t1 = time.perf_counter()
            t3[name] = {"cli_s": round(t1 - t0, 3), "clusters_per_s": round(args.t3_clusters / (t1 - t0), 1),
                        "input_GBs": round(size / (t1 - t0) / 1e9, 2),
                        "out_MB": round(os.path.getsize(mgf_out) / 1e6, 1)}
            print(json.dumps({name: t3[name]}), file=sys.stderr, flush=True)
        out["tier3"] = t3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
