#!/usr/bin/env python3
"""Stage times of the binning CLI's native path (binning._main_mgf) on a tier-3
file (profiling aid): parse -> CSR, H2D, kernels, readback, MGF write.

    python tools/tier3_stages.py [--clusters 100000] [--tmpdir DIR]"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=100000)
    ap.add_argument("--tmpdir", default=None)
    ap.add_argument("--seed", type=int, default=6)
    a = ap.parse_args()
    import numpy as np
    import torch

    from specpride_amd import binning, engine, mgf_native
    from specpride_amd.synthetic import make_clusters_torch

    def write_mgf(path, n_clusters, seed):
        t = make_clusters_torch(n_clusters, seed=seed)
        h = {k: engine.to_host_array(t[k]) for k in ("cluster_off", "spec_off", "mz", "inten", "prec_mz", "charge",
                                                      "rt")}
        del t
        torch.cuda.empty_cache()
        owner = np.repeat(np.arange(n_clusters), np.diff(h["cluster_off"]))
        titles = [f"cluster-{c};mzspec:PXDSYN:synthetic:scan:{s}" for s, c in enumerate(owner.tolist())]
        mgf_native.write_records(path, mgf_native.STYLE_MEDOID, titles, h["spec_off"], h["mz"], h["inten"],
                                 h["prec_mz"], h["charge"], h["rt"])

    res = {}
    with tempfile.TemporaryDirectory(dir=a.tmpdir) as td:
        src, dst = os.path.join(td, "in.mgf"), os.path.join(td, "out.mgf")
        write_mgf(src, a.clusters, a.seed)
        res["mgf_GB"] = round(os.path.getsize(src) / 1e9, 2)
        rsc = binning.RepresentativeSpectrumCreator()
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ids, csr = binning._flat_clusters(src)
            t1 = time.perf_counter()
            batch = engine.DeviceBatch.from_host(csr, rsc.device)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            r = engine.bin_mean(batch)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            h = r.to_host()
            t4 = time.perf_counter()
            mgf_native.write_records(dst, mgf_native.STYLE_BINNING, ids, h["out_off"], h["out_mz"], h["out_int"],
                                     h["prec"], h["charge"])
            t5 = time.perf_counter()
            res[f"run{rep}"] = {"parse_s": round(t1 - t0, 3), "h2d_s": round(t2 - t1, 3), "kernel_s": round(t3 - t2, 3),
                                "readback_s": round(t4 - t3, 3), "write_s": round(t5 - t4, 3),
                                "total_s": round(t5 - t0, 3)}
            del batch, r, h, csr
            print(json.dumps(res[f"run{rep}"]), file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        binning.main(["--mgf_file", src, "--out", dst])
        res["cli_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
