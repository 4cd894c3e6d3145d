#!/usr/bin/env python3
"""Time the REFERENCE on the tier-3 file shape (tools/bench_tiers.py), single
threaded, in the build container; it never reaches the GPU box.  Prints one
JSON line.

* binning.py CLI (binning.py:250-302) end to end: the reference's own code
  (its MGF path needs none of the import stand-ins in tests/golden/stubs).
* average_spectrum_clustering.py: its I/O is pyteomics IndexedMGF/mgf.write,
  absent offline, so only its COMPUTE is timed -- the reference's own
  get_pepmass/get_rt/average_spectrum per consecutive-title cluster
  (:151-165, default helpers lower_median_mass + lower_median_mass_rt), on
  spectra read beforehand by specpride_amd.mgf.iter_mgf (untimed).
* most_similar_representative.py: its scorer is OpenMS C++ (absent); a Python
  stand-in would not time OpenMS, so no reference figure -- bench.py's
  cpu_baseline times the C restatement (oracle/spx_oracle.c) instead.

    python tools/time_reference_cli.py [--clusters 2000]
"""
import argparse
import contextlib
import io
import json
import os
import platform
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_SRC = "/root/reference/src"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=5)
    args = ap.parse_args()
    if not os.path.isdir(REF_SRC):
        raise SystemExit("the reference is only present in the build container")
    sys.path.insert(0, REPO)
    from specpride_amd.mgf import write_csr_mgf
    from specpride_amd.synthetic import make_clusters_np

    small = make_clusters_np(args.clusters, seed=args.seed + 1)  # tier 3's file
    sys.path.insert(0, os.path.join(REPO, "tests", "golden", "stubs"))
    sys.path.insert(0, REF_SRC)
    import binning  # the reference's module

    with tempfile.TemporaryDirectory() as td:
        mgf_in, mgf_out = os.path.join(td, "in.mgf"), os.path.join(td, "out.mgf")
        write_csr_mgf(small, mgf_in)
        argv = sys.argv
        sys.argv = ["binning.py", "--mgf_file", mgf_in, "--out", mgf_out]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                t0 = time.perf_counter()
                binning.main()
                t1 = time.perf_counter()
        finally:
            sys.argv = argv
        res = {"reference_cli": "binning.py --mgf_file (the reference's own code)",
               "clusters": int(small.n_clusters), "peaks": int(small.n_peaks),
               "mgf_MB": round(os.path.getsize(mgf_in) / 1e6, 1), "cli_s": round(t1 - t0, 2),
               "clusters_per_s": round(small.n_clusters / (t1 - t0), 2), "cores": 1,
               "host": f"{platform.processor() or platform.machine()}, {os.cpu_count()} vCPUs "
                       "(build container, not the GPU box)"}
        from itertools import groupby

        import average_spectrum_clustering as asc  # the reference's module
        from specpride_amd.mgf import read_mgf

        spectra = read_mgf(mgf_in)
        with contextlib.redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            n = 0
            for cid, grp in groupby(spectra, lambda s: asc.get_cluster_id(s["params"]["title"])):
                grp = list(grp)
                mz, c = asc.lower_median_mass(grp)
                rt = asc.lower_median_mass_rt(grp)
                asc.average_spectrum(grp, cid, pepmass=mz, charge=c, rtinseconds=rt)
                n += 1
            t1 = time.perf_counter()
        res["reference_gap_average_compute"] = {
            "what": "average_spectrum_clustering.py :151-165 compute only (pyteomics I/O absent)",
            "clusters": n, "s": round(t1 - t0, 2), "clusters_per_s": round(n / (t1 - t0), 2), "cores": 1}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
