#!/usr/bin/env python3
"""Time the REFERENCE's own binning.py CLI (binning.py:250-302) end to end on a
synthetic clustered MGF of the tier-3 shape (tools/bench_tiers.py), single
threaded, in the build container.  The reference is imported from
/root/reference/src with the import stand-ins of tests/golden/stubs (its MGF
path needs none of them); it never reaches the GPU box.  Prints one JSON line.

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
        print(json.dumps({"reference_cli": "binning.py --mgf_file (the reference's own code)",
                          "clusters": int(small.n_clusters), "peaks": int(small.n_peaks),
                          "mgf_MB": round(os.path.getsize(mgf_in) / 1e6, 1), "cli_s": round(t1 - t0, 2),
                          "clusters_per_s": round(small.n_clusters / (t1 - t0), 2), "cores": 1,
                          "host": f"{platform.processor() or platform.machine()}, {os.cpu_count()} vCPUs "
                                  "(build container, not the GPU box)"}), flush=True)


if __name__ == "__main__":
    main()
