#!/usr/bin/env python3
"""Drop-in for the reference's ``src/binning.py`` (bin-mean consensus), running
the per-cluster numeric core on MI355X through ``spx_bin_mean``.

Kept from the reference (same names, arguments, return shapes, errors):

* ``RepresentativeSpectrumCreator(verbose=None)`` (binning.py:19-28)
* ``.read_spectra_clustered_mgf(path) -> {cluster_id: [peaklist, ...]}``
  (binning.py:122-167): line-oriented parse, cluster order = first appearance,
  members merged wherever they appear.
* ``.combine_bin_mean(peaklists, minimum=100, maximum=2000, binsize=0.02,
  apply_peak_quorum=True)`` (binning.py:170-231): dict with ``minimum``,
  ``maximum``, ``binsize``, ``intensities``/``mzs`` (float64 arrays),
  ``precursor_mz`` (np.float64), ``precursor_charge``; raises
  ``AssertionError("Not all precursor charges in cluster are equal")``.
* ``.write_spectrum(spectra, fh)`` (binning.py:234-245): byte-identical text.
* ``main()`` CLI (binning.py:250-302): ``--mgf_file``, ``--out``
  (default ``merged_spectra.mgf``), ``--verbose``, ``--version``; exit 10
  without ``--mgf_file``; nothing is written if a cluster fails.

Added: ``.combine_bin_mean_batch(clusters, ...)`` -- all clusters in one GPU
pass (the CLI uses it).  There is no CPU fallback: without the HIP engine the
numeric calls raise.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

from . import engine
from .csr import SpectraCSR


def eprint(*args, **kwargs):
    print(*args, file=sys.stderr, **kwargs)


MIXED_CHARGE_MSG = "Not all precursor charges in cluster are equal"


class RepresentativeSpectrumCreator:
    """Bin-mean consensus creator (binning.py:19)."""

    def __init__(self, verbose=None):
        self.verbose = 0 if verbose is None else verbose
        self.device = "cuda"

    # ------------------------------------------------------------- MGF input
    def read_spectra_clustered_mgf(self, clustered_mgf_file):
        """Read a clustered MGF -> ``{cluster_id: [peaklist, ...]}`` (binning.py:122-167).

        A peaklist starts at each ``TITLE=`` line (``cluster_id;usi``), picks up
        ``PEPMASS=`` (float) and ``CHARGE=`` (int, '+' stripped), appends every
        line starting with a digit as ``mz intensity`` and is stored at
        ``END IONS``.  Uses the native parser when available (identical result)."""
        from . import mgf_native

        spectra = mgf_native.read_binning_mgf(clustered_mgf_file)
        clusters = {}
        for pl in spectra:
            clusters.setdefault(pl["cluster_id"], []).append(pl)
        return clusters

    # ---------------------------------------------------------- numeric core
    def combine_bin_mean(self, peaklists, minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True):
        """Bin-mean consensus of one cluster (binning.py:170-231) on the GPU."""
        return self.combine_bin_mean_batch([peaklists], minimum, maximum, binsize, apply_peak_quorum)[0]

    def combine_bin_mean_batch(self, clusters, minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True):
        """:meth:`combine_bin_mean` for a list of clusters in one device pass.
        Raises the reference's AssertionError for the first failing cluster."""
        clusters = list(clusters)
        for pl in clusters:
            for p in pl:  # the reference indexes these keys (KeyError if absent)
                p["precursor mz"], p["precursor charge"]
        csr = SpectraCSR.from_clusters(clusters)
        res = engine.bin_mean(engine.DeviceBatch.from_host(csr, self.device), minimum, maximum, binsize,
                              apply_peak_quorum).to_host()
        out = []
        for c, pl in enumerate(clusters):
            st = res["status"][c]
            if st == engine.STATUS_MIXED_CHARGE:
                raise AssertionError(MIXED_CHARGE_MSG)
            if st != engine.STATUS_OK:
                # empty cluster: the reference fails on charges[0]
                raise IndexError("list index out of range")
            a, b = res["out_off"][c], res["out_off"][c + 1]
            out.append({"minimum": minimum, "maximum": maximum, "binsize": binsize,
                        "intensities": res["out_int"][a:b].copy(), "mzs": res["out_mz"][a:b].copy(),
                        "precursor_mz": np.float64(res["prec"][c]),
                        "precursor_charge": pl[0]["precursor charge"]})
        return out

    # ------------------------------------------------------------ MGF output
    def write_spectrum(self, spectra, mgf_file):
        """Write consensus spectra exactly as binning.py:234-245 does
        (``repr`` floats; NaN intensities skipped)."""
        from . import mgf_native

        mgf_native.write_binning_mgf(spectra, mgf_file)


def main(argv=None):
    """CLI of binning.py:250-302."""
    argparser = argparse.ArgumentParser(description="Creates an index for an MSP spectral library file")
    argparser.add_argument("--verbose", action="count", help="If set, print more information about ongoing processing")
    argparser.add_argument("--version", action="version", version="%(prog)s 0.5")
    argparser.add_argument("--mgf_file", action="store", help="Name of the clustered MGF file")
    argparser.add_argument("--out", action="store", default="merged_spectra.mgf", help="Name of the output mgf file")
    params = argparser.parse_args(argv)
    verbose = 1 if params.verbose is None else params.verbose
    if not params.mgf_file:
        print("Example: representative_spectrum_creator.py --mgf_file=../data/clustered_mgf.mgf")
        print("Or use --help for additional usage information")
        sys.exit(10)
    rsc = RepresentativeSpectrumCreator(verbose=verbose)
    print("Reading spectra...")
    clusters = rsc.read_spectra_clustered_mgf(params.mgf_file)
    print("Clustering...")
    ids = list(clusters.keys())
    merged = rsc.combine_bin_mean_batch([clusters[k] for k in ids], minimum=100, maximum=2000, binsize=0.02)
    for cid, spec in zip(ids, merged):
        spec["cluster_id"] = cid
    with open(params.out, "wt") as mgf_file:
        rsc.write_spectrum(merged, mgf_file)


if __name__ == "__main__":
    main()
