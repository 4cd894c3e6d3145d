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

mzML + MaRaCluster input path:

* ``.read_cluster_list(file)`` (binning.py:35-52): a cluster ends at each blank
  line (a trailing cluster with no blank line after it is dropped, as there);
  column 2 of each line is the scan number (kept as a string).
* ``.read_spectra(mzml_file, scan_list)`` (binning.py:57-119): MS2 peaklists
  by Thermo scan id from a plain or ``.gz`` mzML (``specpride_amd.mzml``, a
  pyteomics stand-in), same INFO/ERROR prints.
* CLI ``--mara_file`` / ``--mzml_file`` / ``--cluster``: the options the
  reference keeps commented out (binning.py:253-255, 281-282), run over every
  cluster (or one) in a single GPU pass; titles are the cluster numbers.

Added: ``.combine_bin_mean_batch(clusters, ...)`` -- all clusters in one GPU
pass (the CLI uses it).  There is no CPU fallback: without the HIP engine the
numeric calls raise.
"""
from __future__ import annotations

import argparse
import sys
import timeit

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

    # ----------------------------------------------------- mzML + MaRaCluster
    def read_cluster_list(self, file):
        """MaRaCluster TSV -> list of clusters, each a list of scan strings (binning.py:35-52)."""
        clusters, cluster = [], []
        with open(file) as infile:
            for line in infile:
                columns = line.rstrip().split()
                if len(columns) == 0:
                    clusters.append(cluster)
                    cluster = []
                    continue
                cluster.append(columns[1])
        return clusters

    def read_spectra(self, mzml_file, scan_list, reader=None):
        """MS2 peaklists for ``scan_list`` from an mzML file (binning.py:57-119)."""
        from . import mzml

        t0 = timeit.default_timer()
        n_spectra = 0
        if self.verbose >= 1:
            eprint(f"INFO: Reading {len(scan_list)} scans from mzML file {mzml_file}")
        spectra = []
        ids = [f"controllerType=0 controllerNumber=1 scan={scan}" for scan in scan_list]
        rd = reader if reader is not None else mzml.read(mzml_file, ids=ids)
        for scan in scan_list:
            spectrum = rd.get_by_id(f"controllerType=0 controllerNumber=1 scan={scan}")
            if spectrum["ms level"] == 2 and "m/z array" in spectrum:
                ion = spectrum["precursorList"]["precursor"][0]["selectedIonList"]["selectedIon"][0]
                precursor_mz, precursor_charge = ion["selected ion m/z"], ion["charge state"]
                print(f"INFO: Reading {scan}. Precursor m/z = {precursor_mz}. n peaks={len(spectrum['m/z array'])}")
                spectra.append({"m/z array": spectrum["m/z array"], "intensity array": spectrum["intensity array"],
                                "precursor mz": precursor_mz, "precursor charge": precursor_charge})
            else:
                print(f"ERROR: scan {scan} is not ms_level=2! Skipping")
            n_spectra += 1
        if self.verbose >= 1:
            eprint("")
        t1 = timeit.default_timer()
        print(f"INFO: Read {n_spectra} spectra from {mzml_file}")
        print(f"INFO: Elapsed time: {t1 - t0}")
        print(f"INFO: Processed {n_spectra / max(t1 - t0, 1e-12)} spectra per second")
        return spectra

    def read_spectra_clusters(self, mzml_file, clusters):
        """read_spectra for several scan lists with ONE parse of the mzML file."""
        from . import mzml

        ids = [f"controllerType=0 controllerNumber=1 scan={scan}" for scans in clusters for scan in scans]
        rd = mzml.read(mzml_file, ids=ids)  # only the listed scans are kept (and decoded lazily)
        return [self.read_spectra(mzml_file, scans, reader=rd) for scans in clusters]

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
        return self._combine_csr(SpectraCSR.from_clusters(clusters), clusters, minimum, maximum, binsize,
                                 apply_peak_quorum)

    def _combine_host(self, csr, minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True):
        """The device pass over a packed batch: the dense host result of
        :meth:`engine.PeaksResult.to_host`, after raising the reference's error for
        the first failing cluster (AssertionError on mixed charges, binning.py:205-206)."""
        batch = engine.DeviceBatch.from_host(csr, self.device)
        # a batch small enough for the one-copy readback (the per-cluster calls) runs
        # the large-cluster chain only if a cluster needs it (spx_bin_mean_stage)
        res = engine.bin_mean(batch, minimum, maximum, binsize, apply_peak_quorum,
                              staged=engine.packed_readback(batch)).to_host()
        bad = np.flatnonzero(res["status"] != engine.STATUS_OK)
        if len(bad):
            if res["status"][bad[0]] == engine.STATUS_MIXED_CHARGE:
                raise AssertionError(MIXED_CHARGE_MSG)
            # empty cluster: the reference fails on charges[0]
            raise IndexError("list index out of range")
        return res

    def _combine_csr(self, csr, clusters, minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True):
        """The device pass over a packed batch; ``clusters[c]`` (peaklists) or None
        per cluster -- the output's precursor_charge is its first member's charge."""
        res = self._combine_host(csr, minimum, maximum, binsize, apply_peak_quorum)
        out = []
        for c, pl in enumerate(clusters):
            a, b = res["out_off"][c], res["out_off"][c + 1]
            out.append({"minimum": minimum, "maximum": maximum, "binsize": binsize,
                        "intensities": res["out_int"][a:b].copy(), "mzs": res["out_mz"][a:b].copy(),
                        "precursor_mz": np.float64(res["prec"][c]),
                        "precursor_charge": pl[0]["precursor charge"] if pl is not None
                        else int(csr.charge[csr.cluster_off[c]])})
        return out

    # ------------------------------------------------------------ MGF output
    def write_spectrum(self, spectra, mgf_file):
        """Write consensus spectra exactly as binning.py:234-245 does
        (``repr`` floats; NaN intensities skipped)."""
        from . import mgf_native

        mgf_native.write_binning_mgf(spectra, mgf_file)


def _flat_clusters(path):
    """read_spectra_clustered_mgf + packing without per-spectrum Python objects:
    the native parser's flat arrays grouped by cluster natively (first appearance,
    members in file order: binning.py:122-167) -- no copy when the
    clusters are contiguous in the file.  None when the file is outside the native
    subset or a spectrum lacks the fields the reference indexes (the dict path then
    raises exactly as the reference does)."""
    from . import mgf_native
    from .csr import concat_ranges

    try:
        flat = mgf_native.parse_native(path, group=mgf_native.GROUP_BINNING)
    except ValueError:  # includes a TITLE without ';' (the reference's parts[1] raises)
        return None
    if flat is None or len(flat["spec_off"]) < 2 or not (flat["has_prec"].all() and flat["has_charge"].all()):
        return None
    key, ids = flat["key"], flat["group_ids"]
    cluster_off = np.zeros(len(ids) + 1, np.int64)
    np.cumsum(np.bincount(key, minlength=len(ids)), out=cluster_off[1:])
    if np.all(key[1:] >= key[:-1]):  # contiguous clusters: the parse order is the CSR order
        return ids, SpectraCSR(cluster_off, flat["spec_off"], flat["mz"], flat["inten"], flat["prec_mz"],
                               flat["charge"].astype(np.int32), np.full(len(key), np.nan))
    perm = np.argsort(key, kind="stable")
    so = flat["spec_off"]
    lens = (so[1:] - so[:-1])[perm]
    spec_off = np.zeros(len(perm) + 1, np.int64)
    np.cumsum(lens, out=spec_off[1:])
    idx = concat_ranges(so[:-1][perm], lens)
    csr = SpectraCSR(cluster_off, spec_off, flat["mz"][idx], flat["inten"][idx], flat["prec_mz"][perm],
                     flat["charge"][perm].astype(np.int32), np.full(len(perm), np.nan))
    return ids, csr


def main(argv=None):
    """CLI of binning.py:250-302."""
    argparser = argparse.ArgumentParser(description="Creates an index for an MSP spectral library file")
    argparser.add_argument("--verbose", action="count", help="If set, print more information about ongoing processing")
    argparser.add_argument("--version", action="version", version="%(prog)s 0.5")
    argparser.add_argument("--mara_file", action="store", help="Name of the mara clusters file")
    argparser.add_argument("--mzml_file", action="store", help="Name of the mzml file")
    argparser.add_argument("--cluster", action="store", help="Cluster number to combine (default: all)")
    argparser.add_argument("--mgf_file", action="store", help="Name of the clustered MGF file")
    argparser.add_argument("--out", action="store", default="merged_spectra.mgf", help="Name of the output mgf file")
    params = argparser.parse_args(argv)
    verbose = 1 if params.verbose is None else params.verbose
    if not params.mgf_file and params.mara_file and params.mzml_file:
        rsc = RepresentativeSpectrumCreator(verbose=verbose)
        clusters = rsc.read_cluster_list(params.mara_file)
        ids = [int(params.cluster)] if params.cluster is not None else list(range(len(clusters)))
        peaklists = rsc.read_spectra_clusters(params.mzml_file, [clusters[i] for i in ids])
        merged = rsc.combine_bin_mean_batch(peaklists, minimum=100, maximum=2000, binsize=0.02)
        for cid, spec in zip(ids, merged):
            spec["cluster_id"] = str(cid)
        with open(params.out, "wt") as mgf_file:
            rsc.write_spectrum(merged, mgf_file)
        return
    if not params.mgf_file:
        print("Example: representative_spectrum_creator.py --mgf_file=../data/clustered_mgf.mgf")
        print("Or use --help for additional usage information")
        sys.exit(10)
    from . import sharded_cli

    if sharded_cli.launched_distributed():  # torchrun: rank-local ingest, one GPU per rank
        sharded_cli.run_cli(sharded_cli.binning, lambda: _main_mgf(params.mgf_file, params.out, verbose),
                            params.mgf_file, params.out)
        return
    _main_mgf(params.mgf_file, params.out, verbose)


def _main_mgf(mgf_file, out, verbose):
    """The single-process ``--mgf_file`` CLI body (binning.py:286-302)."""
    from . import mgf_native

    rsc = RepresentativeSpectrumCreator(verbose=verbose)
    print("Reading spectra...")
    flat = _flat_clusters(mgf_file)
    if flat is not None:  # native parse straight to the cluster-segmented CSR, native writer
        ids, csr = flat
        print("Clustering...")
        res = rsc._combine_host(csr, minimum=100, maximum=2000, binsize=0.02)
        mgf_native.write_records(out, mgf_native.STYLE_BINNING, ids, res["out_off"], res["out_mz"], res["out_int"],
                                 res["prec"], res["charge"])
        return
    # the reference's own line loop decides (malformed or unusual input)
    clusters = rsc.read_spectra_clustered_mgf(mgf_file)
    print("Clustering...")
    ids = list(clusters.keys())
    merged = rsc.combine_bin_mean_batch([clusters[k] for k in ids], minimum=100, maximum=2000, binsize=0.02)
    for cid, spec in zip(ids, merged):
        spec["cluster_id"] = cid
    with open(out, "wt") as fh:
        rsc.write_spectrum(merged, fh)


if __name__ == "__main__":
    main()
