#!/usr/bin/env python3
"""Drop-in for the reference's ``src/most_similar_representative.py`` (medoid
representative), running the all-pairs xcorr + summed-distance argmin on
MI355X through ``spx_medoid``.

Kept from the reference:

* ``distance(spec1, spec2, method='xcorr')`` (:13-19): ``1 - xcorr`` with
  OpenMS ``XQuestScores::xCorrelationPrescore(spec1, spec2, 0.1)`` semantics
  (restated); any other ``method`` returns 0.  Spectra may be
  pyteomics/binning-style dicts, ``(mz, intensity)`` tuples or bare m/z arrays.
* ``main(argv)`` (:22-115): ``-i <input> -o <output>`` (``-h`` usage, exit 2 on a
  bad option); cluster names in first-appearance order; each cluster is the
  FIRST contiguous run at or after the previous cluster's run (the reference's
  ``range_start`` scan, :64-75 -- later runs of a split cluster are ignored,
  SURVEY.md A.4); singletons pass through; the representative is the lowest
  index among the minima of ``(rowsum + colsum)/n`` of the upper-triangular
  distance matrix (pairwise-summation order, :98-110).  Prints the cluster
  name and size per cluster and the final count, as the reference does.
  Output: the chosen spectra, written back verbatim as MGF (OpenMS
  ``MascotGenericFile.store`` formatting is not reproduced: parity is on the
  chosen spectrum and its title).

All clusters of a file are scored in ONE device pass.
"""
from __future__ import annotations

import getopt
import sys

import numpy as np

from . import engine
from .csr import SpectraCSR
from .mgf import format_charge, read_mgf

TOLERANCE = 0.1  # most_similar_representative.py:15


def _mz_of(spec):
    if isinstance(spec, dict):
        return np.asarray(spec["m/z array"], np.float64)
    if isinstance(spec, tuple) and len(spec) == 2:
        return np.asarray(spec[0], np.float64)
    return np.asarray(spec, np.float64)


def distance(spec1, spec2, method="xcorr"):
    """1.0 - XQuestScores().xCorrelationPrescore(spec1, spec2, 0.1), on the GPU."""
    if method != "xcorr":
        return 0
    m1, m2 = _mz_of(spec1), _mz_of(spec2)
    csr = SpectraCSR.from_clusters([[{"m/z array": m1, "intensity array": np.zeros_like(m1)},
                                     {"m/z array": m2, "intensity array": np.zeros_like(m2)}]])
    batch = engine.DeviceBatch.from_host(csr)
    d = engine.xcorr_distance(batch, _pair01(batch.device), TOLERANCE)
    return float(d.cpu().numpy()[0])


_PAIR01 = {}


def _pair01(device):
    """The device pair (0, 1), made once per device (no H2D per distance call)."""
    import torch

    t = _PAIR01.get(str(device))
    if t is None:
        t = _PAIR01[str(device)] = torch.tensor([[0, 1]], dtype=torch.int64, device=device)
    return t


def _first_runs(names):
    """The reference's cluster scan (most_similar_representative.py:49-75)."""
    order = list(dict.fromkeys(names))
    runs, range_start = [], 0
    for cl in order:
        members, reached = [], False
        for i in range(range_start, len(names)):
            if names[i] == cl:
                members.append(i)
                reached = True
            elif reached:
                range_start = i - 1
                break
        runs.append((cl, members))
    return runs


def write_record(fh, title, pepmass, charge, rt, mz, inten):
    """One output spectrum (fields that are None are omitted)."""
    parts = ["BEGIN IONS\n"]
    if title is not None:
        parts.append(f"TITLE={title}\n")
    if pepmass is not None:
        parts.append(f"PEPMASS={float(pepmass)!r}\n")
    if charge is not None:
        parts.append(f"CHARGE={format_charge(charge)}\n")
    if rt is not None:
        parts.append(f"RTINSECONDS={float(rt)!r}\n")
    parts.extend(f"{float(a)!r} {float(b)!r}\n" for a, b in zip(mz, inten))
    parts.append("END IONS\n\n")
    fh.write("".join(parts))


def _write_spectra(spectra, path):
    with open(path, "w") as fh:
        for sp in spectra:
            p = sp["params"]
            ch = p.get("charge")
            write_record(fh, p.get("title"), p["pepmass"][0] if "pepmass" in p else None,
                         ch if ch is not None and len(ch) else None, p.get("rtinseconds"),
                         sp["m/z array"], sp["intensity array"])


def representatives(spectra, names):
    """Indices (into ``spectra``) of the representative of every cluster run."""
    runs = [(cl, m) for cl, m in _first_runs(names) if m]
    csr = SpectraCSR.from_clusters([[spectra[i] for i in members] for _cl, members in runs])
    return _choose(csr, runs)


def _choose(csr, runs):
    rep, _ = engine.medoid(engine.DeviceBatch.from_host(csr), TOLERANCE).to_host()
    if np.any(rep < 0):
        raise RuntimeError("medoid engine could not resolve a cluster (see DESIGN.md limits)")
    out = []
    for c, (cl, members) in enumerate(runs):
        out.append((cl, members, members[int(rep[c] - csr.cluster_off[c])]))
    return out


def _main_native(inputfile, outputfile):
    """main() over the native parse: records straight into the CSR, the reference's
    cluster scan done natively (spx_mgf_group mode 2), the chosen records written
    from the flat arrays.  False when the file is outside the native subset or a
    record has no TITLE (the dict path then decides)."""
    from . import ingest, mgf_native

    try:
        flat = mgf_native.parse_general(inputfile, group=mgf_native.GROUP_FIRST_RUNS)
    except ValueError:
        return False
    if flat is None or not flat["has_title"].all():
        return False
    key, ids = flat["key"], flat["group_ids"]
    records = np.flatnonzero(key >= 0)  # each id's first run, runs in file order
    sizes = np.bincount(key[records], minlength=len(ids))
    csr = ingest.csr_from_flat(flat, sizes, None if len(records) == len(key) else records)
    rep, _ = engine.medoid(engine.DeviceBatch.from_host(csr), TOLERANCE).to_host()
    if np.any(rep < 0):
        raise RuntimeError("medoid engine could not resolve a cluster (see DESIGN.md limits)")
    print("".join(f"{cl}\n{n}\n" for cl, n in zip(ids, sizes.tolist())), end="")
    print(len(ids))
    write_chosen(outputfile, flat, records[rep])
    return True


def write_chosen(outputfile, flat, chosen):
    """The chosen records of a native parse, verbatim, through the native
    multithreaded writer (the text of :func:`write_record`)."""
    from . import mgf_native
    from .csr import concat_ranges

    so = flat["spec_off"]
    lens = so[chosen + 1] - so[chosen]
    off = np.zeros(len(chosen) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    idx = concat_ranges(so[chosen], lens)
    flags = (flat["has_prec"][chosen].astype(np.int32) * mgf_native.FLAG_PEPMASS |
             flat["has_charge"][chosen].astype(np.int32) * mgf_native.FLAG_CHARGE |
             flat["has_rt"][chosen].astype(np.int32) * mgf_native.FLAG_RT | mgf_native.FLAG_TITLE)
    mgf_native.write_records(outputfile, mgf_native.STYLE_MEDOID, [flat.title(s) for s in chosen], off,
                             flat["mz"][idx], flat["inten"][idx], flat["prec_mz"][chosen], flat["charge"][chosen],
                             flat["rt"][chosen], flags)


def _main_dicts(inputfile, outputfile):
    """main() over the dict reader (``specpride_amd.mgf.read_mgf``): the path for
    input outside the native parser's subset.  Same cluster scan, prints and
    output as :func:`_main_native`; a record without TITLE fails as the
    reference's ``getMetaValue("TITLE").decode()`` does (:50)."""
    spectra = read_mgf(inputfile)
    names = []
    for sp in spectra:
        title = sp["params"].get("title")
        if title is None:
            raise AttributeError("'NoneType' object has no attribute 'decode'")
        names.append(title.split(";")[0])
    chosen = []
    for cl, members, best in representatives(spectra, names):
        print(cl)
        print(len(members))
        chosen.append(spectra[best])
    print(len(chosen))
    _write_spectra(chosen, outputfile)


def main_single(inputfile, outputfile):
    """The single-process CLI body: native ingest, else the dict path (never
    re-enters the torchrun dispatch: the sharded CLI's rank-0 fallback runs this)."""
    if not _main_native(inputfile, outputfile):
        _main_dicts(inputfile, outputfile)


def main(argv):
    inputfile, outputfile = "", ""
    try:
        opts, _args = getopt.getopt(argv, "hi:o:")
    except getopt.GetoptError:
        print("most_similar_representative.py -i <inputfile> -o <outputfile>")
        sys.exit(2)
    for opt, arg in opts:
        if opt == "-h":
            print("most_similar_representative.py -i <inputfile> -o <outputfile>")
            sys.exit()
        elif opt in ("-i",):
            inputfile = arg
        elif opt in ("-o",):
            outputfile = arg
    from . import sharded_cli

    if sharded_cli.launched_distributed():  # torchrun: rank-local ingest, one GPU per rank
        sharded_cli.run_cli(sharded_cli.medoid, lambda: main_single(inputfile, outputfile), inputfile, outputfile)
        return
    main_single(inputfile, outputfile)


if __name__ == "__main__":
    main(sys.argv[1:])
