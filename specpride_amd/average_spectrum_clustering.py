#!/usr/bin/env python3
"""Drop-in for the reference's ``src/average_spectrum_clustering.py``
(gap-average consensus), running the per-cluster numeric core on MI355X
through ``spx_gap_average``.

Kept from the reference (same names, arguments, return shapes, errors):

* constants ``DIFF_THRESH``, ``DYN_RANGE``, ``MIN_FRACTION``, ``H`` (:6, :21-23)
* ``average_spectrum(spectra, title='', pepmass='', rtinseconds='', charge='',
  **kwargs)`` (:26-103) -> ``{'params': {...}, 'm/z array', 'intensity array'}``;
  raises ``IndexError`` when the pooled peaks have no gap >= mz_accuracy and
  ``ValueError`` when every group is dropped (max of an empty array).
* precursor helpers ``lower_median_mass``, ``lower_median_mass_rt``,
  ``naive_average_mass_and_charge``, ``neutral_average_mass_and_charge``,
  ``median_rt``, ``get_cluster_id`` (:106-148): small host-side scalar
  helpers over pyteomics-shaped spectra (the batched path computes the same
  quantities on the device, see ``spx_gap_params.pepmass_mode``).
* ``process_maracluster_mgf(fname, get_cluster, get_pepmass, get_rt, **kw)``
  (:151-165): consecutive-title grouping (``itertools.groupby``), one output
  per run, all clusters averaged in ONE device pass.
* ``main()`` CLI (:168-210): ``input [output]``, ``--single`` |
  ``--encodedclusters``, ``--dyn-range``, ``--min-fraction``,
  ``--mz-accuracy``, ``--append``, ``--rt``, ``--pepmass``.

Consensus values agree with the reference within 1e-9 relative (the group
sums are exact fixed-point on the device; the reference uses cumulative-sum
differences); group boundaries and counts are exact.
"""
from __future__ import annotations

import argparse
from itertools import groupby

import numpy as np

from . import engine
from .csr import SpectraCSR
from .mgf import read_mgf, write_pyteomics_style

H = engine.PROTON  # pyteomics mass.nist_mass['H+'][0][0]

DIFF_THRESH = 0.01
DYN_RANGE = 1000
MIN_FRACTION = 0.5

_NO_GAP_MSG = "list index out of range"
_EMPTY_MSG = "zero-size array to reduction operation maximum which has no identity"


def _raise_for(status):
    if status == engine.STATUS_NO_GAP:
        raise IndexError(_NO_GAP_MSG)
    if status == engine.STATUS_EMPTY:
        raise ValueError(_EMPTY_MSG)
    if status == engine.STATUS_MIXED_CHARGE:
        raise ValueError("There are different charge states in the cluster. Cannot average precursor m/z.")
    raise RuntimeError(f"gap-average failed with status {status}")


def _flat(s):
    p = s.get("params", {})
    pm = p.get("pepmass", (np.nan,))
    ch = p.get("charge", [0])
    return {"m/z array": s["m/z array"], "intensity array": s["intensity array"],
            "precursor mz": pm[0] if isinstance(pm, (tuple, list)) else pm,
            "precursor charge": ch[0] if isinstance(ch, (tuple, list)) and len(ch) else 0,
            "rt": p.get("rtinseconds", np.nan)}


def _average_batch(clusters, mz_accuracy, dyn_range, min_fraction, pepmass="lower_median",
                   rt="mass_lower_median", device="cuda"):
    csr = SpectraCSR.from_clusters([[_flat(s) for s in sp] for sp in clusters], rt_key="rt")
    return engine.gap_average(engine.DeviceBatch.from_host(csr, device), mz_accuracy, dyn_range,
                              min_fraction, pepmass=pepmass, rt=rt).to_host()


def average_spectrum(spectra, title="", pepmass="", rtinseconds="", charge="", **kwargs):
    """Average spectrum of one cluster (average_spectrum_clustering.py:26-103), on the GPU."""
    spectra = list(spectra)
    r = _average_batch([spectra], kwargs.get("mz_accuracy", DIFF_THRESH), kwargs.get("dyn_range", DYN_RANGE),
                       kwargs.get("min_fraction", MIN_FRACTION))
    if r["status"][0] != engine.STATUS_OK:
        _raise_for(r["status"][0])
    return {"params": {"title": title, "pepmass": pepmass, "rtinseconds": rtinseconds, "charge": charge},
            "m/z array": r["out_mz"].copy(), "intensity array": r["out_int"].copy()}


# ------------------------------------------------------- precursor helpers
def _neutral_masses(spectra):
    mzs = [s["params"]["pepmass"][0] for s in spectra]
    charges = [s["params"]["charge"][0] for s in spectra if len(s["params"]["charge"]) == 1]
    return [(m * c - c * H) for m, c in zip(mzs, charges)], charges


def _lower_median_mass_index(masses):
    order = np.argsort(masses)
    k = order[(len(masses) - 1) // 2]
    return k, masses[k]


def lower_median_mass(spectra):
    masses, charges = _neutral_masses(spectra)
    i, m = _lower_median_mass_index(masses)
    z = charges[i]
    return (m + z * H) / z, z


def lower_median_mass_rt(spectra):
    masses, _ = _neutral_masses(spectra)
    i, _m = _lower_median_mass_index(masses)
    return [s["params"]["rtinseconds"] for s in spectra][i]


def get_cluster_id(title):
    return title.split(";", 1)[0]


def naive_average_mass_and_charge(spectra):
    mzs = [s["params"]["pepmass"][0] for s in spectra]
    charges = {tuple(s["params"]["charge"]) for s in spectra}
    if len(charges) > 1:
        raise ValueError("There are different charge states in the cluster. Cannot average precursor m/z.")
    return sum(mzs) / len(mzs), charges.pop()[0]


def neutral_average_mass_and_charge(spectra):
    masses, charges = _neutral_masses(spectra)
    z = int(round(sum(charges) / len(charges)))
    return (sum(masses) / len(masses) + z * H) / z, z


def median_rt(spectra):
    return np.median([s["params"]["rtinseconds"] for s in spectra])


# ------------------------------------------------------------ batch driver
def process_maracluster_mgf(fname, get_cluster=get_cluster_id, get_pepmass=naive_average_mass_and_charge,
                            get_rt=median_rt, **kwargs):
    """Average every consecutive-title cluster of an MGF (:151-165) in one GPU pass.

    With the standard helpers the file goes through the native parser straight
    into the CSR (no per-spectrum Python objects); custom callables, or a file
    outside the native subset, take the dict path."""
    # the standard helpers run on the device in the same pass; custom callables on the host
    pm_mode = {lower_median_mass: "lower_median", naive_average_mass_and_charge: "naive_average",
               neutral_average_mass_and_charge: "neutral_average"}.get(get_pepmass)
    rt_mode = {median_rt: "median", lower_median_mass_rt: "mass_lower_median"}.get(get_rt)
    on_device = pm_mode is not None and rt_mode is not None
    acc = kwargs.get("mz_accuracy", DIFF_THRESH)
    dyn = kwargs.get("dyn_range", DYN_RANGE)
    frac = kwargs.get("min_fraction", MIN_FRACTION)
    native = _native_pass(fname, get_cluster, get_pepmass, get_rt, **kwargs)
    if native is not None:
        return _outputs(*native[::-1])
    spectra = read_mgf(fname)
    runs = []
    for cluster_id, grp in groupby(spectra, lambda s: get_cluster(s["params"]["title"])):
        runs.append((cluster_id, list(grp)))
    r = _average_batch([sp for _cid, sp in runs], acc, dyn, frac,
                       pepmass=pm_mode or "lower_median", rt=rt_mode or "mass_lower_median")
    if on_device:
        return _outputs(r, [cid for cid, _sp in runs])
    outputs = []
    for c, (cluster_id, sp) in enumerate(runs):
        (mz, ch), rt = get_pepmass(sp), get_rt(sp)
        if r["status"][c] != engine.STATUS_OK:
            _raise_for(r["status"][c])
        a, b = r["out_off"][c], r["out_off"][c + 1]
        outputs.append({"params": {"title": cluster_id, "pepmass": mz, "rtinseconds": rt, "charge": ch},
                        "m/z array": r["out_mz"][a:b].copy(), "intensity array": r["out_int"][a:b].copy()})
    return outputs


def _outputs(r, ids):
    """Output spectra of a device pass whose precursor fields came from the device."""
    outputs = []
    for c, cluster_id in enumerate(ids):
        if r["status"][c] != engine.STATUS_OK:
            _raise_for(r["status"][c])
        a, b = r["out_off"][c], r["out_off"][c + 1]
        outputs.append({"params": {"title": cluster_id, "pepmass": float(r["prec"][c]),
                                   "rtinseconds": float(r["rt"][c]), "charge": int(r["charge"][c])},
                        "m/z array": r["out_mz"][a:b].copy(), "intensity array": r["out_int"][a:b].copy()})
    return outputs


def _native_pass(fname, get_cluster=get_cluster_id, get_pepmass=naive_average_mass_and_charge, get_rt=median_rt,
                 **kwargs):
    """process_maracluster_mgf's device pass over the native parse: (run ids, host
    result with the precursor fields computed on the device), or None when the
    helpers are custom callables or the file is outside the native subset."""
    pm_mode = {lower_median_mass: "lower_median", naive_average_mass_and_charge: "naive_average",
               neutral_average_mass_and_charge: "neutral_average"}.get(get_pepmass)
    rt_mode = {median_rt: "median", lower_median_mass_rt: "mass_lower_median"}.get(get_rt)
    if pm_mode is None or rt_mode is None or get_cluster is not get_cluster_id:
        return None
    native = _native_runs(fname)
    if native is None:
        return None
    ids, csr = native
    r = engine.gap_average(engine.DeviceBatch.from_host(csr), kwargs.get("mz_accuracy", DIFF_THRESH),
                           kwargs.get("dyn_range", DYN_RANGE), kwargs.get("min_fraction", MIN_FRACTION),
                           pepmass=pm_mode, rt=rt_mode).to_host()
    return ids, r


def _native_runs(fname):
    """Native parse -> (run ids, CSR of the consecutive-title runs), or None when
    the file is outside the native subset or a record has no TITLE."""
    from . import ingest, mgf_native

    try:
        flat = mgf_native.parse_general(fname, group=mgf_native.GROUP_RUNS)
    except ValueError:
        return None
    if flat is None or not flat["has_title"].all():
        return None
    ids = flat["group_ids"]  # itertools.groupby runs of get_cluster_id(title), in file order
    return ids, ingest.csr_from_flat(flat, np.bincount(flat["key"], minlength=len(ids)))


def write_outputs_native(r, ids, output, file_mode="w"):
    """mgf.write of the outputs (average_spectrum_clustering.py:207-208) straight
    from a device result: the reference's error for the first failing run, then
    the native multithreaded writer (the same text as write_pyteomics_style)."""
    from . import mgf_native

    bad = np.flatnonzero(r["status"] != engine.STATUS_OK)
    if len(bad):
        _raise_for(r["status"][bad[0]])
    mgf_native.write_records(output, mgf_native.STYLE_GAP_AVERAGE, ids, r["out_off"], r["out_mz"], r["out_int"],
                             r["prec"], r["charge"], r["rt"], append=file_mode == "a")


def main(argv=None):
    pars = argparse.ArgumentParser()
    pars.add_argument("input", help="MGF file with clustered spectra.")
    pars.add_argument("output", nargs="?", help="Output file (default is stdout).")
    mode = pars.add_mutually_exclusive_group(required=True)
    mode.add_argument("--single", action="store_true",
                      help="If specified, input is interpreted as containing a single cluster.")
    mode.add_argument("--encodedclusters", action="store_true",
                      help="Process an MGF with cluster IDs encoded in titles.")
    pars.add_argument("--dyn-range", type=float, default=DYN_RANGE, help="Dynamic range to apply to output spectra")
    pars.add_argument("--min-fraction", type=float, default=MIN_FRACTION,
                      help="Minimum fraction of cluster spectra where MS/MS peak is present.")
    pars.add_argument("--mz-accuracy", type=float, default=DIFF_THRESH,
                      help="Minimum distance between MS/MS peak clusters.")
    pars.add_argument("--append", action="store_true", help="Append to output file instead of replacing it.")
    pars.add_argument("--rt", choices=["median", "mass_lower_median"], default="median")
    pars.add_argument("--pepmass", choices=["naive_average", "neutral_average", "lower_median"],
                      default="lower_median")
    args = pars.parse_args(argv)
    if args.pepmass == "lower_median":
        args.rt = "mass_lower_median"
    get_rt = {"median": median_rt, "mass_lower_median": lower_median_mass_rt}[args.rt]
    get_pepmass = {"naive_average": naive_average_mass_and_charge,
                   "neutral_average": neutral_average_mass_and_charge,
                   "lower_median": lower_median_mass}[args.pepmass]
    kwargs = {"mz_accuracy": args.mz_accuracy, "dyn_range": args.dyn_range, "min_fraction": args.min_fraction}
    mode = "wa"[args.append]
    if args.single:
        spectra = read_mgf(args.input)
        mz, c = get_pepmass(spectra)
        rt = get_rt(spectra)
        write_pyteomics_style([average_spectrum(spectra, title=args.output, pepmass=mz, charge=c, rtinseconds=rt,
                                                **kwargs)], args.output, file_mode=mode)
    elif args.encodedclusters:
        def single():
            native = _native_pass(args.input, get_pepmass=get_pepmass, get_rt=get_rt, **kwargs) \
                if args.output is not None else None
            if native is not None:  # native ingest -> one device pass -> native writer
                write_outputs_native(native[1], native[0], args.output, file_mode=mode)
                return
            write_pyteomics_style(process_maracluster_mgf(args.input, get_pepmass=get_pepmass, get_rt=get_rt,
                                                          **kwargs), args.output, file_mode=mode)

        from . import sharded_cli

        if sharded_cli.launched_distributed():  # torchrun: rank-local ingest, one GPU per rank
            sharded_cli.run_cli(sharded_cli.gap_average, single, args.input, args.output, pepmass=args.pepmass,
                                rt=args.rt, file_mode=mode, **kwargs)
        else:
            single()
    else:
        raise NotImplementedError("This mode is not implemented yet.")


if __name__ == "__main__":
    main()
