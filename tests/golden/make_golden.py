#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only where /root/reference exists (the build container).  It imports the
reference's own modules from /root/reference/src -- ``binning``,
``average_spectrum_clustering`` and ``most_similar_representative`` -- with the
import stand-ins under tests/golden/stubs (pyteomics / pyopenms are absent
offline; see the stub docstrings), feeds them deterministic inputs and writes
inputs + reference outputs as data (compressed .npz without pickles, JSON, MGF).
No reference source is copied: only values it computed.

    python tests/golden/make_golden.py            # regenerate everything

Fixtures:
  bin_mean_<set>.npz        combine_bin_mean() per cluster (binning.py:170-231)
  bin_mean_cli_in.mgf/out   binning.py main() end to end (binning.py:250-302)
  gap_average_<set>.npz     average_spectrum() per cluster (average_spectrum_clustering.py:26-103)
  *_nonfinite*              NaN / inf m/z and intensities: combine_bin_mean, average_spectrum and the
                            binning CLI (``python tests/golden/make_golden.py nonfinite`` regenerates them)
  precursor_helpers.npz     lower_median_mass & co (average_spectrum_clustering.py:106-148)
  medoid_<set>.npz          most_similar_representative.main() reps (most_similar_representative.py:22-115)
  pairwise_sum.npz          numpy pairwise summation (the reduction pandas .sum() runs)
  binned_cosine.npz         cos_dist / average_cos_dist per cluster (benchmark.py:10-38)
  best_spectrum_*           best_spectrum() end to end + get_best_representative (best_spectrum.py:43-175)
  maracluster_*             binning.read_cluster_list (binning.py:35-52) and convert_mgf_cluster.py's
                            read_clusters / read_peptides / buid_usi_accession / convert-mq-marcluster (:14-79)
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
STUBS = os.path.join(HERE, "stubs")

sys.path.insert(0, REPO)
from specpride_amd.csr import SpectraCSR  # noqa: E402
from specpride_amd.mgf import write_csr_mgf  # noqa: E402
from specpride_amd.synthetic import make_clusters_np  # noqa: E402

STATUS_OK, STATUS_MIXED_CHARGE, STATUS_NO_GAP, STATUS_EMPTY = 0, 1, 2, 3


def _import_reference():
    sys.path.insert(0, STUBS)
    sys.path.insert(0, REF_SRC)
    import binning  # noqa: F401
    import average_spectrum_clustering  # noqa: F401
    import most_similar_representative  # noqa: F401
    return binning, average_spectrum_clustering, most_similar_representative


def _csr_arrays(csr: SpectraCSR, prefix=""):
    return {prefix + "cluster_off": csr.cluster_off, prefix + "spec_off": csr.spec_off,
            prefix + "mz": csr.mz, prefix + "inten": csr.inten, prefix + "prec_mz": csr.prec_mz,
            prefix + "charge": csr.charge, prefix + "rt": csr.rt}


def _concat(parts, dtype=np.float64):
    return np.concatenate(parts).astype(dtype) if parts else np.zeros(0, dtype)


# ----------------------------------------------------------------- inputs
EXAMPLE_PEAKS = [  # file_formats.md:10-52 (the only in-repo spectrum: cluster-1, 43 peaks)
    (1.5, 8.84), (5.8, 0.75), (8.285, 1.34), (17.4, 0.32), (97.999, 1.1), (132.017, 445.98),
    (158.996, 235.36), (169.955, 4235.4), (175.045, 518.94), (185.063, 336.05), (209.069, 186.72),
    (260.189, 1255.96), (268.922, 159.25), (277.729, 3557.77), (286.234, 510.24), (334.264, 3129.8),
    (339.303, 328.09), (346.855, 400.5), (350.224, 199.13), (383.827, 5392.89), (402.894, 272.86),
    (411.354, 1636.43), (417.31, 2169.19), (420.341, 446.95), (491.367, 214.35), (519.401, 325.75),
    (521.779, 35.4), (537.578, 32.16), (554.307, 1514.12), (592.429, 35.01), (600.643, 1.7),
    (627.992, 6.41), (647.458, 2.33), (667.572, 61.7), (677.451, 3.69), (713.578, 0.65),
    (761.149, 0.54), (795.495, 0.72), (808.411, 0.68), (839.005, 1.06), (850.931, 1.57),
    (869.944, 0.86), (879.392, 0.61)]


def _spec(mz, it, prec=500.0, z=2, rt=100.0):
    return {"m/z array": list(map(float, mz)), "intensity array": list(map(float, it)),
            "precursor mz": float(prec), "precursor charge": int(z), "rt": float(rt)}


def bin_mean_edge_clusters(rng):
    ex_mz, ex_int = zip(*EXAMPLE_PEAKS)
    cl = []
    cl.append([_spec(ex_mz, ex_int, 318.185, 2)])                          # single example spectrum
    cl.append([_spec(ex_mz, ex_int, 318.185, 2),                           # example + jittered copies
               _spec(np.array(ex_mz) + 0.004, np.array(ex_int) * 1.5, 318.19, 2),
               _spec(np.array(ex_mz) - 0.011, np.array(ex_int) * 0.5, 318.18, 2)])
    cl.append([_spec([150.001, 150.005, 150.011], [10, 20, 40], 400, 3),  # A.1 item 8: last wins
               _spec([150.003], [1], 401, 3)])
    cl.append([_spec([100.0, 99.99999, 1999.99999, 2000.0, 150.0], [1, 2, 3, 4, 5], 600, 2),  # range edges
               _spec([100.0, 1999.99999, 2000.00001], [7, 8, 9], 600.5, 2)])
    for n in (3, 4, 5, 7, 8, 9):                                           # quorum boundaries
        base = np.sort(rng.uniform(100, 2000, 30))
        sp = []
        for k in range(n):
            take = rng.random(30) < (0.3 + 0.7 * (k / max(1, n - 1)))
            sp.append(_spec(np.round(base[take] + rng.normal(0, 0.004, take.sum()), 5),
                            np.round(rng.lognormal(4, 1, take.sum()), 2), 700 + k * 0.01, 2))
        cl.append(sp)
    # unsorted spectra with non-adjacent duplicates in one bin (last in FILE order wins)
    cl.append([_spec([300.011, 500.0, 300.001, 250.0, 300.013], [1, 2, 3, 4, 5], 500, 2),
               _spec([500.001, 300.005, 250.015, 300.019], [10, 20, 30, 40], 500, 2),
               _spec([300.0, 300.002, 499.999], [6, 7, 8], 500, 2)])
    # an empty spectrum inside a cluster, and identical spectra
    cl.append([_spec([], [], 420, 2), _spec([200.0, 300.0], [1, 2], 421, 2), _spec([200.0, 300.0], [1, 2], 422, 2)])
    cl.append([_spec([123.456, 456.789], [3.0, 4.0], 333, 3)] * 4)
    # large intensities (f32 accumulation rounding visible) and tiny ones
    cl.append([_spec([1000.00001, 1500.5], [1.23456789e9, 3.3e-7], 900, 2),
               _spec([1000.00002, 1500.50001], [9.87654321e8, 1.1e-7], 900, 2)])
    return cl


def csr_to_peaklists(csr: SpectraCSR):
    out = []
    for c in range(csr.n_clusters):
        pl = []
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            mz, it = csr.spectrum(s)
            pl.append({"m/z array": [float(x) for x in mz], "intensity array": [float(x) for x in it],
                       "precursor mz": float(csr.prec_mz[s]), "precursor charge": int(csr.charge[s]),
                       "rt": float(csr.rt[s])})
        out.append(pl)
    return out


def peaklists_to_csr(clusters):
    return SpectraCSR.from_clusters(clusters, rt_key="rt")


# ---------------------------------------------------------------- bin-mean
def gen_bin_mean(binning):
    rsc = binning.RepresentativeSpectrumCreator(verbose=0)
    rng = np.random.default_rng(101)
    sets = {
        "edge": (bin_mean_edge_clusters(rng), dict()),
        "synthetic": (csr_to_peaklists(make_clusters_np(32, seed=7)), dict()),
        "params_b": (csr_to_peaklists(make_clusters_np(16, seed=8, max_size=20)),
                     dict(minimum=150, maximum=1500, binsize=0.05, apply_peak_quorum=False)),
        "params_c": (csr_to_peaklists(make_clusters_np(12, seed=9, max_size=12)),
                     dict(minimum=0, maximum=3000, binsize=0.01, apply_peak_quorum=True)),
    }
    mixed = [[_spec([200.0], [1.0], 400, 2), _spec([200.0], [1.0], 400, 3)],
             [_spec([210.0, 220.0], [1.0, 2.0], 410, 2), _spec([210.0], [1.0], 410, 2)]]
    sets["mixed_charge"] = (mixed, dict())
    for name, (clusters, kw) in sets.items():
        out_mz, out_int, out_off, prec, charge, status = [], [], [0], [], [], []
        for pl in clusters:
            try:
                r = rsc.combine_bin_mean(pl, **kw)
            except AssertionError:
                status.append(STATUS_MIXED_CHARGE)
                out_off.append(out_off[-1])
                prec.append(np.nan)
                charge.append(0)
                continue
            status.append(STATUS_OK)
            assert r["mzs"].dtype == np.float64 and r["intensities"].dtype == np.float64
            out_mz.append(r["mzs"])
            out_int.append(r["intensities"])
            out_off.append(out_off[-1] + len(r["mzs"]))
            prec.append(float(r["precursor_mz"]))
            charge.append(int(r["precursor_charge"]))
        csr = peaklists_to_csr(clusters)
        params = dict(minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True)
        params.update(kw)
        np.savez_compressed(os.path.join(HERE, f"bin_mean_{name}.npz"), **_csr_arrays(csr),
                            out_off=np.array(out_off, np.int64), out_mz=_concat(out_mz),
                            out_int=_concat(out_int), out_prec=np.array(prec), out_charge=np.array(charge, np.int32),
                            status=np.array(status, np.int32),
                            params=np.array([params["minimum"], params["maximum"], params["binsize"],
                                             float(params["apply_peak_quorum"])], np.float64))
        print(f"bin_mean_{name}: {len(clusters)} clusters, {out_off[-1]} output peaks")


def gen_bin_mean_cli():
    csr = make_clusters_np(20, seed=11, n_template=40)
    ex_mz, ex_int = zip(*EXAMPLE_PEAKS)
    extra = SpectraCSR.from_clusters([[_spec(ex_mz, ex_int, 318.185, 2), _spec(ex_mz, ex_int, 318.185, 2)]],
                                     cluster_ids=["cluster-ex"], rt_key="rt")
    in_path = os.path.join(HERE, "bin_mean_cli_in.mgf")
    out_path = os.path.join(HERE, "bin_mean_cli_out.mgf")
    with open(in_path, "w") as fh:
        write_csr_mgf(csr, fh)
        # a second run of cluster-3 after the others (binning.py merges by id: A.4)
        extra_titles = [f"cluster-ex;mzspec:PXD004732:ex.raw:scan:{k}" for k in range(2)]
        write_csr_mgf(extra, fh, titles=extra_titles, sequences=["VLHPLEGAVVIIFK/2", ""])
        late = csr.select([3])
        write_csr_mgf(late, fh, titles=[f"cluster-3;mzspec:PXDSYN:synthetic:scan:late{k}"
                                        for k in range(late.n_spectra)])
    env = dict(os.environ, PYTHONPATH=STUBS)
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([sys.executable, os.path.join(REF_SRC, "binning.py"), "--mgf_file", in_path,
                            "--out", os.path.join(td, "out.mgf")], env=env, cwd=td, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr)
        with open(os.path.join(td, "out.mgf")) as src, open(out_path, "w") as dst:
            dst.write(src.read())
        r2 = subprocess.run([sys.executable, os.path.join(REF_SRC, "binning.py")], env=env, cwd=td,
                            capture_output=True, text=True)
    with open(os.path.join(HERE, "bin_mean_cli.json"), "w") as fh:
        json.dump({"stdout": r.stdout, "no_args_returncode": r2.returncode, "no_args_stdout": r2.stdout}, fh, indent=1)
    print("bin_mean_cli: ok", os.path.getsize(in_path), os.path.getsize(out_path))


# ------------------------------------------------------------- gap-average
def gap_edge_clusters(rng):
    S = lambda mz, it: {"m/z array": np.array(mz, float), "intensity array": np.array(it, float)}  # noqa: E731
    cl = []
    cl.append([S([500.0, 100.0, 300.0], [5.0, 1.0, 0.001])])                       # n=1 passthrough (unsorted)
    cl.append([S([100.0, 100.001], [1, 2]), S([100.002], [3])])                     # one group -> IndexError
    cl.append([S([100.0, 200.0], [1, 2]), S([100.001, 200.001], [3, 4])])           # two groups
    cl.append([S([100.0, 200.0, 300.0], [1, 2, 3]), S([100.001, 200.001, 300.001], [1, 2, 3])])  # merge quirk
    cl.append([S([100, 150, 200, 250, 300, 350], [1, 2, 3, 4, 5, 6]),
               S([100.005, 200.005, 300.005], [1, 1, 1]), S([150.002, 350.001], [9, 9])])     # min_fraction drops
    cl.append([S([100.0, 300.0], [1, 1]), S([200.0, 400.0], [1, 1]), S([500.0], [1])])        # merged tail survives
    cl.append([S([100.0], [1]), S([200.0], [1]), S([300.0], [1]), S([400.0], [1]), S([500.0], [1])])  # all dropped -> ValueError
    cl.append([S([100.0, 200.0, 300.0, 400.0], [1000.0, 1.0, 0.999, 500.0]),
               S([100.0, 200.0, 300.0, 400.0], [1000.0, 1.0, 1.001, 500.0])])  # dyn-range: 2000/1000 = 2.0 boundary
    cl.append([S([], []), S([], [])])                                               # no peaks -> IndexError
    cl.append([S([], [])])                                                          # n=1 empty -> ValueError
    cl.append([S([100.0, 100.0, 100.0, 200.0], [1, 2, 3, 4]), S([100.0, 200.0], [5, 6])])  # mz ties
    cl.append([S([100.00, 100.01, 100.02, 100.035], [1, 2, 3, 4]), S([100.005, 100.03], [5, 6])])  # gaps ~ acc
    big = rng.uniform(100, 2000, 40)
    cl.append([S(np.round(np.sort(big + rng.normal(0, 0.002, 40)), 5), np.round(rng.lognormal(5, 1.5, 40), 2))
               for _ in range(6)])
    return cl


def _pyteo_spectra(csr: SpectraCSR):
    out = []
    for c in range(csr.n_clusters):
        sp = []
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            mz, it = csr.spectrum(s)
            sp.append({"m/z array": mz.copy(), "intensity array": it.copy(),
                       "params": {"title": f"cluster-{c};scan:{s}", "pepmass": (float(csr.prec_mz[s]), None),
                                  "charge": [int(csr.charge[s])], "rtinseconds": float(csr.rt[s])}})
        out.append(sp)
    return out


def gen_gap_average(asc):
    rng = np.random.default_rng(202)
    sets = {
        "edge": (gap_edge_clusters(rng), dict()),
        "synthetic": (_pyteo_spectra(make_clusters_np(32, seed=17)), dict()),
        "params_b": (_pyteo_spectra(make_clusters_np(16, seed=18, max_size=20)),
                     dict(mz_accuracy=0.02, dyn_range=100, min_fraction=0.3)),
        "params_c": (_pyteo_spectra(make_clusters_np(12, seed=19, max_size=30)),
                     dict(mz_accuracy=0.005, dyn_range=10000, min_fraction=0.75)),
    }
    for name, (clusters, kw) in sets.items():
        out_mz, out_int, out_off, status = [], [], [0], []
        for sp in clusters:
            try:
                r = asc.average_spectrum(sp, "t", **kw)
            except IndexError:
                status.append(STATUS_NO_GAP)
                out_off.append(out_off[-1])
                continue
            except ValueError:
                status.append(STATUS_EMPTY)
                out_off.append(out_off[-1])
                continue
            status.append(STATUS_OK)
            out_mz.append(np.asarray(r["m/z array"], np.float64))
            out_int.append(np.asarray(r["intensity array"], np.float64))
            out_off.append(out_off[-1] + len(r["m/z array"]))
        csr = SpectraCSR.from_clusters(clusters)
        p = dict(mz_accuracy=asc.DIFF_THRESH, dyn_range=asc.DYN_RANGE, min_fraction=asc.MIN_FRACTION)
        p.update(kw)
        np.savez_compressed(os.path.join(HERE, f"gap_average_{name}.npz"), **_csr_arrays(csr),
                            out_off=np.array(out_off, np.int64), out_mz=_concat(out_mz), out_int=_concat(out_int),
                            status=np.array(status, np.int32),
                            params=np.array([p["mz_accuracy"], p["dyn_range"], p["min_fraction"]], np.float64))
        print(f"gap_average_{name}: {len(clusters)} clusters, {out_off[-1]} output peaks, status {status[:12]}")


NAN, INF = float("nan"), float("inf")


def gap_nonfinite_clusters(rng):
    """NaN / +-inf m/z and intensities (no reference test covers them; these pin
    what average_spectrum returns: argsort puts NaN last, diff >= acc is False
    across NaN, the cumsum differences go inf/NaN, np.max propagates NaN)."""
    S = lambda mz, it: {"m/z array": np.array(mz, float), "intensity array": np.array(it, float)}  # noqa: E731
    cl = []
    cl.append([S([100, NAN, 200], [1, 2, 3]), S([100, 200], [1, 3])])             # NaN m/z joins the last group
    cl.append([S([100, 200], [1, NAN]), S([100, 200], [1, 1])])                    # NaN intensity: max NaN -> empty
    cl.append([S([100, 200, 300], [NAN, 1, 1]), S([100, 200, 300], [1, 1, 1])])    # NaN in the first group
    cl.append([S([100, 150, 200, 300], [1, NAN, 2, 3]), S([100, 200, 300], [1, 2, 3]),
               S([100, 200, 300], [1, 2, 3])])                                     # NaN in a dropped group
    cl.append([S([100, 200, 300, 400], [1, 2, 3, 4]), S([100, 200, 300, 400, 500], [1, 2, 3, 4, NAN]),
               S([100, 200, 300, 400], [1, 2, 3, 4]), S([100, 200, 300, 400], [1, 2, 3, 4]),
               S([100, 200, 300, 400], [1, 2, 3, 4])])                             # NaN in a dropped LAST group
    cl.append([S([100, 200, 300], [1, INF, 3]), S([100, 200, 300], [1, 2, 3])])    # +inf intensity: keep inf only
    cl.append([S([100, 200, 300, 400], [1, INF, 3, 4]), S([100, 200, 300, 400], [1, 2, 3, 4])])  # inf - inf
    cl.append([S([100, 200, 300], [1, -INF, 3]), S([100, 200, 300], [1, 2, 3])])   # -inf intensity dropped
    cl.append([S([100, 200, 300], [1, -INF, 3]), S([100, 200, 300], [1, INF, 3])])  # inf + -inf in one group
    cl.append([S([100, 200, 300, 400], [-INF, 1, 3, 1]), S([100, 200, 300, 400], [1, 2, 3, 1])])  # -inf first
    cl.append([S([100, 200, INF], [1, 2, 3]), S([100, 200], [1, 2])])             # +inf m/z
    cl.append([S([100, 200, 300, INF], [1, 2, 3, 9]), S([100, 200, 300], [1, 2, 3])])  # +inf m/z, 3 groups
    cl.append([S([-INF, 100, 200], [5, 1, 2]), S([100, 200], [1, 2])])            # -inf m/z
    cl.append([S([-INF, 100, 200, 300], [5, 1, 2, 3]), S([-INF, 100, 200, 300], [5, 1, 2, 3])])
    cl.append([S([-INF], [1]), S([INF], [1])])                                     # -inf | +inf
    cl.append([S([-INF, NAN], [1, 2]), S([INF], [1])])
    cl.append([S([-INF], [1]), S([-INF], [1])])                                    # no gap (NaN diff)
    cl.append([S([NAN, NAN], [1, 2]), S([NAN], [3])])                              # all NaN -> IndexError
    cl.append([S([100], [1]), S([NAN], [2])])                                      # finite + NaN -> IndexError
    cl.append([S([100, 200, INF, NAN], [1, 1, 1, 1]), S([100, 200], [1, 1])])     # +inf then NaN
    cl.append([S([100, 200, INF], [1, 1, 1]), S([150, INF, INF], [1, 1, 1])])      # inf - inf diff
    cl.append([S([100, 200, NAN, NAN], [1, 2, 3, 4]), S([100, 200, NAN], [1, 2, 5]), S([100, 300], [1, 2])])
    cl.append([S([100, 200, 300], [1, NAN, 3])])                                   # n=1: NaN max -> empty
    cl.append([S([100, 200, 300], [1, INF, 3])])                                   # n=1: inf max
    cl.append([S([NAN, 200, INF], [1, 2, 3])])                                     # n=1: m/z passthrough
    cl.append([S([100, 200, 300], [-INF, 2, 3])])                                  # n=1: -inf dropped
    cl.append([S([100, 200, 300], [5, 2, 3]), S([100, 200, 300], [NAN, NAN, NAN])])
    cl.append([S([100, 100.004, 100.008, 200], [1, NAN, 1, 2]), S([100.002, 200], [1, 2])])
    # synthetic clusters with a few entries replaced (m/z and intensity, all kinds)
    base = make_clusters_np(40, seed=55, max_size=12, n_template=30)
    for c in range(base.n_clusters):
        sp = []
        for s in range(base.cluster_off[c], base.cluster_off[c + 1]):
            mz, it = base.spectrum(s)
            mz, it = mz.copy(), it.copy()
            if c % 4 != 0:
                k = int(rng.integers(0, 3))
                for _ in range(k):
                    j = int(rng.integers(0, len(mz))) if len(mz) else 0
                    if not len(mz):
                        break
                    v = [NAN, INF, -INF][int(rng.integers(0, 3))]
                    if (c + s) % 3 == 0:
                        it[j] = v
                    else:
                        mz[j] = v
            sp.append(S(mz, it))
        cl.append(sp)
    return cl


def bin_mean_nonfinite_clusters():
    cl = []
    cl.append([_spec([100.5, NAN, 200.0], [1, 2, 3]), _spec([100.5, 200.0], [1, 2])])       # NaN m/z masked
    cl.append([_spec([100.5, INF, -INF, 300.0], [1, 2, 3, 4]), _spec([100.5, 300.0], [5, 6])])  # inf m/z masked
    cl.append([_spec([100.5, 200.0], [NAN, 2]), _spec([100.5, 200.0], [1, 2])])             # NaN intensity bin
    cl.append([_spec([100.5, 200.0], [INF, 2]), _spec([100.5, 200.0], [1, 2])])             # +inf bin
    cl.append([_spec([100.5, 200.0], [-INF, 2]), _spec([100.5, 200.0], [INF, 2])])          # inf + -inf -> NaN
    cl.append([_spec([100.5, 200.0], [1e39, 2]), _spec([100.5, 200.0], [1, 2])])            # f32 overflow
    cl.append([_spec([150.001, NAN, 150.005], [10, 20, 40]), _spec([150.003], [1])])        # last wins past NaN
    cl.append([_spec([150.001, 150.005], [10, NAN]), _spec([150.003], [1])])                # last is NaN
    cl.append([_spec([150.001, 150.005], [NAN, 10]), _spec([150.003], [1])])                # NaN overwritten
    cl.append([_spec([NAN, NAN], [1, 2]), _spec([NAN], [3])])                               # nothing in range
    cl.append([_spec([200.0, 300.0], [1, 2])] * 3 + [_spec([200.0, 300.0], [NAN, INF])])  # 4 spectra, quorum 2
    return cl


def gen_nonfinite(binning, asc):
    """bin_mean_nonfinite.npz / gap_average_nonfinite.npz: the reference run on
    NaN / inf m/z and intensity (same layouts as the other bin_mean_* / gap_average_* sets)."""
    rsc = binning.RepresentativeSpectrumCreator(verbose=0)
    clusters = bin_mean_nonfinite_clusters()
    out_mz, out_int, out_off, prec, charge, status = [], [], [0], [], [], []
    with np.errstate(all="ignore"):
        for pl in clusters:
            r = rsc.combine_bin_mean(pl)
            status.append(STATUS_OK)
            out_mz.append(r["mzs"])
            out_int.append(r["intensities"])
            out_off.append(out_off[-1] + len(r["mzs"]))
            prec.append(float(r["precursor_mz"]))
            charge.append(int(r["precursor_charge"]))
    csr = peaklists_to_csr(clusters)
    np.savez_compressed(os.path.join(HERE, "bin_mean_nonfinite.npz"), **_csr_arrays(csr),
                        out_off=np.array(out_off, np.int64), out_mz=_concat(out_mz),
                        out_int=_concat(out_int), out_prec=np.array(prec), out_charge=np.array(charge, np.int32),
                        status=np.array(status, np.int32),
                        params=np.array([100, 2000, 0.02, 1.0], np.float64))
    print(f"bin_mean_nonfinite: {len(clusters)} clusters, {out_off[-1]} output peaks")

    # the binning CLI end to end on non-finite number tokens (float() spellings)
    in_path = os.path.join(HERE, "bin_mean_cli_nonfinite_in.mgf")
    out_path = os.path.join(HERE, "bin_mean_cli_nonfinite_out.mgf")
    recs = [("c1", "u1", ["100.5 nan", "200.0 2.0", "300.0 inf"]),
            ("c1", "u2", ["100.5 1.0", "200.0 -inf", "300.0 3.0"]),
            ("c2", "u3", ["150.0 NaN", "1e999 5.0", "250.0 Infinity", "260.0 1e999"]),
            ("c2", "u4", ["150.0 4.0", "250.0 -Infinity", "260.0 2.5"]),
            ("c3", "u5", ["120.0 1e39", "130.0 -nan", "140.0 +inf"]),
            ("c3", "u6", ["120.0 1.0", "130.0 2.0", "140.0 INF"])]
    with open(in_path, "w") as fh:
        for cid, usi, peaks in recs:
            fh.write(f"BEGIN IONS\nTITLE={cid};{usi}\nPEPMASS=500.25\nCHARGE=2+\n")
            fh.write("".join(p + "\n" for p in peaks))
            fh.write("END IONS\n\n")
    env = dict(os.environ, PYTHONPATH=STUBS)
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([sys.executable, os.path.join(REF_SRC, "binning.py"), "--mgf_file", in_path,
                            "--out", os.path.join(td, "out.mgf")], env=env, cwd=td, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr)
        with open(os.path.join(td, "out.mgf")) as src, open(out_path, "w") as dst:
            dst.write(src.read())
    print("bin_mean_cli_nonfinite: ok")

    rng = np.random.default_rng(606)
    sets = {"nonfinite": (gap_nonfinite_clusters(rng), dict())}
    sets["nonfinite_b"] = (sets["nonfinite"][0], dict(mz_accuracy=0.02, dyn_range=100, min_fraction=0.3))
    for name, (clusters, kw) in sets.items():
        out_mz, out_int, out_off, status = [], [], [0], []
        for sp in clusters:
            try:
                with np.errstate(all="ignore"):
                    r = asc.average_spectrum(sp, "t", **kw)
            except IndexError:
                status.append(STATUS_NO_GAP)
                out_off.append(out_off[-1])
                continue
            except ValueError:
                status.append(STATUS_EMPTY)
                out_off.append(out_off[-1])
                continue
            status.append(STATUS_OK)
            out_mz.append(np.asarray(r["m/z array"], np.float64))
            out_int.append(np.asarray(r["intensity array"], np.float64))
            out_off.append(out_off[-1] + len(r["m/z array"]))
        csr = SpectraCSR.from_clusters(clusters)
        p = dict(mz_accuracy=asc.DIFF_THRESH, dyn_range=asc.DYN_RANGE, min_fraction=asc.MIN_FRACTION)
        p.update(kw)
        np.savez_compressed(os.path.join(HERE, f"gap_average_{name}.npz"), **_csr_arrays(csr),
                            out_off=np.array(out_off, np.int64), out_mz=_concat(out_mz), out_int=_concat(out_int),
                            status=np.array(status, np.int32),
                            params=np.array([p["mz_accuracy"], p["dyn_range"], p["min_fraction"]], np.float64))
        print(f"gap_average_{name}: {len(clusters)} clusters, {out_off[-1]} output peaks, status {status[:30]}")


def gen_precursor_helpers(asc):
    csr = make_clusters_np(40, seed=23, max_size=9, n_template=5)
    csr.charge[csr.cluster_off[5]] = 3 if csr.charge[csr.cluster_off[5]] == 2 else 2  # one mixed-charge cluster
    clusters = _pyteo_spectra(csr)
    res = {k: [] for k in ("lm_mz", "lm_z", "lm_rt", "na_mz", "na_z", "na_status", "ne_mz", "ne_z", "med_rt")}
    for sp in clusters:
        m, z = asc.lower_median_mass(sp)
        res["lm_mz"].append(m)
        res["lm_z"].append(z)
        res["lm_rt"].append(asc.lower_median_mass_rt(sp))
        try:
            m, z = asc.naive_average_mass_and_charge(sp)
            res["na_mz"].append(m)
            res["na_z"].append(z)
            res["na_status"].append(0)
        except ValueError:
            res["na_mz"].append(np.nan)
            res["na_z"].append(0)
            res["na_status"].append(1)
        m, z = asc.neutral_average_mass_and_charge(sp)
        res["ne_mz"].append(m)
        res["ne_z"].append(z)
        res["med_rt"].append(float(asc.median_rt(sp)))
    np.savez_compressed(os.path.join(HERE, "precursor_helpers.npz"), **_csr_arrays(csr),
                        **{k: np.array(v) for k, v in res.items()}, H=np.array(asc.H))
    print("precursor_helpers: ok")


# ------------------------------------------------------------------ medoid
def medoid_cases():
    sizes = [1, 2, 3, 9, 17, 130, 300, 5, 4, 33, 64, 65, 7, 8, 129]
    csr = make_clusters_np(len(sizes), seed=31, sizes=np.array(sizes), n_template=60)
    clusters = [[(m.copy(), i.copy()) for (m, i) in csr.cluster(c)] for c in range(csr.n_clusters)]
    prec = [[float(csr.prec_mz[s]) for s in range(csr.cluster_off[c], csr.cluster_off[c + 1])]
            for c in range(csr.n_clusters)]
    # identical spectra (ties -> lowest index) and a spectrum with two peaks in one 0.1 bin
    base_mz = np.array([200.01, 300.02, 400.03, 500.04])
    clusters.append([(base_mz.copy(), np.ones(4)) for _ in range(5)])
    prec.append([500.0] * 5)
    clusters.append([(np.array([200.01, 200.05, 300.0]), np.ones(3)), (np.array([200.03, 300.0]), np.ones(2)),
                     (np.array([200.09, 300.02, 300.07, 450.0]), np.ones(4)), (np.array([450.0]), np.ones(1))])
    prec.append([500.0] * 4)
    big = make_clusters_np(1, seed=32, sizes=np.array([1000]), n_template=30)
    clusters.append([(m.copy(), i.copy()) for (m, i) in big.cluster(0)])
    prec.append([float(x) for x in big.prec_mz])
    return clusters, prec


def _write_medoid_mgf(path, order):
    """order: list of (cluster_name, mz, inten, prec, scan)."""
    with open(path, "w") as fh:
        for name, mz, it, p, scan in order:
            fh.write(f"BEGIN IONS\nTITLE={name};mzspec:PXDSYN:synthetic:scan:{scan}\nPEPMASS={p!r}\nCHARGE=2+\n")
            fh.write("".join(f"{float(a)!r} {float(b)!r}\n" for a, b in zip(mz, it)))
            fh.write("END IONS\n\n")


def _run_medoid_main(msr, in_path):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "out.txt")
        with contextlib.redirect_stdout(io.StringIO()):
            msr.main(["-i", in_path, "-o", out])
        with open(out) as fh:
            rows = [ln.rstrip("\n").split("\t") for ln in fh if ln.strip()]
    return [(int(i), t) for i, t in rows]


def gen_medoid(msr):
    clusters, prec = medoid_cases()
    order, scan = [], 0
    for c, (sp, pr) in enumerate(zip(clusters, prec)):
        for (mz, it), p in zip(sp, pr):
            order.append((f"cluster-{c}", mz, it, p, scan))
            scan += 1
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "in.mgf")
        _write_medoid_mgf(path, order)
        reps = _run_medoid_main(msr, path)
    csr = SpectraCSR.from_clusters([[{"m/z array": m, "intensity array": i} for (m, i) in sp] for sp in clusters])
    np.savez_compressed(os.path.join(HERE, "medoid_main.npz"), **_csr_arrays(csr),
                        rep_index=np.array([r[0] for r in reps], np.int64))
    print("medoid_main:", [r[0] for r in reps])

    # non-contiguous cluster order (A.4): A A B A C C B D -> first runs only
    rng = np.random.default_rng(33)
    names = ["A", "A", "B", "A", "C", "C", "B", "D", "D", "D", "A"]
    order = []
    for k, nm in enumerate(names):
        mz = np.round(np.sort(rng.uniform(100, 600, 12)), 3)
        order.append((nm, mz, np.ones(12), 400.0 + k, k))
    for k in (1, 3):  # make some members similar so the choice is non-trivial
        order[k] = (order[k][0], order[0][1].copy(), np.ones(12), order[k][3], k)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "in.mgf")
        _write_medoid_mgf(path, order)
        reps = _run_medoid_main(msr, path)
        with open(path) as fh:
            mgf_text = fh.read()
    with open(os.path.join(HERE, "medoid_noncontiguous.mgf"), "w") as fh:
        fh.write(mgf_text)
    with open(os.path.join(HERE, "medoid_noncontiguous.json"), "w") as fh:
        json.dump({"names": names, "rep_index": [r[0] for r in reps], "titles": [r[1] for r in reps]}, fh, indent=1)
    print("medoid_noncontiguous:", reps)


def gen_pairwise():
    """numpy/pandas pairwise-summation tree (what `.iloc[i,:].sum()` evaluates,
    most_similar_representative.py:98-100): random vectors with zeros kept in
    place, several lengths crossing the n<8 / n<=128 / recursive-split regimes."""
    import pandas as pd

    rng = np.random.default_rng(44)
    lens = [1, 2, 5, 7, 8, 9, 15, 16, 17, 31, 64, 127, 128, 129, 130, 200, 255, 256, 257, 300, 1000, 1031, 4097]
    vals, offs, sums_np, sums_pd = [], [0], [], []
    for n in lens:
        v = rng.random(n) * (10.0 ** rng.uniform(-3, 3, n))
        v[rng.random(n) < 0.3] = 0.0
        vals.append(v)
        offs.append(offs[-1] + n)
        sums_np.append(np.add.reduce(v))
        m = np.zeros((n, n))
        m[0, :] = v
        sums_pd.append(pd.DataFrame(m).iloc[0, :].sum())
    assert all(a == b for a, b in zip(sums_np, sums_pd))
    np.savez_compressed(os.path.join(HERE, "pairwise_sum.npz"), off=np.array(offs, np.int64),
                        vals=np.concatenate(vals), sums=np.array(sums_np))
    print("pairwise_sum: ok")


def binned_cosine_cases(rng):
    """Representative + members per cluster: synthetic clusters with a member
    or a jittered copy as the representative, plus the binning edge cases."""
    import importlib
    bench = importlib.import_module("benchmark")
    s = bench.mz_space
    start = -s / 2.
    clusters, reps = [], []
    csr = make_clusters_np(40, seed=31, n_template=120)
    for c in range(csr.n_clusters):
        spectra = []
        for k in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            a, b = csr.spec_off[k], csr.spec_off[k + 1]
            spectra.append((csr.mz[a:b].copy(), csr.inten[a:b].copy()))
        clusters.append(spectra)
        if c % 3 == 0:
            reps.append(spectra[0])
        else:  # a consensus-like representative: jittered, re-sorted
            mz = np.sort(np.round(spectra[-1][0] + rng.normal(0, 0.002, len(spectra[-1][0])), 5))
            reps.append((mz, np.round(rng.lognormal(5, 1, len(mz)), 2)))

    def edge(i):  # np.arange's i-th value (numpy DOUBLE_fill)
        return start if i == 0 else (start + s if i == 1 else start + i * ((start + s) - start))

    # on the rightmost edge: the pair's max m/z puts a member peak within 1e-9 of the last edge
    M = 1500.0
    L = int(np.ceil((M - start) / s))
    e_last = edge(L - 1)
    rep = (np.array([100.0, 700.5, 1200.25, M]), np.array([10.0, 20.0, 30.0, 40.0]))
    mem = (np.array([100.001, 700.501, e_last, e_last + 3e-9, e_last + 2e-7]), np.array([1.0, 2.0, 3.0, 4.0, 5.0]))
    clusters.append([mem, rep])
    reps.append(rep)
    # peaks sharing bins (sum order), a peak at 0.0 and one below the first edge
    clusters.append([(np.array([-0.01, 0.0, 0.001, 0.002, 500.0, 500.001]), np.array([1., 2., 3., 4., 5., 6.])),
                     (np.array([0.0005, 500.0004]), np.array([7., 8.]))])
    reps.append((np.array([0.0, 0.0015, 500.0, 800.0]), np.array([2.0, 3.0, 5.0, 1.0])))
    # no shared bin (0.0), zero intensities (a == 0 -> 0.0), identical spectra (1.0)
    clusters.append([(np.array([300.0, 400.0]), np.array([1.0, 1.0])),
                     (np.array([200.0, 250.0]), np.array([0.0, 0.0])),
                     (np.array([200.0, 250.0, 900.0]), np.array([3.0, 4.0, 5.0]))])
    reps.append((np.array([200.0, 250.0, 900.0]), np.array([3.0, 4.0, 5.0])))
    # unsorted member and unsorted representative
    clusters.append([(np.array([900.0, 200.0, 250.0, 200.001]), np.array([5.0, 3.0, 4.0, 1.0]))])
    reps.append((np.array([250.0, 200.0, 900.0, 200.002]), np.array([4.0, 3.0, 5.0, 2.0])))
    # no members (average 0.0), an empty member (IndexError)
    clusters.append([])
    reps.append((np.array([100.0]), np.array([1.0])))
    clusters.append([(np.array([100.0]), np.array([1.0])), (np.zeros(0), np.zeros(0))])
    reps.append((np.array([100.0]), np.array([1.0])))
    return bench, clusters, reps


def gen_binned_cosine():
    from types import SimpleNamespace

    rng = np.random.default_rng(17)
    bench, clusters, reps = binned_cosine_cases(rng)
    cos, avg, status = [], [], []
    for spectra, (rm, ri) in zip(clusters, reps):
        rep = SimpleNamespace(mz=rm, intensity=ri)
        members = [SimpleNamespace(mz=m, intensity=i) for m, i in spectra]
        try:
            cs = [bench.cos_dist(rep, mem) for mem in members]
            avg.append(bench.average_cos_dist(rep, members))
            cos.extend(cs)
            status.append(STATUS_OK)
        except IndexError:  # mz[-1] of an empty spectrum (benchmark.py:20)
            cos.extend([np.nan] * len(spectra))
            avg.append(np.nan)
            status.append(STATUS_EMPTY)
    csr = SpectraCSR.from_clusters([[{"m/z array": m, "intensity array": i} for m, i in sp] for sp in clusters])
    rep_off = np.zeros(len(reps) + 1, np.int64)
    np.cumsum([len(r[0]) for r in reps], out=rep_off[1:])
    np.savez_compressed(os.path.join(HERE, "binned_cosine.npz"), **_csr_arrays(csr),
                        rep_off=rep_off, rep_mz=np.concatenate([r[0] for r in reps]),
                        rep_int=np.concatenate([r[1] for r in reps]), mz_space=np.float64(bench.mz_space),
                        cos=np.array(cos, np.float64), avg=np.array(avg, np.float64),
                        status=np.array(status, np.int32))
    print(f"binned_cosine: {len(clusters)} clusters, {len(cos)} members")


# ----------------------------------------------------------- best spectrum
def best_spectrum_cases(rng):
    """An MGF of clusters (members interleaved across the file) and a MaxQuant
    msms.txt: duplicate PSMs per scan, NaN scores, unscored members, equal
    scores across USIs (ties: first USI in string order, 'scan:10' < 'scan:9')."""
    raws = ["runB", "runA", "run_10", "run_9"]
    spectra, rows = [], []
    n_clusters = 60
    members = {c: [] for c in range(n_clusters)}
    scan = 0
    for c in range(n_clusters):
        for _ in range(int(rng.integers(1, 9))):
            members[c].append((raws[int(rng.integers(0, len(raws)))], scan))
            scan += int(rng.integers(1, 4))
    order = [(c, r, sc) for c in members for r, sc in members[c]]
    perm = rng.permutation(len(order))  # non-contiguous clusters
    order = [order[i] for i in perm]
    for c, r, sc in order:
        npk = int(rng.integers(1, 5))
        mz = np.sort(np.round(rng.uniform(100, 1500, npk), 4))
        it = np.round(rng.lognormal(4, 1, npk), 2)
        spectra.append((f"cluster-{c}", f"mzspec:PXD004732:{r}.raw::scan:{sc}", mz, it,
                        float(np.round(rng.uniform(400, 1200), 4)), int(rng.integers(2, 4)),
                        float(np.round(rng.uniform(0, 3600), 3))))
        kind = c % 6
        if kind == 0:  # unscored cluster -> skipped (ValueError)
            continue
        k = int(rng.integers(0, 4))
        for _ in range(k if kind != 5 else max(k, 1)):
            v = float(rng.integers(0, 4)) * 10.0  # few distinct values: many ties
            if kind == 4 and rng.random() < 0.5:
                v = float("nan")
            rows.append((r, sc, v))
    # a cluster whose PSM scores are all NaN crashes the reference (KeyError, pinned
    # separately below): give every scored cluster one real score
    usi_cluster = {(r, sc): c for c, r, sc in order}
    real = {usi_cluster[(r, sc)] for r, sc, v in rows if v == v}
    for c in sorted({usi_cluster[(r, sc)] for r, sc, _ in rows} - real):
        rows.append((members[c][0][0], members[c][0][1], 20.0))
    # PSMs for scans that are in no cluster
    rows += [("runZ", 99999, 50.0), ("runA", 88888, float("nan"))]
    rows = [rows[i] for i in rng.permutation(len(rows))]
    return spectra, rows


def _write_best_inputs(spectra, rows, mgf_path, msms_path):
    with open(mgf_path, "w") as fh:
        for cl, usi, mz, it, pm, z, rt in spectra:
            fh.write(f"BEGIN IONS\nTITLE={cl};{usi}\nPEPMASS={pm!r}\nCHARGE={z}+\nRTINSECONDS={rt!r}\n")
            fh.write("".join(f"{float(a)!r} {float(b)!r}\n" for a, b in zip(mz, it)))
            fh.write("END IONS\n\n")
    with open(msms_path, "w") as fh:
        fh.write("Raw file\tScan number\tSequence\tScore\n")
        for r, sc, v in rows:
            fh.write(f"{r}\t{sc}\tPEPTIDEK\t{'NaN' if v != v else repr(v)}\n")


def gen_best_spectrum():
    import importlib
    from types import SimpleNamespace

    from specpride_amd.mgf import iter_mgf

    bs = importlib.import_module("best_spectrum")
    written = []
    # pyteomics.mgf is absent: its reader is replaced by the build's (parse parity is
    # not what this pins); write() captures the reference's spectrum dicts
    bs.mgf = SimpleNamespace(read=lambda fn: iter_mgf(fn), write=lambda sp, fh: written.extend(sp))
    rng = np.random.default_rng(23)
    spectra, rows = best_spectrum_cases(rng)
    mgf_path = os.path.join(HERE, "best_spectrum_in.mgf")
    msms_path = os.path.join(HERE, "best_spectrum_msms.txt")
    _write_best_inputs(spectra, rows, mgf_path, msms_path)
    with tempfile.TemporaryDirectory() as td:
        bs.best_spectrum(mgf_path, os.path.join(td, "out.mgf"), msms_path)
    out = [{"title": d["params"]["title"], "pepmass": float(d["params"]["pepmass"]),
            "rtinseconds": float(d["params"]["rtinseconds"]), "charge": int(d["params"]["charge"]),
            "mz": [float(x) for x in d["m/z array"]], "intensity": [float(x) for x in d["intensity array"]]}
           for d in written]
    # per cluster (split_into_clusters order): the chosen USI or the exception type
    scores = bs.get_scores(msms_path)
    per_cluster = []
    for cl in bs.split_into_clusters(bs.get_cluster_spectra(mgf_path)):
        try:
            per_cluster.append(bs.get_best_representative(cl, scores).identifier)
        except ValueError:
            per_cluster.append("ValueError")
    # a cluster whose only PSM scores are NaN: idxmax -> nan, spectra[nan] -> KeyError
    nan_cluster = {u: SimpleNamespace(identifier=u) for u in ["mzspec:PXD004732:runA.raw::scan:88888"]}
    try:
        bs.get_best_representative(nan_cluster, scores)
        nan_case = "no error"
    except KeyError:
        nan_case = "KeyError"
    with open(os.path.join(HERE, "best_spectrum.json"), "w") as fh:
        json.dump({"output": out, "per_cluster": per_cluster, "nan_only_cluster": list(nan_cluster),
                   "nan_only_result": nan_case}, fh, indent=0)
    print(f"best_spectrum: {len(per_cluster)} clusters, {len(out)} representatives, nan case {nan_case}")


# ------------------------------------------------ MaRaCluster / convert_mgf_cluster
MARA_TSV = ("run.raw\t11\t0.5\nrun.raw\t3\t0.5\nrun.raw\t7\t0.1\n\n"
            "run.raw\t5\t0.2\n\n\nrun.raw\t012\t0.3\nrun.raw\t1\t0.3\n\n"
            "run.raw\t20\t0.9\nrun.raw\t21\t0.9\n")  # double blank line; last cluster has no blank after it
MSMS_TXT = ("Raw file\tScan number\tx\ty\tz\tw\tv\tModified sequence\tScore\n"
            "run\t11\ta\tb\tc\td\te\t_PEPTIDEK_\t50\n"
            "run\t5\ta\tb\tc\td\te\t_M(ox)AAK_\t20\n"
            "run\t11\ta\tb\tc\td\te\t_OTHERR_\t40\n"
            "run\t20\ta\tb\tc\td\te\t_LASTK_\t10\n")


def gen_maracluster(binning):
    import importlib
    from types import SimpleNamespace

    from specpride_amd.mgf import iter_mgf

    cmc = importlib.import_module("convert_mgf_cluster")
    tsv = os.path.join(HERE, "maracluster_clusters.tsv")
    msms = os.path.join(HERE, "maracluster_msms.txt")
    mgf_in = os.path.join(HERE, "maracluster_in.mgf")
    with open(tsv, "w") as fh:
        fh.write(MARA_TSV)
    with open(msms, "w") as fh:
        fh.write(MSMS_TXT)
    rng = np.random.default_rng(41)
    with open(mgf_in, "w") as fh:  # scans 1..21 plus a duplicate title and a 'xscan=5' look-alike
        for scan in list(range(1, 22)) + [11, 55]:
            title = f"run.{scan}.{scan}.2 File:run.raw, NativeID:controllerType=0 controllerNumber=1 scan={scan}"
            if scan == 55:
                title = "run.55 NativeID:xscan=5"
            mz = np.sort(np.round(rng.uniform(150, 1400, 4), 4))
            fh.write(f"BEGIN IONS\nTITLE={title}\nPEPMASS={500 + scan}.25\nCHARGE={2 + scan % 2}+\n")
            fh.write("".join(f"{a!r} {b!r}\n" for a, b in zip(mz, np.round(rng.lognormal(4, 1, 4), 2))))
            fh.write("END IONS\n\n")
    written = []
    cmc.mgf = SimpleNamespace(read=lambda fn: iter_mgf(fn), write=lambda sp, out: written.extend(sp))
    with contextlib.redirect_stdout(io.StringIO()):
        cmc.convert_mq_mracluster_mgf.callback(msms, tsv, mgf_in, "unused.mgf", "PXD000001", "run")
    rsc = binning.RepresentativeSpectrumCreator(verbose=0)
    g = {"read_cluster_list": rsc.read_cluster_list(tsv),
         "read_clusters": {str(k): v for k, v in cmc.read_clusters(tsv).items()},
         "read_peptides": {str(k): v for k, v in cmc.read_peptides(msms).items()},
         "usi": [cmc.buid_usi_accession("cluster-3", None, 7, "PXD1", "raw", 2),
                 cmc.buid_usi_accession("cluster-3", "PEPK", 7, "PXD1", "raw", 2)],
         "converted_titles": [sp["params"]["title"] for sp in written],
         "converted_pepmass": [float(sp["params"]["pepmass"][0]) for sp in written]}
    with open(os.path.join(HERE, "maracluster.json"), "w") as fh:
        json.dump(g, fh, indent=0)
    print(f"maracluster: {len(g['read_cluster_list'])} clusters, {len(written)} converted spectra")


def main():
    if not os.path.isdir(REF_SRC):
        raise SystemExit("reference not present; fixtures are committed under tests/golden/")
    binning, asc, msr = _import_reference()
    if sys.argv[1:] == ["best_spectrum"]:  # regenerate one set only
        gen_best_spectrum()
        return
    if sys.argv[1:] == ["maracluster"]:
        gen_maracluster(binning)
        return
    if sys.argv[1:] == ["nonfinite"]:
        gen_nonfinite(binning, asc)
        return
    gen_bin_mean(binning)
    gen_bin_mean_cli()
    gen_gap_average(asc)
    gen_nonfinite(binning, asc)
    gen_precursor_helpers(asc)
    gen_pairwise()
    gen_medoid(msr)
    gen_binned_cosine()
    gen_best_spectrum()
    gen_maracluster(binning)


if __name__ == "__main__":
    main()
