"""ctypes front-end of oracle/build/libspx_oracle.so.  TEST INFRASTRUCTURE ONLY
(see spx_oracle.c's header: tests/, smoke() and bench.py's cpu_baseline only)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libspx_oracle.so")
_lib = None

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_dbl = ctypes.c_double


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.spxo_pairwise_sum.restype = _dbl
        _lib.spxo_pairwise_sum.argtypes = [_p, _i64]
        _lib.spxo_bin_mean.argtypes = [_i64, _p, _p, _p, _p, _p, _p, _dbl, _dbl, _dbl, ctypes.c_int,
                                       _p, _p, _p, _p, _p, _p]
        _lib.spxo_gap_average.argtypes = [_i64, _p, _p, _p, _p, _dbl, _dbl, _dbl, _p, _p, _p, _p]
        _lib.spxo_medoid.argtypes = [_i64, _p, _p, _p, _dbl, ctypes.c_int, _p, _p]
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def pairwise_sum(v) -> float:
    v = np.ascontiguousarray(v, np.float64)
    return lib().spxo_pairwise_sum(_ptr(v), len(v))


def bin_mean(csr, minimum=100.0, maximum=2000.0, binsize=0.02, apply_peak_quorum=True):
    C = csr.n_clusters
    out_off = np.zeros(C + 1, np.int64)
    cap = max(1, csr.n_peaks)
    out_mz, out_int = np.empty(cap), np.empty(cap)
    prec, charge, status = np.empty(C), np.zeros(C, np.int32), np.zeros(C, np.int32)
    rc = lib().spxo_bin_mean(C, _ptr(csr.cluster_off), _ptr(csr.spec_off), _ptr(csr.mz), _ptr(csr.inten),
                             _ptr(csr.prec_mz), _ptr(csr.charge), float(minimum), float(maximum),
                             float(binsize), int(bool(apply_peak_quorum)), _ptr(out_off), _ptr(out_mz),
                             _ptr(out_int), _ptr(prec), _ptr(charge), _ptr(status))
    if rc:
        raise MemoryError("spxo_bin_mean")
    n = out_off[-1]
    return dict(out_off=out_off, out_mz=out_mz[:n].copy(), out_int=out_int[:n].copy(), prec=prec,
                charge=charge, status=status)


def gap_average(csr, mz_accuracy=0.01, dyn_range=1000.0, min_fraction=0.5):
    C = csr.n_clusters
    out_off = np.zeros(C + 1, np.int64)
    cap = max(1, csr.n_peaks)
    out_mz, out_int, status = np.empty(cap), np.empty(cap), np.zeros(C, np.int32)
    rc = lib().spxo_gap_average(C, _ptr(csr.cluster_off), _ptr(csr.spec_off), _ptr(csr.mz), _ptr(csr.inten),
                                float(mz_accuracy), float(dyn_range), float(min_fraction), _ptr(out_off),
                                _ptr(out_mz), _ptr(out_int), _ptr(status))
    if rc:
        raise MemoryError("spxo_gap_average")
    n = out_off[-1]
    return dict(out_off=out_off, out_mz=out_mz[:n].copy(), out_int=out_int[:n].copy(), status=status)


def medoid(csr, tol=0.1, dense_tables=False, with_totals=False):
    rep = np.zeros(csr.n_clusters, np.int64)
    totals = np.zeros(max(1, csr.n_spectra)) if with_totals else None
    rc = lib().spxo_medoid(csr.n_clusters, _ptr(csr.cluster_off), _ptr(csr.spec_off), _ptr(csr.mz), float(tol),
                           int(bool(dense_tables)), _ptr(rep), _ptr(totals) if with_totals else None)
    if rc:
        raise MemoryError("spxo_medoid")
    return (rep, totals[:csr.n_spectra]) if with_totals else rep


def medoid_parallel(csr, tol=0.1, with_totals=False, threads=None):
    """:func:`medoid` over cluster chunks in a thread pool (ctypes releases the GIL
    during the C call): the same per-cluster results, for large test batches."""
    from concurrent.futures import ThreadPoolExecutor

    C = csr.n_clusters
    threads = threads or min(16, os.cpu_count() or 1)
    sizes = np.diff(csr.cluster_off).astype(np.float64)
    cost = np.cumsum(sizes * sizes + 1.0)
    bounds = np.searchsorted(cost, np.linspace(0, cost[-1] if C else 0, 4 * threads + 1)[1:-1])
    edges = np.unique(np.concatenate([[0], bounds, [C]])).astype(np.int64)
    # the largest clusters on their own, first: they bound the wall time
    order = np.argsort(-sizes)[:threads]
    chunks = [np.array([c]) for c in order]
    rest = np.setdiff1d(np.arange(C), order)
    for a, b in zip(edges[:-1], edges[1:]):
        part = rest[(rest >= a) & (rest < b)]
        if len(part):
            chunks.append(part)
    rep = np.zeros(C, np.int64)
    totals = np.zeros(csr.n_spectra) if with_totals else None

    def run(cl):
        sub = csr.select(cl)
        r = medoid(sub, tol, with_totals=with_totals)
        return cl, sub, r

    with ThreadPoolExecutor(threads) as ex:
        for cl, sub, r in ex.map(run, chunks):
            rr, tt = (r if with_totals else (r, None))
            base = csr.cluster_off[cl]
            rep[cl] = np.where(rr >= 0, rr - sub.cluster_off[:-1] + base, rr)
            if with_totals:
                from specpride_amd.csr import concat_ranges

                totals[concat_ranges(base, np.diff(sub.cluster_off))] = tt
    return (rep, totals) if with_totals else rep
