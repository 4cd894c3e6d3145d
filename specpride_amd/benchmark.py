"""Drop-in for the reference's evaluation module ``src/benchmark.py`` (binned
cosine, benchmark.py:7-38) on the MI355X engine (``spx_binned_cosine``).

Same names and argument meanings as the reference: spectra are objects with
``.mz`` and ``.intensity`` arrays (spectrum_utils ``MsmsSpectrum`` or anything
alike).  ``cos_dist`` / ``average_cos_dist`` evaluate one representative;
``average_cos_dist_batch`` evaluates every cluster of a file in one device pass.
An empty spectrum raises IndexError, as the reference's ``mz[-1]`` does.
``fraction_of_by`` (spectrum_utils peptide annotation) is outside the engine's
scope.
"""
from __future__ import annotations

import numpy as np

from . import engine
from .csr import SpectraCSR

mz_unit = 1.000508         # benchmark.py:7
mz_space = mz_unit * .005  # benchmark.py:8


def _arrays(spec):
    return np.asarray(spec.mz, np.float64), np.asarray(spec.intensity, np.float64)


def average_cos_dist_batch(representatives, clusters, mz_space=mz_space, device="cuda"):
    """[average_cos_dist(representatives[c], clusters[c]) for every c] and the
    per-member cosines, from ONE engine call.  Returns (avg [C], cos: list of
    per-cluster arrays)."""
    import torch

    csr = SpectraCSR.from_clusters([[{"m/z array": _arrays(s)[0], "intensity array": _arrays(s)[1]} for s in cl]
                                    for cl in clusters])
    reps = [_arrays(r) for r in representatives]
    if len(reps) != csr.n_clusters:
        raise ValueError("one representative per cluster")
    rep_off = np.zeros(len(reps) + 1, np.int64)
    np.cumsum([len(m) for m, _ in reps], out=rep_off[1:])
    rep_mz = np.concatenate([m for m, _ in reps]) if reps else np.zeros(0)
    rep_int = np.concatenate([i for _, i in reps]) if reps else np.zeros(0)
    batch = engine.DeviceBatch.from_host(csr, device=device)
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=device)  # noqa: E731
    t_off, t_mz, t_int = dev(rep_off), dev(rep_mz if len(rep_mz) else np.zeros(1)), dev(
        rep_int if len(rep_int) else np.zeros(1))
    cos, avg, status = engine.binned_cosine(batch, t_off, t_mz, t_int, mz_space=mz_space).to_host()
    for c, st in enumerate(status[:csr.n_clusters]):
        if st == engine.STATUS_EMPTY:
            raise IndexError("index -1 is out of bounds for axis 0 with size 0")  # benchmark.py:20 mz[-1]
        if st != engine.STATUS_OK:
            raise RuntimeError(f"cluster {c}: binned cosine unresolved (status {st})")
    return avg[:csr.n_clusters], [cos[csr.cluster_off[c]:csr.cluster_off[c + 1]] for c in range(csr.n_clusters)]


def cos_dist(representative_spectrum, cluster_member):
    """benchmark.py:19-29: binned cosine of a representative and one member."""
    _, cos = average_cos_dist_batch([representative_spectrum], [[cluster_member]])
    return float(cos[0][0])


def average_cos_dist(representative_spectrum, cluster_members):
    """benchmark.py:31-38: mean cosine of the representative to the members (0.0 if none)."""
    avg, _ = average_cos_dist_batch([representative_spectrum], [list(cluster_members)])
    return float(avg[0])
