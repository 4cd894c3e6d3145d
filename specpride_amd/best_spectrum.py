"""Drop-in for the reference's ``src/best_spectrum.py`` (score-based
representative) on the MI355X engine (``spx_best_score``).

Same names, argument meanings and errors as the reference:

* :func:`get_cluster_spectra` (best_spectrum.py:10-40) -- MGF -> ``{usi: spectrum}``;
  ``ValueError`` on a non-unique USI, the title must be ``<cluster>;<usi>``;
* :func:`get_scores` (:43-64) -- MaxQuant ``msms.txt`` -> USI-sorted score Series
  (pandas, as in the reference; the PXD accession is hard-coded there too);
* :func:`get_best_representative` (:67-100) -- ``ValueError`` if no member has a
  score; ties go to the first USI in sorted order (``idxmax``);
* :func:`split_into_clusters` (:126-148), :func:`write_mgf` (:103-123),
  :func:`best_spectrum` (:151-175) and the three-argument CLI (:178-179).

:func:`best_representatives` evaluates every cluster of a file in ONE device
call: the host folds the score join into per-spectrum (score, rank) arrays
(``rank`` = the USI's position among the sorted distinct score USIs) and the
kernel does the segmented argmax.  When every matching score of a cluster is
NaN, pandas' ``idxmax`` returns NaN and the reference's ``spectra[nan]`` raises
``KeyError`` -- reproduced here.

``spectrum_utils`` is not installed offline: :class:`MsmsSpectrum` is a plain
container with the attributes the reference reads (identifier, precursor_mz,
precursor_charge, mz, intensity, retention_time, cluster).
"""
from __future__ import annotations

import collections
import sys
from typing import Dict, Iterable, List

import numpy as np

from . import engine
from .mgf import iter_mgf, write_pyteomics_style


class MsmsSpectrum:
    """The fields of ``spectrum_utils.spectrum.MsmsSpectrum`` the reference uses."""

    def __init__(self, identifier, precursor_mz, precursor_charge, mz, intensity, retention_time=None):
        self.identifier = identifier
        self.precursor_mz = precursor_mz
        self.precursor_charge = precursor_charge
        self.mz = np.asarray(mz, np.float64)
        self.intensity = np.asarray(intensity, np.float64)
        self.retention_time = retention_time
        self.cluster = None


def get_cluster_spectra(mgf_filename: str) -> Dict[str, MsmsSpectrum]:
    """best_spectrum.py:10-40: ``{usi: spectrum}`` in file order."""
    spectra = {}
    for spectrum_dict in iter_mgf(mgf_filename):
        params = spectrum_dict["params"]
        cluster, usi = params["title"].split(";")
        spectrum = MsmsSpectrum(usi, params["pepmass"][0], params["charge"][0], spectrum_dict["m/z array"],
                                spectrum_dict["intensity array"], retention_time=params["rtinseconds"])
        spectrum.cluster = cluster
        if usi in spectra:
            raise ValueError(f"Non-unique USI: {usi}")
        spectra[usi] = spectrum
    return spectra


def get_scores(score_filename: str):
    """best_spectrum.py:43-64: MaxQuant msms.txt -> Series(Score, index=USI), sorted."""
    import pandas as pd

    scores = pd.read_csv(score_filename, sep="\t", usecols=["Raw file", "Scan number", "Score"])
    scores["usi"] = ("mzspec:PXD004732:" + scores["Raw file"] + ".raw::scan:" + scores["Scan number"].astype(str))
    scores = scores.set_index("usi")
    return scores["Score"].sort_index()


def _score_arrays(usis: List[str], scores):
    """Per spectrum: (max non-NaN PSM score, rank of its USI among the sorted
    distinct score USIs or -1).  The Series filter + idxmax of :97-100 become a
    segmented argmax over (score desc, rank asc)."""
    per_usi = scores.groupby(level=0, sort=True).max()  # NaN-skipping max; sorted distinct USIs
    pos = per_usi.index.get_indexer(usis) if len(usis) else np.zeros(0, np.int64)
    pos = np.asarray(pos, np.int64)
    vals = np.asarray(per_usi.to_numpy(dtype=np.float64, na_value=np.nan), np.float64)
    score = np.where(pos >= 0, vals[np.maximum(pos, 0)] if len(vals) else np.nan, np.nan).astype(np.float64)
    return score, pos


def best_representatives(clusters: List[Dict[str, MsmsSpectrum]], scores, device="cuda"):
    """[get_best_representative(cluster, scores) for cluster in clusters] from ONE
    engine call.  Returns a list with the chosen spectrum, or None where the
    reference raises ValueError (no member has a score)."""
    import torch

    usis = [u for cl in clusters for u in cl]
    off = np.zeros(len(clusters) + 1, np.int64)
    np.cumsum([len(cl) for cl in clusters], out=off[1:])
    score, rank = _score_arrays(usis, scores)
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=device)  # noqa: E731
    res = engine.best_score(dev(off), dev(score if len(score) else np.zeros(1)),
                            dev(rank if len(rank) else np.full(1, -1, np.int64)))
    best, status = res.to_host()
    flat = [sp for cl in clusters for sp in cl.values()]
    out = []
    for c in range(len(clusters)):
        st = int(status[c])
        if st == engine.STATUS_OK:
            out.append(flat[int(best[c])])
        elif st == engine.STATUS_EMPTY:
            out.append(None)
        else:  # only NaN scores: idxmax() -> nan, spectra[nan] (best_spectrum.py:100)
            raise KeyError(np.nan)
    return out


def get_best_representative(spectra: Dict[str, MsmsSpectrum], scores) -> MsmsSpectrum:
    """best_spectrum.py:67-100 for one cluster."""
    rep = best_representatives([spectra], scores)[0]
    if rep is None:
        raise ValueError("No scores found for the given scan numbers")
    return rep


def write_mgf(filename: str, spectra: List[MsmsSpectrum]) -> None:
    """best_spectrum.py:103-123 (pyteomics ``mgf.write`` text format: unpinned, A.5)."""
    write_pyteomics_style(
        ({"m/z array": s.mz, "intensity array": s.intensity,
          "params": {"title": f"{s.cluster};{s.identifier}", "pepmass": s.precursor_mz,
                     "rtinseconds": s.retention_time, "charge": s.precursor_charge}} for s in spectra),
        filename)


def split_into_clusters(spectra: Dict[str, MsmsSpectrum]) -> Iterable[Dict[str, MsmsSpectrum]]:
    """best_spectrum.py:126-148: clusters in first-appearance order, members in file order."""
    clusters = collections.defaultdict(list)
    for spectrum in spectra.values():
        clusters[spectrum.cluster].append(spectrum.identifier)
    for cluster_members in clusters.values():
        yield {usi: spectra[usi] for usi in cluster_members}


def best_spectrum(mgf_in_filename: str, mgf_out_filename: str, scores_filename: str) -> None:
    """best_spectrum.py:151-175: every cluster's highest-scoring member, one device pass."""
    scores = get_scores(scores_filename)
    spectra = get_cluster_spectra(mgf_in_filename)
    reps = best_representatives(list(split_into_clusters(spectra)), scores)
    write_mgf(mgf_out_filename, [r for r in reps if r is not None])


if __name__ == "__main__":
    best_spectrum(sys.argv[1], sys.argv[2], sys.argv[3])
