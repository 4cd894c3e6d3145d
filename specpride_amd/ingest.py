"""Native MGF ingest straight to the cluster-segmented CSR, for the three CLIs
(SURVEY.md §8(f) ranks 1-3), single-process and rank-local.

Each CLI groups spectra into clusters its own way; the groupings are restated
here over title lists so they can run on an index (titles + byte ranges, no
numbers parsed) as well as on a full parse:

* bin-mean (binning.py:122-167): cluster id = ``title.split(';')[0]``, clusters
  in first-appearance order, members merged wherever they appear, in file order.
* gap-average (average_spectrum_clustering.py:151-165): ``itertools.groupby`` of
  consecutive records by ``get_cluster_id(title)`` -- a split cluster yields
  several runs.
* medoid (most_similar_representative.py:49-75): names in first-appearance order,
  each the FIRST contiguous run at or after the previous cluster's run
  (:func:`specpride_amd.most_similar_representative._first_runs`).

Each returns ``(ids, records, sizes)``: cluster ids, the record indices in CSR
order (cluster-major) and the member count per cluster.
"""
from __future__ import annotations

from itertools import groupby

import numpy as np

from .csr import SpectraCSR, concat_ranges


def binning_groups(titles):
    order, cl = {}, np.empty(len(titles), np.int64)
    for i, t in enumerate(titles):
        cl[i] = order.setdefault(t.split(";")[0], len(order))
    records = np.argsort(cl, kind="stable")
    return list(order.keys()), records, np.bincount(cl, minlength=len(order)).astype(np.int64)


def gap_average_groups(titles):
    ids, sizes = [], []
    for cid, grp in groupby(titles, lambda t: t.split(";", 1)[0]):
        ids.append(cid)
        sizes.append(sum(1 for _ in grp))
    return ids, np.arange(len(titles), dtype=np.int64), np.asarray(sizes, np.int64)


def medoid_groups(titles):
    from .most_similar_representative import _first_runs

    runs = [(cl, m) for cl, m in _first_runs([t.split(";")[0] for t in titles]) if m]
    records = np.asarray([i for _cl, m in runs for i in m], np.int64)
    return [cl for cl, _m in runs], records, np.asarray([len(m) for _cl, m in runs], np.int64)


def csr_from_flat(flat: dict, sizes, records=None) -> SpectraCSR:
    """Pack a native parse (``mgf_native`` flat dict) into a CSR whose clusters
    have ``sizes`` members taken in ``records`` order (None = parse order)."""
    so = flat["spec_off"]
    sizes = np.asarray(sizes, np.int64)
    cluster_off = np.zeros(len(sizes) + 1, np.int64)
    np.cumsum(sizes, out=cluster_off[1:])
    rt = flat.get("rt")
    if records is None:
        S = len(so) - 1
        rt = rt if rt is not None else np.full(S, np.nan)
        return SpectraCSR(cluster_off, so, flat["mz"], flat["inten"], flat["prec_mz"],
                          flat["charge"].astype(np.int32), rt)
    records = np.asarray(records, np.int64)
    lens = so[records + 1] - so[records]
    spec_off = np.zeros(len(records) + 1, np.int64)
    np.cumsum(lens, out=spec_off[1:])
    idx = concat_ranges(so[records], lens)
    rt = rt[records] if rt is not None else np.full(len(records), np.nan)
    return SpectraCSR(cluster_off, spec_off, flat["mz"][idx], flat["inten"][idx], flat["prec_mz"][records],
                      flat["charge"][records].astype(np.int32), rt)


def cluster_starts(sizes) -> np.ndarray:
    off = np.zeros(len(sizes) + 1, np.int64)
    np.cumsum(sizes, out=off[1:])
    return off
