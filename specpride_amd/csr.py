"""Cluster-segmented CSR batch: the one data layout every kernel consumes.

Layout (SURVEY.md §8(b) "C-ABI the engine exports")::

    cluster_off[C+1]  int64   offsets into spectra  (cluster c = spectra [cluster_off[c], cluster_off[c+1]))
    spec_off[S+1]     int64   offsets into peaks    (spectrum s = peaks  [spec_off[s],  spec_off[s+1]))
    mz[P], inten[P]   float64 peaks in file order, NOT re-sorted
    prec_mz[S]        float64 precursor m/z
    charge[S]         int32   precursor charge
    rt[S]             float64 retention time (seconds; NaN if absent)

A host batch holds numpy arrays; :meth:`SpectraCSR.to_device` mirrors it into
torch tensors on a HIP device (torch is only used as the HBM allocator here).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np


def concat_ranges(starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """concatenate(arange(s, s + n) for s, n in zip(starts, lens)), vectorised."""
    starts = np.asarray(starts, np.int64)
    lens = np.asarray(lens, np.int64)
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    first = np.zeros(len(lens), np.int64)
    np.cumsum(lens[:-1], out=first[1:])
    return np.repeat(starts - first, lens) + np.arange(total, dtype=np.int64)


@dataclass
class SpectraCSR:
    cluster_off: np.ndarray
    spec_off: np.ndarray
    mz: np.ndarray
    inten: np.ndarray
    prec_mz: np.ndarray
    charge: np.ndarray
    rt: np.ndarray
    cluster_ids: list = field(default_factory=list)
    titles: list = field(default_factory=list)

    def __post_init__(self):
        self.cluster_off = np.ascontiguousarray(self.cluster_off, np.int64)
        self.spec_off = np.ascontiguousarray(self.spec_off, np.int64)
        self.mz = np.ascontiguousarray(self.mz, np.float64)
        self.inten = np.ascontiguousarray(self.inten, np.float64)
        self.prec_mz = np.ascontiguousarray(self.prec_mz, np.float64)
        self.charge = np.ascontiguousarray(self.charge, np.int32)
        self.rt = np.ascontiguousarray(self.rt, np.float64)
        self.validate()

    # ------------------------------------------------------------------ shape
    @property
    def n_clusters(self) -> int:
        return len(self.cluster_off) - 1

    @property
    def n_spectra(self) -> int:
        return len(self.spec_off) - 1

    @property
    def n_peaks(self) -> int:
        return len(self.mz)

    def validate(self) -> None:
        C, S, P = self.n_clusters, self.n_spectra, self.n_peaks
        if C < 0 or S < 0:
            raise ValueError("offset arrays must have at least one element")
        if self.cluster_off[0] != 0 or self.cluster_off[-1] != S:
            raise ValueError("cluster_off must start at 0 and end at n_spectra")
        if self.spec_off[0] != 0 or self.spec_off[-1] != P:
            raise ValueError("spec_off must start at 0 and end at n_peaks")
        if C and np.any(np.diff(self.cluster_off) < 0):
            raise ValueError("cluster_off must be non-decreasing")
        if S and np.any(np.diff(self.spec_off) < 0):
            raise ValueError("spec_off must be non-decreasing")
        if len(self.inten) != P:
            raise ValueError("mz and inten must have the same length")
        for name in ("prec_mz", "charge", "rt"):
            if len(getattr(self, name)) != S:
                raise ValueError(f"{name} must have n_spectra entries")

    # -------------------------------------------------------------- builders
    @classmethod
    def from_clusters(cls, clusters: Sequence[Sequence[dict]], cluster_ids: Sequence[str] | None = None,
                      mz_key="m/z array", int_key="intensity array", prec_key="precursor mz",
                      charge_key="precursor charge", rt_key=None, title_key=None) -> "SpectraCSR":
        """Pack nested python spectra (``clusters[c][s]`` dicts) into one batch.

        Missing precursor fields become NaN / 0 so packing never raises; the
        callers that need them (bin-mean's charge check) validate themselves."""
        sizes = np.fromiter((len(c) for c in clusters), np.int64, len(clusters))
        cluster_off = np.zeros(len(clusters) + 1, np.int64)
        np.cumsum(sizes, out=cluster_off[1:])
        flat = [s for c in clusters for s in c]
        lens = np.fromiter((len(s[mz_key]) for s in flat), np.int64, len(flat))
        spec_off = np.zeros(len(flat) + 1, np.int64)
        np.cumsum(lens, out=spec_off[1:])
        if flat and spec_off[-1]:
            mz = np.concatenate([np.asarray(s[mz_key], np.float64) for s in flat])
            inten = np.concatenate([np.asarray(s[int_key], np.float64) for s in flat])
        else:
            mz = np.zeros(0)
            inten = np.zeros(0)

        def _get(s, key, default):
            if key is None:
                return default
            v = s.get(key, default) if isinstance(s, dict) else default
            return default if v is None else v

        prec = np.array([float(_get(s, prec_key, np.nan)) for s in flat], np.float64)
        charge = np.array([int(_get(s, charge_key, 0)) for s in flat], np.int32)
        rt = np.array([float(_get(s, rt_key, np.nan)) for s in flat], np.float64)
        titles = [str(_get(s, title_key, "")) for s in flat] if title_key else []
        return cls(cluster_off, spec_off, mz, inten, prec, charge, rt,
                   cluster_ids=list(cluster_ids) if cluster_ids is not None else [],
                   titles=titles)

    # --------------------------------------------------------------- helpers
    def cluster_sizes(self) -> np.ndarray:
        return np.diff(self.cluster_off)

    def cluster_peaks(self) -> np.ndarray:
        return self.spec_off[self.cluster_off[1:]] - self.spec_off[self.cluster_off[:-1]]

    def spectrum(self, s: int):
        a, b = self.spec_off[s], self.spec_off[s + 1]
        return self.mz[a:b], self.inten[a:b]

    def cluster(self, c: int):
        """List of (mz, inten) views of cluster ``c``'s spectra."""
        return [self.spectrum(s) for s in range(self.cluster_off[c], self.cluster_off[c + 1])]

    def select(self, clusters: Iterable[int]) -> "SpectraCSR":
        """A new batch holding only ``clusters`` (in the given order)."""
        clusters = np.asarray(list(clusters) if not isinstance(clusters, np.ndarray) else clusters, np.int64)
        sizes = self.cluster_off[clusters + 1] - self.cluster_off[clusters]
        cluster_off = np.zeros(len(clusters) + 1, np.int64)
        np.cumsum(sizes, out=cluster_off[1:])
        spectra = concat_ranges(self.cluster_off[clusters], sizes)
        lens = self.spec_off[spectra + 1] - self.spec_off[spectra]
        spec_off = np.zeros(len(spectra) + 1, np.int64)
        np.cumsum(lens, out=spec_off[1:])
        idx = concat_ranges(self.spec_off[spectra], lens)
        ids = [self.cluster_ids[c] for c in clusters] if self.cluster_ids else []
        titles = [self.titles[s] for s in spectra] if self.titles else []
        return SpectraCSR(cluster_off, spec_off, self.mz[idx], self.inten[idx], self.prec_mz[spectra],
                          self.charge[spectra], self.rt[spectra], cluster_ids=ids, titles=titles)

    def to_device(self, device="cuda"):
        """Mirror the numeric arrays into torch tensors on ``device`` (HBM)."""
        import torch

        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return dict(cluster_off=t(self.cluster_off), spec_off=t(self.spec_off), mz=t(self.mz),
                    inten=t(self.inten), prec_mz=t(self.prec_mz), charge=t(self.charge), rt=t(self.rt),
                    n_clusters=self.n_clusters, n_spectra=self.n_spectra, n_peaks=self.n_peaks)

    @classmethod
    def from_device(cls, d: dict) -> "SpectraCSR":
        g = lambda k: d[k].detach().cpu().numpy()  # noqa: E731
        return cls(g("cluster_off"), g("spec_off"), g("mz"), g("inten"), g("prec_mz"), g("charge"), g("rt"))

    @staticmethod
    def select_on_device(d: dict, clusters, host_cluster_off=None, host_spec_off=None) -> dict:
        """A new DEVICE batch (the dict layout of :meth:`to_device`) holding only
        ``clusters`` (in the given order) of the device batch ``d``: offsets are
        rebuilt on the host from the (optionally passed) host offsets, the peaks and
        per-spectrum fields are gathered in HBM.  This is how a rank keeps its share
        of a batch every rank generated identically (bench.py strong scaling)."""
        import torch

        clusters = np.asarray(clusters, np.int64)
        co = d["cluster_off"].cpu().numpy() if host_cluster_off is None else np.asarray(host_cluster_off, np.int64)
        so = d["spec_off"].cpu().numpy() if host_spec_off is None else np.asarray(host_spec_off, np.int64)
        sizes = co[clusters + 1] - co[clusters]
        cluster_off = np.zeros(len(clusters) + 1, np.int64)
        np.cumsum(sizes, out=cluster_off[1:])
        spectra = concat_ranges(co[clusters], sizes)
        lens = so[spectra + 1] - so[spectra]
        spec_off = np.zeros(len(spectra) + 1, np.int64)
        np.cumsum(lens, out=spec_off[1:])
        dev = d["mz"].device
        idx = torch.from_numpy(concat_ranges(so[spectra], lens)).to(dev)
        sidx = torch.from_numpy(spectra).to(dev)
        out = {k: d[k].index_select(0, sidx) for k in ("prec_mz", "charge", "rt")}
        out["mz"] = d["mz"].index_select(0, idx)
        out["inten"] = d["inten"].index_select(0, idx)
        del idx
        out["cluster_off"] = torch.from_numpy(cluster_off).to(dev)
        out["spec_off"] = torch.from_numpy(spec_off).to(dev)
        out.update(n_clusters=len(clusters), n_spectra=len(spectra), n_peaks=int(spec_off[-1]))
        return out

    @classmethod
    def select_from_device(cls, d: dict, clusters) -> "SpectraCSR":
        """Host copy of only ``clusters`` (in the given order) of a device batch:
        the peaks are gathered on the device, so a batch of tens of GB need not
        cross PCIe to check a sample of it."""
        import torch

        clusters = np.asarray(clusters, np.int64)
        co = d["cluster_off"].cpu().numpy()
        so = d["spec_off"].cpu().numpy()
        sizes = co[clusters + 1] - co[clusters]
        cluster_off = np.zeros(len(clusters) + 1, np.int64)
        np.cumsum(sizes, out=cluster_off[1:])
        spectra = concat_ranges(co[clusters], sizes)
        lens = so[spectra + 1] - so[spectra]
        spec_off = np.zeros(len(spectra) + 1, np.int64)
        np.cumsum(lens, out=spec_off[1:])
        dev = d["mz"].device
        idx = torch.from_numpy(concat_ranges(so[spectra], lens)).to(dev)
        sidx = torch.from_numpy(spectra).to(dev)
        g = lambda k, i: d[k].index_select(0, i).cpu().numpy()  # noqa: E731
        return cls(cluster_off, spec_off, g("mz", idx), g("inten", idx), g("prec_mz", sidx), g("charge", sidx),
                   g("rt", sidx))

