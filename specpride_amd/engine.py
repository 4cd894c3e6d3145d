"""Batched device engine: the Python face of the C-ABI (include/specpride.h).

A :class:`DeviceBatch` holds one cluster-segmented CSR batch resident in HBM
(torch tensors are used purely as the allocator) plus the host-side facts the
workspace queries need.  :func:`bin_mean`, :func:`gap_average` and
:func:`medoid` enqueue the HIP kernels on the current torch stream and return
device-resident results; ``.to_host()`` packs them (device compaction, then
one D2H copy).

This module is the product path: it never imports the oracle and has no CPU
fallback -- without the HIP library it raises (see :mod:`specpride_amd._lib`).
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from .csr import SpectraCSR

STATUS_OK, STATUS_MIXED_CHARGE, STATUS_NO_GAP, STATUS_EMPTY, STATUS_NON_FINITE = 0, 1, 2, 3, 4
STATUS_UNRESOLVED = 100
PROTON = 1.00727646677  # pyteomics nist_mass['H+'][0][0] (average_spectrum_clustering.py:6)

PEPMASS_MODES = {"lower_median": 0, "naive_average": 1, "neutral_average": 2}
RT_MODES = {"median": 0, "mass_lower_median": 1}


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream_handle(stream=None) -> Optional[int]:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream or None


# Small batches (the per-cluster shim calls: one cluster, one pair) cross PCIe
# as ONE packed copy each way through a reused pinned buffer, instead of one
# pageable copy per array: the per-call cost is then launches + two copies.
PACKED_MAX_BYTES = 64 << 20


class _Pinned(threading.local):
    """A grow-only pinned host staging buffer (one per direction and host thread:
    two threads reading results back at once must not share it).  Every copy
    through it is waited for before the call returns, so it is free again."""

    def __init__(self):
        self.buf = None

    def take(self, nbytes: int):
        import torch

        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(int(nbytes), 1 << 16) * 2, dtype=torch.uint8, pin_memory=True)
        return self.buf


_H2D, _D2H = _Pinned(), _Pinned()


def _layout(items):
    """Byte offsets (256-aligned) of (name, numpy array) items; total bytes."""
    off, o = {}, 0
    for name, a in items:
        off[name] = o
        o += (a.nbytes + 255) & ~255
    return off, o


class DeviceBatch:
    """A SpectraCSR mirrored into HBM, with the host metadata the ABI needs."""

    def __init__(self, tensors: dict, host_cluster_off: np.ndarray, host_spec_off: np.ndarray,
                 max_mz_span: float, cluster_ids=None, titles=None, buffers: Optional[dict] = None):
        self.t = tensors
        self.n_clusters = int(tensors["n_clusters"])
        self.n_spectra = int(tensors["n_spectra"])
        self.n_peaks = int(tensors["n_peaks"])
        self.host_cluster_off = np.ascontiguousarray(host_cluster_off, np.int64)
        self.host_spec_off = np.ascontiguousarray(host_spec_off, np.int64)
        sizes = np.diff(self.host_cluster_off)
        peaks = self.host_spec_off[self.host_cluster_off[1:]] - self.host_spec_off[self.host_cluster_off[:-1]]
        self.info = _lib.SpxBatchInfo(int(peaks.max(initial=0)), int(sizes.max(initial=0)), float(max_mz_span))
        self.csr = _lib.SpxCsr(self.n_clusters, self.n_spectra, self.n_peaks,
                               _ptr(tensors["cluster_off"]), _ptr(tensors["spec_off"]), _ptr(tensors["mz"]),
                               _ptr(tensors["inten"]), _ptr(tensors["prec_mz"]), _ptr(tensors["charge"]),
                               _ptr(tensors.get("rt")))
        self.cluster_ids = cluster_ids or []
        self.titles = titles or []
        self._ws = {}  # host-side facts of THIS batch (workspace sizes, large-path flags)
        # workspace tensors by entry point; a caller streaming many batches through the
        # same device memory (pipeline.HostPipeline) passes one dict to all of them
        self._bufs = buffers if buffers is not None else {}

    @classmethod
    def from_host(cls, csr: SpectraCSR, device="cuda") -> "DeviceBatch":
        items = [("cluster_off", csr.cluster_off), ("spec_off", csr.spec_off), ("mz", csr.mz),
                 ("inten", csr.inten), ("prec_mz", csr.prec_mz), ("charge", csr.charge), ("rt", csr.rt)]
        off, total = _layout(items)
        if total > PACKED_MAX_BYTES:
            # large batches: the span is reduced in HBM after the copy (a host
            # pass over the m/z array costs more than its transfer)
            tensors = _staged_to_device(items, off, total, device)
            span = _device_span(tensors["mz"])
        else:
            # the m/z span over FINITE values only: a NaN/inf peak makes its cluster
            # SPX_NON_FINITE, it must not blow up the workspace sizing of the others
            fin = csr.mz[np.isfinite(csr.mz)] if csr.n_peaks else csr.mz
            span = float(fin.max() - fin.min()) if len(fin) else 0.0
            tensors = _packed_to_device(items, off, total, device)
        tensors.update(n_clusters=csr.n_clusters, n_spectra=csr.n_spectra, n_peaks=csr.n_peaks)
        return cls(tensors, csr.cluster_off, csr.spec_off, span, cluster_ids=csr.cluster_ids, titles=csr.titles)

    @classmethod
    def from_device(cls, tensors: dict) -> "DeviceBatch":
        """Wrap tensors already in HBM (e.g. synthetic.make_clusters_torch)."""
        import torch

        return cls(tensors, tensors["cluster_off"].cpu().numpy(), tensors["spec_off"].cpu().numpy(),
                   _device_span(tensors["mz"]))

    def workspace(self, key: str, nbytes: int):
        import torch

        ws = self._bufs.get(key)
        if ws is None or ws.numel() < nbytes:
            self._bufs.pop(key, None)
            ws = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.t["mz"].device)
            self._bufs[key] = ws
        return ws

    @property
    def device(self):
        return self.t["mz"].device


def _device_span(mz) -> float:
    """max - min over the finite values of a device m/z tensor (0.0 if none)."""
    import torch

    if not mz.numel():
        return 0.0
    fin = torch.isfinite(mz)
    inf = torch.tensor(float("inf"), dtype=mz.dtype, device=mz.device)
    hi = torch.where(fin, mz, -inf).max()
    lo = torch.where(fin, mz, inf).min()
    return float((hi - lo).clamp(min=0.0).item()) if bool(fin.any().item()) else 0.0


def _packed_to_device(items, off, total, device):
    """One pinned staging copy + one H2D for all of ``items``; device views."""
    import torch

    host = _H2D.take(total)
    hv = host.numpy()
    for name, a in items:
        hv[off[name]:off[name] + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    dev = torch.empty(max(total, 256), dtype=torch.uint8, device=device)
    dev[:total].copy_(host[:total], non_blocking=True)
    # ordered before later work on this stream, and waited for here like the
    # pageable copies it replaces (so any stream may consume the batch)
    torch.cuda.current_stream(dev.device).synchronize()
    return _views(dev, items, off)


_TORCH_DT = {np.dtype(np.int64): "int64", np.dtype(np.float64): "float64", np.dtype(np.int32): "int32"}


def _views(dev, items, off):
    import torch

    return {name: dev[off[name]:off[name] + a.nbytes].view(getattr(torch, _TORCH_DT[a.dtype]))
            for name, a in items}


def _staged_to_device(items, off, total, device):
    """Large batches: one device allocation, each array copied by spx_copy_h2d
    (pinned staging pool, several host threads, DMA overlapped with the staging
    copies) straight from the caller's pageable numpy memory; waited for here
    like the pageable copies it replaces."""
    import torch

    dev = torch.empty(max(total, 256), dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(dev.device)
    L = _lib.lib()
    with torch.cuda.device(dev.device):
        for name, a in items:
            a = np.ascontiguousarray(a)
            _lib.check(L.spx_copy_h2d(dev.data_ptr() + off[name], a.ctypes.data, a.nbytes, stream.cuda_stream),
                       "spx_copy_h2d")
    stream.synchronize()
    return _views(dev, items, off)


def to_host_array(t) -> np.ndarray:
    """A device tensor's contents as a new numpy array: spx_copy_d2h (pinned
    staging, overlapped) above PACKED_MAX_BYTES, ``.cpu()`` below."""
    import torch

    n = t.numel() * t.element_size()
    if n <= PACKED_MAX_BYTES or t.device.type != "cuda":
        return t.cpu().numpy()
    t = t.contiguous()
    np_dt = {torch.int64: np.int64, torch.float64: np.float64, torch.int32: np.int32}[t.dtype]
    out = np.empty(t.numel(), np_dt)
    with torch.cuda.device(t.device):
        _lib.check(_lib.lib().spx_copy_d2h(out.ctypes.data, t.data_ptr(), n,
                                           torch.cuda.current_stream(t.device).cuda_stream), "spx_copy_d2h")
    return out


def _packed_to_host(tensors):
    """One device concatenation + one D2H of the (name, tensor) list (8-byte
    dtypes first, so every piece stays aligned); numpy copies."""
    import torch

    tensors = sorted(tensors, key=lambda nt: -nt[1].element_size())
    flat = [t.reshape(-1).view(torch.uint8) for _, t in tensors]
    dev = torch.cat(flat) if flat else torch.zeros(0, dtype=torch.uint8)
    n = dev.numel()
    host = _D2H.take(n)
    host[:n].copy_(dev, non_blocking=True)
    torch.cuda.current_stream(dev.device).synchronize()
    hv = host.numpy()
    res, o = {}, 0
    for name, t in tensors:
        nb = t.numel() * t.element_size()
        np_dt = {torch.int64: np.int64, torch.float64: np.float64, torch.int32: np.int32}[t.dtype]
        res[name] = hv[o:o + nb].view(np_dt).copy()
        o += nb
    return res


def packed_readback(batch) -> bool:
    """Results of this batch come back in one packed D2H (PeaksResult.to_host)."""
    return 16 * batch.n_peaks + 32 * batch.n_clusters <= PACKED_MAX_BYTES


@dataclass
class PeaksResult:
    """Per-cluster peak lists in the capacity layout (cluster c at its input
    peak offset), plus per-cluster scalars, all device tensors."""
    batch: DeviceBatch
    mz: object
    inten: object
    count: object
    status: object
    prec: object
    charge: object
    rt: object = None
    stream: object = None  # the torch stream the producing kernel was enqueued on
    # bin_mean(staged=True): enqueues spx_bin_mean_stage(2); to_host() runs it when a
    # cluster came back SPX_UNRESOLVED from stage 1
    pending: object = None

    def compact(self, stream=None, total: Optional[int] = None):
        """Dense device arrays: (out_off [C+1], mz, inten).  Enqueued on ``stream``
        (default: the stream the producing kernel ran on, so compaction never
        reads a result that is still being written).  ``total`` = the known number
        of kept peaks skips the one host read of the count sum (no sync)."""
        import torch

        st = stream if stream is not None else (self.stream or torch.cuda.current_stream(self.count.device))
        C = self.batch.n_clusters
        with torch.cuda.stream(st):
            out_off = torch.zeros(C + 1, dtype=torch.int64, device=self.count.device)
            if C:
                torch.cumsum(self.count[:C], 0, out=out_off[1:])
            n = total if total is not None else (int(out_off[-1].item()) if C else 0)
            dmz = torch.empty(max(n, 1), dtype=torch.float64, device=self.count.device)
            dint = torch.empty_like(dmz)
            src = _lib.SpxPeaksOut(_ptr(self.mz), _ptr(self.inten), _ptr(self.count))
            _lib.check(_lib.lib().spx_compact_peaks(ctypes.byref(self.batch.csr), ctypes.byref(src), _ptr(out_off),
                                                    _ptr(dmz), _ptr(dint), _stream_handle(st)), "spx_compact_peaks")
        return out_off, dmz[:n], dint[:n]

    def to_host(self) -> dict:
        d = self._to_host()
        if self.pending is not None:
            finish, self.pending = self.pending, None
            if np.any(d["status"] == STATUS_UNRESOLVED):
                finish()
                d = self._to_host()
        return d

    def _to_host(self) -> dict:
        import torch

        if packed_readback(self.batch):
            return self._to_host_small()
        out_off, mz, inten = self.compact()
        if self.stream is not None:  # the readback copies run on the batch device's current stream
            torch.cuda.current_stream(self.batch.device).wait_stream(self.stream)
        d = dict(out_off=out_off.cpu().numpy(), out_mz=to_host_array(mz), out_int=to_host_array(inten),
                 status=self.status.cpu().numpy(), prec=self.prec.cpu().numpy(), charge=self.charge.cpu().numpy())
        if self.rt is not None:
            d["rt"] = self.rt.cpu().numpy()
        return d

    def _to_host_small(self) -> dict:
        """Small batches: the capacity-layout arrays and the scalars in one D2H
        (after the producing stream), compacted on the host."""
        import torch

        C, P = self.batch.n_clusters, self.batch.n_peaks
        if self.stream is not None:
            torch.cuda.current_stream(self.batch.device).wait_stream(self.stream)
        items = [("count", self.count[:C]), ("status", self.status[:C]), ("prec", self.prec[:C]),
                 ("charge", self.charge[:C]), ("mz", self.mz[:P]), ("inten", self.inten[:P])]
        if self.rt is not None:
            items.append(("rt", self.rt[:C]))
        h = _packed_to_host(items)
        count = h["count"]
        out_off = np.zeros(C + 1, np.int64)
        np.cumsum(count, out=out_off[1:])
        base = self.batch.host_spec_off[self.batch.host_cluster_off[:C]]
        idx = np.repeat(base - out_off[:-1], count) + np.arange(out_off[-1], dtype=np.int64)
        d = dict(out_off=out_off, out_mz=h["mz"][idx], out_int=h["inten"][idx], status=h["status"],
                 prec=h["prec"], charge=h["charge"])
        if self.rt is not None:
            d["rt"] = h["rt"]
        return d


def _alloc_peaks(batch: DeviceBatch):
    import torch

    dev = batch.device
    P, C = max(batch.n_peaks, 1), max(batch.n_clusters, 1)
    return (torch.empty(P, dtype=torch.float64, device=dev), torch.empty(P, dtype=torch.float64, device=dev),
            torch.zeros(C, dtype=torch.int64, device=dev), torch.zeros(C, dtype=torch.int32, device=dev),
            torch.empty(C, dtype=torch.float64, device=dev), torch.zeros(C, dtype=torch.int32, device=dev))


def bin_mean(batch: DeviceBatch, minimum=100.0, maximum=2000.0, binsize=0.02, apply_peak_quorum=True,
             out: Optional[PeaksResult] = None, stream=None, staged: bool = False) -> PeaksResult:
    """combine_bin_mean (binning.py:170-231) for every cluster of the batch.

    ``staged``: enqueue only stage 1 of ``spx_bin_mean_stage`` (the register and wide
    kernels); :meth:`PeaksResult.to_host` runs stage 2 (the large-cluster chain) if a
    cluster needs it.  For callers that copy the result back anyway (the per-cluster
    shims): 17 fewer empty launches per call.  Device-side consumers of the result
    must not use it."""
    L = _lib.lib()
    prm = _lib.SpxBinParams(float(minimum), float(maximum), float(binsize), int(apply_peak_quorum is True))
    need = L.spx_bin_mean_workspace_size(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info))
    ws = batch.workspace("bin_mean", need)
    if out is None:
        mz, it, cnt, st, prec, ch = _alloc_peaks(batch)
        out = PeaksResult(batch, mz, it, cnt, st, prec, ch)
    out.stream = stream
    po = _lib.SpxPeaksOut(_ptr(out.mz), _ptr(out.inten), _ptr(out.count))

    def launch(stage):
        _lib.check(L.spx_bin_mean_stage(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info),
                                        ctypes.byref(po), _ptr(out.prec), _ptr(out.charge), _ptr(out.status),
                                        _ptr(ws), ws.numel(), _stream_handle(stream), stage), "spx_bin_mean")

    launch(1 if staged else 0)
    out.pending = (lambda: launch(2)) if staged else None
    return out


def gap_average(batch: DeviceBatch, mz_accuracy=0.01, dyn_range=1000.0, min_fraction=0.5,
                pepmass="lower_median", rt="mass_lower_median", proton=PROTON,
                out: Optional[PeaksResult] = None, stream=None) -> PeaksResult:
    """average_spectrum (average_spectrum_clustering.py:26-103) + precursor helpers for every cluster."""
    import torch

    L = _lib.lib()
    if batch.t.get("rt") is None:
        raise ValueError("gap_average needs per-spectrum RT (NaN where absent)")
    prm = _lib.SpxGapParams(float(mz_accuracy), float(dyn_range), float(min_fraction), float(proton),
                            PEPMASS_MODES[pepmass], RT_MODES[rt])
    need = L.spx_gap_average_workspace_size(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info))
    ws = batch.workspace("gap_average", need)
    if out is None:
        mz, it, cnt, st, prec, ch = _alloc_peaks(batch)
        out = PeaksResult(batch, mz, it, cnt, st, prec, ch,
                          rt=torch.empty(max(batch.n_clusters, 1), dtype=torch.float64, device=batch.device))
    out.stream = stream
    po = _lib.SpxPeaksOut(_ptr(out.mz), _ptr(out.inten), _ptr(out.count))
    _lib.check(L.spx_gap_average(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info),
                                 ctypes.byref(po), _ptr(out.prec), _ptr(out.charge), _ptr(out.rt), _ptr(out.status),
                                 _ptr(ws), ws.numel(), _stream_handle(stream)), "spx_gap_average")
    return out


REP_EMPTY, REP_RANGE, REP_ARENA, REP_DEFERRED = -1, -2, -3, -4  # include/specpride.h SPX_REP_*


@dataclass
class MedoidResult:
    rep: object     # [C] int64 global spectrum index, or a REP_* code (< 0)
    totals: object  # [S] f64 or None

    def to_host(self):
        return self.rep.cpu().numpy(), (None if self.totals is None else self.totals.cpu().numpy())


def _medoid_launch(batch: DeviceBatch, tolerance, large_path: bool, out: MedoidResult, extra, stream):
    L = _lib.lib()
    key = ("medoid_size", tuple(extra))
    need = batch._ws.get(key)
    if need is None:
        ex = np.ascontiguousarray(extra, np.int64)
        need = L.spx_medoid_workspace_size(batch.host_cluster_off.ctypes.data_as(ctypes.c_void_p),
                                           batch.host_spec_off.ctypes.data_as(ctypes.c_void_p), batch.n_clusters,
                                           ex.ctypes.data_as(ctypes.c_void_p) if len(ex) else None, len(ex))
        if need == 0:
            raise ValueError("spx_medoid_workspace_size: invalid offsets")
        batch._ws[key] = need
    ws = batch.workspace("medoid", need)
    prm = _lib.SpxMedoidParams(float(tolerance), int(bool(large_path)))
    _lib.check(L.spx_medoid(ctypes.byref(batch.csr), ctypes.byref(prm), _ptr(out.rep), _ptr(out.totals), _ptr(ws),
                            ws.numel(), _stream_handle(stream)), "spx_medoid")


def medoid_needs_large_path(batch: DeviceBatch) -> bool:
    """True if some cluster takes the large (MFMA) path by size alone (host query, cached)."""
    v = batch._ws.get("medoid_needs_large")
    if v is None:
        v = bool(_lib.lib().spx_medoid_needs_large_path(batch.host_cluster_off.ctypes.data_as(ctypes.c_void_p),
                                                         batch.host_spec_off.ctypes.data_as(ctypes.c_void_p),
                                                         batch.n_clusters))
        batch._ws["medoid_needs_large"] = v
    return v


def medoid(batch: DeviceBatch, tolerance=0.1, with_totals=False, out: Optional[MedoidResult] = None,
           stream=None, check: bool = True) -> MedoidResult:
    """distance() + the medoid loop (most_similar_representative.py:13-111) for every cluster.

    The large-cluster passes are launched only when some cluster is large by size
    (spx_medoid_needs_large_path).  With ``check`` (the default) the call then waits
    for the result and, if a cluster was deferred at run time (REP_DEFERRED) or
    ran out of arena (REP_ARENA), re-runs with the large path on and those clusters
    budgeted in the arena, so every cluster comes back resolved or REP_RANGE.
    ``check=False`` only enqueues (timed loops that were checked once)."""
    import torch

    if out is None:
        out = MedoidResult(torch.empty(max(batch.n_clusters, 1), dtype=torch.int64, device=batch.device),
                           torch.empty(max(batch.n_spectra, 1), dtype=torch.float64, device=batch.device)
                           if with_totals else None)
    large = medoid_needs_large_path(batch)
    extra = batch._ws.get("medoid_extra", ())
    _medoid_launch(batch, tolerance, large or bool(extra), out, extra, stream)
    if not check or batch.n_clusters == 0:
        return out
    for _ in range(2):
        rep = out.rep[:batch.n_clusters]
        bad = torch.nonzero((rep == REP_DEFERRED) | (rep == REP_ARENA)).flatten().cpu().numpy()
        if len(bad) == 0:
            break
        arena = np.flatnonzero(out.rep[:batch.n_clusters].cpu().numpy() == REP_ARENA)
        extra = tuple(sorted(set(extra) | set(int(c) for c in arena)))
        batch._ws["medoid_extra"] = extra
        _medoid_launch(batch, tolerance, True, out, extra, stream)
    return out


def bin_mean_medoid(batch: DeviceBatch, minimum=100.0, maximum=2000.0, binsize=0.02, apply_peak_quorum=True,
                    tolerance=0.1, out_bm: Optional[PeaksResult] = None, out_md: Optional[MedoidResult] = None,
                    stream=None, check: bool = True):
    """bin_mean() and medoid() of the same batch in one pass (spx_bin_mean_medoid: each
    cluster's two register bodies share one workgroup); results identical to the two
    calls.  ``check`` as in :func:`medoid` (run-time deferrals re-run by medoid()).
    Returns (PeaksResult, MedoidResult).

    A checked call runs stage 1 of spx_bin_mean_medoid_stage (the fused register pass),
    reads how many clusters each register body handed on, and enqueues stage 2 (both
    leftover chains) only if either count is non-zero.  The counts depend only on the
    batch and the parameters, so the batch remembers a zero result: later unchecked
    calls with the same parameters then run stage 1 alone (~22 empty launches fewer),
    and otherwise the whole pass (stage 0).  The batch's input tensors must not be
    changed in place after construction (nothing in this package does)."""
    import torch

    L = _lib.lib()
    prm = _lib.SpxBinParams(float(minimum), float(maximum), float(binsize), int(apply_peak_quorum is True))
    need = L.spx_bin_mean_workspace_size(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info))
    ws_bm = batch.workspace("bin_mean", need)
    if out_bm is None:
        mz, it, cnt, st, prec, ch = _alloc_peaks(batch)
        out_bm = PeaksResult(batch, mz, it, cnt, st, prec, ch)
    out_bm.stream = stream
    out_bm.pending = None
    if out_md is None:
        out_md = MedoidResult(torch.empty(max(batch.n_clusters, 1), dtype=torch.int64, device=batch.device), None)
    large = medoid_needs_large_path(batch)
    extra = batch._ws.get("medoid_extra", ())
    key = ("medoid_size", tuple(extra))
    need_md = batch._ws.get(key)
    if need_md is None:
        ex = np.ascontiguousarray(extra, np.int64)
        need_md = L.spx_medoid_workspace_size(batch.host_cluster_off.ctypes.data_as(ctypes.c_void_p),
                                              batch.host_spec_off.ctypes.data_as(ctypes.c_void_p), batch.n_clusters,
                                              ex.ctypes.data_as(ctypes.c_void_p) if len(ex) else None, len(ex))
        if need_md == 0:
            raise ValueError("spx_medoid_workspace_size: invalid offsets")
        batch._ws[key] = need_md
    ws_md = batch.workspace("medoid", need_md)
    mprm = _lib.SpxMedoidParams(float(tolerance), int(bool(large or extra)))
    po = _lib.SpxPeaksOut(_ptr(out_bm.mz), _ptr(out_bm.inten), _ptr(out_bm.count))

    def launch(stage, handoff=None):
        _lib.check(L.spx_bin_mean_medoid_stage(ctypes.byref(batch.csr), ctypes.byref(prm), ctypes.byref(batch.info),
                                               ctypes.byref(po), _ptr(out_bm.prec), _ptr(out_bm.charge),
                                               _ptr(out_bm.status), _ptr(ws_bm), ws_bm.numel(), ctypes.byref(mprm),
                                               _ptr(out_md.rep), _ptr(out_md.totals), _ptr(ws_md), ws_md.numel(),
                                               _stream_handle(stream), stage, _ptr(handoff)), "spx_bin_mean_medoid")

    clean_key = ("fused_clean", prm.minimum, prm.maximum, prm.binsize, prm.apply_peak_quorum, mprm.tolerance,
                 mprm.large_path)
    if not check or not batch.n_clusters:
        launch(1 if batch._ws.get(clean_key) else 0)
        return out_bm, out_md
    hand = batch.workspace("handoff", 8)[:8].view(torch.int32)
    launch(1, hand)
    if stream is not None:
        torch.cuda.current_stream(batch.device).wait_stream(stream)
    n_bm, n_md = (int(x) for x in hand.cpu())
    if n_bm or n_md:
        launch(2)
    batch._ws[clean_key] = not (n_bm or n_md)
    if check and batch.n_clusters:
        rep = out_md.rep[:batch.n_clusters]
        if bool(((rep == REP_DEFERRED) | (rep == REP_ARENA)).any().item()):
            medoid(batch, tolerance=tolerance, out=out_md, stream=stream, check=True)
    return out_bm, out_md


def wire_count_bytes(max_count: int) -> int:
    """Bytes per peak count of the gather wire format for clusters of <= max_count
    spectra: 1 (<= 255) or 2 (<= 65,535); 0 = the compact format does not apply."""
    return 1 if max_count <= 255 else (2 if max_count <= 65535 else 0)


def wire_pack(mz, inten, max_count: int, stream=None, mi=None, cnt=None, n_fail=None):
    """spx_wire_pack: dense bin-mean consensus peaks (f64 device tensors) -> the gather's
    wire format, (mi float32 [2n] = the f32 bin sums M, I; cnt uint8/int16 [n];
    n_fail int32 [1], peaks no count <= max_count rebuilds).  Enqueued on ``stream``;
    the buffers may be passed in (reused across steps)."""
    import torch

    n = int(mz.numel())
    cb = wire_count_bytes(max_count)
    if cb == 0:
        raise ValueError("wire_pack: clusters past 65,535 spectra need the f64 format")
    dev = mz.device
    if mi is None or mi.numel() < 2 * n:
        mi = torch.empty(max(2 * n, 2), dtype=torch.float32, device=dev)
    if cnt is None or cnt.numel() < n:
        cnt = torch.empty(max(n, 1), dtype=torch.uint8 if cb == 1 else torch.int16, device=dev)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    if n_fail is None:
        n_fail = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().spx_wire_pack(_ptr(mz), _ptr(inten), n, int(max_count), _ptr(mi), _ptr(cnt), cb,
                                        _ptr(n_fail), _stream_handle(st)), "spx_wire_pack")
    return mi[:2 * n], cnt[:n], n_fail


def wire_unpack(mi, cnt, mz=None, inten=None, stream=None):
    """spx_wire_unpack: the wire format back to the f64 consensus peaks, bit for bit."""
    import torch

    n = int(cnt.numel())
    dev = cnt.device
    if mz is None:
        mz = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    if inten is None:
        inten = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    _lib.check(_lib.lib().spx_wire_unpack(_ptr(mi), _ptr(cnt), cnt.element_size(), n, _ptr(mz), _ptr(inten),
                                          _stream_handle(st)), "spx_wire_unpack")
    return mz[:n], inten[:n]


def xcorr_distance(batch: DeviceBatch, pairs, tolerance=0.1, stream=None):
    """1 - xcorr prescore (most_similar_representative.py:13-19) for (global
    spectrum index) pairs; returns a device f64 tensor."""
    import torch

    if isinstance(pairs, torch.Tensor):
        pairs_t = pairs.to(device=batch.device, dtype=torch.int64).reshape(-1, 2).contiguous()
    else:
        pairs_t = torch.as_tensor(np.asarray(pairs, np.int64).reshape(-1, 2), device=batch.device).contiguous()
    out = torch.empty(max(len(pairs_t), 1), dtype=torch.float64, device=batch.device)
    prm = _lib.SpxMedoidParams(float(tolerance), 0)
    _lib.check(_lib.lib().spx_xcorr_distance(ctypes.byref(batch.csr), ctypes.byref(prm), _ptr(pairs_t),
                                             len(pairs_t), _ptr(out), _stream_handle(stream)), "spx_xcorr_distance")
    return out[:len(pairs_t)]


MZ_SPACE = 1.000508 * .005  # benchmark.py:7-8 (mz_unit * .005)


@dataclass
class CosineResult:
    cos: object     # [S] f64: cos_dist(representative, member) per member spectrum
    avg: object     # [C] f64: average_cos_dist per cluster
    status: object  # [C] i32 (STATUS_EMPTY: an empty spectrum)

    def to_host(self):
        return self.cos.cpu().numpy(), self.avg.cpu().numpy(), self.status.cpu().numpy()


def binned_cosine(batch: DeviceBatch, rep_off, rep_mz, rep_int, mz_space=MZ_SPACE,
                  out: Optional[CosineResult] = None, stream=None, max_rep_peaks: Optional[int] = None) -> CosineResult:
    """cos_dist / average_cos_dist (benchmark.py:19-38) for every cluster of the
    batch: cluster c's representative is the device peak list
    [rep_off[c], rep_off[c+1]) of rep_mz / rep_int, its members are its spectra.
    ``max_rep_peaks`` (an upper bound on the representatives' lengths) sizes the
    workspace for representatives past the LDS path's 512 peaks; if omitted it
    is read from ``rep_off`` (one small device reduction and host read)."""
    import torch

    dev = batch.device
    C = batch.n_clusters
    if out is None:
        out = CosineResult(torch.empty(max(batch.n_spectra, 1), dtype=torch.float64, device=dev),
                           torch.empty(max(C, 1), dtype=torch.float64, device=dev),
                           torch.empty(max(C, 1), dtype=torch.int32, device=dev))
    if max_rep_peaks is None:
        max_rep_peaks = int((rep_off[1:C + 1] - rep_off[:C]).max().item()) if C else 0
    L = _lib.lib()
    need = L.spx_binned_cosine_workspace_size(C, int(max_rep_peaks))
    ws = batch.workspace("binned_cosine", need)
    prm = _lib.SpxCosineParams(float(mz_space))
    _lib.check(L.spx_binned_cosine(ctypes.byref(batch.csr), _ptr(rep_off), _ptr(rep_mz), _ptr(rep_int),
                                   ctypes.byref(prm), _ptr(out.cos), _ptr(out.avg), _ptr(out.status),
                                   int(max_rep_peaks), _ptr(ws), ws.numel(), _stream_handle(stream)),
               "spx_binned_cosine")
    return out


@dataclass
class BestScoreResult:
    best: object    # [C] i64: global spectrum index of the highest-scoring member (-1: none)
    status: object  # [C] i32 (STATUS_EMPTY: no member has a PSM; STATUS_NON_FINITE: only NaN scores)

    def to_host(self):
        return self.best.cpu().numpy(), self.status.cpu().numpy()


def best_score(cluster_off, score, rank, out: Optional[BestScoreResult] = None, stream=None) -> BestScoreResult:
    """get_best_representative (best_spectrum.py:67-100) for every cluster at once.

    Device tensors: ``cluster_off`` [C+1] i64 over the member spectra, ``score``
    [S] f64 (max non-NaN PSM score per spectrum's USI), ``rank`` [S] i64 (the USI's
    position in sorted order, -1 = no PSM).  Only offsets are needed, no peaks."""
    import torch

    C = int(cluster_off.numel()) - 1
    S = int(score.numel())
    if C < 0 or int(rank.numel()) != S:
        raise ValueError("best_score: cluster_off must have C+1 entries and score/rank one per spectrum")
    dev = cluster_off.device
    if out is None:
        out = BestScoreResult(torch.empty(max(C, 1), dtype=torch.int64, device=dev),
                              torch.empty(max(C, 1), dtype=torch.int32, device=dev))
    csr = _lib.SpxCsr(C, S, 0, _ptr(cluster_off), _ptr(cluster_off), None, None, None, None, None)
    _lib.check(_lib.lib().spx_best_score(ctypes.byref(csr), _ptr(score), _ptr(rank), _ptr(out.best),
                                         _ptr(out.status), _stream_handle(stream)), "spx_best_score")
    return out
