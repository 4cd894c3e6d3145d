"""Host-inclusive streaming of a pageable host CSR through HBM (SURVEY.md §8(d) tier 2).

The reference's CLI flow parses every cluster into host memory and then runs the
per-cluster cores over them (binning.py:286-302).  When the batch already sits in
host memory as a packed CSR, the cost on the device side is the PCIe transfer:
32 GB of peaks at ~50 GB/s against ~14 ms of kernels (configs[4]).  This module
keeps the transfer the only cost:

* the host CSR is cut into chunks of whole clusters (``chunk_bytes`` of peaks);
* two device slots -- inputs, outputs and the entry points' workspaces -- are
  allocated once and reused by every chunk of every call (no allocation inside
  the timed window; a ``HostPipeline`` is meant to live across batches);
* chunk k+1's H2D (``spx_copy_h2d``: pinned staging on host threads, DMA on a copy
  stream) runs while chunk k's kernels run on the compute stream, and chunk k-1's
  results are compacted and copied back on a third stream meanwhile; the offsets
  are rebased to the chunk on the device.

Results land in host arrays in the same layout :meth:`engine.PeaksResult.to_host`
returns for one batch (dense ``out_off`` / ``out_mz`` / ``out_int`` + per-cluster
scalars), so the chunking is invisible to the caller.
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib, engine
from .csr import SpectraCSR

_IN_FIELDS = (("cluster_off", np.int64), ("spec_off", np.int64), ("mz", np.float64), ("inten", np.float64),
              ("prec_mz", np.float64), ("charge", np.int32), ("rt", np.float64))


def plan_chunks(cluster_off: np.ndarray, spec_off: np.ndarray, chunk_bytes: int):
    """Cluster ranges [c0, c1) whose peaks take about ``chunk_bytes`` (16 B per peak);
    a cluster larger than that is a chunk of its own."""
    C = len(cluster_off) - 1
    if C <= 0:
        return []
    peaks_at = spec_off[cluster_off]  # [C+1] first peak of each cluster
    per = max(1, int(chunk_bytes) // 16)
    bounds = [0]
    while bounds[-1] < C:
        c0 = bounds[-1]
        c1 = int(np.searchsorted(peaks_at, peaks_at[c0] + per, side="right")) - 1
        bounds.append(min(C, max(c1, c0 + 1)))
    return list(zip(bounds[:-1], bounds[1:]))


@dataclass
class _Slot:
    raw: object                     # one uint8 device tensor: the chunk's input arrays
    views: dict                     # name -> typed device view (capacity)
    bm: object = None               # engine.PeaksResult (capacity)
    md: object = None               # engine.MedoidResult (capacity)
    bufs: dict = field(default_factory=dict)  # shared workspaces of the entry points
    done: object = None             # event: this slot's kernels finished
    chunk: tuple = None             # (c0, c1) it holds


def _offsets(cap_c, cap_s, cap_p):
    sizes = {"cluster_off": 8 * (cap_c + 1), "spec_off": 8 * (cap_s + 1), "mz": 8 * cap_p, "inten": 8 * cap_p,
             "prec_mz": 8 * cap_s, "charge": 4 * cap_s, "rt": 8 * cap_s}
    off, o = {}, 0
    for name, _ in _IN_FIELDS:
        off[name] = o
        o += (sizes[name] + 255) & ~255
    return off, o


class HostPipeline:
    """bin-mean + medoid (the headline's step) over a host CSR, chunked and overlapped."""

    def __init__(self, device="cuda", chunk_bytes: int = 2 << 30):
        import torch

        self.device = torch.device(device)
        self.chunk_bytes = int(chunk_bytes)
        self.slots = []
        self.cap = (0, 0, 0)
        self.copy_stream = torch.cuda.Stream(self.device)
        self.compute_stream = torch.cuda.Stream(self.device)
        self.back_stream = torch.cuda.Stream(self.device)
        self.timing = {}

    # ------------------------------------------------------------ device slots
    def _ensure_slots(self, cap_c, cap_s, cap_p):
        import torch

        if self.slots and cap_c <= self.cap[0] and cap_s <= self.cap[1] and cap_p <= self.cap[2]:
            return
        self.slots = []
        torch.cuda.empty_cache()
        off, total = _offsets(cap_c, cap_s, cap_p)
        sizes = {"cluster_off": cap_c + 1, "spec_off": cap_s + 1, "mz": cap_p, "inten": cap_p, "prec_mz": cap_s,
                 "charge": cap_s, "rt": cap_s}
        for _ in range(2):
            raw = torch.empty(max(total, 256), dtype=torch.uint8, device=self.device)
            views = {name: raw[off[name]:off[name] + sizes[name] * np.dtype(dt).itemsize].view(
                getattr(torch, np.dtype(dt).name)) for name, dt in _IN_FIELDS}
            self.slots.append(_Slot(raw, views))
        self.cap = (cap_c, cap_s, cap_p)

    def _h2d(self, slot: _Slot, csr: SpectraCSR, c0: int, c1: int):
        """Chunk [c0, c1) of the host CSR into the slot, offsets rebased (copy stream)."""
        import torch

        L = _lib.lib()
        s0, s1 = int(csr.cluster_off[c0]), int(csr.cluster_off[c1])
        p0, p1 = int(csr.spec_off[s0]), int(csr.spec_off[s1])
        parts = {"cluster_off": csr.cluster_off[c0:c1 + 1], "spec_off": csr.spec_off[s0:s1 + 1],
                 "mz": csr.mz[p0:p1], "inten": csr.inten[p0:p1], "prec_mz": csr.prec_mz[s0:s1],
                 "charge": csr.charge[s0:s1], "rt": csr.rt[s0:s1]}
        st = self.copy_stream
        if slot.done is not None:
            st.wait_event(slot.done)  # the slot's previous chunk is no longer read
        with torch.cuda.device(self.device):
            for name, a in parts.items():
                a = np.ascontiguousarray(a)
                if a.nbytes:
                    _lib.check(L.spx_copy_h2d(slot.views[name].data_ptr(), a.ctypes.data, a.nbytes,
                                              st.cuda_stream), "spx_copy_h2d")
        with torch.cuda.stream(st):
            slot.views["cluster_off"][:c1 - c0 + 1].sub_(s0)
            slot.views["spec_off"][:s1 - s0 + 1].sub_(p0)
        ev = torch.cuda.Event()
        ev.record(st)
        slot.chunk = (c0, c1)
        return ev

    def _batch(self, slot: _Slot, csr: SpectraCSR):
        c0, c1 = slot.chunk
        s0, s1 = int(csr.cluster_off[c0]), int(csr.cluster_off[c1])
        p0 = int(csr.spec_off[s0])
        C, S, P = c1 - c0, s1 - s0, int(csr.spec_off[s1]) - p0
        t = {name: slot.views[name][:n] for name, n in (("cluster_off", C + 1), ("spec_off", S + 1), ("mz", P),
                                                          ("inten", P), ("prec_mz", S), ("charge", S), ("rt", S))}
        t.update(n_clusters=C, n_spectra=S, n_peaks=P)
        return engine.DeviceBatch(t, csr.cluster_off[c0:c1 + 1] - s0, csr.spec_off[s0:s1 + 1] - p0, 0.0,
                                  buffers=slot.bufs)

    def _outputs(self, slot: _Slot, batch):
        """Capacity output tensors of the slot, sized for the largest chunk."""
        import torch

        cap_c, _, cap_p = self.cap
        if slot.bm is None:
            dev = self.device
            slot.bm = engine.PeaksResult(None, torch.empty(max(cap_p, 1), dtype=torch.float64, device=dev),
                                         torch.empty(max(cap_p, 1), dtype=torch.float64, device=dev),
                                         torch.zeros(max(cap_c, 1), dtype=torch.int64, device=dev),
                                         torch.zeros(max(cap_c, 1), dtype=torch.int32, device=dev),
                                         torch.empty(max(cap_c, 1), dtype=torch.float64, device=dev),
                                         torch.zeros(max(cap_c, 1), dtype=torch.int32, device=dev))
            slot.md = engine.MedoidResult(torch.empty(max(cap_c, 1), dtype=torch.int64, device=dev), None)
        slot.bm.batch = batch
        return slot.bm, slot.md

    # ------------------------------------------------------------------- run
    def run(self, csr: SpectraCSR) -> dict:
        """bin_mean + medoid of every cluster; host results:
        out_off / out_mz / out_int / status / prec / charge (bin-mean), rep (medoid)."""
        import torch

        chunks = plan_chunks(csr.cluster_off, csr.spec_off, self.chunk_bytes)
        co, so = csr.cluster_off, csr.spec_off
        cap_c = max((c1 - c0 for c0, c1 in chunks), default=0)
        cap_s = max((int(co[c1] - co[c0]) for c0, c1 in chunks), default=0)
        cap_p = max((int(so[co[c1]] - so[co[c0]]) for c0, c1 in chunks), default=0)
        self._ensure_slots(cap_c, cap_s, cap_p)
        C = csr.n_clusters
        res = {"out_off": np.zeros(C + 1, np.int64), "out_mz": np.empty(max(csr.n_peaks, 1)),
               "out_int": np.empty(max(csr.n_peaks, 1)), "status": np.empty(C, np.int32),
               "prec": np.empty(C), "charge": np.empty(C, np.int32), "rep": np.empty(C, np.int64)}
        kept = [0]
        redo = []  # chunks whose medoid deferred clusters at run time
        tm = {"h2d_host_s": 0.0, "readback_s": 0.0, "kernel_ms": 0.0, "chunks": len(chunks)}
        kev = []

        def launch(i):
            slot = self.slots[i % 2]
            batch = self._batch(slot, csr)
            bm, md = self._outputs(slot, batch)
            st = self.compute_stream
            st.wait_event(in_ev[i])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            engine.bin_mean(batch, out=bm, stream=st)
            engine.medoid(batch, out=md, stream=st, check=False)
            e1.record(st)
            slot.done = e1
            kev.append((e0, e1))
            return batch

        def readback(i, batch):
            slot = self.slots[i % 2]
            c0, c1 = slot.chunk
            t0 = time.perf_counter()
            bs = self.back_stream
            bs.wait_event(slot.done)
            with torch.cuda.device(self.device):
                out_off, dmz, dint = slot.bm.compact(stream=bs)
                n = int(dmz.numel())
                L = _lib.lib()
                k0 = kept[0]
                for dst, src in ((res["out_mz"], dmz), (res["out_int"], dint)):
                    if n:
                        _lib.check(L.spx_copy_d2h(dst.ctypes.data + 8 * k0, src.data_ptr(), 8 * n, bs.cuda_stream),
                                   "spx_copy_d2h")
                with torch.cuda.stream(bs):
                    Cc = c1 - c0
                    res["out_off"][c0 + 1:c1 + 1] = k0 + out_off[1:Cc + 1].cpu().numpy()
                    res["status"][c0:c1] = slot.bm.status[:Cc].cpu().numpy()
                    res["prec"][c0:c1] = slot.bm.prec[:Cc].cpu().numpy()
                    res["charge"][c0:c1] = slot.bm.charge[:Cc].cpu().numpy()
                    rep = slot.md.rep[:Cc].cpu().numpy()
                res["rep"][c0:c1] = np.where(rep >= 0, rep + co[c0], rep)
                kept[0] = k0 + n
                # the medoid's run-time deferrals (REP_DEFERRED / REP_ARENA): the chunk is
                # re-run by the checked call after the overlapped loop (redo), so the
                # copy and compute streams never drain here
                if np.any((rep == engine.REP_DEFERRED) | (rep == engine.REP_ARENA)):
                    redo.append(i)
            tm["readback_s"] += time.perf_counter() - t0

        def resolve(i):
            """Chunk i again, after the loop: H2D into slot 0, the checked medoid."""
            slot = self.slots[0]
            ev = self._h2d(slot, csr, *chunks[i])
            ev.synchronize()
            batch = self._batch(slot, csr)
            _, md = self._outputs(slot, batch)
            c0, c1 = slot.chunk
            with torch.cuda.device(self.device):
                md = engine.medoid(batch, out=md, check=True)  # the current stream, synchronised reads
                # the slot's next H2D (_h2d waits on slot.done) is ordered after this medoid
                # by an event, not by the implicit sync of the read below
                done = torch.cuda.Event()
                done.record(torch.cuda.current_stream(self.device))
                slot.done = done
                r2 = md.rep[:c1 - c0].cpu().numpy()
            res["rep"][c0:c1] = np.where(r2 >= 0, r2 + co[c0], r2)

        in_ev = [None] * len(chunks)
        batches = [None] * len(chunks)
        if chunks:
            t0 = time.perf_counter()
            self.slots[0].done = None
            self.slots[1].done = None
            in_ev[0] = self._h2d(self.slots[0], csr, *chunks[0])
            tm["h2d_host_s"] += time.perf_counter() - t0
        for i in range(len(chunks)):
            batches[i] = launch(i)
            if i >= 1:
                readback(i - 1, batches[i - 1])
                batches[i - 1] = None
            if i + 1 < len(chunks):
                t0 = time.perf_counter()
                in_ev[i + 1] = self._h2d(self.slots[(i + 1) % 2], csr, *chunks[i + 1])
                tm["h2d_host_s"] += time.perf_counter() - t0
        if chunks:
            readback(len(chunks) - 1, batches[-1])
        torch.cuda.synchronize(self.device)
        tm["redo_chunks"] = len(redo)
        for i in redo:
            t0 = time.perf_counter()
            resolve(i)
            tm["readback_s"] += time.perf_counter() - t0
        tm["kernel_ms"] = sum(a.elapsed_time(b) for a, b in kev)
        self.timing = tm
        res["out_mz"] = res["out_mz"][:kept[0]]
        res["out_int"] = res["out_int"][:kept[0]]
        return res
