"""Multi-GPU driver: clusters sharded over ranks, one gather to rank 0.

Clusters are independent, so the hot path has no data-path collective: each
rank owns a cost-balanced subset of clusters (LPT greedy bucketing -- the
longest job goes to the least-loaded rank), packs its own CSR, runs the
kernels on its own GPU, and the only exchange is a gatherv of the results to
rank 0, which reorders them by global cluster ordinal so the output order is
the reference's.  On MI355X the process group is ``nccl`` (= RCCL): the gather
is point-to-point ``isend/irecv`` of device tensors over xGMI, one link per
peer, no ring.  The same code runs under ``gloo`` on CPU tensors, which is how
the CPU test suite covers it (tests/test_distributed.py).

Per-rank compute is injectable (``compute=``) so the sharding, gather and
reassembly logic can be tested without a GPU; the default is the HIP engine.

Cost model: consensus paths are HBM-bound, cost = Σpeaks;
medoid is Gram-bound, cost = n² · K_c with K_c approximated by the cluster's
peak count / n (mean distinct bins per spectrum) times n, i.e. n · Σpeaks.
"""
from __future__ import annotations

import heapq
from typing import Callable, Optional

import numpy as np

from .csr import SpectraCSR, concat_ranges

CONSENSUS_KEYS = ("count", "status", "prec", "charge", "rt")


# ------------------------------------------------------------------ planning
def costs_from_sizes(sizes, peaks, method: str) -> np.ndarray:
    """Per-cluster cost from spectrum and peak counts (what an MGF index gives
    before any number is parsed)."""
    peaks = np.asarray(peaks, np.float64)
    n = np.asarray(sizes, np.float64)
    if method in ("bin_mean", "gap_average"):
        return peaks + 1.0
    if method == "medoid":
        return n * peaks + 1.0
    if method == "both":
        return peaks + n * peaks / 64.0 + 1.0
    raise ValueError(f"unknown method {method!r}")


def cluster_costs(csr: SpectraCSR, method: str) -> np.ndarray:
    return costs_from_sizes(csr.cluster_sizes(), csr.cluster_peaks(), method)


def plan_costs(cost, world: int, rank0_weight: float = 1.0) -> list:
    """LPT greedy assignment: rank -> ascending array of cluster ids.  Each cluster, longest
    first, goes to the rank that would finish it first.  ``rank0_weight`` < 1 makes rank 0
    a slower machine (it finishes a load L at L / rank0_weight): bench.py's multi-GPU rank 0
    also rebuilds the other ranks' gathered peaks, so it takes a smaller share."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if not 0.0 < rank0_weight <= 1.0:
        raise ValueError("rank0_weight must be in (0, 1]")
    cost = np.asarray(cost, np.float64)
    order = np.argsort(-cost, kind="stable")
    owner = np.empty(len(cost), np.int64)
    if rank0_weight == 1.0 or world == 1:
        heap = [(0.0, r) for r in range(world)]
        for c in order:
            load, r = heapq.heappop(heap)
            owner[c] = r
            heapq.heappush(heap, (load + float(cost[c]), r))
    else:
        heap = [(0.0, r) for r in range(1, world)]
        load0 = 0.0
        for c in order:
            x = float(cost[c])
            if (load0 + x) / rank0_weight <= heap[0][0] + x:
                owner[c] = 0
                load0 += x
            else:
                load, r = heapq.heappop(heap)
                owner[c] = r
                heapq.heappush(heap, (load + x, r))
    return [np.flatnonzero(owner == r) for r in range(world)]


def plan(csr: SpectraCSR, world: int, method: str = "bin_mean") -> list:
    """LPT greedy assignment of ``csr``'s clusters: rank -> ascending global cluster ids."""
    return plan_costs(cluster_costs(csr, method), world)


def world_rank(group=None):
    """(world size, rank) of ``group``; (1, 0) without an initialised process group."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def all_true(flag: bool, group=None) -> bool:
    """Logical AND of ``flag`` over the ranks (a tensor on the backend's device)."""
    import torch
    import torch.distributed as dist

    if world_rank(group)[0] == 1:
        return bool(flag)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


# ---------------------------------------------------------------- collectives
def gatherv(tensors: list, root: int = 0, group=None) -> Optional[list]:
    """Gather a list of 1-D tensors (same dtypes on every rank, any lengths) to
    ``root``.  Returns ``out[rank][i]`` on root, None elsewhere.  Lengths travel
    first (one small all_gather), then payloads point-to-point."""
    import torch
    import torch.distributed as dist

    world, rank = world_rank(group)
    if world == 1:
        return [list(tensors)]
    dev = tensors[0].device if tensors else torch.device("cpu")
    lens = torch.tensor([t.numel() for t in tensors], dtype=torch.int64, device=dev)
    all_lens = [torch.empty_like(lens) for _ in range(world)]
    dist.all_gather(all_lens, lens, group=group)
    all_lens = [x.cpu().tolist() for x in all_lens]
    if rank != root:
        reqs = [dist.isend(t.contiguous(), dst=root, group=group) for t in tensors if t.numel()]
        for q in reqs:
            q.wait()
        return None
    out, reqs = [], []
    for r in range(world):
        if r == root:
            out.append([t for t in tensors])
            continue
        bufs = [torch.empty(n, dtype=t.dtype, device=dev) for n, t in zip(all_lens[r], tensors)]
        reqs += [dist.irecv(b, src=r, group=group) for b in bufs if b.numel()]
        out.append(bufs)
    for q in reqs:
        q.wait()
    return out


def allgatherv(arrays: list, group=None) -> list:
    """All-gather a list of 1-D numpy arrays (same dtypes on every rank, any
    lengths): returns ``out[rank][i]`` on every rank.  Lengths travel first, then
    one padded all_gather per array (device tensors under ``nccl``)."""
    import torch
    import torch.distributed as dist

    world, rank = world_rank(group)
    if world == 1:
        return [list(arrays)]
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    lens = torch.tensor([len(a) for a in arrays], dtype=torch.int64, device=dev)
    all_lens = [torch.empty_like(lens) for _ in range(world)]
    dist.all_gather(all_lens, lens, group=group)
    all_lens = [x.cpu().tolist() for x in all_lens]
    out = [[None] * len(arrays) for _ in range(world)]
    for i, a in enumerate(arrays):
        m = max(max(lr[i] for lr in all_lens), 1)
        buf = torch.zeros(m, dtype=torch.from_numpy(np.zeros(0, a.dtype)).dtype, device=dev)
        if len(a):
            buf[:len(a)] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        bufs = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf, group=group)
        for r in range(world):
            out[r][i] = bufs[r][:all_lens[r][i]].cpu().numpy()
    return out


class StepGatherer:
    """Per-step gather of a rank's results to rank 0 (bench.py's multi-GPU step),
    on its own stream so step k's gather overlaps step k+1's kernels.

    Each rank compacts its consensus peaks (capacity layout -> dense, through the
    result's ``compact(stream=, total=)``) and sends counts, representatives and
    peaks point-to-point (RCCL over xGMI under ``nccl``); rank 0 receives every
    peer's shard into buffers of its own, kept in :attr:`recv` (reordering into
    global cluster order is a host-side index, not part of the device pass).  The
    per-rank cluster and kept-peak counts are exchanged once (:meth:`plan`).

    On a GPU group, with ``wire_max_count`` (the largest cluster size, <= 65,535), the
    peaks travel in the wire format of ``csrc/wire.hip``: the f32 bin sums and a 1- or
    2-byte count, 9-10 bytes a peak instead of 16, and rank 0 rebuilds the f64 peaks
    bit for bit on its gather stream (engine.wire_pack / wire_unpack); counts and
    representatives travel as int32.  The link into rank 0 is what bounds a
    strong-scaled step, so that is 1.6-1.8x less time on it.  :meth:`check` reads
    the senders' pack-failure counters (0 for bin-mean output) after a run.
    On a CPU group (``gloo``, the test suite) the stream and events are skipped,
    the peaks travel as f64 and the P2P ops are the same."""

    def __init__(self, n_clusters: int, rank: int, world: int, device, group=None, wire_max_count=None,
                 wire_ops=None, stage_host: bool = False):
        import torch

        from . import engine

        self.rank, self.world, self.n, self.group = rank, world, int(n_clusters), group
        # stage_host (bench.py's one-GPU rehearsal of the multi-GPU step under gloo, whose
        # point-to-point ops take host tensors): the same device-side pack / unpack, the
        # payloads staged through host copies around the P2P ops
        self.stage_host = bool(stage_host)
        self._host_bufs = {}
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.dev) if self.cuda else None
        self.recv = {}
        self.recv_sizes = None
        self.send_peaks = 0
        # (pack, unpack) with engine.wire_pack / wire_unpack's signatures: the HIP kernels
        # on a GPU group; a CPU test passes a model of them to drive the same protocol
        self.wire_ops = wire_ops or ((engine.wire_pack, engine.wire_unpack) if self.cuda else None)
        cb = engine.wire_count_bytes(int(wire_max_count)) if wire_max_count else 0
        self.wire = cb if self.wire_ops else 0  # bytes per peak count on the wire; 0 = f64 peaks
        self._wire_bufs = {}  # reused per step: the sender's pack outputs, rank 0's wire receive buffers
        self.n_fail = torch.zeros(1, dtype=torch.int32, device=self.dev) if self.wire else None
        self.wire_max = int(wire_max_count) if self.wire else 0

    def plan(self, kept_peaks: int):
        """Exchange the (fixed) per-rank cluster and kept-peak counts once, so
        every step's receive buffers are sized without a per-step handshake.
        Returns the totals over ranks (clusters, kept peaks)."""
        import torch
        import torch.distributed as dist

        sizes = torch.tensor([self.n, int(kept_peaks), self.wire_max], dtype=torch.int64,
                             device="cpu" if self.stage_host else self.dev)
        allsz = [torch.empty_like(sizes) for _ in range(self.world)]
        dist.all_gather(allsz, sizes, group=self.group)
        got = [tuple(int(v) for v in t.cpu()) for t in allsz]
        self.recv_sizes = [g[:2] for g in got]
        self.send_peaks = int(kept_peaks)
        if self.wire:  # one count width for every rank: the largest cluster anywhere
            from . import engine

            self.wire_max = max(g[2] for g in got)
            self.wire = engine.wire_count_bytes(self.wire_max) if min(g[2] for g in got) > 0 else 0
        return sum(x[0] for x in self.recv_sizes), sum(x[1] for x in self.recv_sizes)

    def wire_bytes_per_step(self) -> int:
        """Bytes rank 0 receives per step (all peers)."""
        per_peak = 8 + self.wire if self.wire else 16
        per_cluster = 8 if self.wire else 16
        return sum(c * per_cluster + p * per_peak for c, p in self.recv_sizes[1:])

    def check(self) -> int:
        """Pack failures of this rank's sends so far (synchronises; 0 unless the peaks
        were not bin-mean output)."""
        return int(self.n_fail.item()) if self.wire else 0

    def launch(self, bm, rep, done_event=None, first=None):
        """Enqueue the gather of one step's results (consensus ``bm`` with
        ``.count`` and ``.compact``, representatives ``rep``) after
        ``done_event``; returns an event that completes when this rank's part of
        the gather has (None on CPU, where the call blocks until it has).

        With ``first`` (the rank's local ``cluster_off[:-1]``) the representatives
        travel as member indices within their cluster (``rep - first``; failure
        codes < 0 pass through), which rank 0 maps to global spectrum indices in
        :meth:`assemble`; without it, as the rank's local spectrum indices."""
        import contextlib

        import torch
        import torch.distributed as dist

        from . import engine

        ctx = torch.cuda.stream(self.stream) if self.cuda else contextlib.nullcontext()
        idt = torch.int32 if self.wire else torch.int64
        with ctx:
            if self.cuda and done_event is not None:
                self.stream.wait_event(done_event)
            if self.rank == 0:
                ops = []
                for r in range(1, self.world):
                    c_r, p_r = self.recv_sizes[r]
                    bufs = self.recv.get(r)
                    if bufs is None:
                        bufs = (torch.empty(max(c_r, 1), dtype=idt, device=self.dev),
                                torch.empty(max(c_r, 1), dtype=idt, device=self.dev),
                                torch.empty(max(p_r, 1), dtype=torch.float64, device=self.dev),
                                torch.empty(max(p_r, 1), dtype=torch.float64, device=self.dev))
                        self.recv[r] = bufs
                    if self.wire:
                        wb = self._wire_bufs.get(r)
                        if wb is None:
                            wb = (torch.empty(max(2 * p_r, 2), dtype=torch.float32, device=self.dev),
                                  torch.empty(max(p_r, 1), dtype=torch.uint8 if self.wire == 1 else torch.int16,
                                              device=self.dev))
                            self._wire_bufs[r] = wb
                        # (2-byte counts travel as bytes: RCCL/NCCL has no 16-bit integer type)
                        ops += [dist.P2POp(dist.irecv, b, r, group=self.group)
                                for b in (bufs[0], bufs[1], wb[0], wb[1].view(torch.uint8))]
                    else:
                        ops += [dist.P2POp(dist.irecv, b, r, group=self.group) for b in bufs]
            else:
                if first is not None:
                    r0 = rep[:self.n]
                    rep = torch.where(r0 >= 0, r0 - first[:self.n], r0)
                # device-side compaction of this rank's consensus peaks (count known: no sync)
                _, dmz, dint = bm.compact(stream=self.stream, total=self.send_peaks)
                one = lambda x: x if x.numel() else torch.zeros(1, dtype=x.dtype, device=x.device)  # noqa: E731
                cnt = bm.count[:self.n].to(idt).contiguous()
                rr = rep[:self.n].to(idt).contiguous()
                if self.wire:
                    wb = self._wire_bufs.get("send")
                    mi, wc, _ = self.wire_ops[0](dmz, dint, self.wire_max, stream=self.stream,
                                                 mi=wb[0] if wb else None, cnt=wb[1] if wb else None,
                                                 n_fail=self.n_fail)
                    self._wire_bufs["send"] = (mi, wc)
                    payload = (cnt, rr, mi, wc.view(torch.uint8))
                else:
                    payload = (cnt, rr, dmz, dint)
                if self.wire and payload[2].numel() == 0:  # no peaks: rank 0 posts 2 floats, 1 count
                    payload = payload[:2] + (torch.zeros(2, dtype=torch.float32, device=self.dev),
                                             torch.zeros(self.wire, dtype=torch.uint8, device=self.dev))
                ops = [dist.P2POp(dist.isend, one(x), 0, group=self.group) for x in payload]
            if self.stage_host and ops:
                ops = self._stage(ops)
            for q in (dist.batch_isend_irecv(ops) if ops else []):
                q.wait()
            if self.stage_host and self.rank == 0:
                for dev_t, host_t in self._recv_pairs:
                    dev_t.copy_(host_t)
            if self.rank == 0 and self.wire:
                for r in range(1, self.world):  # rank 0's rebuild of the f64 peaks, on the gather stream
                    p_r = self.recv_sizes[r][1]
                    if p_r:
                        mi, wc = self._wire_bufs[r]
                        b = self.recv[r]
                        self.wire_ops[1](mi[:2 * p_r], wc[:p_r], b[2], b[3], stream=self.stream)
            if not self.cuda:
                return None
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return ev

    def _stage(self, ops):
        """stage_host: the P2P ops on host copies -- a sender's payloads copied out once its
        gather stream has produced them, rank 0's receives into host buffers that launch()
        copies into the device buffers afterwards (self._recv_pairs)."""
        import torch
        import torch.distributed as dist

        if self.stream is not None:
            self.stream.synchronize()
        staged, self._recv_pairs = [], []
        for k, op in enumerate(ops):
            t = op.tensor
            if op.op is dist.isend:
                staged.append(dist.P2POp(dist.isend, t.cpu(), op.peer, group=self.group))
            else:
                h = self._host_bufs.get(k)
                if h is None or h.shape != t.shape or h.dtype != t.dtype:
                    h = torch.empty(t.shape, dtype=t.dtype)
                    self._host_bufs[k] = h
                staged.append(dist.P2POp(dist.irecv, h, op.peer, group=self.group))
                self._recv_pairs.append((t, h))
        return staged

    def assemble(self, parts: list, cluster_off: np.ndarray, own_bm, own_member) -> dict:
        """Rank 0, after a step's gather has completed: the whole batch's results in
        GLOBAL cluster order from rank 0's own (``own_bm``, ``own_member``) and the
        peers' received buffers (sent with ``first=``).  ``parts[r]`` = the ascending
        global cluster ids of rank r (:func:`plan_costs`), ``cluster_off`` = the global
        spectrum offsets.  Returns host arrays: ``out_off``, ``out_mz``, ``out_int``
        (the compacted consensus peaks), ``count``, ``rep`` (global spectrum index, or
        the failure code).  A host-side index: not part of the timed device pass."""
        if self.rank != 0:
            raise RuntimeError("assemble() runs on rank 0")
        cluster_off = np.asarray(cluster_off, np.int64)
        C = len(cluster_off) - 1
        count = np.zeros(C, np.int64)
        member = np.full(C, -1, np.int64)
        pieces = {}
        for r, ids in enumerate(parts):
            ids = np.asarray(ids, np.int64)
            n = len(ids)
            if r == 0:
                cnt = own_bm.count[:n].to("cpu").numpy()
                _, mz, it = own_bm.compact(total=int(cnt.sum()))
                mem = own_member[:n].to("cpu").numpy()
            else:
                c_r, p_r = self.recv_sizes[r]
                if c_r != n:
                    raise ValueError(f"rank {r} sent {c_r} clusters, the plan gives it {n}")
                b = self.recv[r]
                cnt = b[0][:n].cpu().numpy()
                mem = b[1][:n].cpu().numpy()
                mz, it = b[2][:p_r], b[3][:p_r]
            count[ids] = cnt
            member[ids] = mem
            pieces[r] = (ids, cnt, mz.cpu().numpy(), it.cpu().numpy())
        out_off = np.zeros(C + 1, np.int64)
        np.cumsum(count, out=out_off[1:])
        out_mz = np.empty(int(out_off[-1]), np.float64)
        out_int = np.empty_like(out_mz)
        for ids, cnt, mz, it in pieces.values():
            dst = concat_ranges(out_off[ids], cnt)
            out_mz[dst] = mz[:len(dst)]
            out_int[dst] = it[:len(dst)]
        rep = np.where(member >= 0, cluster_off[:-1] + member, member)
        return dict(out_off=out_off, out_mz=out_mz, out_int=out_int, count=count, rep=rep)


def strong_partition(cluster_off, spec_off, world: int, method: str = "both", rank0_weight: float = 1.0):
    """bench.py's strong-scaling split of ONE batch (the same on every rank: each
    rank computes it from the offsets of the batch it generated identically):
    size-balanced LPT buckets (:func:`plan_costs`) over the per-cluster cost of
    ``method`` -- "both" = Σpeaks (bin-mean) + n·Σpeaks/64 (medoid).  Returns
    ``(parts, loads)``: rank -> ascending global cluster ids, and each rank's cost."""
    co = np.asarray(cluster_off, np.int64)
    so = np.asarray(spec_off, np.int64)
    sizes = np.diff(co)
    peaks = so[co[1:]] - so[co[:-1]]
    cost = costs_from_sizes(sizes, peaks, method)
    parts = plan_costs(cost, world, rank0_weight)
    loads = np.array([float(cost[p].sum()) for p in parts])
    return parts, loads


# ------------------------------------------------------------ default compute
def _engine_consensus(method: str, params: dict, device):
    def run(sub: SpectraCSR) -> dict:
        from . import engine

        batch = engine.DeviceBatch.from_host(sub, device)
        res = getattr(engine, method)(batch, **params)
        out_off, mz, inten = res.compact()
        d = dict(count=res.count[:sub.n_clusters], status=res.status[:sub.n_clusters],
                 prec=res.prec[:sub.n_clusters], charge=res.charge[:sub.n_clusters], mz=mz, inten=inten)
        if res.rt is not None:
            d["rt"] = res.rt[:sub.n_clusters]
        return d
    return run


def _engine_medoid(params: dict, device):
    """Per-rank medoid compute; ``member`` = representative index within its cluster."""
    def run(sub: SpectraCSR) -> dict:
        import torch

        from . import engine

        batch = engine.DeviceBatch.from_host(sub, device)
        res = engine.medoid(batch, **params)
        rep = res.rep[:sub.n_clusters]
        first = batch.t["cluster_off"][:-1]
        member = torch.where(rep >= 0, rep - first, rep)  # index within the cluster (<0 passes through)
        d = dict(member=member)
        if res.totals is not None:
            d["totals"] = res.totals[:sub.n_spectra]
        return d
    return run


# ----------------------------------------------------------------- drivers
def _my_shard(csr: SpectraCSR, method: str, group):
    world, rank = world_rank(group)
    parts = plan(csr, world, method)
    return parts, rank, csr.select(parts[rank])


def gather_consensus(res: dict, parts: list, n_clusters: int, group=None) -> Optional[dict]:
    """Gather every rank's consensus result (``res``: count/status/prec/charge[/rt]
    per local cluster + dense mz/inten) to rank 0 and reorder it into global
    cluster order; rank 0 returns the host dict of :meth:`engine.PeaksResult.to_host`,
    other ranks None."""
    import torch

    with_rt = "rt" in res
    keys = [k for k in CONSENSUS_KEYS if k in res]
    dev = res["count"].device
    payload = [res[k].contiguous() for k in keys] + [res["mz"].contiguous(), res["inten"].contiguous()]
    got = gatherv(payload, group=group)
    if got is None:
        return None
    C = n_clusters
    full = {}
    for i, k in enumerate(keys):
        t0 = got[0][i]
        buf = torch.zeros(C, dtype=t0.dtype, device=dev)
        for r, ids in enumerate(parts):
            if len(ids):
                buf[torch.from_numpy(ids).to(dev)] = got[r][i].to(dev)
        full[k] = buf
    count = full["count"].to(torch.int64).cpu().numpy()
    out_off = np.zeros(C + 1, np.int64)
    np.cumsum(count, out=out_off[1:])
    total = int(out_off[-1])
    mz = np.empty(total, np.float64)
    inten = np.empty(total, np.float64)
    for r, ids in enumerate(parts):
        if not len(ids):
            continue
        ids_np = np.asarray(ids, np.int64)
        dst = concat_ranges(out_off[ids_np], count[ids_np])
        if len(dst):
            mz[dst] = got[r][len(keys)].cpu().numpy()
            inten[dst] = got[r][len(keys) + 1].cpu().numpy()
    out = dict(out_off=out_off, out_mz=mz, out_int=inten, status=full["status"].cpu().numpy(),
               prec=full["prec"].cpu().numpy(), charge=full["charge"].cpu().numpy())
    if with_rt:
        out["rt"] = full["rt"].cpu().numpy()
    return out


def consensus_sharded(csr: SpectraCSR, method: str = "bin_mean", params: Optional[dict] = None,
                      device=None, group=None, compute: Optional[Callable] = None) -> Optional[dict]:
    """Run ``engine.bin_mean`` / ``engine.gap_average`` over the ranks of ``group``;
    rank 0 returns the host dict of :meth:`engine.PeaksResult.to_host` for the
    WHOLE batch in global cluster order; other ranks return None.  Every rank
    passes the same ``csr`` (the CLIs' rank-local ingest instead packs only the
    rank's own clusters and calls :func:`gather_consensus`)."""
    params = params or {}
    parts, rank, sub = _my_shard(csr, method, group)
    run = compute or _engine_consensus(method, params, device)
    return gather_consensus(run(sub), parts, csr.n_clusters, group)


def gather_medoid(res: dict, parts: list, cluster_off: np.ndarray, group=None):
    """Rank 0: ``(rep [C] global spectrum index, totals [S] or None)`` from every
    rank's ``member`` (index within its cluster, <0 = failure code) [+ totals]."""
    with_totals = "totals" in res
    payload = [res["member"].contiguous()] + ([res["totals"].contiguous()] if with_totals else [])
    got = gatherv(payload, group=group)
    if got is None:
        return None
    C, S = len(cluster_off) - 1, int(cluster_off[-1])
    rep = np.full(C, -1, np.int64)
    totals = np.full(S, np.nan) if with_totals else None
    for r, ids in enumerate(parts):
        if not len(ids):
            continue
        member = got[r][0].cpu().numpy()
        first = cluster_off[ids]
        rep[ids] = np.where(member >= 0, first + member, member)
        if with_totals:
            sizes = cluster_off[ids + 1] - first
            totals[concat_ranges(first, sizes)] = got[r][1].cpu().numpy()
    return rep, totals


def medoid_sharded(csr: SpectraCSR, params: Optional[dict] = None, device=None, group=None,
                   compute: Optional[Callable] = None):
    """Sharded ``engine.medoid``: rank 0 returns ``(rep [C] global spectrum index,
    totals [S] or None)`` in global order; other ranks return None."""
    params = params or {}
    parts, rank, sub = _my_shard(csr, "medoid", group)
    run = compute or _engine_medoid(params, device)
    return gather_medoid(run(sub), parts, csr.cluster_off, group)
