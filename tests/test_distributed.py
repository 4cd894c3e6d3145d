"""Multi-rank path on CPU: world_size-2 (and 3) ``gloo`` process groups drive
specpride_amd.shard -- LPT planning, per-rank CSR packing, the gatherv to rank 0
and the reorder by global cluster ordinal -- with the C oracle as the per-rank
compute (no GPU here).  The result on rank 0 must equal the single-process
oracle over the whole batch, bit for bit.  On MI355X the same code runs with
``nccl`` (RCCL) and the HIP engine as compute."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from specpride_amd import shard
from specpride_amd.synthetic import make_clusters_np


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_consensus(method):
    from oracle import c_oracle

    def run(sub):
        r = getattr(c_oracle, method)(sub)
        t = torch.from_numpy
        C = sub.n_clusters
        d = dict(count=t(np.diff(r["out_off"])), status=t(r["status"]), mz=t(r["out_mz"]), inten=t(r["out_int"]))
        d["prec"] = t(r["prec"]) if "prec" in r else torch.zeros(C, dtype=torch.float64)
        d["charge"] = t(r["charge"]) if "charge" in r else torch.zeros(C, dtype=torch.int32)
        return d
    return run


def _oracle_medoid(sub):
    from oracle import c_oracle

    rep, totals = c_oracle.medoid(sub, with_totals=True)
    member = np.where(rep >= 0, rep - sub.cluster_off[:-1], rep)
    return dict(member=torch.from_numpy(member), totals=torch.from_numpy(totals))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        csr = make_clusters_np(37, seed=12)
        out = {}
        for method in ("bin_mean", "gap_average"):
            out[method] = shard.consensus_sharded(csr, method, compute=_oracle_consensus(method))
        out["medoid"] = shard.medoid_sharded(csr, compute=_oracle_medoid)
        if rank == 0:
            q.put(out)
        else:
            assert all(v is None for v in out.values())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_single_process(world):
    from oracle import c_oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = make_clusters_np(37, seed=12)
    for method in ("bin_mean", "gap_average"):
        ref = getattr(c_oracle, method)(csr)
        g = got[method]
        for k in ("out_off", "out_mz", "out_int", "status"):
            np.testing.assert_array_equal(g[k], ref[k], err_msg=f"{method} {k}")
        if method == "bin_mean":
            np.testing.assert_array_equal(g["prec"], ref["prec"])
            np.testing.assert_array_equal(g["charge"], ref["charge"])
    rep, totals = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(got["medoid"][0], rep)
    np.testing.assert_array_equal(got["medoid"][1], totals)


def test_plan_is_balanced_partition():
    csr = make_clusters_np(500, seed=2)
    for method in ("bin_mean", "medoid", "both"):
        parts = shard.plan(csr, 8, method)
        allc = np.sort(np.concatenate(parts))
        np.testing.assert_array_equal(allc, np.arange(csr.n_clusters))
        cost = shard.cluster_costs(csr, method)
        loads = np.array([cost[p].sum() for p in parts])
        assert loads.max() <= loads.mean() + cost.max()  # LPT bound
    assert [len(p) for p in shard.plan(csr, 1)] == [csr.n_clusters]


@pytest.mark.parametrize("w0", [1.0, 0.72, 0.5])
def test_plan_costs_rank0_weight(w0):
    """Rank 0 as a slower machine (bench.py's strong split: it also rebuilds the gathered
    peaks): still a partition, rank 0's load ~w0 x the others', and finishing times
    load/speed within one cluster's cost of each other."""
    cost = shard.cluster_costs(make_clusters_np(800, seed=5), "both")
    parts = shard.plan_costs(cost, 8, rank0_weight=w0)
    np.testing.assert_array_equal(np.sort(np.concatenate(parts)), np.arange(len(cost)))
    loads = np.array([cost[p].sum() for p in parts])
    fin = loads / np.array([w0] + [1.0] * 7)
    assert fin.max() - fin.min() <= cost.max() / w0
    assert abs(loads[0] / loads[1:].mean() - w0) < 0.05


# ------------------------------------------------ bench.py's per-step gatherer
class _FakeConsensus:
    """A consensus result in the capacity layout (cluster c's kept peaks at its
    input peak offset), as engine.PeaksResult holds it; compact() on the host."""

    def __init__(self, count, cap_off, mz, inten):
        self.count, self.cap_off, self.mz, self.inten = count, cap_off, mz, inten

    def compact(self, stream=None, total=None):
        idx = torch.cat([torch.arange(int(a), int(a) + int(n)) for a, n in zip(self.cap_off[:-1], self.count)])
        off = torch.zeros(len(self.count) + 1, dtype=torch.int64)
        off[1:] = torch.cumsum(self.count, 0)
        assert total is None or total == int(off[-1])
        return off, self.mz[idx], self.inten[idx]


def _step_result(rank, step, n_clusters):
    g = torch.Generator().manual_seed(1000 * rank + 17)
    cap = torch.randint(1, 9, (n_clusters,), generator=g)
    count = torch.minimum(cap, torch.randint(0, 9, (n_clusters,), generator=g))  # fixed over steps
    cap_off = torch.zeros(n_clusters + 1, dtype=torch.int64)
    cap_off[1:] = torch.cumsum(cap, 0)
    P = int(cap_off[-1])
    mz = torch.arange(P, dtype=torch.float64) + 0.25 * step + 1e4 * rank
    inten = -mz
    rep = cap_off[:-1] + step % 2
    return _FakeConsensus(count, cap_off, mz, inten), rep


def _gatherer_worker(rank, world, port, q, stage_host=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 5 + 3 * rank
        bm, _ = _step_result(rank, 0, n)
        gat = shard.StepGatherer(n, rank, world, "cpu", stage_host=stage_host)
        totals = gat.plan(int(bm.count.sum()))
        ok = True
        for step in range(3):
            bm, rep = _step_result(rank, step, n)
            assert gat.launch(bm, rep) is None
            if rank == 0:
                for r in range(1, world):
                    wbm, wrep = _step_result(r, step, 5 + 3 * r)
                    _, wmz, wint = wbm.compact()
                    cnt, rp, mz, it = gat.recv[r]
                    ok &= torch.equal(cnt[:len(wbm.count)], wbm.count) and torch.equal(rp[:len(wrep)], wrep)
                    ok &= torch.equal(mz[:len(wmz)], wmz) and torch.equal(it[:len(wint)], wint)
        q.put((rank, ok, totals))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,stage_host", [(2, False), (3, False), (2, True)])
def test_step_gatherer_gloo(world, stage_host):
    """bench.py's multi-GPU step gather (shard.StepGatherer: sizes exchanged once,
    then per step counts + representatives + compacted peaks point-to-point to
    rank 0) under gloo: rank 0 holds every peer's step results, step after step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gatherer_worker, args=(r, world, port, q, stage_host)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (ok, tot)) for r, ok, tot in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for ok, _ in got.values())
    want_c = sum(5 + 3 * r for r in range(world))
    assert all(tot[0] == want_c for _, tot in got.values())


# ------------------------------------------- bench.py's strong-scaling partition
class _OracleConsensus:
    """An oracle bin-mean result with the two members StepGatherer/assemble use:
    ``count`` and ``compact(stream=, total=)`` (dense already)."""

    def __init__(self, r):
        self.count = torch.from_numpy(np.diff(r["out_off"]))
        self._off = torch.from_numpy(r["out_off"])
        self._mz, self._int = torch.from_numpy(r["out_mz"]), torch.from_numpy(r["out_int"])

    def compact(self, stream=None, total=None):
        assert total is None or total == int(self._off[-1])
        return self._off, self._mz, self._int


def _strong_worker(rank, world, port, q, wire=False):
    from oracle import c_oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # every rank builds the same batch and keeps its LPT bucket, as bench.py does
        csr = make_clusters_np(61, seed=23)
        parts, loads = shard.strong_partition(csr.cluster_off, csr.spec_off, world, "both")
        sub = csr.select(parts[rank])
        bm = _OracleConsensus(c_oracle.bin_mean(sub))
        rep = torch.from_numpy(c_oracle.medoid(sub))
        first = torch.from_numpy(sub.cluster_off[:-1])
        if wire:  # the GPU path's wire format, with the numpy model of the kernels
            import wire_model

            gat = shard.StepGatherer(sub.n_clusters, rank, world, "cpu", wire_ops=wire_model.torch_ops(),
                                     wire_max_count=int(sub.cluster_sizes().max()))
        else:
            gat = shard.StepGatherer(sub.n_clusters, rank, world, "cpu")
        gat.plan(int(bm.count.sum()))
        for _ in range(2):  # two steps through the same receive buffers
            assert gat.launch(bm, rep, first=first) is None
        if rank == 0:
            own_member = torch.where(rep >= 0, rep - first, rep)
            q.put((gat.assemble(parts, csr.cluster_off, bm, own_member), loads.tolist(),
                   [len(p) for p in parts], gat.wire, gat.check()))
        else:
            assert gat.check() == 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,wire", [(2, False), (3, False), (2, True), (3, True)])
def test_strong_partition_gather_equals_world1(world, wire):
    """bench.py --scaling strong at world 2/3 under gloo: the size-balanced LPT split
    of ONE batch (shard.strong_partition), per-rank compute on the rank's clusters,
    the per-step gather with member-index representatives, and rank 0's reassembly
    in global order (StepGatherer.assemble) give exactly the world-1 results -- with the
    peaks as f64 (CPU groups) and in the GPU path's 9-byte wire format (f32 bin sums +
    counts, csrc/wire.hip; its numpy model here), rebuilt bit for bit on rank 0."""
    from oracle import c_oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, q, wire)) for r in range(world)]
    for p in procs:
        p.start()
    got, loads, sizes, wbytes, n_fail = q.get(timeout=240)
    assert wbytes == (1 if wire else 0) and n_fail == 0
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    csr = make_clusters_np(61, seed=23)
    ref = c_oracle.bin_mean(csr)
    for k in ("out_off", "out_mz", "out_int"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(got["rep"], c_oracle.medoid(csr))
    assert sum(sizes) == csr.n_clusters and min(sizes) > 0
    cost = shard.costs_from_sizes(csr.cluster_sizes(), csr.cluster_peaks(), "both")
    assert max(loads) <= sum(loads) / world + cost.max()  # the LPT bound
