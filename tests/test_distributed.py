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
