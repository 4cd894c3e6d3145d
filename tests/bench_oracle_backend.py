"""A CPU stand-in for bench.py's HipBackend (test infrastructure only): the same
synthetic law generated on the host, the C oracle as each rank's "kernels", gloo
between ranks and the numpy model of the gather wire format.  tests/test_bench_launcher.py
sets SPX_BENCH_BACKEND=bench_oracle_backend:OracleBackend so that ``bench.py --gpus N``
runs its real launcher, strong split, per-step gather and rank 0's reassembly check
on a machine without a GPU.  The product path never imports this module."""
import numpy as np
import torch

import wire_model
from oracle import c_oracle
from specpride_amd.csr import SpectraCSR
from specpride_amd.synthetic import make_clusters_torch


class _Consensus:
    """An oracle bin-mean result with what bench.py and shard.StepGatherer read:
    ``count``, ``status`` and ``compact(stream=, total=)`` (already dense)."""

    def __init__(self, r):
        self.count = torch.from_numpy(np.diff(r["out_off"]))
        self.status = torch.from_numpy(r["status"].astype(np.int32))
        self._off = torch.from_numpy(r["out_off"])
        self._mz, self._int = torch.from_numpy(r["out_mz"]), torch.from_numpy(r["out_int"])

    def compact(self, stream=None, total=None):
        assert total is None or total == int(self._off[-1])
        return self._off, self._mz, self._int


class _Medoid:
    def __init__(self, rep):
        self.rep = torch.from_numpy(rep)


class OracleBackend:
    kind = "oracle"
    dist_backend = "gloo"

    def __init__(self, local):
        self.dev = torch.device("cpu")
        self.stream = None
        self.wire_ops = wire_model.torch_ops()

    def sync(self):
        pass

    def generate(self, clusters, seed):
        return make_clusters_torch(clusters, seed=seed, device="cpu")

    def select(self, t, ids, co, so):
        return SpectraCSR.select_on_device(t, ids, co, so)

    def batch(self, t):
        return SpectraCSR.from_device(t)

    def _run(self, csr):
        return _Consensus(c_oracle.bin_mean(csr)), _Medoid(c_oracle.medoid(csr))

    def first_step(self, csr):
        bm, md = self._run(csr)
        assert not bool((bm.status != 0).any()) and not bool((md.rep < 0).any())
        return bm, md, None

    def alloc(self, csr):
        return self._run(csr)

    def step(self, csr, bm, md):
        b, m = self._run(csr)
        bm.__dict__.update(b.__dict__)
        md.rep = m.rep

    def record(self):
        return None

    def wait(self, ev):
        pass

    def first(self, csr):
        return torch.from_numpy(csr.cluster_off[:-1])

    def max_cluster_spectra(self, csr):
        return int(csr.cluster_sizes().max())

    def sample_results(self, t, ids, co, so):
        sub = self.batch(self.select(t, ids, co, so))
        r = c_oracle.bin_mean(sub)
        rep = c_oracle.medoid(sub)
        return dict(count=np.diff(r["out_off"]), out_off=r["out_off"], out_mz=r["out_mz"], out_int=r["out_int"],
                    member=np.where(rep >= 0, rep - sub.cluster_off[:-1], rep))
