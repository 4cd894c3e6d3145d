"""Rank-local multi-GPU mode of the three CLIs.

Under ``torchrun`` (WORLD_SIZE > 1) ``binning.main``, ``average_spectrum_clustering
.main --encodedclusters`` and ``most_similar_representative.main`` run here:

1. rank k indexes only byte stripe [k*size/W, (k+1)*size/W) of the input MGF
   (``mgf_native.index_range``: the records whose start line lies in it -- byte
   range, title, peak-line count; no number is parsed; multithreaded), and one
   all-gather of that metadata gives every rank the whole index, from which it
   derives the reference's cluster grouping (:mod:`specpride_amd.ingest`);
2. the clusters are LPT-planned over the ranks from the index's spectrum and
   peak counts (:func:`specpride_amd.shard.plan_costs`) -- every rank computes
   the same plan, no exchange;
3. each rank parses ONLY its own clusters' records (``mgf_native.parse_ranges``)
   straight into its CSR, uploads it to its GPU and runs the kernel -- no rank
   ever holds another rank's peaks;
4. the results (consensus peaks, or the chosen representative spectra) are
   gathered to rank 0 (:func:`specpride_amd.shard.gatherv`: RCCL point-to-point
   over xGMI under ``nccl``, ``gloo`` on CPU), which writes the output file in
   the reference's order with the native multithreaded writer
   (``mgf_native.write_records``), byte-identical to the single-process run.

Per-rank compute is injectable (``compute=``: CSR -> dict of tensors, the
:mod:`specpride_amd.shard` contract) so the CPU test suite drives the same code
with the oracle under ``gloo``; the default is the HIP engine on
``cuda:LOCAL_RANK``.  When the input is outside the native parser's subset (or
a record lacks a field the reference indexes) every rank agrees (one
all-reduce) and the drivers return :data:`FALLBACK`: the CLI then runs the
single-process path on rank 0, which behaves -- or raises -- as the reference.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np

from . import ingest, mgf_native, shard
from .csr import concat_ranges

FALLBACK = "fallback"


# ------------------------------------------------------------------ process group
def launched_distributed() -> bool:
    return int(os.environ.get("WORLD_SIZE", "1")) > 1


def init_from_env():
    """Process group from torchrun's env (nccl = RCCL when a GPU is visible, else
    gloo); returns the device this rank computes on."""
    import torch
    import torch.distributed as dist

    if torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=dev)
        return dev
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return torch.device("cpu")


def run_cli(driver: Callable, fallback: Callable, *args, **kwargs):
    """Run ``driver`` on every rank of a torchrun job; rank 0 runs ``fallback``
    when the drivers report :data:`FALLBACK`.  The group is torn down after."""
    import torch.distributed as dist

    device = init_from_env()
    try:
        rc = driver(*args, device=device, **kwargs)
        rank = dist.get_rank()
        dist.barrier()
    finally:
        dist.destroy_process_group()
    if rc == FALLBACK and rank == 0:
        return fallback()
    return None


# ------------------------------------------------------------------ shared steps
def rank_index(path, general: bool, group=None):
    """The whole file's record index, built rank-locally: this rank indexes its
    byte stripe and the stripes' metadata is all-gathered (stripes are in file
    order, so their concatenation is ``mgf_native.index(path, general)``)."""
    world, rank = shard.world_rank(group)
    size = os.path.getsize(path)
    try:
        mine = mgf_native.index_range(path, general, rank * size // world, (rank + 1) * size // world)
    except ValueError:  # outside the native subset (e.g. a NUL byte in a title): every rank agrees
        mine = None
    if not shard.all_true(mine is not None, group):
        return None
    if world == 1:
        return mine
    titles = "\n".join(mine["titles"]).encode("utf-8", errors="surrogateescape")
    got = shard.allgatherv([mine["begin"], mine["end"], mine["npk"], np.frombuffer(titles, np.uint8)], group)
    X = {k: np.concatenate([g[i] for g in got]) for i, k in enumerate(("begin", "end", "npk"))}
    X["titles"] = [t for g in got if len(g[0])
                   for t in g[3].tobytes().decode("utf-8", errors="surrogateescape").split("\n")]
    return X


def _load_my_clusters(path, general: bool, groups: Callable, method: str, group):
    """Index -> grouping -> plan -> parse own records.  Returns (ids, records,
    sizes, parts, mine, X, flat, ok): cluster ids, record indices in CSR order,
    members per cluster, the plan, this rank's clusters, the index, this rank's
    parse (None if outside the native subset) and whether it is usable; None when
    the file cannot be indexed natively (every rank then falls back)."""
    world, rank = shard.world_rank(group)
    X = rank_index(path, general, group)
    if X is None:
        return None
    ids, records, sizes = groups(X["titles"])
    starts = ingest.cluster_starts(sizes)
    peaks = np.add.reduceat(X["npk"][records], starts[:-1]) if len(records) else np.zeros(0, np.int64)
    parts = shard.plan_costs(shard.costs_from_sizes(sizes, peaks, method), world)
    mine = parts[rank]
    my_records = records[concat_ranges(starts[mine], sizes[mine])] if len(mine) else np.zeros(0, np.int64)
    try:
        flat = mgf_native.parse_ranges(path, X["begin"][my_records], X["end"][my_records], general)
        ok = flat["titles"] == [X["titles"][r] for r in my_records]
    except ValueError:
        flat, ok = None, False
    return ids, records, sizes, parts, mine, X, flat, ok


def _engine_compute(method: str, params: dict, device):
    return shard._engine_medoid(params, device) if method == "medoid" else \
        shard._engine_consensus(method, params, device)


# ------------------------------------------------------------------ bin-mean
def binning(mgf_file: str, out: str, group=None, device=None, compute: Optional[Callable] = None,
            minimum=100, maximum=2000, binsize=0.02):
    """binning.py's ``--mgf_file`` CLI (binning.py:286-302), rank-local."""
    from .binning import MIXED_CHARGE_MSG
    from .engine import STATUS_MIXED_CHARGE, STATUS_OK

    loaded = _load_my_clusters(mgf_file, False, ingest.binning_groups, "bin_mean", group)
    if loaded is None:
        return FALLBACK
    ids, _rec, sizes, parts, mine, X, flat, ok = loaded
    ok = ok and all(";" in t for t in X["titles"]) and bool(flat["has_prec"].all() and flat["has_charge"].all())
    if not shard.all_true(ok, group):
        return FALLBACK
    sub = ingest.csr_from_flat(flat, sizes[mine])
    params = dict(minimum=minimum, maximum=maximum, binsize=binsize)
    res = (compute or _engine_compute("bin_mean", params, device))(sub)
    r = shard.gather_consensus(res, parts, len(ids), group)
    if r is None:
        return None
    bad = np.flatnonzero(r["status"] != STATUS_OK)
    if len(bad):
        if r["status"][bad[0]] == STATUS_MIXED_CHARGE:
            raise AssertionError(MIXED_CHARGE_MSG)
        raise IndexError("list index out of range")
    mgf_native.write_records(out, mgf_native.STYLE_BINNING, ids, r["out_off"], r["out_mz"], r["out_int"], r["prec"],
                             r["charge"])
    return None


# ------------------------------------------------------------------ gap-average
def gap_average(input_mgf: str, output, group=None, device=None, compute: Optional[Callable] = None,
                mz_accuracy=0.01, dyn_range=1000.0, min_fraction=0.5, pepmass="lower_median",
                rt="mass_lower_median", file_mode="w"):
    """average_spectrum_clustering.py ``--encodedclusters`` (:151-165, :201-203), rank-local."""
    from .average_spectrum_clustering import _raise_for, write_outputs_native
    from .engine import STATUS_OK
    from .mgf import write_pyteomics_style

    loaded = _load_my_clusters(input_mgf, True, ingest.gap_average_groups, "gap_average", group)
    if loaded is None:
        return FALLBACK
    ids, _rec, sizes, parts, mine, X, flat, ok = loaded
    ok = ok and bool(flat["has_title"].all())
    if not shard.all_true(ok, group):
        return FALLBACK
    sub = ingest.csr_from_flat(flat, sizes[mine])
    params = dict(mz_accuracy=mz_accuracy, dyn_range=dyn_range, min_fraction=min_fraction, pepmass=pepmass, rt=rt)
    res = (compute or _engine_compute("gap_average", params, device))(sub)
    r = shard.gather_consensus(res, parts, len(ids), group)
    if r is None:
        return None
    if output is not None:
        write_outputs_native(r, ids, output, file_mode=file_mode)
        return None
    outputs = []
    for c, cid in enumerate(ids):
        if r["status"][c] != STATUS_OK:
            _raise_for(r["status"][c])
        a, b = r["out_off"][c], r["out_off"][c + 1]
        outputs.append({"params": {"title": cid, "pepmass": float(r["prec"][c]), "rtinseconds": float(r["rt"][c]),
                                   "charge": int(r["charge"][c])},
                        "m/z array": r["out_mz"][a:b], "intensity array": r["out_int"][a:b]})
    write_pyteomics_style(outputs, output, file_mode=file_mode)
    return None


# ------------------------------------------------------------------ medoid
def medoid(inputfile: str, outputfile: str, group=None, device=None, compute: Optional[Callable] = None,
           tolerance=0.1, verbose=True):
    """most_similar_representative.py main (:22-115), rank-local: each rank sends
    rank 0 only the representative spectra it chose."""
    import torch

    loaded = _load_my_clusters(inputfile, True, ingest.medoid_groups, "medoid", group)
    if loaded is None:
        return FALLBACK
    ids, records, sizes, parts, mine, X, flat, ok = loaded
    ok = ok and bool(flat["has_title"].all())
    if not shard.all_true(ok, group):
        return FALLBACK
    sub = ingest.csr_from_flat(flat, sizes[mine])
    res = (compute or _engine_compute("medoid", dict(tolerance=tolerance), device))(sub)
    member = res["member"].cpu().numpy().astype(np.int64)
    # the chosen spectra of this rank, packed: lengths, scalars, peaks (a failure
    # code travels in ``member``; rank 0 raises after the gather)
    chosen = sub.cluster_off[:-1] + np.maximum(member, 0)
    so = flat["spec_off"]
    lens = so[chosen + 1] - so[chosen]
    idx = concat_ranges(so[chosen], lens)
    flags = (flat["has_prec"][chosen].astype(np.int64) | (flat["has_charge"][chosen].astype(np.int64) << 1) |
             (flat["has_rt"][chosen].astype(np.int64) << 2))
    t = torch.from_numpy
    dev = res["member"].device
    payload = [t(np.ascontiguousarray(a)).to(dev) for a in
               (member, lens, flags, flat["charge"][chosen], flat["prec_mz"][chosen], flat["rt"][chosen],
                flat["mz"][idx], flat["inten"][idx])]
    got = shard.gatherv(payload, group=group)
    if got is None:
        return None
    C = len(ids)
    cols = [None] * 8
    for k in range(6):
        dt = got[0][k].cpu().numpy().dtype
        cols[k] = np.zeros(C, dt)
        for r, cl in enumerate(parts):
            if len(cl):
                cols[k][cl] = got[r][k].cpu().numpy()
    member, lens, flags, charge, prec, rt = cols[:6]
    if np.any(member < 0):
        raise RuntimeError("medoid engine could not resolve a cluster (see DESIGN.md limits)")
    off = ingest.cluster_starts(lens)
    mz, inten = np.empty(off[-1]), np.empty(off[-1])
    for r, cl in enumerate(parts):
        if len(cl):
            dst = concat_ranges(off[cl], lens[cl])
            mz[dst] = got[r][6].cpu().numpy()
            inten[dst] = got[r][7].cpu().numpy()
    starts = ingest.cluster_starts(sizes)
    if verbose:
        print("".join(f"{cl}\n{int(sizes[c])}\n" for c, cl in enumerate(ids)), end="")
        print(C)
    titles = [X["titles"][records[starts[c] + member[c]]] for c in range(C)]
    mgf_native.write_records(outputfile, mgf_native.STYLE_MEDOID, titles, off, mz, inten, prec, charge, rt,
                             flags.astype(np.int32) | mgf_native.FLAG_TITLE)
    return None
