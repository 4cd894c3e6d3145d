"""Rank-local sharded CLIs (specpride_amd.sharded_cli) under ``gloo`` on CPU.

Each rank indexes the MGF, plans, parses ONLY its own clusters' records and
runs the per-rank compute (the C / numpy oracle here; the HIP engine on
MI355X); rank 0 gathers and writes.  Checked:

* the output file of world 2 and 3 is byte-identical to world 1 (same driver,
  no process group) -- and for the bin-mean CLI to the reference's own output
  (tests/golden/bin_mean_cli_out.mgf), for the medoid CLI to the reference
  representatives (tests/golden/medoid_noncontiguous.json);
* no rank parses a record of another rank: the record ranges each rank read are
  disjoint and together cover every record of the file;
* the world-1 driver's output equals the single-process CLI's dict path
  (the reference's line loop) -- see test_host.py for the native-vs-dict checks.

Reference: binning.py:122-167/:286-302, average_spectrum_clustering.py:151-165,
most_similar_representative.py:22-115.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ------------------------------------------------------------ oracle computes
def oracle_compute(method):
    from oracle import c_oracle, np_oracle

    t = torch.from_numpy

    def run(sub):
        C = sub.n_clusters
        if method == "medoid":
            rep = c_oracle.medoid(sub)
            return dict(member=t(np.where(rep >= 0, rep - sub.cluster_off[:-1], rep)))
        r = getattr(c_oracle, method)(sub)
        d = dict(count=t(np.diff(r["out_off"])), status=t(r["status"]), mz=t(r["out_mz"]), inten=t(r["out_int"]))
        if method == "bin_mean":
            d["prec"], d["charge"] = t(r["prec"]), t(r["charge"])
            return d
        prec, charge, rt = np.zeros(C), np.zeros(C, np.int32), np.zeros(C)
        for c in range(C):
            a, b = sub.cluster_off[c], sub.cluster_off[c + 1]
            prec[c], charge[c] = np_oracle.lower_median_mass(sub.prec_mz[a:b], sub.charge[a:b])
            rt[c] = np_oracle.lower_median_mass_rt(sub.prec_mz[a:b], sub.charge[a:b], sub.rt[a:b])
        d.update(prec=t(prec), charge=t(charge), rt=t(rt))
        return d
    return run


def write_records(path, csr, order, titles):
    """An MGF whose records are csr's spectra in ``order`` (interleaving clusters)."""
    with open(path, "w") as fh:
        for s in order:
            mz, it = csr.spectrum(s)
            fh.write(f"BEGIN IONS\nTITLE={titles[s]}\nPEPMASS={float(csr.prec_mz[s])!r}\n"
                     f"CHARGE={int(csr.charge[s])}+\nRTINSECONDS={float(csr.rt[s])!r}\n")
            fh.write("".join(f"{float(a)!r} {float(b)!r}\n" for a, b in zip(mz, it)))
            fh.write("END IONS\n\n")


def synthetic_mgf(path, n_clusters=23, seed=3):
    from specpride_amd.synthetic import make_clusters_np

    csr = make_clusters_np(n_clusters, seed=seed, max_size=12)
    owner = np.repeat(np.arange(csr.n_clusters), np.diff(csr.cluster_off))
    titles = [f"cl{owner[s]};mzspec:PXDSYN:synthetic:scan:{s}" for s in range(csr.n_spectra)]
    # interleave: the bin-mean reader merges a cluster's members wherever they are,
    # the gap-average reader makes one run per contiguous block
    order = np.random.default_rng(seed).permutation(csr.n_spectra)
    order = np.concatenate([np.sort(order[: csr.n_spectra // 2]), order[csr.n_spectra // 2:]])
    write_records(path, csr, order, titles)
    return path


# ------------------------------------------------------------ drivers per CLI
CASES = {
    "bin_mean": ("binning", [os.path.join(GOLD, "bin_mean_cli_in.mgf"), "SYN"]),
    "gap_average": ("gap_average", [os.path.join(GOLD, "bin_mean_cli_in.mgf"), "SYN"]),
    "medoid": ("medoid", [os.path.join(GOLD, "medoid_noncontiguous.mgf"), "SYN"]),
}


def _run_driver(method, src, out, group=None):
    from specpride_amd import mgf_native, sharded_cli

    read, stripes = [], []
    orig, orig_ix = mgf_native.parse_ranges, mgf_native.index_range

    def spy(path, begin, end, general, threads=0):
        read.extend(zip(np.asarray(begin).tolist(), np.asarray(end).tolist()))
        return orig(path, begin, end, general, threads)

    def spy_ix(path, general, lo, hi, threads=0):
        stripes.append((lo, hi))
        return orig_ix(path, general, lo, hi, threads)

    mgf_native.parse_ranges, mgf_native.index_range = spy, spy_ix
    try:
        fn = getattr(sharded_cli, CASES[method][0])
        kw = dict(verbose=False) if method == "medoid" else {}
        rc = fn(src, out, group=group, compute=oracle_compute(method), **kw)
    finally:
        mgf_native.parse_ranges, mgf_native.index_range = orig, orig_ix
    read.append(("stripes", stripes))
    return rc, read


def _worker(rank, world, port, q, method, src, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rc, read = _run_driver(method, src, out)
        q.put((rank, rc, read))
    finally:
        dist.destroy_process_group()


def _sharded(method, src, out, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, method, src, out)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = {}
    for r, rc, read in got:
        assert read[-1][0] == "stripes"
        res[r] = (rc, read[:-1], read[-1][1])
    return res


@pytest.fixture(scope="module")
def syn(tmp_path_factory):
    return synthetic_mgf(str(tmp_path_factory.mktemp("syn") / "clustered.mgf"))


@pytest.mark.parametrize("method", ["bin_mean", "gap_average", "medoid"])
@pytest.mark.parametrize("which", [0, 1])
def test_sharded_cli_byte_identical(method, which, syn, tmp_path):
    from specpride_amd import mgf_native

    src = CASES[method][1][which]
    src = syn if src == "SYN" else src
    one = str(tmp_path / "w1.mgf")
    rc, read1 = _run_driver(method, src, one)
    read1 = read1[:-1]
    assert rc is None
    want = open(one, "rb").read()
    assert want.count(b"BEGIN IONS") > 0
    from specpride_amd import ingest

    titles = mgf_native.index(src, method != "bin_mean")["titles"]
    # the records the CLI uses (the medoid CLI ignores later runs of a split cluster)
    n_records = len(getattr(ingest, f"{'binning' if method == 'bin_mean' else method}_groups")(titles)[1])
    assert len(read1) == n_records
    for world in (2, 3):
        out = str(tmp_path / f"w{world}.mgf")
        res = _sharded(method, src, out, world)
        assert all(rc is None for rc, _, _ in res.values())
        # rank-local indexing: rank r indexed exactly byte stripe [r*size/W, (r+1)*size/W)
        size = os.path.getsize(src)
        assert [res[r][2] for r in range(world)] == [[(r * size // world, (r + 1) * size // world)]
                                                     for r in range(world)]
        assert open(out, "rb").read() == want, f"world {world} output differs"
        # rank-local ingest: disjoint record sets covering the file
        sets = [set(map(tuple, res[r][1])) for r in range(world)]
        assert sum(len(s) for s in sets) == n_records
        assert set().union(*sets) == set(map(tuple, read1))
        assert all(len(s) for s in sets)


def test_sharded_binning_matches_reference_output(tmp_path):
    """bin_mean_cli_out.mgf is the reference binning.py's own output for
    bin_mean_cli_in.mgf (tests/golden/make_golden.py)."""
    out = str(tmp_path / "o.mgf")
    res = _sharded("bin_mean", os.path.join(GOLD, "bin_mean_cli_in.mgf"), out, 2)
    assert all(rc is None for rc, _, _ in res.values())
    assert open(out, "rb").read() == open(os.path.join(GOLD, "bin_mean_cli_out.mgf"), "rb").read()


def test_sharded_medoid_matches_reference_representatives(tmp_path):
    from specpride_amd.mgf import read_mgf

    gold = json.load(open(os.path.join(GOLD, "medoid_noncontiguous.json")))
    out = str(tmp_path / "o.mgf")
    _sharded("medoid", os.path.join(GOLD, "medoid_noncontiguous.mgf"), out, 2)
    assert [s["params"]["title"] for s in read_mgf(out)] == gold["titles"]


def test_sharded_fallback_outside_native_subset(tmp_path):
    """A file the native parser does not take (tab-separated peaks in the binning
    format) makes every rank return FALLBACK, so the CLI runs the reference's
    line loop on rank 0."""
    from specpride_amd import sharded_cli

    src = tmp_path / "tabs.mgf"
    src.write_text("BEGIN IONS\nTITLE=a;u1\nPEPMASS=500.0\nCHARGE=2+\n100.0\t5.0\nEND IONS\n")
    rc, _ = _run_driver("bin_mean", str(src), str(tmp_path / "o.mgf"))
    assert rc == sharded_cli.FALLBACK


def test_sharded_gap_average_raises_like_reference(tmp_path):
    """maracluster_in.mgf has a run whose every group is dropped: the reference
    raises ValueError (max of an empty array); so does the sharded driver."""
    with pytest.raises(ValueError, match="zero-size array"):
        _run_driver("gap_average", os.path.join(GOLD, "maracluster_in.mgf"), str(tmp_path / "o.mgf"))


def test_medoid_cli_titleless_raises_without_recursion(tmp_path):
    """A record without TITLE: the native ingest declines it and the dict path
    fails as the reference does (getMetaValue("TITLE").decode() on None), once
    -- no RecursionError."""
    from specpride_amd import most_similar_representative as msr

    src = tmp_path / "notitle.mgf"
    src.write_text("BEGIN IONS\nPEPMASS=500.0\nCHARGE=2+\n100.0 5.0\nEND IONS\n\n"
                   "BEGIN IONS\nTITLE=a;u2\nPEPMASS=500.0\nCHARGE=2+\n101.0 5.0\nEND IONS\n")
    with pytest.raises(AttributeError, match="decode"):
        msr.main(["-i", str(src), "-o", str(tmp_path / "o.mgf")])


def _torchrun_worker(rank, world, port, q, src, out):
    """One rank of `torchrun most_similar_representative.py` (env-initialised gloo group)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    from specpride_amd import most_similar_representative as msr

    try:
        msr.main(["-i", src, "-o", out])
        q.put((rank, None))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, type(e).__name__))


def test_medoid_cli_torchrun_fallback_runs_rank0_once(tmp_path):
    """Under torchrun (WORLD_SIZE=2) an input the native ingest declines makes
    every rank agree on FALLBACK; rank 0 then runs the single-process body once,
    after the group is gone, without re-entering the torchrun dispatch (which
    would re-initialise a group alone and hang)."""
    src = tmp_path / "notitle.mgf"
    src.write_text("BEGIN IONS\nPEPMASS=500.0\nCHARGE=2+\n100.0 5.0\nEND IONS\n\n"
                   "BEGIN IONS\nTITLE=a;u2\nPEPMASS=500.0\nCHARGE=2+\n101.0 5.0\nEND IONS\n")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_torchrun_worker, args=(r, 2, port, q, str(src), str(tmp_path / "o.mgf")))
             for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got == {0: "AttributeError", 1: None}
