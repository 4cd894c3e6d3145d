"""The three CLIs on the GPU: native ingest (mgf_io.cpp straight to the CSR),
the dict path (the reference's readers) and the rank-local sharded driver over a
world-1 ``nccl`` (RCCL) group with the HIP engine as compute all write the same
bytes.  Inputs: golden files and an interleaved synthetic clustered MGF.

Reference: binning.py:286-302, average_spectrum_clustering.py:151-165/:201-203,
most_similar_representative.py:22-115.
"""
import contextlib
import io
import os
import socket

import pytest

from conftest import GOLDEN
from specpride_amd import average_spectrum_clustering as asc
from specpride_amd import binning, sharded_cli
from specpride_amd import most_similar_representative as msr
from test_sharded_cli import synthetic_mgf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_world1():
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def syn(tmp_path_factory):
    return synthetic_mgf(str(tmp_path_factory.mktemp("syn") / "clustered.mgf"), n_clusters=200, seed=5)


def _src(which, syn, golden):
    return syn if which == "syn" else os.path.join(GOLDEN, golden)


def _quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


@pytest.mark.parametrize("which", ["golden", "syn"])
def test_binning_cli_native_dict_sharded_identical(gpu, rccl_world1, syn, tmp_path, which):
    src = _src(which, syn, "bin_mean_cli_in.mgf")
    native, sharded = tmp_path / "n.mgf", tmp_path / "s.mgf"
    _quiet(binning._main_mgf, src, str(native), 1)
    rsc = binning.RepresentativeSpectrumCreator()
    clusters = rsc.read_spectra_clustered_mgf(src)
    ids = list(clusters.keys())
    merged = rsc.combine_bin_mean_batch([clusters[k] for k in ids])
    for cid, spec in zip(ids, merged):
        spec["cluster_id"] = cid
    with open(tmp_path / "d.mgf", "wt") as fh:
        rsc.write_spectrum(merged, fh)
    assert sharded_cli.binning(src, str(sharded), device=gpu) is None
    want = native.read_bytes()
    assert (tmp_path / "d.mgf").read_bytes() == want
    assert sharded.read_bytes() == want
    if which == "golden":
        assert want == open(os.path.join(GOLDEN, "bin_mean_cli_out.mgf"), "rb").read()


@pytest.mark.parametrize("which", ["golden", "syn"])
def test_gap_average_cli_native_dict_sharded_identical(gpu, rccl_world1, syn, tmp_path, which):
    src = _src(which, syn, "bin_mean_cli_in.mgf")
    native, sharded = tmp_path / "n.mgf", tmp_path / "s.mgf"
    asc.main([src, str(native), "--encodedclusters"])
    # dict path: the same helpers through a lambda (custom get_cluster -> no native ingest)
    outs = asc.process_maracluster_mgf(src, get_cluster=lambda t: asc.get_cluster_id(t),
                                       get_pepmass=asc.lower_median_mass, get_rt=asc.lower_median_mass_rt)
    asc.write_pyteomics_style(outs, str(tmp_path / "d.mgf"))
    assert sharded_cli.gap_average(src, str(sharded), device=gpu) is None
    want = native.read_bytes()
    assert (tmp_path / "d.mgf").read_bytes() == want
    assert sharded.read_bytes() == want


@pytest.mark.parametrize("which", ["golden", "syn"])
def test_medoid_cli_native_dict_sharded_identical(gpu, rccl_world1, syn, tmp_path, which, monkeypatch):
    from specpride_amd import mgf_native

    src = _src(which, syn, "medoid_noncontiguous.mgf")
    native, dicts, sharded = tmp_path / "n.mgf", tmp_path / "d.mgf", tmp_path / "s.mgf"
    out_n = io.StringIO()
    with contextlib.redirect_stdout(out_n):
        msr.main(["-i", src, "-o", str(native)])
    out_s = io.StringIO()
    with contextlib.redirect_stdout(out_s):
        assert sharded_cli.medoid(src, str(sharded), device=gpu) is None
    # dict leg: the native reader is switched off, so main() must take read_mgf
    seen = []
    real_read = msr.read_mgf
    monkeypatch.setattr(mgf_native, "parse_general", lambda *a, **k: None)
    monkeypatch.setattr(msr, "read_mgf", lambda path: seen.append(path) or real_read(path))
    out_d = io.StringIO()
    with contextlib.redirect_stdout(out_d):
        msr.main(["-i", src, "-o", str(dicts)])
    assert seen == [src], "the dict path did not run"
    assert out_n.getvalue() == out_d.getvalue() == out_s.getvalue()
    want = native.read_bytes()
    assert dicts.read_bytes() == want
    assert sharded.read_bytes() == want


def test_medoid_cli_outside_native_subset(gpu, tmp_path):
    """A record with two charges ("2+ and 3+") is outside the native reader's
    subset: main() takes the dict path and still picks the reference's
    representatives (tests/golden/medoid_noncontiguous.json)."""
    import json

    from specpride_amd import mgf_native
    from specpride_amd.mgf import read_mgf

    text = open(os.path.join(GOLDEN, "medoid_noncontiguous.mgf")).read().replace("CHARGE=2+", "CHARGE=2+ and 3+", 1)
    src = tmp_path / "multi_charge.mgf"
    src.write_text(text)
    with pytest.raises(ValueError, match="fallback"):
        mgf_native.parse_general(str(src))
    out = tmp_path / "o.mgf"
    _quiet(msr.main, ["-i", str(src), "-o", str(out)])
    gold = json.load(open(os.path.join(GOLDEN, "medoid_noncontiguous.json")))
    got = read_mgf(str(out))
    assert [s["params"]["title"] for s in got] == gold["titles"]
    assert got[0]["params"]["charge"] == [2, 3]
