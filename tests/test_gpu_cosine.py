"""GPU parity of the binned-cosine evaluation (spx_binned_cosine) against the
reference's own benchmark.cos_dist / average_cos_dist outputs (golden) and the
numpy restatement (oracle/np_oracle.py).  Bar: statuses exact, cosines and
averages within 1e-12 relative (the reference sums its dot products in BLAS
order; the north star allows 1e-5)."""
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import load_golden
from oracle import np_oracle
from specpride_amd import benchmark, engine
from specpride_amd.csr import SpectraCSR
from specpride_amd.synthetic import make_clusters_np

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def _dev(a):
    import torch

    return torch.as_tensor(np.ascontiguousarray(a), device="cuda")


def _run(csr, rep_off, rep_mz, rep_int, mz_space=np_oracle.MZ_SPACE):
    b = engine.DeviceBatch.from_host(csr)
    return engine.binned_cosine(b, _dev(rep_off), _dev(rep_mz if len(rep_mz) else np.zeros(1)),
                                _dev(rep_int if len(rep_int) else np.zeros(1)), mz_space=mz_space).to_host()


def _check(got, want, n_clusters, n_spectra):
    cos, avg, st = got
    wcos, wavg, wst = want
    np.testing.assert_array_equal(st[:n_clusters], wst)
    np.testing.assert_allclose(cos[:n_spectra], wcos, rtol=RTOL, atol=0, equal_nan=True)
    np.testing.assert_allclose(avg[:n_clusters], wavg, rtol=RTOL, atol=0, equal_nan=True)


def test_binned_cosine_matches_reference_golden(gpu):
    z, csr = load_golden("binned_cosine.npz")
    got = _run(csr, z["rep_off"], z["rep_mz"], z["rep_int"], float(z["mz_space"]))
    _check(got, (z["cos"], z["avg"], z["status"]), csr.n_clusters, csr.n_spectra)


def _shuffled_members(csr, seed=5):
    rng = np.random.default_rng(seed)
    mz, it = csr.mz.copy(), csr.inten.copy()
    for s in range(0, csr.n_spectra, 5):
        a, b = csr.spec_off[s], csr.spec_off[s + 1]
        p = rng.permutation(b - a)
        mz[a:b], it[a:b] = mz[a:b][p], it[a:b][p]
    return SpectraCSR(csr.cluster_off, csr.spec_off, mz, it, csr.prec_mz, csr.charge, csr.rt)


@pytest.mark.parametrize("rep_kind", ["bin_mean", "medoid"])
def test_binned_cosine_synthetic_vs_oracle(gpu, rep_kind):
    """Representatives as the pipeline makes them: the bin-mean consensus
    (compacted engine output) or the medoid spectrum; every fifth member
    unsorted (the O(m^2) B.B path)."""
    csr = make_clusters_np(50, seed=77)
    b = engine.DeviceBatch.from_host(csr)
    if rep_kind == "bin_mean":
        r = engine.bin_mean(b).to_host()
        rep_off, rep_mz, rep_int = r["out_off"], r["out_mz"], r["out_int"]
    else:
        rep, _ = engine.medoid(b).to_host()
        lens = csr.spec_off[rep + 1] - csr.spec_off[rep]
        rep_off = np.concatenate([[0], np.cumsum(lens)])
        rep_mz = np.concatenate([csr.mz[csr.spec_off[s]:csr.spec_off[s + 1]] for s in rep])
        rep_int = np.concatenate([csr.inten[csr.spec_off[s]:csr.spec_off[s + 1]] for s in rep])
    mem = _shuffled_members(csr)
    got = _run(mem, rep_off, rep_mz, rep_int)
    want = np_oracle.binned_cosine(mem, rep_off, rep_mz, rep_int)
    _check(got, want, csr.n_clusters, csr.n_spectra)
    assert np.all(got[2][:csr.n_clusters] == 0) and np.all(got[1][:csr.n_clusters] > 0.0)


def test_binned_cosine_long_members_and_runs(gpu):
    """Members longer than a wave (runs carried across 64-peak chunks), many
    peaks per bin, a representative longer than the members."""
    rng = np.random.default_rng(3)
    clusters, reps = [], []
    for k in range(6):
        base = np.sort(rng.uniform(100, 1900, 40))
        members = []
        for _ in range(5 + k):
            mz = np.sort(np.concatenate([base + rng.normal(0, 0.0008, 40) for _ in range(5)]))  # 200 peaks, dense bins
            members.append({"m/z array": np.round(mz, 5), "intensity array": rng.lognormal(5, 1, len(mz))})
        clusters.append(members)
        rm = np.sort(np.concatenate([base, rng.uniform(100, 1990, 300)]))
        reps.append((rm, rng.lognormal(4, 1, len(rm))))
    csr = SpectraCSR.from_clusters(clusters)
    rep_off = np.concatenate([[0], np.cumsum([len(r[0]) for r in reps])])
    rep_mz, rep_int = np.concatenate([r[0] for r in reps]), np.concatenate([r[1] for r in reps])
    _check(_run(csr, rep_off, rep_mz, rep_int), np_oracle.binned_cosine(csr, rep_off, rep_mz, rep_int),
           csr.n_clusters, csr.n_spectra)


def test_benchmark_shim_names(gpu):
    """specpride_amd.benchmark keeps the reference's function names (benchmark.py:19-38)."""
    a = SimpleNamespace(mz=np.array([200.0, 250.0, 900.0]), intensity=np.array([3.0, 4.0, 5.0]))
    b = SimpleNamespace(mz=np.array([200.001, 500.0]), intensity=np.array([1.0, 2.0]))
    assert benchmark.cos_dist(a, a) == pytest.approx(1.0, rel=1e-15)
    want = np_oracle.cos_dist(a.mz, a.intensity, b.mz, b.intensity)
    assert benchmark.cos_dist(a, b) == pytest.approx(want, rel=RTOL)
    assert benchmark.average_cos_dist(a, []) == 0.0
    assert benchmark.average_cos_dist(a, [a, b]) == pytest.approx((1.0 + want) / 2, rel=RTOL)
    with pytest.raises(IndexError):
        benchmark.cos_dist(a, SimpleNamespace(mz=np.zeros(0), intensity=np.zeros(0)))


def test_binned_cosine_representatives_past_lds(gpu):
    """Representatives of 1,025-5,000 peaks (the global-scratch path), mixed with
    ordinary ones in one call; one of them unsorted (the rank sort), one sharing
    bins with every member (runs of several peaks)."""
    rng = np.random.default_rng(41)
    clusters, reps = [], []
    for k, R in enumerate((300, 1025, 2048, 5000, 900, 1500)):
        base = np.sort(rng.uniform(100, 1900, 60))
        members = [{"m/z array": np.round(np.sort(base + rng.normal(0, 0.002, 60)), 5),
                    "intensity array": rng.lognormal(5, 1, 60)} for _ in range(3 + k)]
        clusters.append(members)
        rm = np.concatenate([np.repeat(base, 3) + rng.normal(0, 0.0005, 180), rng.uniform(100, 1990, R - 180)])
        rm = np.round(rm, 5)
        if k != 5:
            rm = np.sort(rm)  # cluster 5: an unsorted representative
        reps.append((rm, rng.lognormal(4, 1, len(rm))))
    csr = SpectraCSR.from_clusters(clusters)
    rep_off = np.concatenate([[0], np.cumsum([len(r[0]) for r in reps])])
    rep_mz, rep_int = np.concatenate([r[0] for r in reps]), np.concatenate([r[1] for r in reps])
    got = _run(csr, rep_off, rep_mz, rep_int)
    assert np.all(got[2][:csr.n_clusters] == 0)
    _check(got, np_oracle.binned_cosine(csr, rep_off, rep_mz, rep_int), csr.n_clusters, csr.n_spectra)
