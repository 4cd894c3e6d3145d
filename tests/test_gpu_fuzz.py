"""Randomised parity: many small batches of varied shape through every kernel
path of the three methods, against the C oracle (bin-mean and medoid bit-exact,
values and totals included; gap-average group structure exact, values within
GAP_RTOL).  Each case draws cluster sizes (1..300, heavy tails), spectrum lengths
(1..900 template peaks), and mutations the reference meets in real files: m/z
snapped to a coarse grid (several peaks per bin, exact m/z ties), unsorted
spectra, empty spectra, a mixed-charge cluster, and non-default bin parameters."""
import numpy as np
import pytest

from oracle import c_oracle
from specpride_amd import engine
from specpride_amd.csr import SpectraCSR
from specpride_amd.synthetic import make_clusters_np
from test_gpu_parity import assert_bin_mean_equal, assert_gap_close

pytestmark = pytest.mark.gpu

N_CASES = 24


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    C = int(rng.integers(4, 40))
    kind = rng.integers(0, 3)
    if kind == 0:
        sizes = rng.integers(1, 60, C)
    elif kind == 1:
        sizes = np.minimum(300, (2 * rng.random(C) ** (-1 / 1.1)).astype(np.int64) + 1)
    else:
        sizes = rng.integers(100, 200, C)
    n_template = int(rng.choice([1, 5, 60, 200, 300, 600, 900]))
    csr = make_clusters_np(C, seed=seed, sizes=sizes, n_template=n_template)
    mz, it, so = csr.mz.copy(), csr.inten.copy(), csr.spec_off
    charge = csr.charge.copy()
    if rng.random() < 0.4:  # coarse grid: duplicate bins and exact m/z ties
        mz = np.round(mz / 0.05) * 0.05
        for s in range(csr.n_spectra):
            a, b = so[s], so[s + 1]
            mz[a:b] = np.sort(mz[a:b])
    if rng.random() < 0.3:  # unsorted spectra
        for s in rng.choice(csr.n_spectra, max(1, csr.n_spectra // 5), replace=False):
            a, b = so[s], so[s + 1]
            p = rng.permutation(b - a)
            mz[a:b], it[a:b] = mz[a:b][p], it[a:b][p]
    if rng.random() < 0.3:  # a mixed-charge cluster
        c = int(rng.integers(0, C))
        s0, s1 = csr.cluster_off[c], csr.cluster_off[c + 1]
        if s1 - s0 > 1:
            charge[s1 - 1] = charge[s0] + 1
    keep_spec = np.ones(csr.n_spectra, bool)
    if rng.random() < 0.3:  # empty spectra (their peaks dropped)
        keep_spec[rng.choice(csr.n_spectra, max(1, csr.n_spectra // 10), replace=False)] = False
    lens = np.where(keep_spec, np.diff(so), 0)
    sel = np.repeat(keep_spec, np.diff(so))
    spec_off = np.zeros(csr.n_spectra + 1, np.int64)
    np.cumsum(lens, out=spec_off[1:])
    out = SpectraCSR(csr.cluster_off, spec_off, mz[sel], it[sel], csr.prec_mz, charge, csr.rt)
    params = [dict(), dict(minimum=float(rng.uniform(50, 300)), maximum=float(rng.uniform(1200, 2500)),
                           binsize=float(rng.choice([0.005, 0.02, 0.05, 0.3])),
                           apply_peak_quorum=bool(rng.random() < 0.7))]
    return out, params


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_bin_mean(gpu, seed):
    csr, params = _case(seed)
    batch = engine.DeviceBatch.from_host(csr)
    for kw in params:
        got = engine.bin_mean(batch, **kw).to_host()
        assert_bin_mean_equal(got, c_oracle.bin_mean(csr, **kw))
        staged = engine.bin_mean(batch, staged=True, **kw).to_host()
        assert_bin_mean_equal(staged, got)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_medoid(gpu, seed):
    csr, _ = _case(seed)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_gap_average(gpu, seed):
    csr, _ = _case(seed)
    got = engine.gap_average(engine.DeviceBatch.from_host(csr)).to_host()
    assert_gap_close(got, c_oracle.gap_average(csr), 1000.0)
