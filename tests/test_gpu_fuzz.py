"""Randomised parity: many small batches of varied shape through every kernel
path of the three methods, against the C oracle (bin-mean and medoid bit-exact,
values and totals included; gap-average group structure exact, values within
GAP_RTOL).  Each case draws cluster sizes (1..300, heavy tails), spectrum lengths
(1..900 template peaks), and mutations the reference meets in real files: m/z
snapped to a coarse grid (several peaks per bin, exact m/z ties), unsorted
spectra, empty spectra, a mixed-charge cluster, m/z past the medoid's register
range and bin range, zero intensities, and non-default bin-mean / gap-average
parameters; the binned cosine, xcorr distance and best score ride along."""
import numpy as np
import pytest

from oracle import c_oracle, np_oracle
from specpride_amd import engine
from specpride_amd.csr import SpectraCSR
from specpride_amd.synthetic import make_clusters_np
from test_gpu_parity import assert_bin_mean_equal, assert_gap_close

pytestmark = pytest.mark.gpu

N_CASES = 40


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
    if rng.random() < 0.25:  # m/z past the medoid's register bitmap (3,276.8) and bin range (6,553.6)
        far = rng.choice(len(mz), max(1, len(mz) // 200), replace=False)
        mz[far] = rng.choice([3300.0, 7000.0, 15000.0]) + rng.uniform(0, 50, len(far))
        for s in range(csr.n_spectra):
            a, b = so[s], so[s + 1]
            o = np.argsort(mz[a:b], kind="stable")
            mz[a:b], it[a:b] = mz[a:b][o], it[a:b][o]
    if rng.random() < 0.2:  # zero intensities
        it[rng.choice(len(it), max(1, len(it) // 50), replace=False)] = 0.0
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
    tol = float(np.random.default_rng(4000 + seed).choice([0.02, 0.05, 0.3, 1.0]))  # other xcorr tolerances
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), tolerance=tol, with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, tol=tol, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_gap_average(gpu, seed):
    csr, _ = _case(seed)
    batch = engine.DeviceBatch.from_host(csr)
    rng = np.random.default_rng(2000 + seed)
    for kw in (dict(), dict(mz_accuracy=float(rng.choice([0.005, 0.02, 0.05])),
                            dyn_range=float(rng.choice([10.0, 100.0, 1e4])),
                            min_fraction=float(rng.choice([0.1, 0.3, 0.8])))):
        got = engine.gap_average(batch, **kw).to_host()
        assert_gap_close(got, c_oracle.gap_average(csr, **kw), kw.get("dyn_range", 1000.0))


@pytest.mark.parametrize("seed", range(0, N_CASES, 2))
def test_fuzz_cosine_xcorr_best(gpu, seed):
    """The side entry points on the same batches: the binned cosine of each
    cluster's bin-mean consensus vs its members (<= 1e-12 rel), the xcorr distance
    of random spectrum pairs (exact), the best-score argmax (exact)."""
    import torch

    csr, _ = _case(seed)
    batch = engine.DeviceBatch.from_host(csr)
    cons = engine.bin_mean(batch).to_host()
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda:0")  # noqa: E731
    cos, avg, st = engine.binned_cosine(batch, dev(cons["out_off"]), dev(cons["out_mz"]),
                                        dev(cons["out_int"])).to_host()
    wcos, wavg, wst = np_oracle.binned_cosine(csr, cons["out_off"], cons["out_mz"], cons["out_int"])
    C = csr.n_clusters
    np.testing.assert_array_equal(st[:C], wst)
    ok = wst == 0
    np.testing.assert_allclose(avg[:C][ok], wavg[ok], rtol=1e-12)
    rng = np.random.default_rng(3000 + seed)
    pairs = rng.integers(0, csr.n_spectra, (min(500, csr.n_spectra * 3), 2))
    d = engine.xcorr_distance(batch, dev(pairs)).cpu().numpy()
    so = csr.spec_off
    want = np.array([1.0 - np_oracle.xcorr(csr.mz[so[a]:so[a + 1]], csr.mz[so[b]:so[b + 1]]) for a, b in pairs])
    np.testing.assert_array_equal(d, want)
    score = rng.integers(0, 4, csr.n_spectra).astype(np.float64)
    score[rng.random(csr.n_spectra) < 0.1] = np.nan
    rank = rng.permutation(csr.n_spectra).astype(np.int64)
    best, bst = engine.best_score(dev(csr.cluster_off), dev(score), dev(rank)).to_host()
    wbest, wbst = np_oracle.best_score(csr.cluster_off, score, rank)
    np.testing.assert_array_equal(best[:C], wbest)
    np.testing.assert_array_equal(bst[:C], wbst)


@pytest.mark.parametrize("seed", range(1, N_CASES, 2))
def test_fuzz_precursor_modes(gpu, seed):
    """The gap-average CLI's precursor choices (average_spectrum_clustering.py:106-148,
    --pepmass / --rt) on the fuzz batches, cluster by cluster against the numpy
    restatement of the reference helpers: pepmass, charge and RT bit-exact
    (tie-free masses: the reference's argsort is unstable on ties past 16)."""
    csr, _ = _case(seed)
    # the synthetic precursors repeat within a cluster (5 decimals); a tie in the
    # neutral masses makes the reference's pick depend on numpy's unstable argsort
    # (and on the host's SIMD sort), so the masses are made distinct here
    csr = SpectraCSR(csr.cluster_off, csr.spec_off, csr.mz, csr.inten,
                     csr.prec_mz + 1e-7 * np.arange(csr.n_spectra), csr.charge, csr.rt)
    batch = engine.DeviceBatch.from_host(csr)
    co = csr.cluster_off
    H = engine.PROTON
    for pm, rtm in (("lower_median", "mass_lower_median"), ("lower_median", "median"),
                    ("neutral_average", "median"), ("naive_average", "mass_lower_median")):
        got = engine.gap_average(batch, pepmass=pm, rt=rtm).to_host()
        for c in range(csr.n_clusters):
            s0, s1 = co[c], co[c + 1]
            if s1 == s0:
                continue
            prec, ch, rt = csr.prec_mz[s0:s1], csr.charge[s0:s1], csr.rt[s0:s1]
            if pm == "naive_average":
                want = np_oracle.naive_average_mass_and_charge(prec, ch)
                if want is None:
                    assert got["status"][c] == engine.STATUS_MIXED_CHARGE, c
                    continue
            elif pm == "neutral_average":
                want = np_oracle.neutral_average_mass_and_charge(prec, ch, H)
            else:
                want = np_oracle.lower_median_mass(prec, ch, H)
            wrt = (np_oracle.lower_median_mass_rt(prec, ch, rt, H) if rtm == "mass_lower_median"
                   else np_oracle.median_rt(rt))
            assert got["prec"][c] == want[0] and got["charge"][c] == want[1], (pm, c)
            assert got["rt"][c] == wrt or (np.isnan(wrt) and np.isnan(got["rt"][c])), (rtm, c)


def test_precursor_picks_large_clusters(gpu):
    """Clusters past GA_RADIX_N (512) spectra take the radix select for the
    precursor picks: the lower-median mass index and the RT median must be the
    stable ranks' picks (ties by index, NaN last, -0 == +0) exactly as the O(n^2)
    rank loops give them.  Ties are dense here (masses on a coarse grid, mixed
    charges, NaN and signed-zero RTs), so the expected pick is numpy's stable
    argsort -- the definition the kernels implement (the reference's
    unstable argsort leaves tied picks parity unpinned)."""
    rng = np.random.default_rng(77)
    sizes = np.array([65, 511, 512, 513, 700, 1025, 3000, 5000, 2, 1])
    csr = make_clusters_np(len(sizes), seed=77, sizes=sizes, n_template=5)
    S = csr.n_spectra
    charge = rng.choice([2, 3], S).astype(csr.charge.dtype)
    prec = np.round(rng.uniform(400, 420, S), 1)  # ~200 distinct values: many ties
    rt = np.round(rng.uniform(0, 50, S), 0)
    rt[rng.random(S) < 0.05] = 0.0
    rt[rng.random(S) < 0.05] = -0.0
    co = csr.cluster_off
    for nan_c in (0, 4, 8):  # NaN RTs off the middle ranks (np.median -> NaN): block, radix and wave paths
        rt[co[nan_c] + 1] = np.nan
    csr = SpectraCSR(csr.cluster_off, csr.spec_off, csr.mz, csr.inten, prec, charge, rt)
    batch = engine.DeviceBatch.from_host(csr)
    H = engine.PROTON
    for rtm in ("mass_lower_median", "median"):
        got = engine.gap_average(batch, pepmass="lower_median", rt=rtm).to_host()
        for c in range(csr.n_clusters):
            s0, s1 = co[c], co[c + 1]
            n = s1 - s0
            z = charge[s0:s1].astype(np.float64)
            mass = prec[s0:s1] * z - z * H
            lm = int(np.argsort(mass, kind="stable")[(n - 1) // 2])
            zl = int(charge[s0 + lm])
            assert got["charge"][c] == zl, (rtm, c)
            assert got["prec"][c] == (mass[lm] + zl * H) / zl, (rtm, c)
            wrt = rt[s0 + lm] if rtm == "mass_lower_median" else np_oracle.median_rt(rt[s0:s1])
            assert got["rt"][c] == wrt or (np.isnan(wrt) and np.isnan(got["rt"][c])), (rtm, c)


def test_gap_average_giant_pipeline(gpu):
    """Clusters past GA_GIANT_N (16,384) peaks go from the global kernel to the
    tiled giant pipeline.  24 clusters here: 21 giants -- with a NaN intensity, NaN / +inf
    m/z, -inf m/z, +-inf m/z with a -inf intensity, an +inf intensity with a NaN m/z (since
    round 6 all of them through the tiled passes, the reference's NaN arithmetic in the
    flat emit), every m/z NaN (one workgroup, gap_body_nf) -- giants on a coarse m/z grid
    (exact ties, several peaks per bucket), a 2-spectrum giant, and small clusters
    between them.  Against the C oracle (the reference's NaN arithmetic): group
    structure exact, values within GAP_RTOL, under the default and non-default
    parameters."""
    rng = np.random.default_rng(91)
    sizes = np.array([300, 5, 400, 2, 260, 280, 3, 350] + [270] * 14 + [1, 330])
    csr = make_clusters_np(len(sizes), seed=91, sizes=sizes, n_template=300)
    mz, it = csr.mz.copy(), csr.inten.copy()
    so, co = csr.spec_off, csr.cluster_off
    it[so[co[4]] + 17] = np.nan  # cluster 4: a NaN intensity
    mz[so[co[7]] + 3] = np.nan   # cluster 7: NaN and +inf m/z (the merged last group)
    mz[so[co[7] + 5] + 9] = np.inf
    mz[so[co[13] + 9] + 1] = -np.inf  # cluster 13: -inf m/z (group 0; every later m/z NaN)
    mz[so[co[15] + 2] + 5] = -np.inf  # cluster 15: -inf AND +inf m/z, and a -inf intensity
    mz[so[co[15] + 7] + 11] = np.inf
    it[so[co[15] + 4] + 20] = -np.inf
    it[so[co[16] + 1] + 30] = np.inf  # cluster 16: +inf intensity in a middle group, NaN m/z
    mz[so[co[16] + 3] + 2] = np.nan
    for s_ in range(co[17], co[18]):  # cluster 17: every m/z NaN (no finite m/z: one workgroup)
        mz[so[s_]:so[s_ + 1]] = np.nan
    top = so[co[10]] + int(np.argmax(mz[so[co[10]]:so[co[11]]]))
    it[top] = np.inf  # cluster 10: +inf intensity in the last group
    for c in (5, 9, 12):  # coarse grid, spectra kept sorted
        for s in range(co[c], co[c + 1]):
            a, b = so[s], so[s + 1]
            mz[a:b] = np.sort(np.round(mz[a:b] / 0.02) * 0.02)
    # cluster 3: two spectra of 40,000 peaks each
    big = [np.sort(rng.uniform(100, 2000, 40000)) for _ in range(2)]
    parts_mz, parts_it, lens = [], [], []
    for s in range(csr.n_spectra):
        if co[3] <= s < co[4]:
            m = big[s - co[3]]
            parts_mz.append(m)
            parts_it.append(rng.uniform(1, 1e4, len(m)))
        else:
            parts_mz.append(mz[so[s]:so[s + 1]])
            parts_it.append(it[so[s]:so[s + 1]])
        lens.append(len(parts_mz[-1]))
    spec_off = np.zeros(csr.n_spectra + 1, np.int64)
    np.cumsum(lens, out=spec_off[1:])
    csr = SpectraCSR(co, spec_off, np.concatenate(parts_mz), np.concatenate(parts_it), csr.prec_mz,
                     csr.charge, csr.rt)
    N = np.diff(spec_off[co])
    assert (N > 16384).sum() >= 21
    batch = engine.DeviceBatch.from_host(csr)
    for kw in (dict(), dict(mz_accuracy=0.02, dyn_range=100.0, min_fraction=0.3)):
        got = engine.gap_average(batch, **kw).to_host()
        # cluster 17 has no finite m/z: no diff reaches mz_accuracy, the reference's
        # ind_list[0] raises IndexError (average_spectrum_clustering.py:69) -> SPX_NO_GAP
        assert got["status"][17] == engine.STATUS_NO_GAP
        assert not np.delete(got["status"], 17).any()
        assert got["out_off"][5] == got["out_off"][4]  # the NaN intensity: max NaN -> nothing kept
        o = got["out_off"]
        assert o[14] > o[13] and np.isnan(got["out_mz"][o[13]:o[14]]).all()  # after -inf: cm differences NaN
        assert np.isfinite(got["out_int"][o[13]:o[14]]).all()
        assert_gap_close(got, c_oracle.gap_average(csr, **kw), kw.get("dyn_range", 1000.0))


def test_gap_average_giant_overflow(gpu):
    """More giants than the pipeline's GA_GMAX (256) records: 272 clusters of
    ~18k peaks, each with one peak past the LDS and wide kernels' bucket range
    (m/z 2,700) so that all of them reach the global kernel.  256 go through the
    pipeline, the rest stay in the global kernel, and every one matches the C
    oracle."""
    C = 272
    csr = make_clusters_np(C, seed=93, sizes=np.full(C, 60), n_template=300)
    mz = csr.mz.copy()
    so, co = csr.spec_off, csr.cluster_off
    for c in range(C):
        s0 = co[c]
        mz[so[s0 + 1] - 1] = 2700.0 + 0.5 * (c % 7)  # the first spectrum's last peak
    csr = SpectraCSR(co, so, mz, csr.inten, csr.prec_mz, csr.charge, csr.rt)
    N = np.diff(so[co])
    assert (N > 16384).sum() > 256
    batch = engine.DeviceBatch.from_host(csr)
    got = engine.gap_average(batch).to_host()
    assert_gap_close(got, c_oracle.gap_average(csr), 1000.0)


def test_gap_average_giant_intake_overflow(gpu):
    """The giant intake (round 6): clusters past SPX_GA_WMAXN (65,536) peaks are
    registered up front and their pipeline runs on the call's second stream beside the
    LDS and wide kernels.  260 such clusters here (230 spectra of ~300 peaks) plus small
    ones between them: the intake's table takes 256, the other 4 go to the global kernel,
    which hands them to its own table's pipeline on the caller's stream.  Every cluster
    matches the C oracle, and a second call on a reused output gives the same bits."""
    sizes = np.array([230, 230, 3] * 130)
    csr = make_clusters_np(len(sizes), seed=97, sizes=sizes, n_template=300)
    N = np.diff(csr.spec_off[csr.cluster_off])
    assert (N > 65536).sum() == 260
    batch = engine.DeviceBatch.from_host(csr)
    res = engine.gap_average(batch)
    got = res.to_host()
    assert not got["status"].any()
    assert_gap_close(got, c_oracle.gap_average(csr), 1000.0)
    again = engine.gap_average(batch, out=res).to_host()
    for k in ("out_off", "out_mz", "out_int", "status", "prec", "rt"):
        np.testing.assert_array_equal(again[k], got[k])
