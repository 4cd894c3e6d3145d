"""GPU parity: the HIP engine (through the C-ABI) against the reference's golden
vectors and against the oracle on seeded synthetic batches.

Bar (BASELINE.json north_star): bin indices, peak counts and representative
indices bit-exact; consensus values within 1e-5 relative.  Achieved here:
bin-mean bit-exact (values too), medoid bit-exact (indices AND totals),
gap-average counts/boundaries exact and values within GAP_RTOL."""
import numpy as np
import pytest

from conftest import BIN_SETS, GAP_SETS, bin_params, gap_params, load_golden
from oracle import c_oracle, np_oracle
from specpride_amd import engine
from specpride_amd.csr import SpectraCSR
from specpride_amd.synthetic import make_clusters_np

pytestmark = pytest.mark.gpu

GAP_RTOL = 1e-9  # fixed-point group sums vs numpy cumsum differences (north star: 1e-5)


def _bin_mean(csr, **kw):
    return engine.bin_mean(engine.DeviceBatch.from_host(csr), **kw).to_host()


def assert_bin_mean_equal(got, ref):
    np.testing.assert_array_equal(got["status"], ref["status"])
    np.testing.assert_array_equal(got["out_off"], ref["out_off"])
    np.testing.assert_array_equal(got["out_mz"], ref["out_mz"])
    np.testing.assert_array_equal(got["out_int"], ref["out_int"])
    ok = ref["status"] == 0
    np.testing.assert_array_equal(got["prec"][ok], ref["prec"][ok])
    np.testing.assert_array_equal(got["charge"][ok], ref["charge"][ok])


def assert_gap_close(got, ref, dyn_range, rtol=GAP_RTOL):
    """Exact statuses and group structure; values within rtol.  A peak may be
    present on one side only if its intensity sits within rtol of the
    dynamic-range threshold (a near-tie the reference's own rounding decides)."""
    np.testing.assert_array_equal(got["status"], ref["status"])
    for c in range(len(ref["status"])):
        a, b = ref["out_off"][c], ref["out_off"][c + 1]
        ga, gb = got["out_off"][c], got["out_off"][c + 1]
        rm, ri = ref["out_mz"][a:b], ref["out_int"][a:b]
        gm, gi = got["out_mz"][ga:gb], got["out_int"][ga:gb]
        if len(rm) == len(gm):
            np.testing.assert_allclose(gm, rm, rtol=rtol, err_msg=f"cluster {c} mz")
            np.testing.assert_allclose(gi, ri, rtol=rtol, err_msg=f"cluster {c} int")
            continue
        thr = ri.max() / dyn_range
        rset = {round(x, 6): y for x, y in zip(rm, ri)}
        gset = {round(x, 6): y for x, y in zip(gm, gi)}
        for k in set(rset) ^ set(gset):
            v = rset.get(k, gset.get(k))
            assert abs(v - thr) <= rtol * abs(thr) * 10, f"cluster {c}: unmatched peak {k} int {v} thr {thr}"


# ------------------------------------------------------------------ goldens
@pytest.mark.parametrize("name", BIN_SETS)
def test_bin_mean_matches_reference_golden(gpu, name):
    z, csr = load_golden(f"bin_mean_{name}.npz")
    got = _bin_mean(csr, **bin_params(z))
    ref = dict(status=z["status"], out_off=z["out_off"], out_mz=z["out_mz"], out_int=z["out_int"],
               prec=z["out_prec"], charge=z["out_charge"])
    assert_bin_mean_equal(got, ref)


@pytest.mark.parametrize("name", GAP_SETS)
def test_gap_average_matches_reference_golden(gpu, name):
    z, csr = load_golden(f"gap_average_{name}.npz")
    p = gap_params(z)
    got = engine.gap_average(engine.DeviceBatch.from_host(csr), **p).to_host()
    ref = dict(status=z["status"], out_off=z["out_off"], out_mz=z["out_mz"], out_int=z["out_int"])
    assert_gap_close(got, ref, p["dyn_range"])


def test_medoid_matches_reference_golden(gpu):
    z, csr = load_golden("medoid_main.npz")
    res = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True)
    rep, totals = res.to_host()
    np.testing.assert_array_equal(rep, z["rep_index"])
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(totals, ref_tot)  # the reference's f64 epilogue, bit for bit


def test_precursor_helpers_on_gpu(gpu):
    z, csr = load_golden("precursor_helpers.npz")
    b = engine.DeviceBatch.from_host(csr)
    H = float(z["H"])
    r = engine.gap_average(b, pepmass="lower_median", rt="mass_lower_median", proton=H).to_host()
    np.testing.assert_array_equal(r["prec"], z["lm_mz"])
    np.testing.assert_array_equal(r["charge"], z["lm_z"])
    np.testing.assert_array_equal(r["rt"], z["lm_rt"])
    r = engine.gap_average(b, pepmass="neutral_average", rt="median", proton=H).to_host()
    np.testing.assert_array_equal(r["prec"], z["ne_mz"])
    np.testing.assert_array_equal(r["charge"], z["ne_z"])
    np.testing.assert_array_equal(r["rt"], z["med_rt"])
    r = engine.gap_average(b, pepmass="naive_average", rt="median", proton=H).to_host()
    mixed = z["na_status"] == 1
    assert np.all(r["status"][mixed] == engine.STATUS_MIXED_CHARGE)
    np.testing.assert_array_equal(r["prec"][~mixed], z["na_mz"][~mixed])


# ---------------------------------------------------------- synthetic vs oracle
@pytest.fixture(scope="module")
def synth():
    return make_clusters_np(1500, seed=1234)


def test_bin_mean_synthetic_vs_oracle(gpu, synth):
    assert_bin_mean_equal(_bin_mean(synth), c_oracle.bin_mean(synth))


def test_bin_mean_other_params_vs_oracle(gpu, synth):
    sub = synth.select(range(300))
    for kw in (dict(minimum=150.0, maximum=1500.0, binsize=0.05, apply_peak_quorum=False),
               dict(minimum=0.0, maximum=3000.0, binsize=0.01),          # > LDS bins: global path
               dict(minimum=100.0, maximum=2000.0, binsize=0.0037)):
        assert_bin_mean_equal(_bin_mean(sub, **kw), c_oracle.bin_mean(sub, **kw))


def test_gap_average_synthetic_vs_oracle(gpu, synth):
    sub = synth.select(range(600))
    got = engine.gap_average(engine.DeviceBatch.from_host(sub)).to_host()
    assert_gap_close(got, np_oracle.gap_average(sub), 1000.0)


def test_medoid_synthetic_vs_oracle(gpu, synth):
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(synth), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(synth, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


def _shuffled(csr, seed=3):
    rng = np.random.default_rng(seed)
    mz, it = csr.mz.copy(), csr.inten.copy()
    for s in range(0, csr.n_spectra, 2):  # every other spectrum unsorted
        a, b = csr.spec_off[s], csr.spec_off[s + 1]
        p = rng.permutation(b - a)
        mz[a:b], it[a:b] = mz[a:b][p], it[a:b][p]
    return SpectraCSR(csr.cluster_off, csr.spec_off, mz, it, csr.prec_mz, csr.charge, csr.rt)


def test_unsorted_spectra(gpu, synth):
    sub = _shuffled(synth.select(range(200)))
    assert_bin_mean_equal(_bin_mean(sub), c_oracle.bin_mean(sub))
    rep, _ = engine.medoid(engine.DeviceBatch.from_host(sub)).to_host()
    np.testing.assert_array_equal(rep, c_oracle.medoid(sub))
    got = engine.gap_average(engine.DeviceBatch.from_host(sub)).to_host()
    assert_gap_close(got, np_oracle.gap_average(sub), 1000.0)


def test_large_clusters_fallback_paths(gpu):
    # spectra counts past every LDS limit: n > 64 (medoid), n > 128 (bin-mean mean),
    # > 1536 distinct bins, long tail up to 700
    sizes = np.array([2, 65, 129, 300, 700, 3, 90], np.int64)
    csr = make_clusters_np(len(sizes), seed=77, sizes=sizes, n_template=120)
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)
    got = engine.gap_average(engine.DeviceBatch.from_host(csr)).to_host()
    assert_gap_close(got, np_oracle.gap_average(csr), 1000.0)


def test_wide_mz_range_and_noisy_cluster(gpu):
    # bin range > LDS bitmap (medoid) and many distinct bins (bin-mean D > LDS cap)
    rng = np.random.default_rng(9)
    clusters = []
    for n, hi in ((6, 9000.0), (40, 2000.0)):
        sp = [{"m/z array": np.round(np.sort(rng.uniform(100.0, hi, 400)), 5),
               "intensity array": np.round(rng.lognormal(5, 1.5, 400), 2), "precursor mz": 500.0,
               "precursor charge": 2} for _ in range(n)]
        clusters.append(sp)
    csr = SpectraCSR.from_clusters(clusters)
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))
    rep, _ = engine.medoid(engine.DeviceBatch.from_host(csr)).to_host()
    np.testing.assert_array_equal(rep, c_oracle.medoid(csr))
    got = engine.gap_average(engine.DeviceBatch.from_host(csr)).to_host()
    assert_gap_close(got, np_oracle.gap_average(csr), 1000.0)


def test_gap_average_deterministic_and_nonfinite(gpu, synth):
    sub = synth.select(range(100))
    b = engine.DeviceBatch.from_host(sub)
    r1 = engine.gap_average(b).to_host()
    r2 = engine.gap_average(b).to_host()
    for k in ("out_off", "out_mz", "out_int", "status"):
        np.testing.assert_array_equal(r1[k], r2[k])
    # NaN sorts last and never opens a gap: [100, 100, NaN] has no gap -> the reference's IndexError
    bad = SpectraCSR.from_clusters([[{"m/z array": [100.0, np.nan], "intensity array": [1.0, 2.0]},
                                     {"m/z array": [100.0], "intensity array": [1.0]}]])
    r = engine.gap_average(engine.DeviceBatch.from_host(bad)).to_host()
    assert r["status"][0] == engine.STATUS_NO_GAP


def test_gap_average_nonfinite_mixed_into_large_batch(gpu, synth):
    """Non-finite peaks sprinkled into a batch of ordinary clusters (every kernel of
    the chain sees its share) against the numpy oracle -- the reference's own
    arithmetic -- and no cluster status other than the oracle's."""
    sub = synth.select(range(400))
    rng = np.random.default_rng(12)
    mz, it = sub.mz.copy(), sub.inten.copy()
    for c in range(0, sub.n_clusters, 3):
        a, b = sub.spec_off[sub.cluster_off[c]], sub.spec_off[sub.cluster_off[c + 1]]
        for j in rng.integers(a, b, size=int(rng.integers(1, 4))):
            v = [np.nan, np.inf, -np.inf][int(rng.integers(0, 3))]
            if rng.random() < 0.5:
                mz[j] = v
            else:
                it[j] = v
    bad = SpectraCSR(sub.cluster_off, sub.spec_off, mz, it, sub.prec_mz, sub.charge, sub.rt)
    for kw in (dict(), dict(mz_accuracy=0.02, dyn_range=100.0, min_fraction=0.3)):
        got = engine.gap_average(engine.DeviceBatch.from_host(bad), **kw).to_host()
        with np.errstate(all="ignore"):
            ref = np_oracle.gap_average(bad, **kw)
        assert_gap_close(got, ref, kw.get("dyn_range", 1000.0))


def test_empty_batch_and_empty_clusters(gpu):
    csr = SpectraCSR.from_clusters([[], [{"m/z array": [], "intensity array": [], "precursor mz": 1.0,
                                          "precursor charge": 2}]])
    b = engine.DeviceBatch.from_host(csr)
    rep, _ = engine.medoid(b).to_host()
    assert list(rep) == [-1, 1 - 1 + csr.cluster_off[1]]
    r = engine.bin_mean(b).to_host()
    assert r["out_off"][-1] == 0


def test_medoid_large_path_skewed_unsorted_and_empty(gpu):
    """MFMA Gram path: config-4-like skewed sizes (one n = 1500 cluster: 12x12
    Gram tiles), unsorted peaks, and empty spectra inside a large cluster."""
    csr = make_clusters_np(400, seed=5, skewed=True, forced_large=1, large_size=1500, n_template=80)
    csr = _shuffled(csr, seed=11)
    rng = np.random.default_rng(2)
    big = [{"m/z array": np.round(rng.uniform(100, 1800, int(k)), 4), "intensity array": np.ones(int(k))}
           for k in rng.integers(0, 40, 200)]
    big[0] = {"m/z array": np.zeros(0), "intensity array": np.zeros(0)}
    big[150] = {"m/z array": np.zeros(0), "intensity array": np.zeros(0)}
    extra = SpectraCSR.from_clusters([big])
    both = SpectraCSR(np.concatenate([csr.cluster_off, csr.cluster_off[-1] + extra.cluster_off[1:]]),
                      np.concatenate([csr.spec_off, csr.spec_off[-1] + extra.spec_off[1:]]),
                      np.concatenate([csr.mz, extra.mz]), np.concatenate([csr.inten, extra.inten]),
                      np.concatenate([csr.prec_mz, extra.prec_mz]), np.concatenate([csr.charge, extra.charge]),
                      np.concatenate([csr.rt, extra.rt]))
    assert np.diff(both.cluster_off).max() == 1500
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(both), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(both, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


def _concat(*parts):
    """Concatenate SpectraCSR batches (cluster order kept)."""
    co, so, n_s, n_p = [np.zeros(1, np.int64)], [np.zeros(1, np.int64)], 0, 0
    for p in parts:
        co.append(p.cluster_off[1:] + n_s)
        so.append(p.spec_off[1:] + n_p)
        n_s += p.n_spectra
        n_p += p.n_peaks
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])  # noqa: E731
    return SpectraCSR(np.concatenate(co), np.concatenate(so), cat("mz"), cat("inten"), cat("prec_mz"),
                      cat("charge"), cat("rt"))


def test_bin_mean_many_clusters_with_special_shapes(gpu):
    """Thousands of clusters with empty clusters, empty spectra, mixed charges, a
    spectrum longer than one fast-path step (252 peaks), an unsorted spectrum and
    a > 128-spectrum cluster scattered through them (deferred to the global kernel)."""
    rng = np.random.default_rng(21)
    base = make_clusters_np(7000, seed=8, min_size=1, max_size=12, n_template=60)
    co = base.cluster_off.copy()
    # empty clusters: repeat some boundaries
    co = np.sort(np.concatenate([co, rng.choice(co[1:-1], 300)]))
    ch = base.charge.copy()
    for c in rng.choice(len(co) - 1, 40, replace=False):  # mixed charges
        a, b = co[c], co[c + 1]
        if b - a >= 2:
            ch[b - 1] = ch[a] + 1
    body = SpectraCSR(co, base.spec_off, base.mz, base.inten, base.prec_mz, ch, base.rt)

    def spec(k, sort=True):
        m = np.round(rng.uniform(100.0, 2000.0, k), 5)
        return {"m/z array": np.sort(m) if sort else m, "intensity array": np.round(rng.lognormal(5, 1.5, k), 2),
                "precursor mz": 600.0, "precursor charge": 2}

    special = SpectraCSR.from_clusters([
        [spec(300), spec(200), spec(280)],                  # longer than a step
        [spec(50), {"m/z array": [], "intensity array": [], "precursor mz": 600.0, "precursor charge": 2},
         spec(40)],                                         # an empty spectrum
        [spec(30, sort=False), spec(30)],                   # unsorted
        [spec(20) for _ in range(140)],                     # > 128 spectra
        [],
    ])
    parts = [body.select(range(0, 3000)), special, body.select(range(3000, 5000)), special,
             body.select(range(5000, body.n_clusters))]
    csr = _concat(*parts)
    assert csr.n_clusters > 5 * 1280
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))


def _edge_batch():
    """Edge shapes: spectra longer than a fast-path step, clusters of 100-128 spectra, every peak
    in one bin (D = 1: three empty ranges), no in-range peak (D = 0), empty spectra
    inside a cluster, repeated bins inside a spectrum (last wins), peaks on the
    range ends (min, just below max, max itself)."""
    rng = np.random.default_rng(77)
    clusters = []
    # long spectra: 900 sorted peaks over a narrow window -> runs of >> 64 per wave
    clusters.append([{"m/z array": np.sort(rng.uniform(500, 540, 900)), "intensity array": rng.lognormal(3, 1, 900),
                      "precursor mz": 600.0 + k, "precursor charge": 2} for k in range(5)])
    # 100..128 spectra of ~60 peaks
    for nspec in (100, 127, 128):
        t = np.sort(rng.uniform(100, 2000, 60))
        clusters.append([{"m/z array": np.sort(t + rng.normal(0, 0.003, 60)), "intensity array": rng.lognormal(5, 1, 60),
                          "precursor mz": 700.0, "precursor charge": 3} for _ in range(nspec)])
    # every peak in one bin
    clusters.append([{"m/z array": np.array([300.001, 300.005, 300.011]), "intensity array": np.array([1.0, 2.0, 3.0]),
                      "precursor mz": 500.0, "precursor charge": 2} for _ in range(7)])
    # nothing in range
    clusters.append([{"m/z array": np.array([50.0, 99.99, 2000.0, 2500.0]), "intensity array": np.ones(4),
                      "precursor mz": 500.0, "precursor charge": 2} for _ in range(3)])
    # empty spectra between full ones, repeated bins, range ends
    ends = np.array([100.0, 100.0, 100.019, 1234.5671, 1234.5672, 1999.99999, 2000.0])
    clusters.append([{"m/z array": ends, "intensity array": np.arange(1.0, 8.0), "precursor mz": 400.0,
                      "precursor charge": 2},
                     {"m/z array": np.zeros(0), "intensity array": np.zeros(0), "precursor mz": 401.0,
                      "precursor charge": 2},
                     {"m/z array": ends + 0.001, "intensity array": np.arange(2.0, 9.0), "precursor mz": 402.0,
                      "precursor charge": 2},
                     {"m/z array": np.zeros(0), "intensity array": np.zeros(0), "precursor mz": 403.0,
                      "precursor charge": 2}])
    return SpectraCSR.from_clusters(clusters)


def test_bin_mean_edge_shapes(gpu):
    csr = _edge_batch()
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))
    assert_bin_mean_equal(_bin_mean(csr), np_oracle.bin_mean(csr))


def test_bin_mean_chunk_boundaries(gpu):
    """bin_mean_wide_kernel walks long spectra in 252-position chunks: runs of one
    bin straddling a chunk boundary (positions 251/252, 503/504), spectra of exactly
    252 and 504 peaks, an empty spectrum between long ones, 128 spectra of 260 peaks
    (the most a cluster may have there) -- bit-exact against the C oracle."""
    rng = np.random.default_rng(5)

    def spec(mz):
        mz = np.asarray(mz, np.float64)
        return {"m/z array": mz, "intensity array": np.round(rng.lognormal(4, 1, len(mz)), 2),
                "precursor mz": 500.0, "precursor charge": 2}

    def straddle(n, cuts):
        m = np.sort(rng.uniform(120.0, 1900.0, n))
        for k in cuts:  # positions k-2 .. k+1 in one 0.02 bin
            b = 100.0 + 0.02 * np.floor((m[k] - 100.0) / 0.02)
            m[k - 2:k + 2] = b + np.array([0.001, 0.005, 0.009, 0.013])
        return np.sort(m)

    clusters = [
        [spec(straddle(600, [252, 504])), spec(straddle(700, [252, 504])), spec(straddle(300, [252]))],
        [spec(np.sort(rng.uniform(100, 2000, 252))), spec(np.sort(rng.uniform(100, 2000, 504))),
         spec(np.zeros(0)), spec(np.sort(rng.uniform(100, 2000, 253)))],
        [spec(straddle(260, [252])) for _ in range(128)],
    ]
    csr = SpectraCSR.from_clusters(clusters)
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))


def test_bin_mean_skewed_and_unsorted(gpu):
    """Skewed sizes (>128 spectra -> deferred) and shuffled spectra (deferred) mixed
    with regular clusters in one launch: bit-exact against the oracle."""
    csr = make_clusters_np(400, seed=91, skewed=True)
    csr = csr.select([c for c in range(csr.n_clusters) if csr.cluster_off[c + 1] - csr.cluster_off[c] <= 300])
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))
    sub = _shuffled(csr.select(range(120)))
    assert_bin_mean_equal(_bin_mean(sub), c_oracle.bin_mean(sub))


def test_bin_mean_staged(gpu):
    """spx_bin_mean_stage: stage 1 alone (every cluster within the wide kernel's
    caps) and stage 1 + 2 on demand (skewed sizes, shuffled spectra: to_host runs
    stage 2 when a cluster came back SPX_UNRESOLVED) equal the one-call chain and
    the oracle bit for bit; the per-cluster shim takes the staged path."""
    from specpride_amd.binning import RepresentativeSpectrumCreator

    small = make_clusters_np(40, seed=93)
    big = make_clusters_np(400, seed=91, skewed=True)
    big = big.select([c for c in range(big.n_clusters) if big.cluster_off[c + 1] - big.cluster_off[c] <= 300])
    for csr in (small, big, _shuffled(big.select(range(120)))):
        ref = c_oracle.bin_mean(csr)
        batch = engine.DeviceBatch.from_host(csr)
        res = engine.bin_mean(batch, staged=True)
        assert res.pending is not None
        assert_bin_mean_equal(res.to_host(), ref)
        assert res.pending is None
        assert_bin_mean_equal(engine.bin_mean(batch).to_host(), ref)
    sizes = np.diff(big.cluster_off)
    assert sizes.max() > 128  # stage 2 really ran for this batch
    c = int(np.argmax(sizes))
    one = big.select([c])
    clusters = [[{"m/z array": one.mz[one.spec_off[s]:one.spec_off[s + 1]],
                  "intensity array": one.inten[one.spec_off[s]:one.spec_off[s + 1]],
                  "precursor mz": float(one.prec_mz[s]), "precursor charge": int(one.charge[s])}
                 for s in range(one.n_spectra)]]
    got = RepresentativeSpectrumCreator().combine_bin_mean(clusters[0])
    ref = c_oracle.bin_mean(one)
    np.testing.assert_array_equal(got["mzs"], ref["out_mz"])
    np.testing.assert_array_equal(got["intensities"], ref["out_int"])


def test_bin_mean_range_boundaries(gpu):
    """Short spectra (1-3 peaks), spectra entirely below / above parts of the range,
    repeated identical spectra (every bin hit by every spectrum), spectra of 255
    and 256 peaks (around the fast-path step), all bit-exact against the oracle."""
    rng = np.random.default_rng(123)
    clusters = []
    for n0 in (1, 2, 3):
        sp = [{"m/z array": np.sort(rng.uniform(100, 2000, n0)), "intensity array": rng.lognormal(3, 1, n0),
               "precursor mz": 500.0, "precursor charge": 2}]
        for k in range(12):
            lo, hi = [(100, 400), (1500, 2000), (100, 2000), (800, 801)][k % 4]
            m = int(rng.integers(1, 200))
            sp.append({"m/z array": np.sort(rng.uniform(lo, hi, m)), "intensity array": rng.lognormal(3, 1, m),
                       "precursor mz": 500.0 + k, "precursor charge": 2})
        clusters.append(sp)
    for length in (255, 256):
        clusters.append([{"m/z array": np.sort(rng.uniform(100, 2000, length)),
                          "intensity array": rng.lognormal(3, 1, length), "precursor mz": 600.0,
                          "precursor charge": 3} for _ in range(4)])
    # boundary bins hit exactly: every spectrum repeats spectrum 0's peaks
    base = np.sort(rng.uniform(100, 2000, 40))
    clusters.append([{"m/z array": base.copy(), "intensity array": rng.lognormal(3, 1, 40), "precursor mz": 700.0,
                      "precursor charge": 2} for _ in range(9)])
    csr = SpectraCSR.from_clusters(clusters)
    assert_bin_mean_equal(_bin_mean(csr), c_oracle.bin_mean(csr))


def _zero_tail_batches():
    """(a) a batch whose LAST cluster has spectra but no peaks (so its peak range
    starts at n_peaks), (b) a batch with no peaks at all."""
    rng = np.random.default_rng(31)

    def spec(k):
        return {"m/z array": np.round(np.sort(rng.uniform(100.0, 1999.0, k)), 5),
                "intensity array": np.round(rng.lognormal(5, 1.5, k), 2) + 0.01,
                "precursor mz": 500.0, "precursor charge": 2}

    empty = {"m/z array": [], "intensity array": [], "precursor mz": 500.0, "precursor charge": 2}
    a = SpectraCSR.from_clusters([[spec(40), spec(35), spec(50)], [spec(60)], [dict(empty), dict(empty)]])
    b = SpectraCSR.from_clusters([[dict(empty), dict(empty)], [dict(empty)]])
    return a, b


@pytest.mark.parametrize("which", [0, 1])
def test_zero_peak_tail_all_entry_points(gpu, which):
    """Regression for the clamp-to-p0 fault class (a load of index n_peaks): every
    entry point on a batch whose last cluster -- or whole batch -- has no peaks."""
    import torch

    csr = _zero_tail_batches()[which]
    b = engine.DeviceBatch.from_host(csr)
    assert_bin_mean_equal(engine.bin_mean(b).to_host(), c_oracle.bin_mean(csr))
    ga = engine.gap_average(b).to_host()
    want = np_oracle.gap_average(csr)
    np.testing.assert_array_equal(ga["status"], want["status"])
    rep, tot = engine.medoid(b, with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)
    # binned cosine with the bin-mean output as representatives (empty ones included)
    r = engine.bin_mean(b).to_host()
    dev = lambda x: torch.as_tensor(np.ascontiguousarray(x), device="cuda")  # noqa: E731
    rm = r["out_mz"] if len(r["out_mz"]) else np.zeros(1)
    ri = r["out_int"] if len(r["out_int"]) else np.zeros(1)
    cos, avg, st = engine.binned_cosine(b, dev(r["out_off"]), dev(rm), dev(ri)).to_host()
    wcos, wavg, wst = np_oracle.binned_cosine(csr, r["out_off"], r["out_mz"], r["out_int"])
    np.testing.assert_array_equal(st[:csr.n_clusters], wst)
    torch.cuda.synchronize()


def test_medoid_many_runtime_deferrals(gpu):
    """small clusters that the register kernel defers only at run
    time (m/z above 3,276.8 = outside its 32,768-bin table) land in the large-path
    arena; 300 of them must all resolve (the engine re-budgets the workspace on
    SPX_REP_ARENA and re-runs), with representatives and totals equal to the oracle."""
    rng = np.random.default_rng(7)
    clusters = []
    for _c in range(300):
        n = int(rng.integers(2, 24))
        base = np.sort(rng.uniform(100.0, 4500.0, 150))
        spectra = []
        for _s in range(n):
            keep = rng.random(150) > 0.1
            mz = np.sort(np.round(base[keep] + rng.normal(0.0, 0.003, int(keep.sum())), 5))
            spectra.append({"m/z array": mz, "intensity array": np.ones(len(mz))})
        clusters.append(spectra)
    csr = SpectraCSR.from_clusters(clusters)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    want_rep, want_tot = c_oracle.medoid(csr, with_totals=True)
    assert np.all(rep >= 0)
    np.testing.assert_array_equal(rep, want_rep)
    np.testing.assert_array_equal(tot, want_tot)


def test_medoid_wide_bin_overflow_deferrals(gpu):
    """small clusters (n <= 64) whose distinct bins overflow the wide
    kernel's 6,080 are deferred at run time; the workspace query reserves a slot per
    such cluster (up to 256), and all 40 resolve equal to the oracle, totals included."""
    rng = np.random.default_rng(11)
    clusters = []
    for _c in range(40):
        n = int(rng.integers(12, 30))
        spectra = []
        for _s in range(n):
            mz = np.sort(np.round(rng.uniform(100.0, 3200.0, 420), 4))
            spectra.append({"m/z array": mz, "intensity array": rng.uniform(1.0, 9.0, len(mz))})
        clusters.append(spectra)
    csr = SpectraCSR.from_clusters(clusters)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    want_rep, want_tot = c_oracle.medoid(csr, with_totals=True)
    assert np.all(rep >= 0)
    np.testing.assert_array_equal(rep, want_rep)
    np.testing.assert_array_equal(tot, want_tot)


def test_bin_mean_split_path(gpu):
    """Clusters past the register and wide kernels (> 128 spectra, > 4,096 distinct
    bins) through the segmented fold and -- with its arena capped -- the bin-range
    split path: one 3,000-spectrum cluster, long-spectrum clusters, a giant unsorted
    one (-> the global kernel), a giant mixed-charge one and NaN m/z in a long one,
    mixed with ordinary clusters; bit-exact against the C oracle, values included."""
    big = make_clusters_np(1, seed=41, sizes=np.array([3000]))
    longsp = make_clusters_np(12, seed=42, n_template=600, max_size=30)
    plain = make_clusters_np(30, seed=43)
    uns = _shuffled(make_clusters_np(1, seed=44, sizes=np.array([400])), seed=5)
    mixed = make_clusters_np(1, seed=45, sizes=np.array([300]))
    mixed.charge[7] = mixed.charge[0] + 1
    nan = make_clusters_np(1, seed=46, n_template=500, sizes=np.array([20]))
    nan.mz[nan.spec_off[3] + 5] = np.nan

    def cat(parts):
        cl, sp, mz, it, pr, ch, rt = [0], [0], [], [], [], [], []
        for p in parts:
            cl += list(cl[-1] + p.cluster_off[1:])
            sp += list(sp[-1] + p.spec_off[1:])
            mz.append(p.mz); it.append(p.inten); pr.append(p.prec_mz); ch.append(p.charge); rt.append(p.rt)
        return SpectraCSR(np.array(cl), np.array(sp), np.concatenate(mz), np.concatenate(it), np.concatenate(pr),
                          np.concatenate(ch), np.concatenate(rt))

    csr = cat([plain, big, longsp, uns, mixed, nan, plain])
    got = _bin_mean(csr)
    want = c_oracle.bin_mean(csr)
    assert_bin_mean_equal(got, want)
    assert np.any(want["status"] == engine.STATUS_MIXED_CHARGE)
    # a tiny range-record cap (SPX_SPLIT_RANGE_CAP, read by the library per call): the
    # clusters that overflow it -- one straddling the cap among them -- go to the
    # global kernel and their reserved records are dropped, never read unwritten
    import os

    # no quorum: nothing for the kept-bin fold, the segmented fold takes every
    # deferred cluster
    assert_bin_mean_equal(_bin_mean(csr, apply_peak_quorum=False), c_oracle.bin_mean(csr, apply_peak_quorum=False))
    # the segmented fold with the quorum (SPX_KEPT_FOLD=0 turns the kept-bin fold off)
    os.environ["SPX_KEPT_FOLD"] = "0"
    try:
        assert_bin_mean_equal(_bin_mean(csr), want)
    finally:
        del os.environ["SPX_KEPT_FOLD"]
    # the arena (SPX_SEG_ARENA): none (every deferred cluster takes the bin-range
    # split path), room for part of the clusters
    for arena in ("0", "400000"):
        os.environ["SPX_SEG_ARENA"] = arena
        try:
            assert_bin_mean_equal(_bin_mean(csr), want)
            for cap in ("1", "3", "7"):
                os.environ["SPX_SPLIT_RANGE_CAP"] = cap
                try:
                    assert_bin_mean_equal(_bin_mean(csr), want)
                finally:
                    del os.environ["SPX_SPLIT_RANGE_CAP"]
        finally:
            del os.environ["SPX_SEG_ARENA"]


def test_bin_mean_kept_fold(gpu):
    """The kept-bin fold (bin_mean_q.hip) on the clusters the wide kernel defers:
    n = 129 .. 2,500 (blocks of 64 spectra, the last one partial; the intake's list, folded on
    the side stream), 100 spectra of 20k distinct bins (the wide kernel's list), 700-peak spectra
    (blocks of < 64 spectra), more than Q_KCAP = 2,048 kept bins (-> the segmented
    fold), a NaN intensity in a kept bin (that bin dropped), every spectrum empty,
    nothing in range, peaks on the window's ends, a mixed-charge one, an unsorted
    one (-> the global kernel); bit-exact against the C oracle, with and without
    the quorum."""
    rng = np.random.default_rng(17)
    parts = [make_clusters_np(1, seed=60 + k, sizes=np.array([n])) for k, n in enumerate((129, 192, 257, 700, 2500))]
    parts.append(make_clusters_np(2, seed=70, sizes=np.array([140, 200]), n_template=700))
    # 100 spectra of ~2,000 peaks: 20,636 distinct bins, past the wide kernel's 4,096 -- a kept-bin fold
    # of the wide kernel's own leftovers, beside the intake's (clusters past 128 spectra) since round 6
    parts.append(make_clusters_np(1, seed=75, sizes=np.array([100]), n_template=2000))

    def spec(mz, it=None):
        mz = np.asarray(mz, np.float64)
        return {"m/z array": mz, "intensity array": rng.lognormal(4, 1, len(mz)) if it is None else it,
                "precursor mz": 500.0, "precursor charge": 2}

    wide = np.sort(rng.uniform(100, 2000, 2300))
    nan_it = rng.lognormal(4, 1, 50)
    nan_it[10] = np.nan
    base = np.sort(rng.uniform(300, 900, 50))
    ends = np.array([100.0, 100.01, 1999.99, 1999.999])
    special = SpectraCSR.from_clusters([
        [spec(wide) for _ in range(130)],                                  # K = 2,300 > Q_KCAP
        [spec(base, nan_it if k == 3 else None) for k in range(150)],      # NaN intensity in a kept bin
        [spec(np.zeros(0)) for _ in range(131)],                           # every spectrum empty
        [spec(np.array([50.0, 99.0, 2000.0, 3000.0])) for _ in range(135)],  # nothing in range
        [spec(ends) for _ in range(133)],                                  # the window's ends
    ])
    mixed = make_clusters_np(1, seed=71, sizes=np.array([300]))
    mixed.charge[5] = mixed.charge[0] + 1
    uns = _shuffled(make_clusters_np(1, seed=72, sizes=np.array([180])), seed=9)
    csr = _concat(make_clusters_np(20, seed=73), *parts, special, mixed, uns, make_clusters_np(20, seed=74))
    for q in (True, False):
        assert_bin_mean_equal(_bin_mean(csr, apply_peak_quorum=q), c_oracle.bin_mean(csr, apply_peak_quorum=q))


def test_medoid_empty_spectrum_positions(gpu):
    """Empty spectra at every position of small clusters (register kernel), of a
    wide-kernel cluster (600-peak spectra) and of an MFMA-path cluster (n > 64):
    an empty spectrum shares its start offset with the next one, so the peak ->
    spectrum map must not count start offsets (the fuzz test's find: the empty-spectrum
    vote saw lane 0 only).  Representatives and totals bit-exact vs the oracle."""
    rng = np.random.default_rng(77)
    clusters = []

    def spec(n):
        return {"m/z array": np.sort(rng.uniform(100, 2000, n)), "intensity array": rng.lognormal(3, 1, n),
                "precursor mz": 500.0, "precursor charge": 2}

    for n in (2, 3, 5, 9, 26, 50, 64):
        for empties in ([0], [1], [n // 2], [n - 1], [1, 2], list(range(1, n, 3))):
            clusters.append([spec(0) if j in empties else spec(int(rng.integers(150, 250))) for j in range(n)])
    clusters.append([spec(0) if j in (1, 7) else spec(600) for j in range(30)])   # wide kernel
    clusters.append([spec(0) if j in (1, 40) else spec(120) for j in range(90)])  # large path
    csr = SpectraCSR.from_clusters(clusters)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


@pytest.mark.parametrize("shape", ["synth", "mixed"])
def test_fused_bin_mean_medoid_equals_separate_calls(gpu, synth, shape):
    """spx_bin_mean_medoid (one pass, both register bodies per workgroup) against the
    separate entry points and the C oracle: every output bit-identical.  'mixed' adds
    clusters past both register kernels (n > 50 / > 64, long spectra, unsorted,
    mixed charge, empty) so both leftover chains run after the fused head."""
    if shape == "synth":
        csr = synth.select(range(800))
    else:
        sizes = np.array([3, 51, 65, 130, 2, 1, 0, 40, 7, 300], np.int64)
        base = make_clusters_np(len(sizes), seed=17, sizes=sizes, n_template=120)
        long = make_clusters_np(3, seed=18, sizes=np.array([12, 30, 45]), n_template=400)
        csr = _shuffled(SpectraCSR.from_clusters(
            [[{"m/z array": m, "intensity array": i, "precursor mz": float(base.prec_mz[base.cluster_off[c]]),
               "precursor charge": int(base.charge[base.cluster_off[c]])} for m, i in base.cluster(c)]
             for c in range(base.n_clusters)] +
            [[{"m/z array": m, "intensity array": i, "precursor mz": 500.0, "precursor charge": 2}
              for m, i in long.cluster(c)] for c in range(long.n_clusters)]))
        ch = csr.charge.copy()
        ch[csr.cluster_off[0] + 1] += 1  # cluster 0: mixed charges (bin-mean's AssertionError status)
        csr = SpectraCSR(csr.cluster_off, csr.spec_off, csr.mz, csr.inten, csr.prec_mz, ch, csr.rt)
    b = engine.DeviceBatch.from_host(csr)
    bm, md = engine.bin_mean_medoid(b)
    got = bm.to_host()
    rep, _ = md.to_host()
    want = _bin_mean(csr)
    assert_bin_mean_equal(got, want)
    assert_bin_mean_equal(got, c_oracle.bin_mean(csr))
    rep2, _ = engine.medoid(engine.DeviceBatch.from_host(csr)).to_host()
    np.testing.assert_array_equal(rep[:csr.n_clusters], rep2[:csr.n_clusters])
    np.testing.assert_array_equal(rep[:csr.n_clusters], c_oracle.medoid(csr))
    # the checked call ran stage 1, read the hand-off counts and ran stage 2 only if a
    # register body handed a cluster on; an unchecked call then runs stage 1 alone (synth:
    # nothing handed on) or the whole pass (mixed) -- the same outputs either way
    clean = [v for k, v in b._ws.items() if isinstance(k, tuple) and k[0] == "fused_clean"]
    assert clean == [shape == "synth"]
    bm3, md3 = engine.bin_mean_medoid(b, check=False)
    assert_bin_mean_equal(bm3.to_host(), got)
    np.testing.assert_array_equal(md3.rep.cpu().numpy()[:csr.n_clusters], rep[:csr.n_clusters])


def test_bin_mean_mz_representations(gpu, synth):
    """Bit-exact against the C oracle whatever the m/z look like: 5-decimal m/z (the
    synthetic law, an MGF parse), 4- and 2-decimal m/z (many equal m/z, bins shared
    across spectra), full-precision m/z, one m/z per odd cluster moved by 1 ulp,
    6-decimal m/z, m/z on exact bin edges, each with other bin sizes and the
    quorum off.  (Round 4 used this test for the decimal-code variant of the
    register kernel, profiles/r04_ab_decimal_codes.txt.)"""
    sub = synth.select(range(400))
    rng = np.random.default_rng(77)

    def with_mz(mz):
        return SpectraCSR(sub.cluster_off, sub.spec_off, mz, sub.inten, sub.prec_mz, sub.charge, sub.rt)

    def resort(mz):  # keep every spectrum sorted (the register path's precondition)
        out = mz.copy()
        for s in range(sub.n_spectra):
            a, b = sub.spec_off[s], sub.spec_off[s + 1]
            out[a:b] = np.sort(out[a:b])
        return out

    full = resort(sub.mz + rng.uniform(-1e-3, 1e-3, sub.mz.shape))  # not decimal
    mixed = sub.mz.copy()
    for c in range(1, sub.n_clusters, 2):
        s = sub.cluster_off[c] + rng.integers(0, sub.cluster_off[c + 1] - sub.cluster_off[c])
        k = sub.spec_off[s] + (sub.spec_off[s + 1] - sub.spec_off[s]) // 2
        mixed[k] = np.nextafter(mixed[k], np.inf)  # stays sorted: the next peak is >= 1e-5 away
    edges = sub.mz.copy()
    k = rng.choice(len(edges), size=len(edges) // 20, replace=False)
    edges[k] = np.round(100.0 + 0.02 * np.round((edges[k] - 100.0) / 0.02), 5)
    batches = {"dec5": sub.mz, "dec4": resort(np.round(sub.mz, 4)), "dec2": resort(np.round(sub.mz, 2)),
               "full": full, "mixed": mixed, "dec6": resort(np.round(full, 6)), "edges": resort(edges)}
    for name, mz in batches.items():
        csr = with_mz(mz)
        for kw in ({}, dict(binsize=0.05, apply_peak_quorum=False), dict(binsize=0.001), dict(binsize=0.2)):
            got = _bin_mean(csr, **kw)
            ref = c_oracle.bin_mean(csr, **kw)
            try:
                assert_bin_mean_equal(got, ref)
            except AssertionError as e:
                raise AssertionError(f"batch {name} params {kw}: {e}") from None


def test_medoid_large_path_row_widths(gpu):
    """The large path's bit rows are built in LDS up to 512 row words (32,768 columns)
    and with global atomics past that (medoid_fill_kernel); the Gram reads them as FP4
    operands and the leaves kernel takes its quotients from exact reciprocals.  Clusters
    of n = 65..200 spectra whose distinct 0.1-Da bins fall under (28.5k), at (32,768) and
    over (33,000; 56.6k) the LDS row width, spectra of 1 to 9,000 peaks, an empty spectrum and identical spectra
    (count = min size, distance exactly 0): representatives AND totals bit-exact vs
    the C oracle."""
    rng = np.random.default_rng(2024)
    clusters = []

    def spec(mz):
        mz = np.sort(np.asarray(mz, np.float64))
        return {"m/z array": mz, "intensity array": np.ones(len(mz)), "precursor mz": 500.0,
                "precursor charge": 2}

    for n, cols, kmax in ((65, 32000, 3000), (70, 32768, 9000), (80, 33000, 9000), (120, 60000, 3000),
                          (200, 5000, 3000)):
        grid = 0.1 * np.arange(1, cols + 1) - 0.05  # one bin per grid value: ceil(m / 0.1) = k
        members = []
        for j in range(n):
            k = int(rng.integers(1, kmax)) if j % 7 else int(rng.integers(1, 40))
            members.append(spec(rng.choice(grid, size=min(k, cols), replace=False)))
        members[3] = spec([])                 # an empty spectrum
        members[5] = dict(members[4])         # identical spectra
        clusters.append(members)
    csr = SpectraCSR.from_clusters(clusters)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


def test_medoid_large_path_pairwise_tree_shapes(gpu):
    """The large path's totals follow numpy's pairwise tree over n (leaves of <= 128,
    splits at n/2 - (n/2) % 8): medoid_plan2_kernel numbers the leaves and internal
    nodes in post-order by descents from the root, medoid_combine_kernel evaluates the
    tree as a stack machine over those ids.  n at and around every leaf / split boundary
    up to three levels (65 .. 513 spectra of short spectra, so the flat unit and row
    grids hold many small deferred clusters), between ordinary small clusters:
    representatives and totals bit-exact vs the C oracle."""
    ns = [65, 127, 128, 129, 135, 136, 137, 255, 256, 257, 263, 264, 265, 511, 512, 513]
    sizes = []
    for n in ns:
        sizes += [n, 3]
    csr = make_clusters_np(len(sizes), seed=313, sizes=np.array(sizes), n_template=24)
    rep, tot = engine.medoid(engine.DeviceBatch.from_host(csr), with_totals=True).to_host()
    ref_rep, ref_tot = c_oracle.medoid_parallel(csr, with_totals=True)
    np.testing.assert_array_equal(rep, ref_rep)
    np.testing.assert_array_equal(tot, ref_tot)


# ------------------------------------------------------- gather wire format
def _wire_roundtrip(mz, it, max_count):
    import torch

    dev = torch.device("cuda:0")
    dmz = torch.as_tensor(np.ascontiguousarray(mz), device=dev)
    dit = torch.as_tensor(np.ascontiguousarray(it), device=dev)
    mi, cnt, n_fail = engine.wire_pack(dmz, dit, max_count)
    rmz, rit = engine.wire_unpack(mi, cnt)
    torch.cuda.synchronize()
    return rmz.cpu().numpy(), rit.cpu().numpy(), cnt.cpu().numpy(), int(n_fail.item())


def test_gather_wire_format_rebuilds_bin_mean_bits(gpu):
    """spx_wire_pack / spx_wire_unpack (the multi-GPU gather's 9-10 byte peaks) on
    bin-mean consensus peaks: every peak rebuilt bit for bit -- a NaN m/z of a zero m/z
    sum (binning.py:216; minimum below 0 and peaks at m/z 0), infinite intensity sums,
    1-byte counts (clusters <= 255) and 2-byte counts (a 300-spectrum cluster) -- and a
    value that no bin-mean produces reported in n_fail."""
    base = make_clusters_np(200, seed=61)
    rng = np.random.default_rng(3)
    extra = []
    for n, lo in ((4, -1.0), (300, 100.0)):  # zero-m/z bins; a cluster past 255 spectra
        cl = []
        tmpl = np.sort(np.round(rng.uniform(100.0, 900.0, 60), 5))  # every bin reaches the quorum
        for s in range(n):
            mzv = np.round(tmpl + rng.normal(0.0, 0.002, 60), 5) if s % 2 else tmpl.copy()
            mzv = np.sort(mzv)
            if lo < 0:
                mzv = np.concatenate([[0.0, 0.0], mzv])
            itv = np.round(rng.uniform(1.0, 500.0, len(mzv)), 2)
            if s == 1 and lo < 0:
                itv[1] = np.inf  # the zero-m/z bin's contribution: an infinite intensity sum
            cl.append({"m/z array": mzv, "intensity array": itv, "precursor mz": 500.0, "precursor charge": 2})
        extra.append(cl)
    ex = SpectraCSR.from_clusters(extra)
    for csr, kw in ((base, {}), (ex, dict(minimum=-1.0))):
        ref = c_oracle.bin_mean(csr, **kw)
        got = _bin_mean(csr, **kw)
        assert_bin_mean_equal(got, ref)
        mz, it = got["out_mz"], got["out_int"]
        cmax = int(csr.cluster_sizes().max())
        rmz, rit, cnt, n_fail = _wire_roundtrip(mz, it, cmax)
        assert n_fail == 0
        assert cnt.dtype == (np.uint8 if cmax <= 255 else np.int16)
        np.testing.assert_array_equal(rmz.view(np.int64), mz.view(np.int64))
        np.testing.assert_array_equal(rit.view(np.int64), it.view(np.int64))
    assert np.isnan(got["out_mz"]).any() and np.isinf(got["out_int"]).any()
    _, _, _, n_fail = _wire_roundtrip(np.array([np.pi, 100.25]), np.array([np.e, 3.5]), 50)
    assert n_fail == 1
