"""Pin the oracle (numpy + C restatements) to the reference's own outputs.

The golden vectors in tests/golden/ were produced by running the reference
(/root/reference/src) itself -- see tests/golden/make_golden.py.  Bin-mean and
gap-average are bit-exact; medoid indices are exact given the restated OpenMS
xcorr (parity unpinned at that boundary)."""
import numpy as np
import pytest

from conftest import BIN_SETS, GAP_SETS, bin_params, gap_params, load_golden
from oracle import c_oracle, np_oracle


@pytest.mark.parametrize("name", BIN_SETS)
@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_bin_mean_oracle_matches_reference(name, impl):
    z, csr = load_golden(f"bin_mean_{name}.npz")
    r = (np_oracle if impl == "numpy" else c_oracle).bin_mean(csr, **bin_params(z))
    np.testing.assert_array_equal(r["status"], z["status"])
    np.testing.assert_array_equal(r["out_off"], z["out_off"])
    np.testing.assert_array_equal(r["out_mz"], z["out_mz"])          # bit-exact
    np.testing.assert_array_equal(r["out_int"], z["out_int"])
    ok = z["status"] == 0
    np.testing.assert_array_equal(r["prec"][ok], z["out_prec"][ok])
    np.testing.assert_array_equal(r["charge"][ok], z["out_charge"][ok])


@pytest.mark.parametrize("name", GAP_SETS)
def test_gap_average_numpy_oracle_bit_exact(name):
    z, csr = load_golden(f"gap_average_{name}.npz")
    r = np_oracle.gap_average(csr, **gap_params(z))
    np.testing.assert_array_equal(r["status"], z["status"])
    np.testing.assert_array_equal(r["out_off"], z["out_off"])
    np.testing.assert_array_equal(r["out_mz"], z["out_mz"])
    np.testing.assert_array_equal(r["out_int"], z["out_int"])


@pytest.mark.parametrize("name", GAP_SETS)
def test_gap_average_c_oracle(name):
    z, csr = load_golden(f"gap_average_{name}.npz")
    r = c_oracle.gap_average(csr, **gap_params(z))
    np.testing.assert_array_equal(r["status"], z["status"])
    np.testing.assert_array_equal(r["out_off"], z["out_off"])
    np.testing.assert_allclose(r["out_mz"], z["out_mz"], rtol=1e-12)
    np.testing.assert_allclose(r["out_int"], z["out_int"], rtol=1e-12)


def test_precursor_helpers():
    z, csr = load_golden("precursor_helpers.npz")
    H = float(z["H"])
    for c in range(csr.n_clusters):
        s0, s1 = csr.cluster_off[c], csr.cluster_off[c + 1]
        pr, ch, rt = csr.prec_mz[s0:s1], csr.charge[s0:s1], csr.rt[s0:s1]
        m, zz = np_oracle.lower_median_mass(pr, ch, H)
        assert m == z["lm_mz"][c] and zz == z["lm_z"][c]
        assert np_oracle.lower_median_mass_rt(pr, ch, rt, H) == z["lm_rt"][c]
        na = np_oracle.naive_average_mass_and_charge(pr, ch)
        if z["na_status"][c]:
            assert na is None
        else:
            assert na == (z["na_mz"][c], z["na_z"][c])
        assert np_oracle.neutral_average_mass_and_charge(pr, ch, H) == (z["ne_mz"][c], z["ne_z"][c])
        assert np_oracle.median_rt(rt) == z["med_rt"][c]


@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_pairwise_sum_tree(impl):
    z = np.load(__import__("conftest").GOLDEN + "/pairwise_sum.npz")
    f = np_oracle.pairwise_sum if impl == "numpy" else c_oracle.pairwise_sum
    for a, b, s in zip(z["off"][:-1], z["off"][1:], z["sums"]):
        assert f(z["vals"][a:b]) == s


def test_pairwise_sum_matches_numpy_reduce():
    rng = np.random.default_rng(5)
    for n in list(range(0, 300)) + [511, 512, 513, 1024, 2047, 4099, 8191]:
        v = rng.random(n) * 10.0 ** rng.uniform(-5, 5, n)
        assert c_oracle.pairwise_sum(v) == np.add.reduce(v)


@pytest.mark.parametrize("impl", ["numpy", "c", "c_dense"])
def test_medoid_oracle_matches_reference(impl):
    z, csr = load_golden("medoid_main.npz")
    if impl == "numpy":
        rep = np_oracle.medoid(csr)
    else:
        rep = c_oracle.medoid(csr, dense_tables=(impl == "c_dense"))
    np.testing.assert_array_equal(rep, z["rep_index"])


def test_binned_cosine_oracle_matches_reference():
    """benchmark.py cos_dist / average_cos_dist, run by the reference itself
    (scipy binned_statistic) vs the numpy restatement: identical values."""
    z, csr = load_golden("binned_cosine.npz")
    cos, avg, status = np_oracle.binned_cosine(csr, z["rep_off"], z["rep_mz"], z["rep_int"], float(z["mz_space"]))
    np.testing.assert_array_equal(status, z["status"])
    np.testing.assert_array_equal(cos, z["cos"])
    np.testing.assert_array_equal(avg, z["avg"])
    # the golden holds the edge cases it claims: an on-edge member peak, cos 0 and 1, no members
    assert np.any(z["cos"] == 0.0) and np.any(np.isclose(z["cos"], 1.0)) and np.any(z["avg"] == 0.0)


def _best_golden():
    import json
    import os

    import pandas as pd

    from specpride_amd import best_spectrum as bs

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "best_spectrum.json")) as fh:
        g = json.load(fh)
    spectra = bs.get_cluster_spectra(os.path.join(here, "best_spectrum_in.mgf"))
    scores = bs.get_scores(os.path.join(here, "best_spectrum_msms.txt"))
    assert isinstance(scores, pd.Series) and scores.index.is_monotonic_increasing
    return g, [list(cl) for cl in bs.split_into_clusters(spectra)], scores


def test_best_score_oracle_matches_reference():
    """best_spectrum.py:97-100 restated (join + segmented argmax) vs the reference's
    get_best_representative on every cluster of the golden file."""
    g, clusters, scores = _best_golden()
    usis = [u for cl in clusters for u in cl]
    off = np.zeros(len(clusters) + 1, np.int64)
    np.cumsum([len(cl) for cl in clusters], out=off[1:])
    score, rank = np_oracle.score_join(usis, list(scores.index), scores.to_numpy())
    best, status = np_oracle.best_score(off, score, rank)
    got = [usis[b] if st == np_oracle.STATUS_OK else "ValueError" for b, st in zip(best, status)]
    assert got == g["per_cluster"]
    # the NaN-only cluster: the reference raises KeyError (pandas idxmax -> NaN)
    s1, r1 = np_oracle.score_join(g["nan_only_cluster"], list(scores.index), scores.to_numpy())
    assert np_oracle.best_score(np.array([0, 1]), s1, r1)[1][0] == np_oracle.STATUS_NON_FINITE
    assert g["nan_only_result"] == "KeyError"


def test_best_spectrum_host_join_matches_oracle():
    """The shim's pandas join (groupby max + sorted rank) equals the oracle's loops."""
    from specpride_amd import best_spectrum as bs

    _, clusters, scores = _best_golden()
    usis = [u for cl in clusters for u in cl] + ["mzspec:PXD004732:runA.raw::scan:88888", "not-scored"]
    s_host, r_host = bs._score_arrays(usis, scores)
    s_or, r_or = np_oracle.score_join(usis, list(scores.index), scores.to_numpy())
    np.testing.assert_array_equal(r_host, r_or)
    np.testing.assert_array_equal(s_host, s_or)
