"""GPU parity of the drop-in modules (the reference's own entry points) against
the reference's golden outputs and the oracle.

* binning.main            -> byte-identical MGF to the reference CLI run (binning.py:250-302)
* most_similar_representative.representatives / main -> the reference's chosen
  spectra, including its first-contiguous-run cluster scan (:49-75)
* most_similar_representative.distance -> oracle xcorr per pair (:13-19)
* average_spectrum_clustering.average_spectrum -> reference outputs and exception
  types per golden cluster (:26-103)
* average_spectrum_clustering.process_maracluster_mgf -> oracle on a synthetic file
"""
import contextlib
import io
import os

import numpy as np
import pytest

from conftest import GOLDEN, gap_params, load_golden, load_json
from oracle import np_oracle
from specpride_amd import average_spectrum_clustering as asc
from specpride_amd import binning
from specpride_amd import most_similar_representative as msr
from specpride_amd.mgf import read_mgf, write_csr_mgf
from specpride_amd.synthetic import make_clusters_np

pytestmark = pytest.mark.gpu


def test_binning_cli_byte_identical(gpu, tmp_path):
    out = tmp_path / "merged.mgf"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        binning.main(["--mgf_file", os.path.join(GOLDEN, "bin_mean_cli_in.mgf"), "--out", str(out)])
    assert buf.getvalue() == load_json("bin_mean_cli.json")["stdout"]
    with open(os.path.join(GOLDEN, "bin_mean_cli_out.mgf"), "rb") as fh:
        assert out.read_bytes() == fh.read()


def test_binning_cli_nonfinite_byte_identical(gpu, tmp_path):
    """nan / inf / Infinity / 1e999 number tokens (Python float() spellings) through
    the binning CLI: the same file as the reference's run (make_golden.py nonfinite)."""
    out = tmp_path / "merged.mgf"
    with contextlib.redirect_stdout(io.StringIO()):
        binning.main(["--mgf_file", os.path.join(GOLDEN, "bin_mean_cli_nonfinite_in.mgf"), "--out", str(out)])
    with open(os.path.join(GOLDEN, "bin_mean_cli_nonfinite_out.mgf"), "rb") as fh:
        assert out.read_bytes() == fh.read()


def test_average_spectrum_nonfinite_no_error(gpu):
    """The reference returns output on NaN input (no exception): NaN m/z joins the
    last group, a kept NaN intensity makes np.max NaN and keeps nothing."""
    S = lambda mz, it: {"m/z array": np.array(mz, float), "intensity array": np.array(it, float)}  # noqa: E731
    r = asc.average_spectrum([S([100, np.nan, 200], [1, 2, 3]), S([100, 200], [1, 3])])
    np.testing.assert_array_equal(r["m/z array"], [100.0, np.nan])
    np.testing.assert_array_equal(r["intensity array"], [1.0, 4.0])
    r = asc.average_spectrum([S([100, 200], [1, np.nan]), S([100, 200], [1, 1])])
    assert len(r["m/z array"]) == 0 and len(r["intensity array"]) == 0
    r = asc.average_spectrum([S([100, 200, np.inf], [1, 2, 3]), S([100, 200], [1, 2])])
    np.testing.assert_array_equal(r["m/z array"], [100.0, np.inf])
    np.testing.assert_array_equal(r["intensity array"], [1.0, 3.5])


def test_medoid_noncontiguous_runs(gpu, tmp_path):
    g = load_json("medoid_noncontiguous.json")
    spectra = read_mgf(os.path.join(GOLDEN, "medoid_noncontiguous.mgf"))
    names = [s["params"]["title"].split(";")[0] for s in spectra]
    assert names == g["names"]
    got = [best for _cl, _m, best in msr.representatives(spectra, names)]
    assert got == g["rep_index"]
    out = tmp_path / "reps.mgf"
    with contextlib.redirect_stdout(io.StringIO()):
        msr.main(["-i", os.path.join(GOLDEN, "medoid_noncontiguous.mgf"), "-o", str(out)])
    assert [s["params"]["title"] for s in read_mgf(str(out))] == g["titles"]


def test_medoid_main_golden_through_shim(gpu):
    z, csr = load_golden("medoid_main.npz")
    spectra, names = [], []
    for c in range(csr.n_clusters):
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            a, b = csr.spec_off[s], csr.spec_off[s + 1]
            spectra.append({"m/z array": csr.mz[a:b], "intensity array": csr.inten[a:b], "params": {}})
            names.append(f"cluster-{c}")
    got = [best for _cl, _m, best in msr.representatives(spectra, names)]
    np.testing.assert_array_equal(got, z["rep_index"])


def test_distance_matches_oracle(gpu):
    rng = np.random.default_rng(5)
    for _ in range(12):
        n1, n2 = rng.integers(0, 80, 2)
        base = np.sort(rng.uniform(100, 1500, max(n1, n2)))
        m1 = np.round(base[:n1] + rng.normal(0, 0.05, n1), 3)
        m2 = np.round(rng.permutation(base)[:n2], 3)
        want = 1.0 - np_oracle.xcorr(m1, m2, 0.1)
        assert msr.distance(m1, m2) == want
        assert msr.distance({"m/z array": m1}, (m2, np.ones_like(m2))) == want
    assert msr.distance([1.0], [2.0], method="other") == 0


def test_xcorr_distance_batched_pairs_vs_oracle(gpu):
    """spx_xcorr_distance over many pairs: the LDS-bitmap path and, for spectra
    with a bin outside [0, 65,536) (m/z >= 6,553.6 or negative), the scan path."""
    from specpride_amd import engine
    from specpride_amd.csr import SpectraCSR

    rng = np.random.default_rng(11)
    spectra = []
    for k in range(60):
        n = int(rng.integers(0, 300))
        hi = 9000.0 if k % 7 == 3 else 2000.0
        lo = -5.0 if k % 11 == 5 else 100.0
        m = np.round(np.sort(rng.uniform(lo, hi, n)), 4)
        if n > 4 and k % 5 == 0:
            m[1] = m[0]  # a repeated bin inside one spectrum
        spectra.append(m)
    csr = SpectraCSR.from_clusters([[{"m/z array": m, "intensity array": np.ones_like(m)} for m in spectra]])
    pairs = [(i, j) for i in range(60) for j in range(i, 60) if (i * 7 + j) % 3 == 0]
    got = engine.xcorr_distance(engine.DeviceBatch.from_host(csr), pairs, 0.1).cpu().numpy()
    want = np.array([1.0 - np_oracle.xcorr(spectra[i], spectra[j], 0.1) for i, j in pairs])
    np.testing.assert_array_equal(got, want)


def test_average_spectrum_per_cluster_vs_golden(gpu):
    z, csr = load_golden("gap_average_edge.npz")
    kw = gap_params(z)
    for c in range(csr.n_clusters):
        spectra = []
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            a, b = csr.spec_off[s], csr.spec_off[s + 1]
            spectra.append({"m/z array": csr.mz[a:b], "intensity array": csr.inten[a:b],
                            "params": {"pepmass": (csr.prec_mz[s], None), "charge": [int(csr.charge[s])],
                                       "rtinseconds": csr.rt[s]}})
        st = int(z["status"][c])
        if st == 2:
            with pytest.raises(IndexError):
                asc.average_spectrum(spectra, **kw)
            continue
        if st == 3:
            with pytest.raises(ValueError):
                asc.average_spectrum(spectra, **kw)
            continue
        r = asc.average_spectrum(spectra, title="t", pepmass=1.0, rtinseconds=2.0, charge=2, **kw)
        a, b = z["out_off"][c], z["out_off"][c + 1]
        np.testing.assert_allclose(r["m/z array"], z["out_mz"][a:b], rtol=1e-9)
        np.testing.assert_allclose(r["intensity array"], z["out_int"][a:b], rtol=1e-9)
        assert r["params"] == {"title": "t", "pepmass": 1.0, "rtinseconds": 2.0, "charge": 2}


@pytest.mark.parametrize("helpers", [("naive", "median"), ("lower", "mass_lower"), ("neutral", "median")])
def test_process_maracluster_mgf_vs_oracle(gpu, tmp_path, helpers):
    csr = make_clusters_np(40, seed=21, n_template=60)
    path = tmp_path / "in.mgf"
    write_csr_mgf(csr, str(path))
    pm = {"naive": asc.naive_average_mass_and_charge, "lower": asc.lower_median_mass,
          "neutral": asc.neutral_average_mass_and_charge}[helpers[0]]
    rtf = {"median": asc.median_rt, "mass_lower": asc.lower_median_mass_rt}[helpers[1]]
    outs = asc.process_maracluster_mgf(str(path), get_pepmass=pm, get_rt=rtf)
    ref = np_oracle.gap_average(csr)
    assert len(outs) == csr.n_clusters
    for c, o in enumerate(outs):
        a, b = ref["out_off"][c], ref["out_off"][c + 1]
        np.testing.assert_allclose(o["m/z array"], ref["out_mz"][a:b], rtol=1e-9)
        np.testing.assert_allclose(o["intensity array"], ref["out_int"][a:b], rtol=1e-9)
        s0, s1 = csr.cluster_off[c], csr.cluster_off[c + 1]
        pr, ch, rt = csr.prec_mz[s0:s1], csr.charge[s0:s1], csr.rt[s0:s1]
        if helpers[0] == "naive":
            want_mz, want_z = np_oracle.naive_average_mass_and_charge(pr, ch)
        elif helpers[0] == "lower":
            want_mz, want_z = np_oracle.lower_median_mass(pr, ch)
        else:
            want_mz, want_z = np_oracle.neutral_average_mass_and_charge(pr, ch)
        want_rt = np_oracle.median_rt(rt) if helpers[1] == "median" else np_oracle.lower_median_mass_rt(pr, ch, rt)
        assert o["params"]["title"] == f"cluster-{c}"
        assert o["params"]["charge"] == want_z
        np.testing.assert_allclose(o["params"]["pepmass"], want_mz, rtol=1e-12)
        np.testing.assert_allclose(o["params"]["rtinseconds"], want_rt, rtol=1e-12)


def test_shard_driver_with_engine_over_rccl(gpu):
    """specpride_amd.shard with the HIP engine as compute over a world-1 nccl
    (RCCL) group: the gatherv/reorder path on device tensors."""
    import socket

    import torch.distributed as dist

    from oracle import c_oracle
    from specpride_amd import shard

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        csr = make_clusters_np(64, seed=8)
        got = shard.consensus_sharded(csr, "bin_mean", device=gpu)
        ref = c_oracle.bin_mean(csr)
        for k in ("out_off", "out_mz", "out_int", "status", "prec", "charge"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        got = shard.consensus_sharded(csr, "gap_average", device=gpu)
        ref = c_oracle.gap_average(csr)
        np.testing.assert_array_equal(got["out_off"], ref["out_off"])
        np.testing.assert_allclose(got["out_mz"], ref["out_mz"], rtol=1e-9)
        rep, totals = shard.medoid_sharded(csr, {"with_totals": True}, device=gpu)
        want_rep, want_tot = c_oracle.medoid(csr, with_totals=True)
        np.testing.assert_array_equal(rep, want_rep)
        np.testing.assert_array_equal(totals, want_tot)
    finally:
        dist.destroy_process_group()


def test_binning_mzml_maracluster_cli(gpu, tmp_path):
    """The mzML + MaRaCluster input path (binning.py:35-119, the CLI options the
    reference keeps commented out): every cluster through one GPU pass, consensus
    bit-exact against the oracle on the same spectra; an MS1 scan is skipped."""
    from oracle import c_oracle
    from specpride_amd import mgf_native, mzml

    csr = make_clusters_np(12, seed=8)
    spectra, tsv, scan = [], [], 100
    for c in range(csr.n_clusters):
        for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
            m, i = csr.spectrum(s)
            spectra.append({"scan": scan, "ms level": 2, "m/z array": m, "intensity array": i,
                            "precursor mz": float(csr.prec_mz[s]), "precursor charge": int(csr.charge[s])})
            tsv.append(f"run.raw\t{scan}\t0.1\n")
            scan += 1
        tsv.append("\n")
    spectra.append({"scan": 9999, "ms level": 1, "m/z array": np.array([150.0]), "intensity array": np.ones(1)})
    tsv.insert(1, "run.raw\t9999\t0.1\n")  # the MS1 scan sits in cluster 0: skipped with an ERROR line
    path, tpath, out = tmp_path / "run.mzML", tmp_path / "mara.tsv", tmp_path / "out.mgf"
    mzml.write_mzml(str(path), spectra)
    tpath.write_text("".join(tsv))
    with contextlib.redirect_stdout(io.StringIO()) as so:
        binning.main(["--mara_file", str(tpath), "--mzml_file", str(path), "--out", str(out)])
    assert "ERROR: scan 9999 is not ms_level=2! Skipping" in so.getvalue()
    # expected: the oracle on the same clusters (precursors as written to the mzML)
    ref = c_oracle.bin_mean(csr)
    merged = []
    for c in range(csr.n_clusters):
        a, b = ref["out_off"][c], ref["out_off"][c + 1]
        merged.append({"cluster_id": str(c), "mzs": ref["out_mz"][a:b], "intensities": ref["out_int"][a:b],
                       "precursor_mz": np.float64(ref["prec"][c]), "precursor_charge": int(ref["charge"][c])})
    want = tmp_path / "want.mgf"
    with open(want, "wt") as fh:
        mgf_native.write_binning_mgf(merged, fh)
    assert out.read_bytes() == want.read_bytes()


def test_staged_host_transfers_round_trip(gpu):
    """spx_copy_h2d / spx_copy_d2h (pinned staging pool, several host threads,
    DMA overlapped): a batch above the packed-copy size arrives bit for bit, and
    comes back the same way; odd sizes cover partial chunks."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_np

    csr = make_clusters_np(6000, seed=31)
    assert 16 * csr.n_peaks > engine.PACKED_MAX_BYTES
    b = engine.DeviceBatch.from_host(csr)
    for k in ("cluster_off", "spec_off", "mz", "inten", "prec_mz", "charge", "rt"):
        got = engine.to_host_array(b.t[k])
        np.testing.assert_array_equal(got, getattr(csr, k), err_msg=k)
    rng = np.random.default_rng(3)
    for n in (1, (1 << 20) + 3, (9 << 20) + 7, 17 * (1 << 20) + 1):  # f64 elements
        a = rng.standard_normal(n)
        d = torch.empty(n, dtype=torch.float64, device="cuda")
        from specpride_amd import _lib

        _lib.check(_lib.lib().spx_copy_h2d(d.data_ptr(), a.ctypes.data, a.nbytes,
                                           torch.cuda.current_stream().cuda_stream), "h2d")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d.cpu().numpy(), a)
        np.testing.assert_array_equal(engine.to_host_array(d) if a.nbytes > engine.PACKED_MAX_BYTES else
                                      d.cpu().numpy(), a)
    # the results of a large batch come back through spx_copy_d2h too
    res = engine.bin_mean(b).to_host()
    from oracle import c_oracle

    sub = csr.select(range(50))
    ref = c_oracle.bin_mean(sub)
    np.testing.assert_array_equal(res["out_mz"][:res["out_off"][50]], ref["out_mz"])
