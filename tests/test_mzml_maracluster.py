"""mzML + MaRaCluster input path, host side.

* binning.read_cluster_list and convert_mgf_cluster.py's read_clusters /
  read_peptides / buid_usi_accession / convert-mq-marcluster against the
  reference's own outputs (tests/golden/maracluster.json, make_golden.py).
* The mzML reader (a pyteomics stand-in; pyteomics is absent, so its parity is
  unpinned) through round trips of the writer: 64/32-bit, zlib/none, gzip.
"""
import json
import os

import numpy as np
import pytest

from specpride_amd import convert_mgf_cluster as cmc
from specpride_amd import mzml
from specpride_amd.binning import RepresentativeSpectrumCreator
from specpride_amd.mgf import read_mgf

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _g():
    with open(os.path.join(GOLD, "maracluster.json")) as fh:
        return json.load(fh)


def test_read_cluster_list_matches_reference():
    got = RepresentativeSpectrumCreator().read_cluster_list(os.path.join(GOLD, "maracluster_clusters.tsv"))
    assert got == _g()["read_cluster_list"]


def test_convert_helpers_match_reference():
    g = _g()
    assert {str(k): v for k, v in cmc.read_clusters(os.path.join(GOLD, "maracluster_clusters.tsv")).items()} \
        == g["read_clusters"]
    assert {str(k): v for k, v in cmc.read_peptides(os.path.join(GOLD, "maracluster_msms.txt")).items()} \
        == g["read_peptides"]
    assert [cmc.buid_usi_accession("cluster-3", None, 7, "PXD1", "raw", 2),
            cmc.buid_usi_accession("cluster-3", "PEPK", 7, "PXD1", "raw", 2)] == g["usi"]


def test_convert_mq_marcluster_mgf_matches_reference(tmp_path, capsys):
    g = _g()
    out = tmp_path / "clustered.mgf"
    cmc.convert_mq_mracluster_mgf(os.path.join(GOLD, "maracluster_msms.txt"),
                                  os.path.join(GOLD, "maracluster_clusters.tsv"),
                                  os.path.join(GOLD, "maracluster_in.mgf"), str(out), "PXD000001", "run")
    got = read_mgf(str(out))
    assert [s["params"]["title"] for s in got] == g["converted_titles"]
    assert [s["params"]["pepmass"][0] for s in got] == g["converted_pepmass"]
    assert "Number of Clusters: 8" in capsys.readouterr().out


def _spectra(rng, scans):
    out = []
    for k, scan in enumerate(scans):
        n = int(rng.integers(0, 40))
        out.append({"scan": scan, "ms level": 1 if k == 2 else 2, "m/z array": np.sort(rng.uniform(100, 2000, n)),
                    "intensity array": rng.lognormal(4, 2, n), "precursor mz": float(rng.uniform(400, 1200)),
                    "precursor charge": int(rng.integers(1, 5))})
    return out


@pytest.mark.parametrize("bits,compress,suffix", [(64, True, ".mzML"), (64, False, ".mzML"), (32, True, ".mzML"),
                                                  (64, True, ".mzML.gz")])
def test_mzml_round_trip(tmp_path, bits, compress, suffix):
    rng = np.random.default_rng(bits + compress)
    sp = _spectra(rng, [3, 10, 11, 250, 7])
    path = str(tmp_path / ("run" + suffix))
    mzml.write_mzml(path, sp, bits=bits, compress=compress)
    with mzml.read(path) as rd:
        assert len(rd) == len(sp)
        for s in sp:
            got = rd.get_by_id(f"controllerType=0 controllerNumber=1 scan={s['scan']}")
            assert got["ms level"] == s["ms level"]
            dt = np.float64 if bits == 64 else np.float32
            np.testing.assert_array_equal(got["m/z array"], s["m/z array"].astype(dt))
            np.testing.assert_array_equal(got["intensity array"], s["intensity array"].astype(dt))
            if s["ms level"] == 2:
                ion = got["precursorList"]["precursor"][0]["selectedIonList"]["selectedIon"][0]
                assert ion["selected ion m/z"] == s["precursor mz"]
                assert ion["charge state"] == s["precursor charge"]
        with pytest.raises(KeyError):
            rd.get_by_id("controllerType=0 controllerNumber=1 scan=999")


def test_read_spectra_skips_non_ms2(tmp_path, capsys):
    rng = np.random.default_rng(2)
    sp = _spectra(rng, [1, 2, 3, 4])
    path = str(tmp_path / "run.mzML")
    mzml.write_mzml(path, sp)
    rsc = RepresentativeSpectrumCreator(verbose=0)
    got = rsc.read_spectra(path, ["4", "3", "1"])  # scan 3 is MS1 (k == 2)
    out = capsys.readouterr().out
    assert "ERROR: scan 3 is not ms_level=2! Skipping" in out
    assert "INFO: Read 3 spectra from" in out
    assert len(got) == 2
    np.testing.assert_array_equal(got[0]["m/z array"], sp[3]["m/z array"])
    assert got[1]["precursor mz"] == sp[0]["precursor mz"] and got[1]["precursor charge"] == sp[0]["precursor charge"]
