"""Native MGF ingest (csrc/mgf_io.cpp via specpride_amd.mgf_native) against the
Python readers it replaces, on the golden files and synthetic ones.

* ``parse_general`` == :func:`specpride_amd.mgf.iter_mgf` (the gap-average and
  medoid CLIs' reader) value for value, or reports "fallback" where its subset
  ends (several charges, non-decimal numbers, tabs inside the binning format ...).
* ``index`` + ``parse_ranges`` in any record order == the whole-file parse.
* the ingest groupings (specpride_amd.ingest) == the CLIs' own dict groupings.
"""
import os

import numpy as np
import pytest

from specpride_amd import ingest, mgf, mgf_native

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
FILES = ["maracluster_in.mgf", "medoid_noncontiguous.mgf", "best_spectrum_in.mgf", "bin_mean_cli_in.mgf"]


def _check_general_equal(path):
    d = mgf_native.parse_general(path)
    ref = mgf.read_mgf(path)
    assert len(ref) == len(d["titles"])
    so = d["spec_off"]
    for s, r in enumerate(ref):
        np.testing.assert_array_equal(d["mz"][so[s]:so[s + 1]], r["m/z array"])
        np.testing.assert_array_equal(d["inten"][so[s]:so[s + 1]], r["intensity array"])
        p = r["params"]
        assert d["has_title"][s] == ("title" in p) and d["titles"][s] == p.get("title", "")
        assert d["has_prec"][s] == ("pepmass" in p) and d["has_charge"][s] == ("charge" in p)
        assert d["has_rt"][s] == ("rtinseconds" in p)
        if "pepmass" in p:
            assert d["prec_mz"][s] == p["pepmass"][0]
        else:
            assert np.isnan(d["prec_mz"][s])
        assert d["charge"][s] == (p["charge"][0] if "charge" in p else 0)
        if "rtinseconds" in p:
            assert d["rt"][s] == p["rtinseconds"]
    return d


@pytest.mark.parametrize("name", FILES)
def test_parse_general_equals_iter_mgf(name):
    _check_general_equal(os.path.join(GOLD, name))


@pytest.mark.parametrize("name", FILES)
@pytest.mark.parametrize("general", [False, True])
def test_index_and_ranges_equal_whole_parse(name, general):
    path = os.path.join(GOLD, name)
    try:
        whole = mgf_native.parse_general(path) if general else mgf_native.parse_native(path)
    except ValueError:
        pytest.skip("outside the binning parser's subset (TITLE without ';')")
    X = mgf_native.index(path, general)
    assert X["titles"] == whole["titles"]
    np.testing.assert_array_equal(X["npk"], np.diff(whole["spec_off"]))
    perm = np.random.default_rng(0).permutation(len(X["begin"]))
    part = mgf_native.parse_ranges(path, X["begin"][perm], X["end"][perm], general)
    assert part["titles"] == [whole["titles"][i] for i in perm]
    so, po = whole["spec_off"], part["spec_off"]
    for k, i in enumerate(perm):
        np.testing.assert_array_equal(part["mz"][po[k]:po[k + 1]], whole["mz"][so[i]:so[i + 1]])
        np.testing.assert_array_equal(part["inten"][po[k]:po[k + 1]], whole["inten"][so[i]:so[i + 1]])
    for key in ("prec_mz", "charge"):
        np.testing.assert_array_equal(part[key], whole[key][perm])


def test_general_edge_cases(tmp_path):
    """Params iter_mgf keeps or ignores, optional intensities, signed / dotted
    peak lines, CRLF, lines outside blocks, a block without END IONS."""
    text = ("junk before\r\nBEGIN IONS\r\nTITLE=a;1\r\nPEPMASS=500.25 1234.5\r\nCHARGE=3-\r\n"
            "SEQUENCE=PEPTIDE\r\nrtinseconds= 12.5 \r\n100.5 3\r\n.5 2\r\n101.5\r\n+102 7\r\nEND IONS\r\n"
            "between=1\nBEGIN IONS\nTITLE=b;2\n200.0\t4.0\nEND IONS\n"
            "BEGIN IONS\nTITLE=lost\n1 2\nBEGIN IONS\ntitle = x\n  300 5 extra  \nEND IONS\n")
    p = tmp_path / "e.mgf"
    p.write_bytes(text.encode())
    d = _check_general_equal(str(p))
    assert d["titles"] == ["a;1", "b;2", ""]
    X = mgf_native.index(str(p), True)
    assert X["titles"] == d["titles"] and list(X["npk"]) == [4, 1, 1]


@pytest.mark.parametrize("text", [
    "BEGIN IONS\nCHARGE=2+ and 3+\nEND IONS\n",            # several charges
    "BEGIN IONS\nPEPMASS=inf\nEND IONS\n",                 # non-decimal number
    "BEGIN IONS\n1_000 2\nEND IONS\n",
    "END IONS\n",                                          # END IONS outside a block
    "BEGIN IONS\nTITLE=é\nEND IONS\n",                # non-ASCII
    "BEGIN IONS\nPEPMASS=500 x\nEND IONS\n",               # iter_mgf's float(p[1]) raises
])
def test_general_fallback(tmp_path, text):
    p = tmp_path / "f.mgf"
    p.write_text(text, encoding="utf-8")
    with pytest.raises(ValueError, match="fallback"):
        mgf_native.parse_general(str(p))


def test_groupings_match_cli_dict_paths():
    from itertools import groupby

    from specpride_amd.most_similar_representative import _first_runs

    path = os.path.join(GOLD, "medoid_noncontiguous.mgf")
    titles = [s["params"]["title"] for s in mgf.read_mgf(path)]
    ids, records, sizes = ingest.medoid_groups(titles)
    runs = [(cl, m) for cl, m in _first_runs([t.split(";")[0] for t in titles]) if m]
    assert ids == [cl for cl, _ in runs] and list(records) == [i for _, m in runs for i in m]
    ids, records, sizes = ingest.gap_average_groups(titles)
    want = [(k, len(list(g))) for k, g in groupby(t.split(";", 1)[0] for t in titles)]
    assert list(zip(ids, sizes.tolist())) == want
    ids, records, sizes = ingest.binning_groups(titles)
    order = list(dict.fromkeys(t.split(";")[0] for t in titles))
    assert ids == order
    assert [titles[i].split(";")[0] for i in records] == sorted((t.split(";")[0] for t in titles), key=order.index)
