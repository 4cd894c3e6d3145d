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


# ------------------------------------------------------------------ striped index
def _index_concat(path, general, cuts):
    parts = [mgf_native.index_range(path, general, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    return {k: (sum((p[k] for p in parts), []) if k == "titles" else np.concatenate([p[k] for p in parts]))
            for k in ("begin", "end", "npk", "titles")}


@pytest.mark.parametrize("general", [False, True])
def test_index_range_stripes_compose(tmp_path, general):
    """Byte stripes at ANY cut points (mid-line, between CR and LF, inside a
    record) list every record of the whole-file index exactly once, in order --
    the sharded CLIs' rank-local indexing (sharded_cli.rank_index)."""
    text = ("junk\r\n" + "".join(
        f"BEGIN IONS\r\nTITLE=c{k % 7};u{k}\r\nPEPMASS={400 + k}.5\r\nCHARGE=2+\r\n"
        + "".join(f"{100 + j}.25 {j + 1}.0\r\n" for j in range(k % 5)) + "END IONS\r\n\n" for k in range(40))
        + "BEGIN IONS\nTITLE=x;no_end\n1 2\n")
    p = tmp_path / "s.mgf"
    p.write_bytes(text.encode())
    whole = mgf_native.index(str(p), general)
    size = len(text)
    rng = np.random.default_rng(1)
    for world in (1, 2, 3, 7, 16):
        cuts = [w * size // world for w in range(world + 1)]
        got = _index_concat(str(p), general, cuts)
        assert got["titles"] == whole["titles"]
        for k in ("begin", "end", "npk"):
            np.testing.assert_array_equal(got[k], whole[k])
    for _ in range(20):
        cuts = [0] + sorted(rng.integers(0, size, 5).tolist()) + [size]
        got = _index_concat(str(p), general, cuts)
        assert got["titles"] == whole["titles"]
        np.testing.assert_array_equal(got["begin"], whole["begin"])
        np.testing.assert_array_equal(got["end"], whole["end"])
    # a CR/LF boundary exactly at the cut
    cr = text.index("\r\n", 30) + 1
    got = _index_concat(str(p), general, [0, cr, size])
    np.testing.assert_array_equal(got["begin"], whole["begin"])


# ------------------------------------------------------------------ native writers
def _py_binning(ids, off, mz, it, prec, charge):
    """binning.py:234-245's f-string text (numpy floats; NaN intensities skipped)."""
    out = []
    for c, cid in enumerate(ids):
        t = f"BEGIN IONS\nTITLE={cid}\nPEPMASS={np.float64(prec[c])}\nCHARGE={int(charge[c])}+\n"
        for a, b in zip(mz[off[c]:off[c + 1]], it[off[c]:off[c + 1]]):
            if not np.isnan(b):
                t += f"{a} {b}\n"
        out.append(t + "END IONS\n\n")
    return "".join(out)


def _writer_case(C=9000, seed=0):
    rng = np.random.default_rng(seed)
    n = rng.integers(0, 6, C)
    n[::97] = 0
    off = np.zeros(C + 1, np.int64)
    np.cumsum(n, out=off[1:])
    P = int(off[-1])
    vals = np.concatenate([[0.0, -0.0, 1e16, 1e-5, 1e-4, 123456789012345.6, 1.0 / 3, np.nan, np.inf, -np.inf,
                            5e-324, 1.7976931348623157e308, 100.0, 2.5e-7]], axis=None)
    mz = np.where(rng.random(P) < 0.1, rng.choice(vals, P), np.round(rng.uniform(100, 2000, P) * 10.0 ** (d := rng.integers(0, 12, P))) / 10.0 ** d)
    it = np.where(rng.random(P) < 0.1, rng.choice(vals, P), rng.lognormal(5, 2, P))
    prec = np.where(rng.random(C) < 0.1, rng.choice(vals, C), rng.uniform(400, 1200, C))
    charge = rng.integers(-3, 5, C)
    rt = np.where(rng.random(C) < 0.1, np.nan, rng.uniform(0, 3600, C))
    flags = rng.integers(0, 16, C).astype(np.int32)
    titles = [("" if k % 13 == 0 else f"cluster-{k};mzspec:X:{k}") for k in range(C)]
    return titles, off, mz, it, prec, charge, rt, flags


def test_write_records_binning_style_matches_reference_fstring(tmp_path):
    titles, off, mz, it, prec, charge, _rt, _f = _writer_case()
    p = tmp_path / "b.mgf"
    mgf_native.write_records(str(p), mgf_native.STYLE_BINNING, titles, off, mz, it, prec, charge)
    assert p.read_text() == _py_binning(titles, off, mz, it, prec, charge)


def test_write_records_gap_average_style_matches_python_writer(tmp_path):
    titles, off, mz, it, prec, charge, rt, _f = _writer_case(seed=1)
    specs = [{"params": {"title": t, "pepmass": float(prec[c]), "rtinseconds": float(rt[c]), "charge": int(charge[c])},
              "m/z array": mz[off[c]:off[c + 1]], "intensity array": it[off[c]:off[c + 1]]}
             for c, t in enumerate(titles)]
    want = tmp_path / "w.mgf"
    mgf.write_pyteomics_style(specs, str(want))
    got = tmp_path / "g.mgf"
    mgf_native.write_records(str(got), mgf_native.STYLE_GAP_AVERAGE, titles, off, mz, it, prec, charge, rt)
    assert got.read_bytes() == want.read_bytes()
    # --append (average_spectrum_clustering.py:183-184, file_mode 'a')
    mgf.write_pyteomics_style(specs[:50], str(want), file_mode="a")
    mgf_native.write_records(str(got), mgf_native.STYLE_GAP_AVERAGE, titles[:50], off[:51], mz, it, prec[:50],
                             charge[:50], rt[:50], append=True)
    assert got.read_bytes() == want.read_bytes()


def test_write_records_medoid_style_matches_write_record(tmp_path):
    import io

    from specpride_amd.most_similar_representative import write_record

    titles, off, mz, it, prec, charge, rt, flags = _writer_case(seed=2)
    buf = io.StringIO()
    for c, t in enumerate(titles):
        f = int(flags[c])
        write_record(buf, t if f & 8 else None, prec[c] if f & 1 else None, int(charge[c]) if f & 2 else None,
                     rt[c] if f & 4 else None, mz[off[c]:off[c + 1]], it[off[c]:off[c + 1]])
    got = tmp_path / "m.mgf"
    mgf_native.write_records(str(got), mgf_native.STYLE_MEDOID, titles, off, mz, it, prec, charge, rt, flags)
    assert got.read_text() == buf.getvalue()


# ------------------------------------------------------------------ native grouping
def _groupings_from_key(key, ids, mode):
    """(ids, records, sizes) of ingest.*_groups from spx_mgf_group's key."""
    if mode == mgf_native.GROUP_FIRST_RUNS:
        records = np.flatnonzero(key >= 0)
    else:
        records = np.argsort(key, kind="stable")
    return ids, records, np.bincount(key[records], minlength=len(ids))


@pytest.mark.parametrize("name", FILES + ["SYN"])
def test_native_grouping_equals_ingest_groupings(name, tmp_path):
    """spx_mgf_group's three modes == the CLIs' own groupings (ingest.binning_groups,
    gap_average_groups, medoid_groups, which restate binning.py:160-165,
    average_spectrum_clustering.py:158, most_similar_representative.py:49-75)."""
    if name == "SYN":
        from test_sharded_cli import synthetic_mgf

        path = synthetic_mgf(str(tmp_path / "syn.mgf"), n_clusters=40, seed=9)
        # a later run of an earlier cluster, and a cluster that recurs after others
        text = open(path).read()
        recs = text.split("BEGIN IONS\n")[1:]
        path = str(tmp_path / "syn2.mgf")
        open(path, "w").write("".join("BEGIN IONS\n" + r for r in recs + recs[:3] + recs[10:12]))
    else:
        path = os.path.join(GOLD, name)
    for mode, fn in ((mgf_native.GROUP_BINNING, ingest.binning_groups), (mgf_native.GROUP_RUNS,
                     ingest.gap_average_groups), (mgf_native.GROUP_FIRST_RUNS, ingest.medoid_groups)):
        flat = mgf_native.parse_general(path, group=mode)
        want = fn(flat["titles"])
        got = _groupings_from_key(flat["key"], flat["group_ids"], mode)
        assert got[0] == want[0]
        np.testing.assert_array_equal(got[1], want[1])
        np.testing.assert_array_equal(got[2], want[2])
        assert [flat.title(s) for s in range(len(flat["key"]))] == flat["titles"]


def test_float_parse_equals_python_float(tmp_path):
    """parse_float (csrc/mgf_io.cpp) == Python float() bit for bit on the number
    shapes that take each of its three paths: short decimals (Clinger), 16-19
    significant digits (the x87 extended step: repr of random doubles over many
    decades, decimals next to double rounding midpoints), and long / huge-exponent
    forms (strtod)."""
    rng = np.random.default_rng(11)
    vals = []
    x = np.concatenate([rng.uniform(50, 3000, 40000), rng.lognormal(3, 3, 40000),
                        10.0 ** rng.uniform(-20, 25, 40000)])
    vals += [repr(float(v)) for v in x]
    vals += [f"{v:.19g}" for v in x[:20000]]  # 19 digits: w up to 10^19
    vals += [f"{v:.18e}" for v in x[20000:30000]]
    # decimals halfway between adjacent doubles (exact midpoints) and a hair off them
    for v in x[:6000]:
        a = float(v)
        b = float(np.nextafter(a, np.inf))
        from decimal import Decimal, getcontext
        getcontext().prec = 40
        mid = (Decimal(a) + Decimal(b)) / 2
        for d in (mid, mid.next_plus(), mid.next_minus()):
            vals.append(format(d.quantize(Decimal(1).scaleb(-17)) if abs(d) < 1e3 else d, "f")[:21])
    vals += ["0", "0.0", "-0.0", "123456789012345678901234.5", "1e300", "2.5e-310", "1" * 25, "9007199254740993",
             "9007199254740992.5", "18446744073709551615", "0.1", "-17.25"]
    path = tmp_path / "floats.mgf"
    with open(path, "w") as fh:
        for i in range(0, len(vals), 500):
            fh.write(f"BEGIN IONS\nTITLE=c;s{i}\nPEPMASS=500.0\nCHARGE=2+\n")
            for v in vals[i:i + 500]:
                fh.write(f"{1 + i % 7} {v}\n")
            fh.write("END IONS\n")
    d = mgf_native.parse_general(str(path))
    want = np.array([float(v) for v in vals])
    got = d["inten"]
    assert len(got) == len(want)
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert len(bad) == 0, [(vals[i], got[i], want[i]) for i in bad[:5]]


def _rand_num(rng, v, allow_exotic):
    forms = [lambda: f"{v:.5f}", lambda: repr(float(v)), lambda: f"{v:.2f}", lambda: str(int(v)),
             lambda: f"{v:.17g}", lambda: f"{v:.8f}".rstrip("0")]
    if allow_exotic:
        forms += [lambda: f"{v:.3e}", lambda: f"+{v:.4f}", lambda: f"{v:.4E}", lambda: f"{int(v)}."]
    return forms[int(rng.integers(0, len(forms)))]()


def _rand_mgf(rng, general):
    """Random MGF text in the shapes real files take: CRLF / CR / LF line ends,
    trailing blanks, extra peak fields, tab or double separators, exotic number
    forms, optional params, blank lines."""
    eol = ["\n", "\r\n", "\r"][int(rng.integers(0, 3))] if rng.random() < 0.3 else "\n"
    out = []
    for k in range(int(rng.integers(1, 6))):
        out.append("BEGIN IONS")
        out.append(f"TITLE=cluster-{k % 3};mzspec:X:{k}" + (" " if rng.random() < 0.1 else ""))
        if rng.random() < 0.9:
            out.append("PEPMASS=" + _rand_num(rng, rng.uniform(300, 1500), rng.random() < 0.3))
        if rng.random() < 0.9:
            out.append("CHARGE=" + ["2+", "3+", "2", " 2+ "][int(rng.integers(0, 4))])
        if rng.random() < 0.5:
            out.append("RTINSECONDS=" + _rand_num(rng, rng.uniform(0, 3600), False))
        for _ in range(int(rng.integers(0, 30))):
            a = _rand_num(rng, rng.uniform(100, 2000), rng.random() < 0.05)
            b = _rand_num(rng, rng.lognormal(3, 2), rng.random() < 0.05)
            r = rng.random()
            if general:
                sep = " " if r < 0.85 else ["\t", "  ", " \t"][int(rng.integers(0, 3))]
            else:
                sep = " " if r < 0.97 else ["\t", "  "][int(rng.integers(0, 2))]
            line = a + sep + b
            if rng.random() < 0.05:
                line += " 7"
            if rng.random() < 0.05:
                line += " "
            out.append(line)
            if rng.random() < 0.02:
                out.append("")
        out.append("END IONS")
        out.append("")
    return eol.join(out) + eol


@pytest.mark.parametrize("general", [False, True])
def test_random_mgf_text_native_equals_python(tmp_path, general):
    """Native parse == the Python reader on 300 random files per grammar: equal
    values (bit for bit) where the native subset applies, the Python reader's own
    result or exception otherwise (the CLIs' fallback)."""
    rng = np.random.default_rng(5 + general)
    n_native = 0
    for i in range(300):
        p = tmp_path / f"r{i}.mgf"
        p.write_bytes(_rand_mgf(rng, general).encode())
        if general:
            try:
                mgf_native.parse_general(str(p))
            except ValueError as e:
                assert "fallback" in str(e)
                continue
            _check_general_equal(str(p))
            n_native += 1
        else:
            try:
                want = mgf_native._read_binning_py(str(p))
            except Exception as e:  # noqa: BLE001 -- the reference's own exception
                with pytest.raises(type(e)):
                    mgf_native.read_binning_mgf(str(p))
                continue
            assert mgf_native.read_binning_mgf(str(p)) == want
            try:
                mgf_native.parse_native(str(p))
                n_native += 1
            except ValueError:
                pass
    assert n_native > 100  # most files take the native path
