"""CPU tests of the host side: the C-ABI library loads and exports every entry
point include/specpride.h declares (no compute calls -- there is no GPU here),
the native MGF reader/writer against the reference's own line loop and f-string
writer, the reference's cluster-run scan, CSR packing and the CLI's no-argument
behaviour."""
import contextlib
import ctypes
import io
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO, load_json
from specpride_amd import _lib, mgf_native
from specpride_amd.csr import SpectraCSR
from specpride_amd.mgf import read_mgf, write_csr_mgf
from specpride_amd.synthetic import make_clusters_np

HEADER = os.path.join(REPO, "include", "specpride.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(spx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_exported_list():
    assert _declared() == sorted(_lib.EXPORTED)


def test_hip_library_exports_every_declared_symbol():
    path = _lib.build()  # cross-compiles for gfx950 when stale; no GPU needed
    L = ctypes.CDLL(path)
    missing = [s for s in _declared() if not hasattr(L, s)]
    assert not missing, missing
    L.spx_abi_version.restype = ctypes.c_int
    assert L.spx_abi_version() == _lib.SPX_ABI_VERSION == 2


MGF_HEADER = os.path.join(REPO, "include", "spx_mgf.h")


def test_mgf_library_exports_every_declared_symbol():
    text = re.sub(r"/\*.*?\*/", "", open(MGF_HEADER).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(spx_[a-z0-9_]+)\s*\(", text)))
    assert len(declared) == 24, declared
    L = ctypes.CDLL(_lib.build_mgf())
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    # and nothing exported that the header leaves out
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.build_mgf()], capture_output=True, text=True)
    if nm.returncode == 0:
        exported = sorted(set(re.findall(r"\b[TW] (spx_[a-z0-9_]+)$", nm.stdout, flags=re.M)))
        assert exported == declared


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "absent.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError):
        _lib.lib()


# ------------------------------------------------------------------ MGF I/O
def _mgf_lib():
    _lib.build_mgf()
    assert mgf_native._native() is not None


def test_native_mgf_reader_matches_reference_loop():
    _mgf_lib()
    path = os.path.join(GOLDEN, "bin_mean_cli_in.mgf")
    want = mgf_native._read_binning_py(path)
    got = mgf_native.read_binning_mgf(path)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w


def test_native_mgf_reader_on_synthetic_file(tmp_path):
    _mgf_lib()
    csr = make_clusters_np(30, seed=4)
    path = str(tmp_path / "s.mgf")
    write_csr_mgf(csr, path)
    flat = mgf_native.parse_native(path)
    np.testing.assert_array_equal(flat["spec_off"], csr.spec_off)
    np.testing.assert_array_equal(flat["mz"], csr.mz)
    np.testing.assert_array_equal(flat["inten"], csr.inten)
    np.testing.assert_array_equal(flat["prec_mz"], csr.prec_mz)
    np.testing.assert_array_equal(flat["charge"], csr.charge)
    assert mgf_native.read_binning_mgf(path) == mgf_native._read_binning_py(path)


def test_native_reader_defers_outside_its_subset(tmp_path):
    _mgf_lib()
    path = tmp_path / "odd.mgf"
    path.write_text("BEGIN IONS\nTITLE=a;b\nPEPMASS=1.5 200\nCHARGE=2+\n100.0 1.0\nEND IONS\n")
    with pytest.raises(ValueError):
        mgf_native._read_binning_py(str(path))  # the reference raises on "1.5 200"
    with pytest.raises(ValueError):
        mgf_native.read_binning_mgf(str(path))


def test_py_repr_formatter_matches_python():
    _mgf_lib()
    L = mgf_native._native()
    L.spx_py_repr.restype = ctypes.c_int
    L.spx_py_repr.argtypes = [ctypes.c_double, ctypes.c_char_p]
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.uniform(0, 2000, 3000), np.round(rng.uniform(0, 2000, 3000), 5),
                           rng.lognormal(0, 12, 3000), [0.0, -0.0, 1e16, 1e-5, 0.0001, 123456789012345678.0,
                                                        float("inf"), float("-inf"), 5e-324, 1.7976931348623157e308]],
                          ).astype(np.float64)
    buf = ctypes.create_string_buffer(64)
    for v in vals:
        n = L.spx_py_repr(float(v), buf)
        assert buf.raw[:n].decode() == repr(float(v)), v


def test_binning_writer_native_equals_fstring():
    _mgf_lib()
    rng = np.random.default_rng(1)
    spectra = [{"cluster_id": f"c{k}", "precursor_mz": float(rng.uniform(300, 900)), "precursor_charge": 2,
                "mzs": np.round(rng.uniform(100, 2000, 50), 4), "intensities": rng.uniform(0, 1e4, 50)}
               for k in range(5)]
    spectra[2]["intensities"][3] = np.nan
    a, b = io.StringIO(), io.StringIO()
    mgf_native.write_binning_mgf(spectra, a)
    saved = mgf_native._mgf
    try:
        mgf_native._mgf = None
        orig = mgf_native.MGF_LIB
        mgf_native.MGF_LIB = "/nonexistent"
        mgf_native.write_binning_mgf(spectra, b)
    finally:
        mgf_native.MGF_LIB = orig
        mgf_native._mgf = saved
    assert a.getvalue() == b.getvalue()


def test_read_mgf_roundtrip(tmp_path):
    csr = make_clusters_np(12, seed=9)
    path = str(tmp_path / "r.mgf")
    write_csr_mgf(csr, path)
    spectra = read_mgf(path)
    assert len(spectra) == csr.n_spectra
    for s, sp in enumerate(spectra):
        mz, it = csr.spectrum(s)
        np.testing.assert_array_equal(sp["m/z array"], mz)
        np.testing.assert_array_equal(sp["intensity array"], it)
        assert sp["params"]["pepmass"][0] == csr.prec_mz[s]
        assert list(sp["params"]["charge"]) == [csr.charge[s]]


# ----------------------------------------------------------- host logic
def test_first_runs_follows_reference_scan():
    from specpride_amd.most_similar_representative import _first_runs

    g = load_json("medoid_noncontiguous.json")
    runs = _first_runs(g["names"])
    assert [cl for cl, _ in runs] == ["A", "B", "C", "D"]
    assert [m for _, m in runs] == [[0, 1], [2], [4, 5], [7, 8, 9]]
    assert [m[0] for _, m in runs][:1] == g["rep_index"][:1]


def test_csr_from_clusters_and_select():
    csr = make_clusters_np(10, seed=3)
    sub = csr.select([2, 5])
    assert sub.n_clusters == 2
    for k, c in enumerate([2, 5]):
        a, b = csr.cluster_off[c], csr.cluster_off[c + 1]
        assert sub.cluster_off[k + 1] - sub.cluster_off[k] == b - a
        for j in range(b - a):
            np.testing.assert_array_equal(sub.spectrum(sub.cluster_off[k] + j)[0], csr.spectrum(a + j)[0])


def test_binning_cli_without_mgf_file_exits_10():
    from specpride_amd import binning

    g = load_json("bin_mean_cli.json")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), pytest.raises(SystemExit) as e:
        binning.main([])
    assert e.value.code == g["no_args_returncode"]
    assert buf.getvalue() == g["no_args_stdout"]


def test_native_decimal_parse_matches_python_float(tmp_path):
    """The native parser's Clinger fast path and its strtod fallback agree with
    Python's float() bit for bit: short and long significands, exponents, leading
    zeros, signs, subnormal/huge values, 19-20 digit boundaries."""
    import random

    import numpy as np

    from specpride_amd import mgf_native

    rng = random.Random(7)
    fixed = ["0", "0.0", "-0.0", "+1.5", "00012.500", "1e5", "1E-5", "2.5e+3", "123456789012345678",
             "1234567890123456789", "12345678901234567890", "9007199254740993", "9007199254740992.0",
             "0.000123", "1.7976931348623157e308", "5e-324", "2.2250738585072014e-308", "1e22", "1e23",
             "4.35679", "0.1", "0.3", "100.00001", "1999.99999", "3.141592653589793238462643383279"]
    nums = fixed + [f"{rng.uniform(0, 2000):.{rng.randint(0, 12)}f}" for _ in range(3000)]
    nums += [f"{rng.uniform(0, 1):.{rng.randint(13, 25)}f}" for _ in range(500)]
    nums += [f"{rng.uniform(1, 10):.6f}e{rng.randint(-30, 30)}" for _ in range(500)]
    path = tmp_path / "nums.mgf"
    with open(path, "w") as fh:
        for k in range(0, len(nums), 50):
            fh.write(f"BEGIN IONS\nTITLE=c{k % 7};usi{k}\nPEPMASS={nums[k]}\nCHARGE=2+\n")
            block = [n for n in nums[k:k + 50] if n[0].isdigit()]
            fh.write("".join(f"{a} {b}\n" for a, b in zip(block, block[1:] + block[:1])))
            fh.write("END IONS\n\n")
    flat = mgf_native.parse_native(str(path))
    ref = mgf_native._read_binning_py(str(path))
    mz = np.concatenate([np.asarray(s["m/z array"], np.float64) for s in ref])
    it = np.concatenate([np.asarray(s["intensity array"], np.float64) for s in ref])
    assert np.array_equal(flat["mz"].view(np.int64), mz.view(np.int64))
    assert np.array_equal(flat["inten"].view(np.int64), it.view(np.int64))
    prec = np.array([s["precursor mz"] for s in ref])
    assert np.array_equal(flat["prec_mz"].view(np.int64), prec.view(np.int64))


def test_gather_wire_format_model_rebuilds_bin_mean_bits():
    """The gather's wire format (csrc/wire.hip): every bin-mean consensus peak of the
    oracle -- mean = f64(f32 sum) / count, binning.py:198-218 -- is carried by f32
    sums and a count <= the cluster size, and rebuilt bit for bit (incl. the NaN m/z of
    a zero m/z sum, :216); the GPU kernels are checked against the same property in
    tests/test_gpu_parity.py."""
    import wire_model
    from oracle import c_oracle

    csr = make_clusters_np(400, seed=19)
    r = c_oracle.bin_mean(csr)
    mz, it = r["out_mz"], r["out_int"]
    cmax = int(csr.cluster_sizes().max())
    M, I, C = wire_model.pack(mz, it, cmax)
    assert np.all(C > 0) and C.max() <= cmax
    mz2, it2 = wire_model.unpack(M, I, C)
    np.testing.assert_array_equal(mz2.view(np.int64)[~np.isnan(mz)], mz.view(np.int64)[~np.isnan(mz)])
    np.testing.assert_array_equal(it2.view(np.int64), it.view(np.int64))
    # a value that is no f64 quotient of an f32 sum by a small count is not carried
    M, I, C = wire_model.pack(np.array([np.pi]), np.array([np.e]), 50)
    assert C[0] == 0
