"""MGF ingest/emit for the bin-mean CLI path.

``read_binning_mgf`` reproduces the reference's line parser
(src/binning.py:122-167) and ``write_binning_mgf`` its f-string writer
(src/binning.py:234-245) byte for byte.  When the native library
``specpride_amd/lib/libspx_mgf.so`` (csrc/mgf_io.cpp, multithreaded C++) is
built, large files are parsed there -- same values (strtod is correctly
rounded, like Python's float()) and same dict structure -- otherwise the
pure-Python line loop below is used.  These are host I/O helpers, not the
compute path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MGF_LIB = os.path.join(HERE, "lib", "libspx_mgf.so")
_mgf = None


def _native():
    global _mgf
    if _mgf is None and os.path.exists(MGF_LIB):
        L = ctypes.CDLL(MGF_LIB)
        L.spx_mgf_parse.restype = ctypes.c_void_p
        L.spx_mgf_parse.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.spx_mgf_error.restype = ctypes.c_char_p
        L.spx_mgf_error.argtypes = [ctypes.c_void_p]
        for f in ("spx_mgf_n_spectra", "spx_mgf_n_peaks"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.spx_mgf_copy.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        L.spx_mgf_titles.restype = ctypes.c_char_p
        L.spx_mgf_titles.argtypes = [ctypes.c_void_p]
        L.spx_mgf_free.argtypes = [ctypes.c_void_p]
        L.spx_mgf_format_binning.restype = ctypes.c_int64
        L.spx_mgf_format_binning.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p,
                                             ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int]
        _mgf = L
    return _mgf


# ------------------------------------------------------------------ reading
def _read_binning_py(clustered_mgf_file):
    all_spectra = []
    with open(clustered_mgf_file, "rt") as mgf:
        for line in mgf:
            if line[:6] == "TITLE=":
                title = line[6:].strip()
                parts = title.split(";")
                peaklist = {"m/z array": [], "intensity array": [], "cluster_id": parts[0],
                            "spectrum_usi": parts[1]}
            if line[:8] == "PEPMASS=":
                peaklist["precursor mz"] = float(line[8:].strip())
            if line[:7] == "CHARGE=":
                peaklist["precursor charge"] = int(line[7:].strip().strip("+"))
            if line[0].isdigit():
                peak = line.strip().split(" ")
                peaklist["m/z array"].append(float(peak[0]))
                peaklist["intensity array"].append(float(peak[1]))
            if line.strip() == "END IONS":
                all_spectra.append(peaklist)
    return all_spectra


def parse_native(path, threads: int = 0):
    """Native parse into flat arrays; returns None when the library is absent.
    Result: dict(spec_off, mz, inten, prec_mz, charge, has_prec, has_charge, titles).
    Raises ValueError where the reference would raise on a line."""
    L = _native()
    if L is None:
        return None
    h = L.spx_mgf_parse(os.fsencode(path), int(threads))
    try:
        err = L.spx_mgf_error(h)
        if err:
            raise ValueError(err.decode(errors="replace"))
        S, P = L.spx_mgf_n_spectra(h), L.spx_mgf_n_peaks(h)
        spec_off = np.zeros(S + 1, np.int64)
        mz, inten = np.empty(P), np.empty(P)
        prec = np.empty(S)
        charge = np.empty(S, np.int64)
        flags = np.empty(S, np.int32)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        L.spx_mgf_copy(h, p(spec_off), p(mz), p(inten), p(prec), p(charge), p(flags))
        titles = L.spx_mgf_titles(h).decode("utf-8", errors="surrogateescape").split("\n")[:S] if S else []
    finally:
        L.spx_mgf_free(h)
    return dict(spec_off=spec_off, mz=mz, inten=inten, prec_mz=prec, charge=charge,
                has_prec=(flags & 1) != 0, has_charge=(flags & 2) != 0, titles=titles)


def read_binning_mgf(path):
    """Spectra of a clustered MGF as binning.py's peaklist dicts (file order)."""
    try:
        flat = parse_native(path)
    except ValueError:  # outside the native subset: the reference's own line loop decides
        flat = None
    if flat is None:
        return _read_binning_py(path)
    out = []
    so, mz, it = flat["spec_off"], flat["mz"], flat["inten"]
    for s, title in enumerate(flat["titles"]):
        parts = title.split(";")
        pl = {"m/z array": mz[so[s]:so[s + 1]].tolist(), "intensity array": it[so[s]:so[s + 1]].tolist(),
              "cluster_id": parts[0], "spectrum_usi": parts[1]}
        if flat["has_prec"][s]:
            pl["precursor mz"] = float(flat["prec_mz"][s])
        if flat["has_charge"][s]:
            pl["precursor charge"] = int(flat["charge"][s])
        out.append(pl)
    return out


# ------------------------------------------------------------------ writing
def write_binning_mgf(spectra, mgf_file):
    """binning.py:234-245 text, byte for byte."""
    L = _native()
    for spectrum in spectra:
        mzs, ints = spectrum["mzs"], spectrum["intensities"]
        if L is not None and isinstance(mzs, np.ndarray) and mzs.dtype == np.float64 and \
                isinstance(ints, np.ndarray) and ints.dtype == np.float64 and \
                type(spectrum["precursor_mz"]) in (float, np.float64) and \
                type(spectrum["precursor_charge"]) in (int, np.int32, np.int64):
            mzs, ints = np.ascontiguousarray(mzs), np.ascontiguousarray(ints)
            cap = 128 + len(str(spectrum["cluster_id"])) * 4 + 64 * len(mzs)
            buf = ctypes.create_string_buffer(cap)
            n = L.spx_mgf_format_binning(buf, cap, str(spectrum["cluster_id"]).encode(),
                                         str(spectrum["precursor_charge"]).encode(),
                                         float(spectrum["precursor_mz"]), mzs.ctypes.data_as(ctypes.c_void_p),
                                         ints.ctypes.data_as(ctypes.c_void_p), len(mzs), 1)
            if n >= 0:
                mgf_file.write(buf.raw[:n].decode())
                continue
        text = f"""BEGIN IONS
TITLE={spectrum["cluster_id"]}
PEPMASS={spectrum['precursor_mz']}
CHARGE={spectrum['precursor_charge']}+
"""
        text += "".join(f"{mz} {intensity}\n" for mz, intensity in zip(mzs, ints) if not np.isnan(intensity))
        text += "END IONS\n\n"
        mgf_file.write(text)
