"""MGF ingest/emit for the three CLIs.

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
        L.spx_mgf_titles.restype = ctypes.c_void_p  # raw pointer: sliced with the title offsets
        L.spx_mgf_titles.argtypes = [ctypes.c_void_p]
        L.spx_mgf_title_offsets.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.spx_mgf_group.restype = ctypes.c_int64
        L.spx_mgf_group.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.spx_mgf_group_ids.restype = ctypes.c_char_p
        L.spx_mgf_group_ids.argtypes = [ctypes.c_void_p]
        L.spx_mgf_free.argtypes = [ctypes.c_void_p]
        L.spx_mgf_format_binning.restype = ctypes.c_int64
        L.spx_mgf_format_binning.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p,
                                             ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int]
        L.spx_mgf_parse_general.restype = ctypes.c_void_p
        L.spx_mgf_parse_general.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.spx_mgf_copy_rt.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.spx_mgf_index.restype = ctypes.c_void_p
        L.spx_mgf_index.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.spx_mgf_index_error.restype = ctypes.c_char_p
        L.spx_mgf_index_error.argtypes = [ctypes.c_void_p]
        L.spx_mgf_index_n.restype = ctypes.c_int64
        L.spx_mgf_index_n.argtypes = [ctypes.c_void_p]
        L.spx_mgf_index_copy.argtypes = [ctypes.c_void_p] * 4
        L.spx_mgf_index_titles.restype = ctypes.c_char_p
        L.spx_mgf_index_titles.argtypes = [ctypes.c_void_p]
        L.spx_mgf_index_free.argtypes = [ctypes.c_void_p]
        L.spx_mgf_index_range.restype = ctypes.c_void_p
        L.spx_mgf_index_range.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
        L.spx_mgf_write_records.restype = ctypes.c_int
        L.spx_mgf_write_records.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                            ctypes.c_char_p] + [ctypes.c_void_p] * 7 + [ctypes.c_int]
        L.spx_mgf_parse_ranges.restype = ctypes.c_void_p
        L.spx_mgf_parse_ranges.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_int, ctypes.c_int]
        _mgf = L
    return _mgf


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _split_titles(raw, n):
    return raw.decode("utf-8", errors="surrogateescape").split("\n")[:n] if n else []


GROUP_BINNING, GROUP_RUNS, GROUP_FIRST_RUNS = 0, 1, 2  # spx_mgf_group modes


class Flat(dict):
    """A native parse: dict(spec_off, mz, inten, prec_mz, charge, has_prec,
    has_charge[, rt, has_rt, has_title]); ``flat["titles"]`` (every title, a
    list) is decoded on first use from the raw '\n'-joined bytes, and
    :meth:`title` decodes one -- a CLI that groups natively never builds the list."""

    def __missing__(self, key):
        if key != "titles":
            raise KeyError(key)
        raw, S = self["_titles_raw"], len(self["spec_off"]) - 1
        v = raw.decode("utf-8", errors="surrogateescape").split("\n")[:S] if S else []
        self["titles"] = v
        return v

    def title(self, s: int) -> str:
        if "titles" in self:
            return self["titles"][s]
        o = self["_title_off"]
        return self["_titles_raw"][o[s]:o[s + 1] - 1].decode("utf-8", errors="surrogateescape")


def _take_result(L, h, general, group=None):
    """Copy a parse handle's arrays out and free it (ValueError on an error/fallback).
    ``group`` (a GROUP_* mode): also ``key`` [S] and ``group_ids`` (spx_mgf_group)."""
    try:
        err = L.spx_mgf_error(h)
        if err:
            raise ValueError(err.decode(errors="replace"))
        S, P = L.spx_mgf_n_spectra(h), L.spx_mgf_n_peaks(h)
        spec_off = np.zeros(S + 1, np.int64)
        mz, inten = np.empty(P), np.empty(P)
        prec, rt = np.empty(S), np.empty(S)
        charge = np.empty(S, np.int64)
        flags = np.empty(S, np.int32)
        L.spx_mgf_copy(h, _ptr(spec_off), _ptr(mz), _ptr(inten), _ptr(prec), _ptr(charge), _ptr(flags))
        L.spx_mgf_copy_rt(h, _ptr(rt))
        toff = np.zeros(S + 1, np.int64)
        L.spx_mgf_title_offsets(h, _ptr(toff))
        raw = ctypes.string_at(L.spx_mgf_titles(h), int(toff[-1])) if S else b""
        extra = {}
        if group is not None:
            key = np.empty(S, np.int64)
            n = L.spx_mgf_group(h, int(group), _ptr(key))
            ids = L.spx_mgf_group_ids(h).decode("utf-8", errors="surrogateescape").split("\n")[:n] if n else []
            extra = dict(key=key, group_ids=ids)
    finally:
        L.spx_mgf_free(h)
    d = Flat(spec_off=spec_off, mz=mz, inten=inten, prec_mz=prec, charge=charge,
             has_prec=(flags & 1) != 0, has_charge=(flags & 2) != 0, _titles_raw=raw, _title_off=toff, **extra)
    if general:
        d.update(rt=rt, has_rt=(flags & 4) != 0, has_title=(flags & 8) != 0)
    return d


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


def parse_native(path, threads: int = 0, group=None):
    """Native parse into flat arrays; returns None when the library is absent.
    Result: dict(spec_off, mz, inten, prec_mz, charge, has_prec, has_charge, titles)
    (+ key, group_ids with ``group``).  Raises ValueError where the reference would
    raise on a line."""
    L = _native()
    if L is None:
        return None
    return _take_result(L, L.spx_mgf_parse(os.fsencode(path), int(threads)), False, group)


def parse_general(path, threads: int = 0, group=None):
    """Native parse of a general (pyteomics-shaped) MGF -- the subset of
    :func:`specpride_amd.mgf.iter_mgf` whose meaning is unambiguous -- into flat
    arrays: dict(spec_off, mz, inten, prec_mz (NaN if absent), charge (0 if
    absent), rt (NaN if absent), has_prec, has_charge, has_rt, has_title, titles).
    None when the library is absent; ValueError("fallback: ...") outside the subset
    (the caller then reads with iter_mgf, which behaves or raises as before)."""
    L = _native()
    if L is None:
        return None
    return _take_result(L, L.spx_mgf_parse_general(os.fsencode(path), int(threads)), True, group)


def _take_index(L, h):
    try:
        err = L.spx_mgf_index_error(h)
        if err:
            raise ValueError(err.decode(errors="replace"))
        n = L.spx_mgf_index_n(h)
        begin, end, npk = (np.empty(n, np.int64) for _ in range(3))
        L.spx_mgf_index_copy(h, _ptr(begin), _ptr(end), _ptr(npk))
        titles = _split_titles(L.spx_mgf_index_titles(h), n)
    finally:
        L.spx_mgf_index_free(h)
    return dict(begin=begin, end=end, npk=npk, titles=titles)


def index(path, general: bool):
    """Record index of an MGF without parsing any number: dict(begin, end, npk,
    titles) -- record r is bytes [begin[r], end[r]) (from its TITLE= line for the
    binning reader, from BEGIN IONS for the general one, to the next record's
    start), npk its peak-line count.  Only records with an END IONS are listed.
    None when the library is absent."""
    L = _native()
    if L is None:
        return None
    return _take_index(L, L.spx_mgf_index(os.fsencode(path), int(bool(general))))


def index_range(path, general: bool, lo: int, hi: int, threads: int = 0):
    """The records of :func:`index` whose start line lies in bytes [lo, hi): the
    stripes [k*size/W, (k+1)*size/W) of W ranks list every record exactly once,
    and each reads only its stripe (plus the tail of its last record)."""
    L = _native()
    if L is None:
        raise RuntimeError(f"native MGF library missing ({MGF_LIB}); run __graft_entry__.build()")
    return _take_index(L, L.spx_mgf_index_range(os.fsencode(path), int(bool(general)), int(lo), int(hi),
                                                 int(threads)))


def parse_ranges(path, begin, end, general: bool, threads: int = 0):
    """Parse only the records [begin[r], end[r]) of :func:`index` (result in the
    given order) with the binning (general=False) or the general parser; the
    same flat dict as :func:`parse_native` / :func:`parse_general`."""
    L = _native()
    if L is None:
        raise RuntimeError(f"native MGF library missing ({MGF_LIB}); run __graft_entry__.build()")
    begin = np.ascontiguousarray(begin, np.int64)
    end = np.ascontiguousarray(end, np.int64)
    h = L.spx_mgf_parse_ranges(os.fsencode(path), _ptr(begin), _ptr(end), len(begin), int(bool(general)),
                               int(threads))
    return _take_result(L, h, general)


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


STYLE_BINNING, STYLE_GAP_AVERAGE, STYLE_MEDOID = 0, 1, 2
FLAG_PEPMASS, FLAG_CHARGE, FLAG_RT, FLAG_TITLE = 1, 2, 4, 8


def write_records(path, style: int, titles, off, mz, inten, prec, charge, rt=None, flags=None,
                  append: bool = False, threads: int = 0) -> None:
    """Write len(titles) MGF records with the native multithreaded writer
    (``spx_mgf_write_records``): style 0 = binning.py:234-245 text, 1 = the
    gap-average CLI's (:func:`specpride_amd.mgf.write_pyteomics_style`), 2 = the
    medoid CLI's (:func:`specpride_amd.most_similar_representative.write_record`);
    record c's peaks are ``mz/inten[off[c]:off[c+1]]``; ``flags`` (styles 1-2) say
    which of PEPMASS / CHARGE / RTINSECONDS / TITLE are present.  Byte-identical
    to the Python writers (tests/test_mgf_native.py)."""
    L = _native()
    if L is None:
        raise RuntimeError(f"native MGF library missing ({MGF_LIB}); run __graft_entry__.build()")
    C = len(titles)
    if any("\n" in t for t in titles):
        raise ValueError("record titles cannot contain a newline")
    off = np.ascontiguousarray(off, np.int64)
    if len(off) != C + 1:
        raise ValueError("off must have len(titles) + 1 entries")
    mz = np.ascontiguousarray(mz, np.float64)
    inten = np.ascontiguousarray(inten, np.float64)
    if C and (off[0] < 0 or off[-1] > len(mz) or len(inten) < off[-1] or np.any(np.diff(off) < 0)):
        raise ValueError("peak offsets out of range")
    prec = np.ascontiguousarray(prec, np.float64)
    charge = np.ascontiguousarray(charge, np.int64)
    rt = np.ascontiguousarray(rt if rt is not None else np.full(C, np.nan), np.float64)
    flags = np.ascontiguousarray(flags if flags is not None else np.full(C, 15), np.int32)
    for a in (prec, charge, rt, flags):
        if len(a) != C:
            raise ValueError("per-record arrays must have len(titles) entries")
    joined = "\n".join(titles).encode("utf-8", errors="surrogateescape")
    rc = L.spx_mgf_write_records(os.fsencode(path), int(bool(append)), int(style), C, joined, _ptr(flags),
                                 _ptr(prec), _ptr(charge), _ptr(rt), _ptr(off), _ptr(mz), _ptr(inten), int(threads))
    if rc != 0:
        raise OSError(f"spx_mgf_write_records failed writing {path}")
