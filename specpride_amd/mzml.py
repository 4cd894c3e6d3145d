"""Minimal mzML reader for the reference's mzML input path.

The reference reads mzML through pyteomics (``binning.py:57-119``:
``mzml.read(infile)`` then ``reader.get_by_id("controllerType=0
controllerNumber=1 scan=<n>")``).  pyteomics is not installed offline, so this
module parses the subset of mzML 1.1 that code path touches and returns the
same dict shape pyteomics does for it:

* ``spectrum['ms level']`` (cvParam MS:1000511, int)
* ``spectrum['m/z array']`` / ``['intensity array']`` (binaryDataArray with
  MS:1000514 / MS:1000515; 64-bit MS:1000523 or 32-bit MS:1000521 floats,
  zlib MS:1000574 or no compression MS:1000576, base64) as numpy arrays
* ``spectrum['precursorList']['precursor'][i]['selectedIonList']['selectedIon'][j]``
  with ``'selected ion m/z'`` (MS:1000744) and ``'charge state'`` (MS:1000041)

cvParam values convert like pyteomics' (int, else float, else the string).
32-bit arrays are returned as float32 (pyteomics keeps the encoded dtype); the
engine widens them to float64.  Exact pyteomics object types (unitfloat etc.) are
not reproduced: parity for this reader is unpinned (no pyteomics here) and is
checked by round trips through :func:`write_mzml` in the tests.
Host I/O only -- not the compute path.
"""
from __future__ import annotations

import base64
import gzip
import re
import zlib
import xml.etree.ElementTree as ET

import numpy as np

_MS_LEVEL = "MS:1000511"
_MZ_ARRAY, _INT_ARRAY = "MS:1000514", "MS:1000515"
_F64, _F32 = "MS:1000523", "MS:1000521"
_ZLIB, _NOCOMP = "MS:1000574", "MS:1000576"


def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _convert(v: str):
    for f in (int, float):
        try:
            return f(v)
        except ValueError:
            pass
    return v


def _cv(elem) -> dict:
    """cvParams / userParams of elem as {name: value} (valueless -> name: '')."""
    out = {}
    for ch in elem:
        t = _local(ch.tag)
        if t in ("cvParam", "userParam"):
            out[ch.get("name")] = _convert(ch.get("value")) if ch.get("value") not in (None, "") else ""
    return out


def _accessions(elem) -> set:
    return {ch.get("accession") for ch in elem if _local(ch.tag) == "cvParam"}


def _binary_array(bda):
    """(name, accessions, raw base64 text) of a binaryDataArray: decoded later."""
    acc = _accessions(bda)
    raw = ""
    for ch in bda:
        if _local(ch.tag) == "binary":
            raw = ch.text or ""
    name = "m/z array" if _MZ_ARRAY in acc else ("intensity array" if _INT_ARRAY in acc else None)
    return name, acc, raw.strip()


def _decode(acc, raw: str):
    dtype = np.float32 if _F32 in acc else np.float64
    data = base64.b64decode(raw) if raw else b""
    if _ZLIB in acc and data:
        data = zlib.decompress(data)
    return np.frombuffer(data, dtype=dtype).copy()


def _spectrum(elem) -> dict:
    """The spectrum's metadata; its binary arrays stay encoded under '_raw' until
    :meth:`MzML.get_by_id` decodes them."""
    sp = {"id": elem.get("id"), "index": int(elem.get("index", -1))}
    sp.update(_cv(elem))
    raw = {}
    for ch in elem:
        t = _local(ch.tag)
        if t == "precursorList":
            precs = []
            for p in ch:
                if _local(p.tag) != "precursor":
                    continue
                pd = {}
                for q in p:
                    if _local(q.tag) == "selectedIonList":
                        pd["selectedIonList"] = {"count": int(q.get("count", 0)),
                                                 "selectedIon": [_cv(si) for si in q if _local(si.tag) == "selectedIon"]}
                    elif _local(q.tag) == "isolationWindow":
                        pd["isolationWindow"] = _cv(q)
                precs.append(pd)
            sp["precursorList"] = {"count": int(ch.get("count", len(precs))), "precursor": precs}
        elif t == "binaryDataArrayList":
            for bda in ch:
                if _local(bda.tag) == "binaryDataArray":
                    name, acc, text = _binary_array(bda)
                    if name:
                        raw[name] = (acc, text)
    sp["_raw"] = raw
    return sp


class MzML:
    """``with MzML(fh) as reader: reader.get_by_id(id)`` over an mzML byte stream
    (path, file object, or ``.gz`` path).  One streaming pass indexes the spectra
    by id; binary arrays are base64/zlib-decoded only when a spectrum is fetched
    (pyteomics' get_by_id is lazy too).  ``ids`` (optional): keep only these
    spectra -- the caller's MaRaCluster scan list -- so a multi-GB run with MS1
    scans costs memory for the wanted spectra alone."""

    def __init__(self, source, ids=None):
        own = False
        if isinstance(source, str):
            source = gzip.open(source) if re.search(r"\.gz$", source) else open(source, "rb")
            own = True
        keep = None if ids is None else set(ids)
        self._spectra = {}
        self._order = []
        try:
            for _, elem in ET.iterparse(source, events=("end",)):
                if _local(elem.tag) == "spectrum":
                    if keep is None or elem.get("id") in keep:
                        sp = _spectrum(elem)
                        self._spectra[sp["id"]] = sp
                        self._order.append(sp["id"])
                    elem.clear()
        finally:
            if own:
                source.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        return (self.get_by_id(i) for i in self._order)

    def __len__(self):
        return len(self._order)

    def get_by_id(self, spectrum_id: str) -> dict:
        """KeyError for an unknown id (pyteomics raises KeyError too)."""
        sp = self._spectra[spectrum_id]
        raw = sp.pop("_raw", None)
        if raw:
            for name, (acc, text) in raw.items():
                sp[name] = _decode(acc, text)
        return sp


def read(source, ids=None) -> MzML:
    """``pyteomics.mzml.read`` stand-in (the reference uses it as a context manager)."""
    return MzML(source, ids=ids)


# ---------------------------------------------------------------- writer (tests, synthetic inputs)
def _encode(arr, bits: int, compress: bool) -> str:
    data = np.ascontiguousarray(arr, np.float64 if bits == 64 else np.float32).tobytes()
    if compress:
        data = zlib.compress(data)
    return base64.b64encode(data).decode("ascii")


def write_mzml(path: str, spectra, bits: int = 64, compress: bool = True) -> None:
    """Write spectra ``{'scan', 'ms level', 'm/z array', 'intensity array',
    'precursor mz', 'precursor charge'}`` as an indexed-free mzML 1.1 run with
    Thermo-style ids (``controllerType=0 controllerNumber=1 scan=<n>``)."""
    fmt = _F64 if bits == 64 else _F32
    fmt_name = "64-bit float" if bits == 64 else "32-bit float"
    comp = (_ZLIB, "zlib compression") if compress else (_NOCOMP, "no compression")
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wt") as fh:
        fh.write('<?xml version="1.0" encoding="utf-8"?>\n<mzML xmlns="http://psi.hupo.org/ms/mzml" version="1.1.0">\n')
        fh.write(f'<run id="synthetic"><spectrumList count="{len(spectra)}">\n')
        for i, sp in enumerate(spectra):
            mz, it = np.asarray(sp["m/z array"]), np.asarray(sp["intensity array"])
            fh.write(f'<spectrum index="{i}" id="controllerType=0 controllerNumber=1 scan={sp["scan"]}" '
                     f'defaultArrayLength="{len(mz)}">\n')
            fh.write(f'<cvParam cvRef="MS" accession="{_MS_LEVEL}" name="ms level" value="{sp.get("ms level", 2)}"/>\n')
            if sp.get("ms level", 2) == 2:
                fh.write('<precursorList count="1"><precursor><selectedIonList count="1"><selectedIon>'
                         f'<cvParam cvRef="MS" accession="MS:1000744" name="selected ion m/z" '
                         f'value="{float(sp["precursor mz"])!r}"/>'
                         f'<cvParam cvRef="MS" accession="MS:1000041" name="charge state" '
                         f'value="{int(sp["precursor charge"])}"/>'
                         '</selectedIon></selectedIonList></precursor></precursorList>\n')
            fh.write('<binaryDataArrayList count="2">\n')
            for acc, name, arr in ((_MZ_ARRAY, "m/z array", mz), (_INT_ARRAY, "intensity array", it)):
                enc = _encode(arr, bits, compress)
                fh.write(f'<binaryDataArray encodedLength="{len(enc)}">'
                         f'<cvParam cvRef="MS" accession="{fmt}" name="{fmt_name}"/>'
                         f'<cvParam cvRef="MS" accession="{comp[0]}" name="{comp[1]}"/>'
                         f'<cvParam cvRef="MS" accession="{acc}" name="{name}"/>'
                         f'<binary>{enc}</binary></binaryDataArray>\n')
            fh.write('</binaryDataArrayList>\n</spectrum>\n')
        fh.write('</spectrumList></run>\n</mzML>\n')
