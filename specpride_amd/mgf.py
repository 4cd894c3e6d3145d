"""MGF text I/O shared by the shims.

The three reference scripts each use a different MGF stack:

* ``binning.py`` has its own line parser (binning.py:122-167) and f-string
  writer (binning.py:234-245) -- reproduced byte-for-byte in
  :mod:`specpride_amd.binning` (native fast path in ``csrc/mgf_io.cpp``).
* ``average_spectrum_clustering.py`` uses pyteomics ``IndexedMGF``/``mgf.write``
  (absent offline): :func:`read_mgf` / :func:`write_pyteomics_style` below
  reproduce the semantics the reference relies on (title index order,
  ``params['pepmass'][0]``, ``params['charge']`` as a list, ``rtinseconds``
  float).  Exact pyteomics text formatting is **unpinned** (A.5).
* ``most_similar_representative.py`` uses OpenMS ``MascotGenericFile``: output
  formatting **unpinned**; parity is on the chosen spectrum and its title.

This module holds the format-neutral pieces: a tolerant reader returning
pyteomics-shaped dicts and writers using Python ``repr`` floats (shortest
round-trip), so that write -> read is lossless.
"""
from __future__ import annotations

import io
import os
from typing import Iterable, Iterator, TextIO

import numpy as np


def _open(path_or_fh, mode):
    if isinstance(path_or_fh, (str, os.PathLike)):
        return open(path_or_fh, mode), True
    return path_or_fh, False


def _parse_charge(v: str):
    out = []
    for tok in v.replace(" and ", ",").split(","):
        tok = tok.strip()
        if not tok:
            continue
        sign = -1 if tok.endswith("-") else 1
        out.append(sign * int(tok.strip("+-")))
    return out


def iter_mgf(path_or_fh) -> Iterator[dict]:
    """Yield spectra as pyteomics-shaped dicts::

        {'params': {'title': str, 'pepmass': (mz, intensity|None), 'charge': [z, ...],
                    'rtinseconds': float, ...},
         'm/z array': float64[], 'intensity array': float64[]}
    """
    fh, own = _open(path_or_fh, "rt")
    try:
        params, mzs, ints, inside = {}, [], [], False
        for raw in fh:
            line = raw.strip()
            if not line:
                continue
            if line == "BEGIN IONS":
                params, mzs, ints, inside = {}, [], [], True
            elif line == "END IONS":
                yield {"params": params, "m/z array": np.array(mzs, np.float64),
                       "intensity array": np.array(ints, np.float64)}
                inside = False
            elif not inside:
                continue
            elif line[0].isdigit() or (line[0] in "+-." and len(line) > 1 and line[1].isdigit()):
                parts = line.split()
                mzs.append(float(parts[0]))
                ints.append(float(parts[1]) if len(parts) > 1 else 0.0)
            elif "=" in line:
                k, v = line.split("=", 1)
                k = k.lower()
                if k == "pepmass":
                    p = v.split()
                    params[k] = (float(p[0]), float(p[1]) if len(p) > 1 else None)
                elif k == "charge":
                    params[k] = _parse_charge(v)
                elif k == "rtinseconds":
                    params[k] = float(v)
                else:
                    params[k] = v
    finally:
        if own:
            fh.close()


def read_mgf(path_or_fh) -> list:
    return list(iter_mgf(path_or_fh))


def format_charge(z) -> str:
    if isinstance(z, (list, tuple, np.ndarray)):
        return " and ".join(format_charge(v) for v in z)
    z = int(z)
    return f"{abs(z)}{'-' if z < 0 else '+'}"


def write_pyteomics_style(spectra: Iterable[dict], out, file_mode: str = "w") -> None:
    """Write ``{'params':…, 'm/z array':…, 'intensity array':…}`` dicts the way the
    gap-average CLI emits them (average_spectrum_clustering.py:203-208).  Key
    order: TITLE, PEPMASS, RTINSECONDS, CHARGE, then peaks as ``repr repr``."""
    fh, own = _open(out, file_mode) if out is not None else (None, False)
    if fh is None:
        import sys

        fh = sys.stdout
    try:
        for sp in spectra:
            p = sp.get("params", {})
            buf = io.StringIO()
            buf.write("BEGIN IONS\n")
            if p.get("title", "") != "":
                buf.write(f"TITLE={p['title']}\n")
            pm = p.get("pepmass", "")
            if pm != "" and pm is not None:
                pm = pm[0] if isinstance(pm, (tuple, list)) else pm
                buf.write(f"PEPMASS={float(pm)!r}\n")
            rt = p.get("rtinseconds", "")
            if rt != "" and rt is not None:
                buf.write(f"RTINSECONDS={float(rt)!r}\n")
            ch = p.get("charge", "")
            if ch != "" and ch is not None:
                buf.write(f"CHARGE={format_charge(ch)}\n")
            for mz, it in zip(sp["m/z array"], sp["intensity array"]):
                buf.write(f"{float(mz)!r} {float(it)!r}\n")
            buf.write("END IONS\n\n")
            fh.write(buf.getvalue())
    finally:
        if own:
            fh.close()


def write_csr_mgf(csr, out: TextIO | str, titles=None, sequences=None) -> None:
    """Write a clustered MGF (file_formats.md:5-57) from a :class:`SpectraCSR`.

    ``titles[s]`` defaults to ``cluster-<c>;mzspec:PXDSYN:synthetic:scan:<s>``.
    Floats are written with ``repr`` so reading back reproduces the arrays."""
    fh, own = _open(out, "w")
    try:
        for c in range(csr.n_clusters):
            cid = csr.cluster_ids[c] if csr.cluster_ids else f"cluster-{c}"
            for s in range(csr.cluster_off[c], csr.cluster_off[c + 1]):
                title = titles[s] if titles is not None else f"{cid};mzspec:PXDSYN:synthetic:scan:{s}"
                mz, it = csr.spectrum(s)
                buf = [f"BEGIN IONS\nTITLE={title}\nPEPMASS={float(csr.prec_mz[s])!r}\n"
                       f"CHARGE={int(csr.charge[s])}+\n"]
                if not np.isnan(csr.rt[s]):
                    buf.append(f"RTINSECONDS={float(csr.rt[s])!r}\n")
                if sequences is not None and sequences[s]:
                    buf.append(f"SEQUENCE={sequences[s]}\n")
                buf.extend(f"{float(a)!r} {float(b)!r}\n" for a, b in zip(mz, it))
                buf.append("END IONS\n\n")
                fh.write("".join(buf))
    finally:
        if own:
            fh.close()
