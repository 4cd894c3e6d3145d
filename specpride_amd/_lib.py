"""ctypes binding of libspecpride_hip.so (the C-ABI in include/specpride.h).

The library is built in-tree (``specpride_amd/lib/libspecpride_hip.so``) by
:func:`build` / ``__graft_entry__.build()``.  There is no fallback: if the
library is missing or fails to load, :func:`lib` raises -- the product path
never silently degrades to a CPU implementation.

torch is imported before the library is loaded so that both share the one HIP
runtime (libamdhip64.so.7) that torch already mapped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.environ.get("SPX_LIB") or os.path.join(LIB_DIR, "libspecpride_hip.so")
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SPX_OFFLOAD_ARCH", "gfx950")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
             f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_dbl = ctypes.c_double
_sz = ctypes.c_size_t


class SpxCsr(ctypes.Structure):
    _fields_ = [("n_clusters", _i64), ("n_spectra", _i64), ("n_peaks", _i64),
                ("cluster_off", _p), ("spec_off", _p), ("mz", _p), ("inten", _p),
                ("prec_mz", _p), ("charge", _p), ("rt", _p)]


class SpxBatchInfo(ctypes.Structure):
    _fields_ = [("max_cluster_peaks", _i64), ("max_cluster_spectra", _i64), ("max_mz_span", _dbl)]


class SpxPeaksOut(ctypes.Structure):
    _fields_ = [("mz", _p), ("inten", _p), ("count", _p)]


class SpxBinParams(ctypes.Structure):
    _fields_ = [("minimum", _dbl), ("maximum", _dbl), ("binsize", _dbl), ("apply_peak_quorum", _i32)]


class SpxGapParams(ctypes.Structure):
    _fields_ = [("mz_accuracy", _dbl), ("dyn_range", _dbl), ("min_fraction", _dbl), ("proton", _dbl),
                ("pepmass_mode", _i32), ("rt_mode", _i32)]


class SpxMedoidParams(ctypes.Structure):
    _fields_ = [("tolerance", _dbl), ("large_path", _i32)]


class SpxCosineParams(ctypes.Structure):
    _fields_ = [("mz_space", _dbl)]


# every symbol include/specpride.h declares (checked by tests/test_host.py)
EXPORTED = ["spx_bin_mean_workspace_size", "spx_bin_mean", "spx_bin_mean_stage", "spx_gap_average_workspace_size", "spx_gap_average",
            "spx_medoid_workspace_size", "spx_medoid_needs_large_path", "spx_medoid", "spx_bin_mean_medoid", "spx_bin_mean_medoid_stage", "spx_xcorr_distance", "spx_binned_cosine_workspace_size", "spx_binned_cosine", "spx_best_score",
            "spx_compact_peaks", "spx_wire_pack", "spx_wire_unpack", "spx_copy_h2d", "spx_copy_d2h",
            "spx_abi_version", "spx_last_error", "spx_profile_enable", "spx_profile_read",
            "spx_medoid_gram_operand_bits"]

SPX_ABI_VERSION = 2
_lib = None


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp")))


def build_all(force: bool = False):
    return build(force), build_mgf(force)


def build(force: bool = False) -> str:
    """Compile the HIP engine for gfx950 into specpride_amd/lib (cross-compiles without a GPU)."""
    os.makedirs(LIB_DIR, exist_ok=True)
    newest = max(os.path.getmtime(f) for f in sources() + [os.path.join(REPO, "include", "specpride.h")])
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= newest:
        return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, *HIP_FLAGS, "-o", tmp, os.path.join(CSRC, "spx_api.hip")]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


MGF_LIB_PATH = os.path.join(LIB_DIR, "libspx_mgf.so")


def build_mgf(force: bool = False) -> str:
    """Host C++ MGF reader/writer (csrc/mgf_io.cpp) -> specpride_amd/lib/libspx_mgf.so."""
    os.makedirs(LIB_DIR, exist_ok=True)
    src = os.path.join(CSRC, "mgf_io.cpp")
    newest = max(os.path.getmtime(src), os.path.getmtime(os.path.join(REPO, "include", "spx_mgf.h")))
    if not force and os.path.exists(MGF_LIB_PATH) and os.path.getmtime(MGF_LIB_PATH) >= newest:
        return MGF_LIB_PATH
    tmp = MGF_LIB_PATH + ".tmp"
    subprocess.run([os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread",
                    "-Wall", "-o", tmp, src], check=True)
    os.replace(tmp, MGF_LIB_PATH)
    return MGF_LIB_PATH


def lib():
    """Load (once) and return the engine library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- share torch's HIP runtime (see module docstring)

    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"specpride HIP engine not built: {LIB_PATH} is missing "
                           "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = ctypes.CDLL(LIB_PATH)
    L.spx_abi_version.restype = ctypes.c_int
    L.spx_last_error.restype = ctypes.c_char_p
    L.spx_bin_mean_workspace_size.restype = _sz
    L.spx_bin_mean_workspace_size.argtypes = [_p, _p, _p]
    L.spx_bin_mean.argtypes = [_p, _p, _p, _p, _p, _p, _p, _p, _sz, _p]
    L.spx_bin_mean_stage.argtypes = [_p, _p, _p, _p, _p, _p, _p, _p, _sz, _p, _i32]
    L.spx_gap_average_workspace_size.restype = _sz
    L.spx_gap_average_workspace_size.argtypes = [_p, _p, _p]
    L.spx_gap_average.argtypes = [_p, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _p]
    L.spx_medoid_workspace_size.restype = _sz
    L.spx_medoid_workspace_size.argtypes = [_p, _p, _i64, _p, _i64]
    L.spx_medoid_needs_large_path.restype = ctypes.c_int
    L.spx_medoid_needs_large_path.argtypes = [_p, _p, _i64]
    L.spx_medoid.argtypes = [_p, _p, _p, _p, _p, _sz, _p]
    L.spx_compact_peaks.argtypes = [_p, _p, _p, _p, _p, _p]
    L.spx_wire_pack.argtypes = [_p, _p, _i64, _i32, _p, _p, _i32, _p, _p]
    L.spx_wire_unpack.argtypes = [_p, _p, _i32, _i64, _p, _p, _p]
    L.spx_xcorr_distance.argtypes = [_p, _p, _p, _i64, _p, _p]
    L.spx_binned_cosine_workspace_size.restype = _sz
    L.spx_binned_cosine_workspace_size.argtypes = [_i64, _i64]
    L.spx_binned_cosine.argtypes = [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _p, _sz, _p]
    L.spx_best_score.argtypes = [_p, _p, _p, _p, _p, _p]
    L.spx_copy_h2d.argtypes = [_p, _p, _sz, _p]
    L.spx_copy_d2h.argtypes = [_p, _p, _sz, _p]
    # symbols added in ABI 2's round 4 (bound when present: A/B runs load older builds)
    for name, argtypes in (("spx_bin_mean_medoid", [_p, _p, _p, _p, _p, _p, _p, _p, _sz, _p, _p, _p, _p, _sz, _p]),
                           ("spx_bin_mean_medoid_stage",
                            [_p, _p, _p, _p, _p, _p, _p, _p, _sz, _p, _p, _p, _p, _sz, _p, _i32, _p]),
                           ("spx_profile_enable", [_i32]), ("spx_profile_read", [ctypes.c_char_p, _p, _p]),
                           ("spx_medoid_gram_operand_bits", [])):
        if hasattr(L, name):
            getattr(L, name).argtypes = argtypes
    if L.spx_abi_version() != SPX_ABI_VERSION:
        raise RuntimeError(f"libspecpride_hip ABI {L.spx_abi_version()} != {SPX_ABI_VERSION}")
    _lib = L
    return L


def profile_enable(on: bool = True) -> None:
    """Per-kernel event timing of the dominant kernels (spx_profile_enable)."""
    check(lib().spx_profile_enable(int(bool(on))), "spx_profile_enable")


def profile_read(kernel: str):
    """(summed ms, launches) of one profiled kernel since profile_enable."""
    ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
    check(lib().spx_profile_read(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)), "spx_profile_read")
    return ms.value, n.value


def gram_operand_bits() -> int:
    """4 (FP4 e2m1) or 8 (i8): the medoid Gram's MFMA operand encoding (8 for builds
    that predate the query)."""
    L = lib()
    return int(L.spx_medoid_gram_operand_bits()) if hasattr(L, "spx_medoid_gram_operand_bits") else 8


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().spx_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
