"""Shared fixtures.  `-m gpu` tests need a real MI355X; everything else runs on CPU."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from specpride_amd.csr import SpectraCSR  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name))
    csr = SpectraCSR(z["cluster_off"], z["spec_off"], z["mz"], z["inten"], z["prec_mz"], z["charge"], z["rt"])
    return z, csr


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


BIN_SETS = ["edge", "synthetic", "params_b", "params_c", "mixed_charge", "nonfinite"]
GAP_SETS = ["edge", "synthetic", "params_b", "params_c", "nonfinite", "nonfinite_b"]


def bin_params(z):
    p = z["params"]
    return dict(minimum=float(p[0]), maximum=float(p[1]), binsize=float(p[2]), apply_peak_quorum=bool(p[3]))


def gap_params(z):
    p = z["params"]
    return dict(mz_accuracy=float(p[0]), dyn_range=float(p[1]), min_fraction=float(p[2]))


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from specpride_amd import _lib

    _lib.lib()
    return torch.device("cuda:0")
