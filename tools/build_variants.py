#!/usr/bin/env python3
"""Build A/B variants of the HIP engine (profiling aid, CPU-side):

    python tools/build_variants.py name="-DFLAG=1 -DX=2" name2="..."

-> specpride_amd/lib/ab_<name>.so, loadable with SPX_LIB=... (tools/gpu/ab.sh)."""
import os
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from specpride_amd import _lib  # noqa: E402


def build(spec):
    name, flags = spec.split("=", 1)
    out = os.path.join(_lib.LIB_DIR, f"ab_{name}.so")
    cmd = [_lib.HIPCC, *_lib.HIP_FLAGS, *shlex.split(flags), "-o", out, os.path.join(_lib.CSRC, "spx_api.hip")]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(build, sys.argv[1:]):
            print(p)
