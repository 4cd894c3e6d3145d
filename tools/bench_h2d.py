#!/usr/bin/env python3
"""Host -> HBM copy rates (profiling aid): torch pinned -> device (the DMA ceiling),
torch pageable, and spx_copy_h2d / spx_copy_d2h from pageable numpy memory on the
default stream and on a side stream.  Prints one JSON line.

    python tools/bench_h2d.py [--gb 4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    a = ap.parse_args()
    import numpy as np
    import torch

    from specpride_amd import _lib

    n = int(a.gb * 1e9) // 8
    host = np.random.default_rng(0).random(n)  # pageable, resident
    dev = torch.empty(n, dtype=torch.float64, device="cuda")
    L = _lib.lib()
    out = {"bytes": host.nbytes}

    def timed(fn, reps=3):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return round(host.nbytes / best / 1e9, 2)

    pinned = torch.empty(n, dtype=torch.float64, pin_memory=True)
    pinned.numpy()[:] = host
    out["torch_pinned_h2d_GBs"] = timed(lambda: dev.copy_(pinned, non_blocking=True))
    out["torch_pageable_h2d_GBs"] = timed(lambda: dev.copy_(torch.from_numpy(host)))
    side = torch.cuda.Stream()
    for name, st in (("default", torch.cuda.current_stream()), ("side", side)):
        out[f"spx_h2d_{name}_GBs"] = timed(lambda: _lib.check(
            L.spx_copy_h2d(dev.data_ptr(), host.ctypes.data, host.nbytes, st.cuda_stream), "h2d"))
        back = np.empty_like(host)
        out[f"spx_d2h_{name}_GBs"] = timed(lambda: _lib.check(
            L.spx_copy_d2h(back.ctypes.data, dev.data_ptr(), host.nbytes, st.cuda_stream), "d2h"))
    assert np.array_equal(back, host)
    t0 = time.perf_counter()
    np.copyto(np.empty_like(host), host)
    out["host_memcpy_1thread_GBs"] = round(host.nbytes / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
