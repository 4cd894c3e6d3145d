"""Time tools/calib/stream_shapes.hip's read shapes on the bench batch (GB/s)."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402

NAMES = {0: "flat", 1: "cl_flat", 2: "cl_ring_barrier", 3: "cl_ring_nobarrier", 4: "cl_flat_mz_only"}


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libstream_shapes.so"))
    t = make_clusters_torch(100_000, seed=0, device="cuda")
    out = torch.zeros(t["n_clusters"] + 1, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for kind, name in NAMES.items():
        def go():
            rc = lib.stream_shape(kind, ctypes.c_void_p(t["cluster_off"].data_ptr()),
                                  ctypes.c_void_p(t["spec_off"].data_ptr()), ctypes.c_void_p(t["mz"].data_ptr()),
                                  ctypes.c_void_p(t["inten"].data_ptr()), ctypes.c_int64(t["n_clusters"]),
                                  ctypes.c_int64(t["n_peaks"]), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st))
            assert rc == 0
        go()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            go()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        nbytes = t["n_peaks"] * (8 if kind == 4 else 16)
        res[name] = {"ms": round(ms, 4), "GBs": round(nbytes / ms / 1e6, 1)}
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for kind, name in ((5, "pers_range"), (6, "pers_rr"), (7, "cl_ring_lds")):
        def go2():
            rc = lib.stream_shape2(kind, ctypes.c_void_p(t["cluster_off"].data_ptr()),
                                   ctypes.c_void_p(t["spec_off"].data_ptr()), ctypes.c_void_p(t["mz"].data_ptr()),
                                   ctypes.c_void_p(t["inten"].data_ptr()), ctypes.c_int64(t["n_clusters"]),
                                   ctypes.c_int(5 * ncu), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st))
            assert rc == 0
        go2()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            go2()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[name] = {"ms": round(ms, 4), "GBs": round(t["n_peaks"] * 16 / ms / 1e6, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
