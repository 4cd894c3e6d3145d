#!/usr/bin/env python3
"""Does running the step's two kernels concurrently pay?  bin-mean and medoid read
the same batch and write disjoint outputs; serially each leaves the CUs partly idle
(LDS caps bin-mean at 5 workgroups per CU, medoid at 6).  Times K steps serial (one
stream) and overlapped (bin-mean and medoid on two streams, joined per step), with
result digests.  GPU box only.

    python tools/overlap_probe.py [--clusters 385000] [--steps 10]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from specpride_amd import engine  # noqa: E402
from specpride_amd.synthetic import make_clusters_torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=385000)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    batch = engine.DeviceBatch.from_device(make_clusters_torch(a.clusters, seed=0))
    bm = engine.bin_mean(batch)
    md = engine.medoid(batch, check=True)
    torch.cuda.synchronize()
    s0 = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def serial():
        engine.bin_mean(batch, out=bm)
        engine.medoid(batch, out=md, check=False)

    def overlapped():
        ev = torch.cuda.Event()
        ev.record(s0)
        s1.wait_event(ev)
        s2.wait_event(ev)
        engine.bin_mean(batch, out=bm, stream=s1)
        engine.medoid(batch, out=md, check=False, stream=s2)
        s0.wait_stream(s1)
        s0.wait_stream(s2)

    res = {"clusters": a.clusters}
    for name, fn in (("serial", serial), ("overlapped", overlapped), ("serial2", serial), ("overlapped2", overlapped)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for _ in range(a.steps):
            fn()
        e1.record(s0)
        torch.cuda.synchronize()
        res[name + "_ms"] = e0.elapsed_time(e1) / a.steps
        res[name + "_digest"] = [float(bm.count[:batch.n_clusters].sum().item()),
                                 int(md.rep[:batch.n_clusters].sum().item())]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
