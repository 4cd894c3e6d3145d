#!/usr/bin/env python3
"""Rank 0's load in bench.py's 8-GPU strong-scaled step, rehearsed on ONE GPU (profiling
aid; the pool gives no multi-GPU box to this repo).  Rank 0 computes its LPT share of the
configs[4] batch like every rank AND, on its gather stream, rebuilds the other seven
ranks' consensus peaks from the wire format (spx_wire_unpack) while RCCL writes the
received bytes into its HBM.  This times, on one GPU:

  A  the fused step over rank 0's share alone (what every other rank does),
  B  the unpack of 7/8 of the batch's consensus peaks alone,
  C  A and B concurrently on two streams, plus a device copy of the received wire bytes
     on a third (standing in for the DMA of RCCL's receives),

so C / A is rank 0's slowdown against the other ranks, from which bench.py's rank-0 cost
share is chosen.  Prints one JSON line.

    python tools/rank0_probe.py [--world 8] [--reps 10]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--clusters", type=int, default=385_000)
    ap.add_argument("--rank0-weight", type=float, default=1.0)
    a = ap.parse_args()
    import torch

    from specpride_amd import engine, shard
    from specpride_amd.csr import SpectraCSR
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(a.clusters, seed=0)
    co, so = t["cluster_off"].cpu().numpy(), t["spec_off"].cpu().numpy()
    parts, loads = shard.strong_partition(co, so, a.world, "both", rank0_weight=a.rank0_weight)
    full = engine.DeviceBatch.from_device(t)
    bmf = engine.bin_mean(full)
    _, mz, it = bmf.compact()
    mi, cnt, nf = engine.wire_pack(mz, it, int(full.info.max_cluster_spectra))
    torch.cuda.synchronize()
    assert int(nf.item()) == 0
    n_other = int(sum(int(bmf.count[p].sum().item()) for p in parts[1:]))
    del bmf
    b0 = engine.DeviceBatch.from_device(SpectraCSR.select_on_device(t, parts[0], co, so))
    del full, t
    torch.cuda.empty_cache()
    bm, md = engine.bin_mean_medoid(b0)
    out_mz = torch.empty(n_other, dtype=torch.float64, device="cuda")
    out_it = torch.empty_like(out_mz)
    wire = torch.empty(n_other * 9, dtype=torch.uint8, device="cuda")  # the received bytes
    wsrc = torch.empty_like(wire)
    s1, s2, s3 = torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()

    def timed(fn):
        for _ in range(a.reps):  # warm: the clocks ramp under load (a cold first loop read 2x slow)
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        for _ in range(a.reps):
            fn()
        ev2, ev3 = torch.cuda.Event(), torch.cuda.Event()
        ev2.record(s2)
        ev3.record(s3)
        s1.wait_event(ev2)
        s1.wait_event(ev3)
        e1.record(s1)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    step = lambda: engine.bin_mean_medoid(b0, out_bm=bm, out_md=md, check=False)  # noqa: E731
    unpack = lambda: engine.wire_unpack(mi[:2 * n_other], cnt[:n_other], out_mz, out_it, stream=s2)  # noqa: E731

    def both():
        ev = torch.cuda.Event()
        ev.record(s1)
        s2.wait_event(ev)
        s3.wait_event(ev)
        with torch.cuda.stream(s3):
            wire.copy_(wsrc, non_blocking=True)
        unpack()
        step()

    res = {"world": a.world, "rank0_weight": a.rank0_weight, "rank_clusters": [len(p) for p in parts],
           "rank_cost_share": [round(float(x / loads.sum()), 5) for x in loads],
           "other_peaks": n_other, "wire_bytes": n_other * 9}
    for _ in range(2):  # twice, interleaved: the second round is reported
        res["A_step_ms"] = round(timed(step), 4)
        res["B_unpack_ms"] = round(timed(unpack), 4)
        res["C_both_ms"] = round(timed(both), 4)
    res["slowdown_C_over_A"] = round(res["C_both_ms"] / res["A_step_ms"], 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
