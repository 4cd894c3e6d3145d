#!/usr/bin/env python3
"""Headline benchmark: clusters/sec for medoid + bin-mean consensus on MI355X.

BASELINE.json metric: "clusters/sec (whole node) for medoid + binned consensus
at 1/2/4/8 MI355X"; workload = configs[1]: 100k synthetic clusters of U{2..50}
spectra, ~200 peaks per spectrum, generated directly in HBM.

One step = one pass of the hot path over one batch already resident in HBM:
  spx_bin_mean (combine_bin_mean for every cluster) + spx_medoid (medoid
  representative for every cluster), results left in HBM.
Multi-GPU: one process per GPU (torchrun); every rank owns its own 100k-cluster
shard (clusters are independent: no data-path collective), so scaling is weak
and value = all ranks' clusters / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--clusters C]

Prints ONE JSON line (rank 0).  Also: per-kernel HIP-event timing for the
roofline object, and the oracle timed on a bounded host sample (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=2000, help="clusters in the CPU-baseline sample (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def dist_init():
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bin_mean_bytes(batch, kept_peaks: int) -> int:
    """Algorithmic HBM bytes of one spx_bin_mean launch:
    read mz+inten (16 B/peak), spec_off + prec_mz + charge (20 B/spectrum),
    cluster_off (8 B/cluster); write 16 B per kept peak + count/prec/charge/status
    (24 B/cluster)."""
    return 16 * batch.n_peaks + 20 * batch.n_spectra + 8 * batch.n_clusters + 16 * kept_peaks + 24 * batch.n_clusters


def medoid_bytes(batch) -> int:
    """Algorithmic HBM bytes of one spx_medoid launch: mz (8 B/peak), spec_off
    (8 B/spectrum), cluster_off (8 B/cluster), rep out (8 B/cluster)."""
    return 8 * batch.n_peaks + 8 * batch.n_spectra + 16 * batch.n_clusters


def load_pmc_traffic(kernel: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh).get(kernel)
    except (OSError, ValueError):
        return None


def cpu_baseline(n_clusters: int, seed: int):
    """The oracle ('port' of the reference: numpy combine_bin_mean restatement +
    C restatement of the OpenMS dense-table xcorr medoid) on one host core."""
    from oracle import c_oracle, np_oracle
    from specpride_amd.synthetic import make_clusters_np

    csr = make_clusters_np(n_clusters, seed=seed + 99)
    c_oracle.lib()
    t0 = time.perf_counter()
    np_oracle.bin_mean(csr)
    t1 = time.perf_counter()
    c_oracle.medoid(csr, dense_tables=True)
    t2 = time.perf_counter()
    return {"value": n_clusters / (t2 - t0), "unit": "clusters/s", "cores": 1, "kind": "port",
            "sample": (f"{n_clusters} synthetic clusters (U{{2..50}} spectra, ~200 peaks) on 1 host core: "
                       f"numpy combine_bin_mean restatement {t1 - t0:.2f} s + C OpenMS-style dense-table "
                       f"xcorr medoid {t2 - t1:.2f} s")}


_CPU_SAMPLE = None  # the parallel CPU sample, inherited by the forked workers (not pickled per task)


def _cpu_shard(ab):
    """Worker of cpu_baseline_parallel (a forked process, no GPU): the oracle on
    clusters [a, b) of the sample."""
    a, b = ab
    from oracle import c_oracle, np_oracle

    sub = _CPU_SAMPLE.select(range(a, b))
    np_oracle.bin_mean(sub)
    c_oracle.medoid(sub, dense_tables=True)
    return b - a


def cpu_baseline_parallel(n_clusters: int, seed: int):
    """The same port, cluster-parallel over the host cores this process may use
    (the all-cores figure beside the 1-core one).  Runs before
    the process touches the GPU, so the forked workers never inherit a HIP context."""
    import multiprocessing as mp

    from oracle import c_oracle
    from specpride_amd.synthetic import make_clusters_np

    cores = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    global _CPU_SAMPLE
    _CPU_SAMPLE = make_clusters_np(n_clusters, seed=seed + 99)
    c_oracle.lib()
    step = (n_clusters + 4 * cores - 1) // (4 * cores)
    chunks = [(a, min(a + step, n_clusters)) for a in range(0, n_clusters, step)]
    with mp.get_context("fork").Pool(cores) as pool:
        t0 = time.perf_counter()
        done = sum(pool.map(_cpu_shard, chunks))
        dt = time.perf_counter() - t0
    _CPU_SAMPLE = None
    return {"value": done / dt, "unit": "clusters/s", "cores": cores, "kind": "port",
            "sample": (f"{n_clusters} synthetic clusters over {cores} worker processes (the 1-core port, "
                       f"cluster-parallel): {dt:.2f} s")}


def main():
    args = parse()
    import torch

    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    cpu_par = None
    if world0 == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
        cpu_par = cpu_baseline_parallel(4 * args.cpu_sample, args.seed)
    rank, world, local = dist_init()
    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    dev = torch.device("cuda", local)
    t = make_clusters_torch(args.clusters, seed=args.seed + 1000 * rank, device=dev)
    batch = engine.DeviceBatch.from_device(t)
    torch.cuda.synchronize()

    bm = engine.bin_mean(batch)
    md = engine.medoid(batch)
    torch.cuda.synchronize()
    st = bm.status.cpu().numpy()
    if np.any(st != 0) or np.any(md.rep.cpu().numpy() < 0):
        raise RuntimeError(f"unexpected statuses: bin-mean {np.unique(st)}, medoid min rep {md.rep.min().item()}")
    kept = int(bm.count.sum().item())

    def step():
        engine.bin_mean(batch, out=bm)
        engine.medoid(batch, out=md)

    for _ in range(args.warmup):
        step()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    value = world * batch.n_clusters * args.steps / elapsed

    # per-kernel timing (events on the stream the kernels run on)
    stream = torch.cuda.current_stream()
    reps = max(3, args.steps)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    for _ in range(reps):
        engine.bin_mean(batch, out=bm)
    ev[1].record(stream)
    for _ in range(reps):
        engine.medoid(batch, out=md)
    ev[2].record(stream)
    torch.cuda.synchronize()
    bm_ms = ev[0].elapsed_time(ev[1]) / reps
    md_ms = ev[1].elapsed_time(ev[2]) / reps
    bm_gbs = bin_mean_bytes(batch, kept) / (bm_ms * 1e-3) / 1e9
    md_gbs = medoid_bytes(batch) / (md_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic("bin_mean_lds_kernel")

    out = {
        "metric": "clusters/sec (whole node) for medoid + binned consensus",
        "value": round(value, 1),
        "unit": "clusters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d) law, generated in HBM per rank)",
        "config": {"workload": "configs[1]: binning.py bin-mean + most_similar_representative medoid, "
                               "U{2..50} spectra/cluster, ~200 peaks/spectrum",
                   "clusters_per_gpu": batch.n_clusters, "spectra_per_gpu": batch.n_spectra,
                   "peaks_per_gpu": batch.n_peaks, "parallelism": f"cluster-sharded x{world}"},
        "roofline": {"bound": "hbm", "kernel": "spx_bin_mean", "achieved": round(bm_gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bm_gbs / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "launch_ms": round(bm_ms, 4),
                     "algorithmic_bytes": bin_mean_bytes(batch, kept)},
        "kernels": {"spx_bin_mean_ms": round(bm_ms, 4), "spx_medoid_ms": round(md_ms, 4),
                    "spx_medoid_algorithmic_GBs": round(md_gbs, 1)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
        out["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.seed)
        if cpu_par is not None:
            out["cpu_baseline_all_cores"] = cpu_par
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
