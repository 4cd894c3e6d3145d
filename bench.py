#!/usr/bin/env python3
"""Headline benchmark: clusters/sec for medoid + bin-mean consensus on MI355X.

BASELINE.json metric: "clusters/sec (whole node) for medoid + binned consensus
at 1/2/4/8 MI355X".  The metric is quoted on configs[4], the full pipeline on a
PRIDE-scale dataset of ~10M spectra; real PRIDE data is not available offline,
so the workload is its synthetic stand-in: 385k clusters of
U{2..50} spectra (~10.0M spectra, ~2.0G peaks, 32 GB of f64 peaks) generated
directly in HBM on every rank.

One step = one pass of the hot path over the resident batch:
  spx_bin_mean (combine_bin_mean, binning.py:170-231, for every cluster) +
  spx_medoid  (medoid representative, most_similar_representative.py:60-111).
Multi-GPU (torchrun, one process per GPU), default --scaling strong: every rank
generates the SAME seeded configs[4] batch and keeps only the clusters of its
size-balanced LPT bucket (shard.strong_partition: cost = peaks + n*peaks/64, the
reference's serial loops binning.py:291 / most_similar_representative.py:60 split
over the GPUs), so total work is fixed as N grows.  Each step's results --
representatives (as member indices) and the compacted consensus peaks -- are
gathered to rank 0 over RCCL inside the timed region, on a second stream that
overlaps the next step's kernels; after the timed region rank 0 reassembles the
last step in global cluster order and checks it.  value = the batch's clusters /
max-over-ranks time.  --scaling weak gives every rank its own 385k-cluster batch.

Extra keys (single GPU): the gap-average consensus on the same batch, the
north-star run (1M clusters on one MI355X), the configs[3] skewed medoid, bin-mean
off the headline's shape and the host-inclusive tier 2 (pageable host CSR -> H2D
-> kernels -> D2H) at the headline's size.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--clusters C] [--ns-clusters 1000000]

Prints ONE JSON line (rank 0).
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

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
HBM_ACHIEVABLE_GBS = 6290.0  # measured float4 copy ceiling (MI355X_MICROARCH.md chip table)
I8_DENSE_TOPS = 5000.0       # i8 MFMA dense peak, 2x BF16's ~2.5 PF (MI355X_MICROARCH.md MFMA table)
FP4_DENSE_TOPS = 10000.0     # FP4 (e2m1) MFMA dense peak, 4x BF16 per clock (same table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clusters", type=int, default=385_000, help="clusters per GPU (configs[4]: ~10M spectra)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--ns-clusters", type=int, default=1_000_000,
                    help="north-star run size on one GPU (0: skip)")
    ap.add_argument("--no-extras", action="store_true", help="headline only (profiling runs)")
    ap.add_argument("--cpu-sample", type=int, default=2000, help="clusters in the CPU-baseline sample (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tier2-chunk-mb", type=int, default=2048, help="tier-2 pipeline chunk (MB of peaks)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default): ONE configs[4] batch split over the ranks by size-balanced LPT "
                         "buckets; weak: every rank its own --clusters batch")
    ap.add_argument("--tier3-clusters", type=int, default=20000, help="tier-3 MGF size in clusters (0: skip)")
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


def consensus_bytes(batch, kept_peaks: int) -> int:
    """Algorithmic HBM bytes of one spx_bin_mean / spx_gap_average launch:
    read mz+inten (16 B/peak), spec_off + prec_mz + charge (20 B/spectrum),
    cluster_off (8 B/cluster); write 16 B per kept peak + count/prec/charge/status
    (24 B/cluster)."""
    return 16 * batch.n_peaks + 20 * batch.n_spectra + 8 * batch.n_clusters + 16 * kept_peaks + 24 * batch.n_clusters


def medoid_bytes(batch) -> int:
    """Algorithmic HBM bytes of one spx_medoid launch: mz (8 B/peak), spec_off
    (8 B/spectrum), cluster_off (8 B/cluster), rep out (8 B/cluster)."""
    return 8 * batch.n_peaks + 8 * batch.n_spectra + 16 * batch.n_clusters


def load_pmc_traffic(kernel: str, batch):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (collected on
    this configuration), scaled to this batch's peak count if it differs."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    v = d.get(kernel)
    if v is None:
        return None
    peaks = d.get("_peaks")
    return v if not peaks or peaks == batch.n_peaks else v * batch.n_peaks / peaks


def load_shape_traffic(key: str):
    """HBM bytes per call of an off-shape run (all the entry point's kernels), from
    the committed PMC passes of tools/gpu/shapes_pmc.sh over the same synthetic
    batch (profiles/pmc_traffic_shapes.json, keys bm_<shape> / md_<shape> / ga_<shape>)."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic_shapes.json")) as fh:
            return json.load(fh).get(key)
    except (OSError, ValueError):
        return None


def roofline(name, kernel, nbytes, ms, traffic=None, kernel_ms=None):
    """HBM roofline of one entry point: ``nbytes`` algorithmic bytes of the WHOLE batch
    over ``ms``, the time of the launches that process all of them (the entry point's:
    every cluster a first kernel hands on is finished inside it), so nothing deferred is
    counted without its time.  ``kernel_ms`` = the dominant kernel's own launch time
    (spx_profile events; the rocprofv3 kernel stats agree with it), reported beside."""
    gbs = nbytes / (ms * 1e-3) / 1e9
    r = {"bound": "hbm", "kernel": kernel, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(gbs / HBM_PEAK_GBS, 4), "frac_of_achievable": round(gbs / HBM_ACHIEVABLE_GBS, 4),
         "achievable": HBM_ACHIEVABLE_GBS, "traffic": traffic, "launch_ms": round(ms, 4),
         "algorithmic_bytes": int(nbytes), "entry_point": name}
    if kernel_ms is not None:
        r["dominant_kernel_ms"] = round(kernel_ms, 4)
    return r


def time_launches(fn, reps, stream):
    """Average launch duration of fn() by HIP events recorded on its stream."""
    import torch

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def kernel_ms(name: str) -> float:
    """Average duration of one kernel's launches since _lib.profile_enable (HIP events
    the library records around that launch on the caller's stream)."""
    from specpride_amd import _lib

    ms, n = _lib.profile_read(name)
    return ms / n if n else float("nan")


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


def headline(args, rank, world, local, out):
    import torch

    from specpride_amd import engine, shard
    from specpride_amd.csr import SpectraCSR
    from specpride_amd.synthetic import make_clusters_torch

    dev = torch.device("cuda", local)
    strong = args.scaling == "strong"
    parts = loads = None
    global_co = None
    if strong:
        # every rank generates the SAME seeded configs[4] batch and keeps the clusters the
        # size-balanced LPT plan gives it (shard.strong_partition, identical on every rank)
        t = make_clusters_torch(args.clusters, seed=args.seed, device=dev)
        if world > 1:
            global_co = t["cluster_off"].cpu().numpy()
            so = t["spec_off"].cpu().numpy()
            parts, loads = shard.strong_partition(global_co, so, world, "both")
            full, t = t, None
            t = SpectraCSR.select_on_device(full, parts[rank], global_co, so)
            del full, so
            torch.cuda.empty_cache()
    else:
        t = make_clusters_torch(args.clusters, seed=args.seed + 1000 * rank, device=dev)
    batch = engine.DeviceBatch.from_device(t)
    torch.cuda.synchronize()

    # checked once, before timing: every cluster resolved by the launch the step makes, and
    # the fused pass (spx_bin_mean_medoid: each cluster's bin-mean and medoid register
    # bodies in one workgroup, then each method's leftover chain) equal to the two
    # separate entry points, consensus peaks and representatives bit for bit
    bm_sep = engine.bin_mean(batch)
    md_sep = engine.medoid(batch, check=True)
    bm, md = engine.bin_mean_medoid(batch, check=True)
    torch.cuda.synchronize()
    st = bm.status.cpu().numpy()[:batch.n_clusters]
    rep = md.rep.cpu().numpy()[:batch.n_clusters]
    if np.any(st != 0) or np.any(rep < 0):
        raise RuntimeError(f"unexpected statuses: bin-mean {np.unique(st)}, medoid min rep {rep.min()}")
    kept = int(bm.count[:batch.n_clusters].sum().item())
    C = batch.n_clusters
    same = (torch.equal(bm.count[:C], bm_sep.count[:C]) and torch.equal(md.rep[:C], md_sep.rep[:C]) and
            all(torch.equal(a, b) for a, b in zip(bm.compact()[1:], bm_sep.compact()[1:])))
    if not same:
        raise RuntimeError("spx_bin_mean_medoid differs from spx_bin_mean + spx_medoid")
    large = engine.medoid_needs_large_path(batch) or bool(batch._ws.get("medoid_extra"))
    stream = torch.cuda.current_stream()
    first = batch.t["cluster_off"][:-1] if strong else None

    # double-buffered results when gathering (step k's are in flight during step k+1)
    bufs = [(bm, md)]
    gat = None
    if world > 1:
        bufs.append(engine.bin_mean_medoid(batch, check=False))
        gat = shard.StepGatherer(batch.n_clusters, rank, world, batch.device,
                                 wire_max_count=max(1, int(batch.info.max_cluster_spectra)))
        total_c, total_p = gat.plan(kept)

    inflight = [None] * len(bufs)  # per buffer: the event of the gather reading it

    def step(k):
        i = k % len(bufs)
        b, m = bufs[i]
        if inflight[i] is not None:
            stream.wait_event(inflight[i])  # this buffer's previous gather (step k-2) is done
        engine.bin_mean_medoid(batch, out_bm=b, out_md=m, check=False)
        if gat is not None:
            ev = torch.cuda.Event()
            ev.record(stream)
            inflight[i] = gat.launch(b, m.rep, ev, first=first)

    for k in range(args.warmup):
        step(k)
    barrier(world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    if gat is not None:
        gat.stream.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    if gat is not None and gat.check() != 0:
        raise RuntimeError(f"rank {rank}: {gat.check()} consensus peaks the gather wire format could not carry")
    total_clusters = (args.clusters if strong else world * batch.n_clusters)
    value = total_clusters * args.steps / elapsed

    assembled = None
    if gat is not None and strong:
        # rank 0 reassembles the last step's gathered results in global cluster order
        # (host-side index, after the timed region): every representative resolved and
        # the consensus peak count equal to the sum the ranks planned
        last = bufs[(args.warmup + args.steps - 1) % len(bufs)]
        if rank == 0:
            own_member = torch.where(last[1].rep[:batch.n_clusters] >= 0,
                                     last[1].rep[:batch.n_clusters] - first, last[1].rep[:batch.n_clusters])
            a = gat.assemble(parts, global_co, last[0], own_member)
            assembled = {"clusters": int(len(a["rep"])), "reps_resolved": bool(np.all(a["rep"] >= 0)),
                         "consensus_peaks": int(a["out_off"][-1]), "planned_peaks": int(total_p),
                         "ok": bool(np.all(a["rep"] >= 0) and int(a["out_off"][-1]) == int(total_p))}
            del a
        barrier(world)

    # per-kernel timing, after the timed region: HIP events on the stream the kernels
    # are launched on -- around each whole entry point, and (spx_profile_*) around
    # its dominant kernel's own launch inside the library
    from specpride_amd import _lib

    reps = max(3, args.steps)
    _lib.profile_enable(True)
    bm_ms_ep = time_launches(lambda: engine.bin_mean(batch, out=bm_sep), reps, stream)
    md_ms_ep = time_launches(lambda: engine.medoid(batch, out=md_sep, check=False), reps, stream)
    fu_ms_ep = time_launches(lambda: engine.bin_mean_medoid(batch, out_bm=bm, out_md=md, check=False), reps, stream)
    fu_k = kernel_ms("bin_mean_medoid_kernel")
    bm_ms = kernel_ms("bin_mean_reg_kernel")
    md_ms = kernel_ms("medoid_reg_kernel")
    _lib.profile_enable(False)
    bm_bytes = consensus_bytes(batch, kept)
    out.update({
        "metric": "clusters/sec (whole node) for medoid + binned consensus",
        "value": round(value, 1),
        "unit": "clusters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d) law, generated in HBM per rank; stand-in for the ~10M-spectrum PRIDE set)",
        "config": {"workload": "configs[4]: full pipeline (bin-mean consensus + medoid representative) on a "
                               "PRIDE-scale clustered dataset of ~10M spectra, U{2..50} spectra/cluster, "
                               "~200 peaks/spectrum",
                   "clusters": total_clusters, "clusters_this_rank": batch.n_clusters,
                   "spectra_this_rank": batch.n_spectra, "peaks_this_rank": batch.n_peaks,
                   "parallelism": (f"cluster-sharded x{world}, size-balanced LPT buckets of one batch "
                                   "(cost = peaks + n*peaks/64)" if strong and world > 1
                                   else f"cluster-sharded x{world}"),
                   "gather": ("per-step RCCL gather of reps + compacted consensus peaks to rank 0, "
                              "overlapped with the next step" if world > 1 else "none (1 GPU: results stay in HBM)"),
                   "medoid_large_path": bool(large)},
        "roofline": roofline("spx_bin_mean", "bin_mean_reg_kernel", bm_bytes, bm_ms_ep,
                             load_pmc_traffic("bin_mean_reg_kernel", batch), kernel_ms=bm_ms),
        "roofline_medoid": roofline("spx_medoid", "medoid_reg_kernel", medoid_bytes(batch), md_ms_ep,
                                    load_pmc_traffic("medoid_reg_kernel", batch), kernel_ms=md_ms),
        "kernels": {"spx_bin_mean_ms": round(bm_ms_ep, 4), "spx_medoid_ms": round(md_ms_ep, 4),
                    "bin_mean_reg_kernel_ms": round(bm_ms, 4), "medoid_reg_kernel_ms": round(md_ms, 4)},
    })
    if gat is not None:
        out["config"]["gathered_clusters_per_step"] = total_c
        out["config"]["gathered_peaks_per_step"] = total_p
        out["config"]["gather_wire"] = (f"f32 bin sums + {gat.wire}-byte counts, rebuilt to f64 on rank 0 "
                                        "(csrc/wire.hip)" if gat.wire else "f64 peaks")
        out["config"]["rank0_inbound_bytes_per_step"] = gat.wire_bytes_per_step() if rank == 0 else None
    if loads is not None:
        out["config"]["rank_cost_share"] = [round(float(x / loads.sum()), 5) for x in loads]
        out["config"]["cost_max_over_min"] = round(float(loads.max() / max(loads.min(), 1.0)), 5)
        out["config"]["rank_clusters"] = [int(len(p)) for p in parts]
    if assembled is not None:
        out["config"]["assembled_last_step"] = assembled
    out["config"]["step"] = ("spx_bin_mean_medoid: one fused pass per cluster (bin-mean + medoid register bodies "
                             "in one workgroup, then each method's leftover kernels); checked bit-identical to "
                             "spx_bin_mean + spx_medoid before timing")
    out["kernels"]["spx_bin_mean_medoid_ms"] = round(fu_ms_ep, 4)
    out["kernels"]["bin_mean_medoid_kernel_ms"] = round(fu_k, 4)
    if rank == 0 and world == 1 and not args.no_extras:
        # the same step through the two separate entry points (the two CLIs' calls)
        sep_ms = time_launches(lambda: (engine.bin_mean(batch, out=bm_sep),
                                        engine.medoid(batch, out=md_sep, check=False)), reps, stream)
        out["separate_step"] = {"entry_points": "spx_bin_mean + spx_medoid", "ms": round(sep_ms, 4),
                                "clusters_per_s": round(batch.n_clusters / (sep_ms * 1e-3), 1),
                                "fused_ms_per_step": round(elapsed / args.steps * 1e3, 4)}
        # gap-average consensus on the same resident batch (average_spectrum_clustering.py:26-148)
        ga = engine.gap_average(batch)
        torch.cuda.synchronize()
        gst = ga.status.cpu().numpy()[:batch.n_clusters]
        gkept = int(ga.count[:batch.n_clusters].sum().item())
        _lib.profile_enable(True)
        ga_ms = time_launches(lambda: engine.gap_average(batch, out=ga), reps, stream)
        ga_k = kernel_ms("gap_average_lds_kernel")
        _lib.profile_enable(False)
        out["gap_average"] = {"clusters_per_s": round(batch.n_clusters / (ga_ms * 1e-3), 1), "launch_ms": round(ga_ms, 4),
                              "lds_kernel_ms": round(ga_k, 4), "ok_clusters": int((gst == 0).sum()),
                              "roofline": roofline("spx_gap_average", "gap_average_lds_kernel",
                                                   consensus_bytes(batch, gkept), ga_ms,
                                                   load_pmc_traffic("gap_average_lds_kernel", batch), kernel_ms=ga_k)}
        del ga
    del bm, md, bm_sep, md_sep, bufs, batch, t
    torch.cuda.empty_cache()


def north_star(args, out):
    """BASELINE.json north_star: 1M synthetic clusters on one MI355X (configs[2]'s
    size), bin-mean + medoid, inputs resident in HBM (5.2G peaks, 83 GB)."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(args.ns_clusters, seed=args.seed + 7)
    batch = engine.DeviceBatch.from_device(t)
    bm, md = engine.bin_mean_medoid(batch, check=True)  # the headline's step (fused pass)
    torch.cuda.synchronize()
    ok = bool(np.all(bm.status.cpu().numpy()[:batch.n_clusters] == 0) and
              np.all(md.rep.cpu().numpy()[:batch.n_clusters] >= 0))
    steps = max(3, args.steps // 2)
    engine.bin_mean_medoid(batch, out_bm=bm, out_md=md, check=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        engine.bin_mean_medoid(batch, out_bm=bm, out_md=md, check=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["north_star_1m"] = {"clusters": batch.n_clusters, "spectra": batch.n_spectra, "peaks": batch.n_peaks,
                            "clusters_per_s": round(batch.n_clusters * steps / dt, 1),
                            "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "all_resolved": ok,
                            "hbm_gb_resident": round(torch.cuda.max_memory_allocated() / 1e9, 1)}
    del bm, md
    torch.cuda.empty_cache()
    # configs[2]'s method on the same 1M clusters: gap-average (average_spectrum_clustering.py:151-165);
    # configs[2] shards it over 8 GPUs, here one MI355X holds all of it
    ga = engine.gap_average(batch)
    torch.cuda.synchronize()
    gst = ga.status.cpu().numpy()[:batch.n_clusters]
    gkept = int(ga.count[:batch.n_clusters].sum().item())
    from specpride_amd import _lib

    _lib.profile_enable(True)
    ga_ms = time_launches(lambda: engine.gap_average(batch, out=ga), 3, torch.cuda.current_stream())
    ga_k = kernel_ms("gap_average_lds_kernel")
    _lib.profile_enable(False)
    out["north_star_1m"]["gap_average"] = {
        "ms": round(ga_ms, 3), "clusters_per_s": round(batch.n_clusters / (ga_ms * 1e-3), 1),
        "ok_clusters": int((gst == 0).sum()), "lds_kernel_ms": round(ga_k, 3),
        "roofline": roofline("spx_gap_average", "gap_average_lds_kernel", consensus_bytes(batch, gkept), ga_ms,
                             kernel_ms=ga_k),
        "hbm_gb_resident": round(torch.cuda.max_memory_allocated() / 1e9, 1)}
    del ga, batch, t
    torch.cuda.empty_cache()


def config3(args, out):
    """configs[3]: medoid on the skewed long tail (MFMA dense-Gram path)."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(20000, seed=4, skewed=True, forced_large=4, large_size=5000)
    batch = engine.DeviceBatch.from_device(t)
    md = engine.medoid(batch, check=True)
    torch.cuda.synchronize()
    ok = bool(np.all(md.rep.cpu().numpy()[:batch.n_clusters] >= 0))
    from specpride_amd import _lib

    _lib.profile_enable(True)
    ms = time_launches(lambda: engine.medoid(batch, out=md, check=False), 5, torch.cuda.current_stream())
    gram_ms = kernel_ms("medoid_gram_kernel")
    _lib.profile_enable(False)
    sizes = np.diff(batch.host_cluster_off)
    ops = gram_ops(t, batch)
    tops = ops / (gram_ms * 1e-3) / 1e12
    bits = _lib.gram_operand_bits()
    peak = FP4_DENSE_TOPS if bits == 4 else I8_DENSE_TOPS
    out["config3_medoid"] = {"clusters": batch.n_clusters, "spectra": batch.n_spectra, "max_n": int(sizes.max()),
                             "large_clusters": int((sizes > 64).sum()), "medoid_ms": round(ms, 3),
                             "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1), "all_resolved": ok,
                             "roofline": {"bound": "mfma", "kernel": "medoid_gram_reg_kernel",
                                          "achieved": round(tops, 1), "peak": peak, "unit": "TOP/s",
                                          "frac": round(tops / peak, 4), "traffic": None,
                                          "operands": "fp4 e2m1 0/1 (v_mfma_f32_32x32x64_f8f6f4)" if bits == 4
                                          else "i8 0/1 (v_mfma_i32_32x32x32_i8)",
                                          "frac_of_i8_peak": round(tops / I8_DENSE_TOPS, 4),
                                          "launch_ms": round(gram_ms, 4), "algorithmic_ops": int(ops),
                                          "ops_definition": "sum over the large-path clusters of 2*n(n+1)/2*K_c, "
                                                            "K_c = distinct ceil(mz/0.1) bins of the cluster",
                                          "entry_point": "spx_medoid"}}
    del md, batch, t
    torch.cuda.empty_cache()


def gram_ops(t, batch) -> int:
    """Algorithmic int ops of the large-cluster Gram: 2*n(n+1)/2*K_c
    per cluster the MFMA path takes (n > 64 or past the small kernels' peak cap),
    K_c its distinct ceil(mz/0.1) bins (most_similar_representative.py:88-93)."""
    from specpride_amd.csr import SpectraCSR

    co, so = batch.host_cluster_off, batch.host_spec_off
    n = np.diff(co)
    p = so[co[1:]] - so[co[:-1]]
    big = np.flatnonzero((n > 64) | (p > 32768))
    sub = SpectraCSR.select_from_device(t, big)
    ops = 0
    for k in range(sub.n_clusters):
        a, b = sub.spec_off[sub.cluster_off[k]], sub.spec_off[sub.cluster_off[k + 1]]
        kc = len(np.unique(np.ceil(sub.mz[a:b] / 0.1)))
        nn = int(sub.cluster_off[k + 1] - sub.cluster_off[k])
        ops += 2 * (nn * (nn + 1) // 2) * kc
    return ops


def medoid_shapes(args, out):
    """Medoid on 600-peak spectra: U{2..50} clusters whose
    peaks (> 12,288) or distinct 0.1-bins (> 1,728) exceed the register kernel's
    caps from n ~ 20 on, so the MFMA Gram path runs at mid-size n."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    t = make_clusters_torch(20000, seed=6, n_template=600)
    batch = engine.DeviceBatch.from_device(t)
    md = engine.medoid(batch, check=True)
    torch.cuda.synchronize()
    ok = bool(np.all(md.rep.cpu().numpy()[:batch.n_clusters] >= 0))
    ms = time_launches(lambda: engine.medoid(batch, out=md, check=False), 5, torch.cuda.current_stream())
    co, so = batch.host_cluster_off, batch.host_spec_off
    sizes, peaks = np.diff(co), so[co[1:]] - so[co[:-1]]
    large = (sizes > 64) | (peaks > 12288)
    out["medoid_shapes"] = {"long_spectra_600": {
        "clusters": batch.n_clusters, "spectra": batch.n_spectra, "peaks": batch.n_peaks,
        "large_path_by_size": int(large.sum()), "ms": round(ms, 3),
        "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1), "all_resolved": ok,
        "roofline": roofline("spx_medoid", "all medoid kernels", medoid_bytes(batch), ms,
                             load_shape_traffic("md_long_spectra_600"))}}
    del md, batch, t
    torch.cuda.empty_cache()


def bin_mean_shapes(args, out):
    """Bin-mean off the headline's shape: the configs[3]
    skewed size law (clusters up to n = 5,000: the LDS and global-scratch paths)
    and spectra longer than the register path's 252 peaks (600-peak templates)."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    res = {}
    for name, kw in (("skewed_config3", dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000)),
                     ("long_spectra_600", dict(n_clusters=20000, seed=6, n_template=600))):
        t = make_clusters_torch(**kw)
        batch = engine.DeviceBatch.from_device(t)
        bm = engine.bin_mean(batch)
        torch.cuda.synchronize()
        st = bm.status.cpu().numpy()[:batch.n_clusters]
        kept = int(bm.count[:batch.n_clusters].sum().item())
        ms = time_launches(lambda: engine.bin_mean(batch, out=bm), 5, torch.cuda.current_stream())
        sizes = np.diff(batch.host_cluster_off)
        so = batch.host_spec_off
        res[name] = {"clusters": batch.n_clusters, "spectra": batch.n_spectra, "peaks": batch.n_peaks,
                     "max_n": int(sizes.max()), "max_spectrum_peaks": int(np.diff(so).max()),
                     "ms": round(ms, 3), "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1),
                     "all_ok": bool(np.all(st == 0)),
                     "roofline": roofline("spx_bin_mean", "all bin-mean kernels", consensus_bytes(batch, kept), ms,
                                          load_shape_traffic(f"bm_{name}"))}
        del bm, batch, t
        torch.cuda.empty_cache()
    out["bin_mean_shapes"] = res


def gap_average_shapes(args, out):
    """Gap-average off the headline's shape, the same batches as bin_mean_shapes:
    600-peak spectra (thousands of occupied 0.01-Da buckets per cluster: the wide
    kernel) and the configs[3] skewed law (its giants: the tiled giant pipeline)."""
    import torch

    from specpride_amd import engine
    from specpride_amd.synthetic import make_clusters_torch

    res = {}
    for name, kw in (("skewed_config3", dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000)),
                     ("long_spectra_600", dict(n_clusters=20000, seed=6, n_template=600))):
        t = make_clusters_torch(**kw)
        batch = engine.DeviceBatch.from_device(t)
        ga = engine.gap_average(batch)
        torch.cuda.synchronize()
        st = ga.status.cpu().numpy()[:batch.n_clusters]
        kept = int(ga.count[:batch.n_clusters].sum().item())
        ms = time_launches(lambda: engine.gap_average(batch, out=ga), 3, torch.cuda.current_stream())
        res[name] = {"clusters": batch.n_clusters, "peaks": batch.n_peaks, "ms": round(ms, 3),
                     "clusters_per_s": round(batch.n_clusters / (ms * 1e-3), 1),
                     "ok_clusters": int((st == 0).sum()),
                     "roofline": roofline("spx_gap_average", "all gap-average kernels", consensus_bytes(batch, kept),
                                          ms, load_shape_traffic(f"ga_{name}"))}
        del ga, batch, t
        torch.cuda.empty_cache()
    out["gap_average_shapes"] = res


def tier2(args, out):
    """SURVEY.md §8(d) tier 2 at the headline's size (configs[4], 385k clusters, a
    32 GB packed host CSR in pageable memory) through pipeline.HostPipeline: chunks of
    whole clusters, H2D of chunk k+1 (spx_copy_h2d) overlapped with chunk k's
    spx_bin_mean + spx_medoid and chunk k-1's compaction + D2H, device slots allocated
    once (the first pass) and reused.  Timed: the second pass, host CSR in -> host
    results out.  Never `value`."""
    import torch

    from specpride_amd.csr import SpectraCSR
    from specpride_amd.pipeline import HostPipeline
    from specpride_amd.synthetic import make_clusters_torch
    from specpride_amd import engine

    t = make_clusters_torch(args.clusters, seed=args.seed + 11)
    h = {k: engine.to_host_array(t[k]) for k in ("cluster_off", "spec_off", "mz", "inten", "prec_mz", "charge", "rt")}
    del t
    torch.cuda.empty_cache()
    csr = SpectraCSR(h["cluster_off"], h["spec_off"], h["mz"], h["inten"], h["prec_mz"], h["charge"], h["rt"])
    nbytes = sum(a.nbytes for a in h.values())
    pipe = HostPipeline(chunk_bytes=args.tier2_chunk_mb << 20)
    best = None
    for rep_i in range(3):  # pass 0 allocates the device slots and the pinned staging pool
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = pipe.run(csr)
        dt = time.perf_counter() - t0
        if rep_i == 0:
            continue
        ok = bool(np.all(r["status"] == 0) and np.all(r["rep"] >= 0))
        tm = pipe.timing
        cur = {"clusters": csr.n_clusters, "host_bytes": int(nbytes), "total_s": round(dt, 4),
               "clusters_per_s": round(csr.n_clusters / dt, 1), "host_GBs": round(nbytes / dt / 1e9, 2),
               "chunks": tm["chunks"], "chunk_mb": args.tier2_chunk_mb,
               "h2d_issue_s": round(tm["h2d_host_s"], 4), "readback_s": round(tm["readback_s"], 4),
               "kernels_s": round(tm["kernel_ms"] * 1e-3, 4),
               "d2h_bytes": int(16 * r["out_off"][-1] + 8 * len(r["rep"])), "all_ok": ok}
        if best is None or cur["clusters_per_s"] > best["clusters_per_s"]:
            best = cur
        del r
    out["tier2_host_inclusive"] = best
    del pipe, csr, h
    torch.cuda.empty_cache()


def tier3(args, out):
    """SURVEY.md §8(d) tier 3: each of the three CLIs MGF text -> MGF text on one
    synthetic clustered MGF (configs law, --tier3-clusters clusters, written once
    before the timed region by the native writer): binning.py (binning.py:250-302),
    average_spectrum_clustering.py --encodedclusters (:168-210) and
    most_similar_representative.py (:22-115).  Each CLI runs once on a 200-cluster
    file first (code objects, allocator, pinned staging), then is timed on the big
    one.  The reference's own binning CLI on the same file shape, timed in the
    build container (the reference never reaches the GPU box), is reported beside
    it from profiles/r02_reference_cli_container.json.  Never `value`."""
    import contextlib
    import io
    import tempfile

    import torch

    from specpride_amd import average_spectrum_clustering as asc
    from specpride_amd import binning
    from specpride_amd import most_similar_representative as msr
    from specpride_amd.synthetic import write_clustered_mgf

    clis = {"binning": lambda i, o: binning.main(["--mgf_file", i, "--out", o]),
            "average_spectrum_clustering": lambda i, o: asc.main([i, o, "--encodedclusters"]),
            "most_similar_representative": lambda i, o: msr.main(["-i", i, "-o", o])}
    res = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        warm_in, mgf_in, mgf_out = (os.path.join(td, x) for x in ("w.mgf", "in.mgf", "out.mgf"))
        write_clustered_mgf(warm_in, 200, args.seed + 22)
        t0 = time.perf_counter()
        S, P = write_clustered_mgf(mgf_in, args.tier3_clusters, args.seed + 21)
        size = os.path.getsize(mgf_in)
        res.update(clusters=args.tier3_clusters, spectra=S, peaks=P, mgf_bytes=int(size),
                   input_write_s=round(time.perf_counter() - t0, 2))
        torch.cuda.empty_cache()
        for name, cli in clis.items():
            with contextlib.redirect_stdout(io.StringIO()):
                cli(warm_in, mgf_out)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                cli(mgf_in, mgf_out)
                dt = time.perf_counter() - t0
            res[name] = {"cli_s": round(dt, 3), "clusters_per_s": round(args.tier3_clusters / dt, 1),
                         "mgf_in_GBs": round(size / dt / 1e9, 3), "mgf_out_bytes": int(os.path.getsize(mgf_out))}
    try:
        with open(os.path.join(REPO, "profiles", "r02_reference_cli_container.json")) as fh:
            ref = json.load(fh)
        res["reference_binning_cli"] = {"clusters_per_s": ref["clusters_per_s"], "cores": ref["cores"],
                                        "where": ref["host"], "file": f"{ref['clusters']} clusters, "
                                                                      f"{ref['mgf_MB']} MB MGF"}
        res["binning_vs_reference_cli"] = round(res["binning"]["clusters_per_s"] / ref["clusters_per_s"], 1)
    except (OSError, ValueError, KeyError):
        pass
    out["tier3_mgf_to_mgf"] = res


def main():
    args = parse()
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    want_cpu = world0 == 1 and not args.no_cpu_baseline and args.cpu_sample > 0
    cpu_par = cpu_baseline_parallel(4 * args.cpu_sample, args.seed) if want_cpu else None
    rank, world, local = dist_init()
    out = {}
    headline(args, rank, world, local, out)
    if rank == 0 and world == 1 and not args.no_extras:
        config3(args, out)
        bin_mean_shapes(args, out)
        medoid_shapes(args, out)
        gap_average_shapes(args, out)
        tier2(args, out)
        if args.tier3_clusters > 0:
            tier3(args, out)
        if args.ns_clusters > 0:
            north_star(args, out)
    if rank == 0 and want_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.seed)
        out["cpu_baseline_all_cores"] = cpu_par
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
