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
    ap.add_argument("--rank0-weight", type=float, default=None,
                    help="strong scaling: rank 0's relative speed in the LPT plan (default rank0_weight(N))")
    return ap.parse_args()


class HipBackend:
    """The product path of one rank: the HIP engine on ``cuda:LOCAL_RANK`` (inputs
    generated in HBM), RCCL between ranks.  bench.py's step, timing and gather code
    only talks to a backend through these methods; the CPU test suite swaps in a
    stand-in (``SPX_BENCH_BACKEND``, tests/bench_oracle_backend.py) to drive the
    launcher, the strong split, the gather and rank 0's reassembly under gloo."""
    kind = "hip"
    dist_backend = "nccl"

    def __init__(self, local: int):
        import torch

        if rehearsal():  # every rank on GPU 0, gloo between them (host-staged P2P)
            local = 0
            self.dist_backend = "gloo"
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.stream = torch.cuda.current_stream()

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def generate(self, clusters: int, seed: int):
        from specpride_amd.synthetic import make_clusters_torch

        return make_clusters_torch(clusters, seed=seed, device=self.dev)

    def select(self, t, ids, co, so):
        from specpride_amd.csr import SpectraCSR

        return SpectraCSR.select_on_device(t, ids, co, so)

    def batch(self, t):
        from specpride_amd import engine

        return engine.DeviceBatch.from_device(t)

    def first_step(self, batch):
        """The step once, checked: every cluster resolved by the launch the step makes,
        and the fused pass (spx_bin_mean_medoid) equal to the two separate entry points,
        consensus peaks and representatives bit for bit.  Returns (bm, md, separate)."""
        import torch

        from specpride_amd import engine

        bm_sep = engine.bin_mean(batch)
        md_sep = engine.medoid(batch, check=True)
        bm, md = engine.bin_mean_medoid(batch, check=True)
        torch.cuda.synchronize()
        C = batch.n_clusters
        st = bm.status.cpu().numpy()[:C]
        rep = md.rep.cpu().numpy()[:C]
        if np.any(st != 0) or np.any(rep < 0):
            raise RuntimeError(f"unexpected statuses: bin-mean {np.unique(st)}, medoid min rep {rep.min()}")
        same = (torch.equal(bm.count[:C], bm_sep.count[:C]) and torch.equal(md.rep[:C], md_sep.rep[:C]) and
                all(torch.equal(a, b) for a, b in zip(bm.compact()[1:], bm_sep.compact()[1:])))
        if not same:
            raise RuntimeError("spx_bin_mean_medoid differs from spx_bin_mean + spx_medoid")
        return bm, md, (bm_sep, md_sep)

    def alloc(self, batch):
        from specpride_amd import engine

        return engine.bin_mean_medoid(batch, check=False)

    def step(self, batch, bm, md):
        from specpride_amd import engine

        engine.bin_mean_medoid(batch, out_bm=bm, out_md=md, check=False)

    def record(self):
        import torch

        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def wait(self, ev):
        self.stream.wait_event(ev)

    def first(self, batch):
        return batch.t["cluster_off"][:-1]

    def max_cluster_spectra(self, batch) -> int:
        return int(batch.info.max_cluster_spectra)

    def sample_results(self, t, ids, co, so) -> dict:
        """World-1 results of clusters ``ids`` of the full batch ``t`` (rank 0, before
        the strong split): the fused pass over just those clusters, on the host."""
        sub = self.batch(self.select(t, ids, co, so))
        bm, md, _ = self.first_step(sub)
        h = bm.to_host()
        first = sub.host_cluster_off[:-1]
        rep = md.rep.cpu().numpy()[:sub.n_clusters]
        return dict(count=np.diff(h["out_off"]), out_off=h["out_off"], out_mz=h["out_mz"], out_int=h["out_int"],
                    member=np.where(rep >= 0, rep - first, rep))


def rehearsal() -> bool:
    """SPX_BENCH_REHEARSE=1: the multi-GPU step rehearsed on ONE GPU (a profiling and test aid;
    the pool gives this repo one GPU per box, and RCCL takes one rank per device): every rank
    runs the HIP engine on GPU 0 and the ranks talk over gloo, the gather's payloads staged
    through host copies (shard.StepGatherer(stage_host=True)).  Everything but RCCL itself --
    the split, the per-rank fused steps, the device-side wire pack / unpack, rank 0's
    reassembly and its bit-for-bit check -- runs as on the node; the timing is not the
    node's and the line says so."""
    return os.environ.get("SPX_BENCH_REHEARSE") == "1"


def make_backend(local: int):
    """HipBackend, unless SPX_BENCH_BACKEND=module:Class names a test stand-in (the CPU
    suite's launcher test; never set on the GPU box)."""
    spec = os.environ.get("SPX_BENCH_BACKEND")
    if not spec:
        return HipBackend(local)
    import importlib

    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)(local)


def dist_init(be):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        kw = {"device_id": torch.device("cuda", local)} if be.dist_backend == "nccl" else {}
        dist.init_process_group(be.dist_backend, **kw)
    return rank, world, local


def barrier(world, be):
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    be.sync()


def max_over_ranks(x: float, world: int, be) -> float:
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if be.dist_backend == "gloo" else be.dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def launch_ranks(args) -> int:
    """``bench.py --gpus N`` outside a torchrun launch: start N fresh worker processes
    of this script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set
    (rendezvous on 127.0.0.1), before this process makes any GPU call.  Rank 0 prints
    the JSON line on this process's stdout; the other ranks' stdout goes to stderr.
    Returns the first non-zero worker exit status (the others are then stopped), or 0.
    More ranks than visible devices is an error: it never falls back to fewer GPUs."""
    import signal
    import socket
    import subprocess
    import threading

    n = args.gpus
    if not os.environ.get("SPX_BENCH_BACKEND") and not rehearsal():
        import torch  # device_count() does not initialise HIP on this image

        have = torch.cuda.device_count()
        if n > have:
            print(f"bench.py: --gpus {n} but only {have} HIP device(s) are visible", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs, rank_of = [], {}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=r == 0))
        rank_of[procs[-1].pid] = r
    relay = threading.Thread(target=_relay_rank0, args=(procs[0].stdout,), daemon=True)
    relay.start()
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {rank_of[p.pid]} exited with {code}; stopping the others",
                          file=sys.stderr, flush=True)
                    for q in procs:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for q in procs:  # only on an exception in this loop: our own children, by PID
            q.kill()
    relay.join(timeout=30)
    return rc


def _relay_rank0(pipe):
    """Rank 0's stdout: the JSON line to this process's stdout, anything else the
    communication libraries print (e.g. gloo's connection notice) to stderr."""
    for line in pipe:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        (sys.stdout if line.startswith("{") else sys.stderr).flush()


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


def fused_bytes(batch, kept_peaks: int) -> int:
    """Algorithmic HBM bytes of one fused step (spx_bin_mean_medoid): both methods'
    bytes, as two separate launches would move them (the medoid reads the m/z again)."""
    return consensus_bytes(batch, kept_peaks) + medoid_bytes(batch)


def one_read_bytes(batch, kept_peaks: int) -> int:
    """The step's single-read floor: every input read once (the consensus bytes, which
    already read each m/z and intensity) plus the representative written (8 B/cluster)."""
    return consensus_bytes(batch, kept_peaks) + 8 * batch.n_clusters


def sample_ids(parts, per_rank: int = 512):
    """Global cluster ids rank 0 checks the reassembled step against (every rank's
    share, spread over its list)."""
    pick = [p[np.linspace(0, len(p) - 1, min(per_rank, len(p))).astype(np.int64)] for p in parts if len(p)]
    return np.unique(np.concatenate(pick)) if pick else np.zeros(0, np.int64)


def check_assembled(a, want, ids, total_p):
    """Rank 0's check of the reassembled last step: every representative resolved, the
    planned peak total, and the sampled clusters bit-identical (counts, f64 peak bits,
    member index) to a world-1 run of the same clusters.  Raises on any difference."""
    ok_rep = bool(np.all(a["rep"] >= 0))
    ok_total = int(a["out_off"][-1]) == int(total_p)
    cnt = np.diff(a["out_off"])[ids]
    same = np.array_equal(cnt, want["count"])
    if same:
        from specpride_amd.csr import concat_ranges

        sel = concat_ranges(a["out_off"][ids], cnt)
        same = (np.array_equal(a["out_mz"][sel].view(np.int64), want["out_mz"].view(np.int64)) and
                np.array_equal(a["out_int"][sel].view(np.int64), want["out_int"].view(np.int64)))
    member = a["rep"][ids] - a["cluster_off"][ids]
    same_rep = np.array_equal(member, want["member"])
    res = {"clusters": int(len(a["rep"])), "reps_resolved": ok_rep, "consensus_peaks": int(a["out_off"][-1]),
           "planned_peaks": int(total_p), "sample_clusters": int(len(ids)),
           "sample_equal_world1": bool(same and same_rep)}
    res["ok"] = bool(ok_rep and ok_total and same and same_rep)
    if not res["ok"]:
        raise RuntimeError(f"rank 0's reassembled step differs from the plan or from world 1: {res}")
    return res


def rank0_weight(world: int) -> float:
    """Rank 0's relative speed in the strong-scaling LPT plan.  Besides its share, rank 0
    rebuilds the other ranks' gathered consensus peaks from the wire format (spx_wire_unpack,
    25 B of HBM traffic per peak) while RCCL writes them into its HBM (9 B per peak); on one
    GPU that load, run beside rank 0's step, added 0.38 / 0.55 / 0.66 ms to a 5.6 / 2.8 /
    1.4 ms step at N = 2 / 4 / 8 (tools/rank0_probe.py, profiles/r06_rank0_probe.txt), against
    ~0.13-0.25 ms of packing and compaction on the other ranks: equal finishing times need
    rank 0 at ~0.98 / ~0.88 / ~0.73 of the others' share."""
    return max(0.5, 1.0 - 0.04 * (world - 1))


def headline(args, rank, world, local, out, be):
    import torch

    from specpride_amd import shard

    strong = args.scaling == "strong"
    parts = loads = None
    global_co = None
    want = ids = None
    if strong:
        # every rank generates the SAME seeded configs[4] batch and keeps the clusters the
        # size-balanced LPT plan gives it (shard.strong_partition, identical on every rank)
        t = be.generate(args.clusters, args.seed)
        if world > 1:
            global_co = t["cluster_off"].cpu().numpy()
            so = t["spec_off"].cpu().numpy()
            w0 = args.rank0_weight if args.rank0_weight is not None else rank0_weight(world)
            parts, loads = shard.strong_partition(global_co, so, world, "both", rank0_weight=w0)
            if rank == 0:  # world-1 results of a sample of every rank's clusters, for the check
                ids = sample_ids(parts)
                want = be.sample_results(t, ids, global_co, so)
            full, t = t, None
            t = be.select(full, parts[rank], global_co, so)
            del full, so
            if be.kind == "hip":
                torch.cuda.empty_cache()
    else:
        t = be.generate(args.clusters, args.seed + 1000 * rank)
    batch = be.batch(t)
    be.sync()

    # checked once, before timing (HipBackend.first_step: statuses, fused == separate)
    bm, md, separate = be.first_step(batch)
    kept = int(bm.count[:batch.n_clusters].sum().item())
    first = be.first(batch) if strong else None

    # double-buffered results when gathering (step k's are in flight during step k+1)
    bufs = [(bm, md)]
    gat = None
    if world > 1:
        bufs.append(be.alloc(batch))
        gat = shard.StepGatherer(batch.n_clusters, rank, world, be.dev,
                                 wire_max_count=max(1, be.max_cluster_spectra(batch)),
                                 wire_ops=getattr(be, "wire_ops", None),
                                 stage_host=be.kind == "hip" and be.dist_backend == "gloo")
        total_c, total_p = gat.plan(kept)

    inflight = [None] * len(bufs)  # per buffer: the event of the gather reading it

    def step(k):
        i = k % len(bufs)
        b, m = bufs[i]
        if inflight[i] is not None:
            be.wait(inflight[i])  # this buffer's previous gather (step k-2) is done
        be.step(batch, b, m)
        if gat is not None:
            inflight[i] = gat.launch(b, m.rep, be.record(), first=first)

    for k in range(args.warmup):
        step(k)
    barrier(world, be)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    if gat is not None and gat.stream is not None:
        gat.stream.synchronize()
    barrier(world, be)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, be)
    if gat is not None and gat.check() != 0:
        raise RuntimeError(f"rank {rank}: {gat.check()} consensus peaks the gather wire format could not carry")
    total_clusters = (args.clusters if strong else world * batch.n_clusters)
    value = total_clusters * args.steps / elapsed

    assembled = None
    if gat is not None and strong:
        # rank 0 reassembles the last step's gathered results in global cluster order
        # (host-side index, after the timed region) and checks it (check_assembled)
        last = bufs[(args.warmup + args.steps - 1) % len(bufs)]
        if rank == 0:
            r = last[1].rep[:batch.n_clusters]
            own_member = torch.where(r >= 0, r - first, r)
            a = gat.assemble(parts, global_co, last[0], own_member)
            a["cluster_off"] = global_co
            assembled = check_assembled(a, want, ids, total_p)
            del a
        barrier(world, be)

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
                                   "(cost = peaks + n*peaks/64; rank 0, which also rebuilds the gathered peaks, "
                                   "weighted by rank0_weight)" if strong and world > 1
                                   else f"cluster-sharded x{world}"),
                   "rehearsal": ("SPX_BENCH_REHEARSE=1: every rank on GPU 0, gloo with host-staged P2P -- "
                                 "not the node's timing" if rehearsal() and world > 1 else None),
                   "launcher": ("bench.py --gpus N (own worker processes)" if os.environ.get("SPX_BENCH_SPAWNED")
                                else ("external (torchrun)" if world > 1 else "single process")),
                   "gather": ("per-step RCCL gather of reps + compacted consensus peaks to rank 0, "
                              "overlapped with the next step" if world > 1 else "none (1 GPU: results stay in HBM)")},
    })
    if gat is not None:
        out["config"]["gathered_clusters_per_step"] = total_c
        out["config"]["gathered_peaks_per_step"] = total_p
        out["config"]["gather_wire"] = (f"f32 bin sums + {gat.wire}-byte counts, rebuilt to f64 on rank 0 "
                                        "(csrc/wire.hip)" if gat.wire else "f64 peaks")
        out["config"]["rank0_inbound_bytes_per_step"] = gat.wire_bytes_per_step() if rank == 0 else None
    if loads is not None:
        out["config"]["rank0_weight"] = w0
        out["config"]["rank_cost_share"] = [round(float(x / loads.sum()), 5) for x in loads]
        out["config"]["cost_max_over_min"] = round(float(loads.max() / max(loads.min(), 1.0)), 5)
        out["config"]["rank_clusters"] = [int(len(p)) for p in parts]
    if assembled is not None:
        out["config"]["assembled_last_step"] = assembled
    out["config"]["step"] = ("spx_bin_mean_medoid: one fused pass per cluster (bin-mean + medoid register bodies "
                             "in one workgroup); the leftover chains only when a register body handed a cluster "
                             "on (spx_bin_mean_medoid_stage); checked bit-identical to spx_bin_mean + spx_medoid "
                             "before timing")
    if be.kind == "hip":
        kernel_lines(args, rank, world, out, be, batch, bm, md, separate, kept)
    del bm, md, separate, bufs, batch, t
    if be.kind == "hip":
        torch.cuda.empty_cache()


def kernel_lines(args, rank, world, out, be, batch, bm, md, separate, kept):
    """Per-kernel timing after the timed region: HIP events on the stream the kernels
    are launched on -- around each whole entry point, and (spx_profile_*) around its
    dominant kernel's own launch inside the library.  ``roofline`` is the fused step's
    (the kernel the headline times); the separate entry points' lines beside it."""
    import torch

    from specpride_amd import _lib, engine

    bm_sep, md_sep = separate
    stream = be.stream
    large = engine.medoid_needs_large_path(batch) or bool(batch._ws.get("medoid_extra"))
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
    fu = roofline("spx_bin_mean_medoid", "bin_mean_medoid_kernel", fused_bytes(batch, kept), fu_ms_ep,
                  load_pmc_traffic("bin_mean_medoid_kernel", batch), kernel_ms=fu_k)
    one = one_read_bytes(batch, kept)
    fu["one_read_bytes"] = int(one)
    fu["one_read_frac"] = round(one / (fu_ms_ep * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    fu["bytes_definition"] = ("bin-mean (16 B/peak + 20 B/spectrum + 32 B/cluster + 16 B/kept peak) + medoid "
                              "(8 B/peak + 8 B/spectrum + 16 B/cluster), as the two separate launches move them; "
                              "one_read_frac: the single-read floor (each input once + 8 B/cluster rep)")
    out["config"]["medoid_large_path"] = bool(large)
    out["roofline"] = fu
    out["roofline_bin_mean"] = roofline("spx_bin_mean", "bin_mean_reg_kernel", bm_bytes, bm_ms_ep,
                                        load_pmc_traffic("bin_mean_reg_kernel", batch), kernel_ms=bm_ms)
    out["roofline_medoid"] = roofline("spx_medoid", "medoid_reg_kernel", medoid_bytes(batch), md_ms_ep,
                                      load_pmc_traffic("medoid_reg_kernel", batch), kernel_ms=md_ms)
    out["kernels"] = {"spx_bin_mean_medoid_ms": round(fu_ms_ep, 4), "bin_mean_medoid_kernel_ms": round(fu_k, 4),
                      "spx_bin_mean_ms": round(bm_ms_ep, 4), "spx_medoid_ms": round(md_ms_ep, 4),
                      "bin_mean_reg_kernel_ms": round(bm_ms, 4), "medoid_reg_kernel_ms": round(md_ms, 4)}
    if rank == 0 and world == 1 and not args.no_extras:
        # the same step through the two separate entry points (the two CLIs' calls)
        sep_ms = time_launches(lambda: (engine.bin_mean(batch, out=bm_sep),
                                        engine.medoid(batch, out=md_sep, check=False)), reps, stream)
        out["separate_step"] = {"entry_points": "spx_bin_mean + spx_medoid", "ms": round(sep_ms, 4),
                                "clusters_per_s": round(batch.n_clusters / (sep_ms * 1e-3), 1),
                                "fused_ms_per_step": out["ms_per_step"]}
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
    if rehearsal() and os.environ.get("SPX_BENCH_TRACE_AFTER"):  # where each rank is, if a rehearsal stalls
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["SPX_BENCH_TRACE_AFTER"]), exit=False)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        os.environ["SPX_BENCH_SPAWNED"] = "1"
        sys.exit(launch_ranks(args))
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world0 != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world0}")
    want_cpu = world0 == 1 and not args.no_cpu_baseline and args.cpu_sample > 0
    cpu_par = cpu_baseline_parallel(4 * args.cpu_sample, args.seed) if want_cpu else None
    be = make_backend(int(os.environ.get("LOCAL_RANK", "0")))
    rank, world, local = dist_init(be)
    out = {}
    headline(args, rank, world, local, out, be)
    if rank == 0 and world == 1 and not args.no_extras and be.kind == "hip":
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
