"""Deterministic synthetic clustered spectra.

Real PRIDE data is not available offline, so every benchmark and most parity
tests run on synthetic clusters with the shape the survey prescribes:

* cluster sizes U{2..50} (or the skewed long-tail law of config 4),
* a 200-peak template per cluster, m/z ~ U[100, 2000), sorted,
* each member = template + N(0, 0.003 Da) jitter, ~10 % peak dropout and
  ~10 % uniform noise peaks, sorted ascending, m/z rounded to 5 decimals,
* intensities lognormal(5, 1.5) rounded to 2 decimals, strictly > 0,
* precursor m/z U[400, 1200] per cluster (+ tiny per-member jitter),
  charge in {2, 3} constant within a cluster, RT ~ U[0, 3600].

Two generators share that law: :func:`make_clusters_np` (numpy, host; used
for golden fixtures, CPU tests and the CPU baseline sample) and
:func:`make_clusters_torch` (torch, on the GPU; used by ``bench.py`` so that a
100k-cluster batch is created directly in HBM).  They are not bit-identical to
each other -- nothing depends on that; parity tests always hand the *same*
arrays to the GPU path and the oracle.

The result is a cluster-segmented CSR batch (:class:`specpride_amd.csr.SpectraCSR`).
"""
from __future__ import annotations

import numpy as np

N_TEMPLATE = 200
MZ_LO, MZ_HI = 100.0, 2000.0
JITTER_SD = 0.003
DROPOUT = 0.10
NOISE_FRAC = 0.10


def cluster_sizes(n_clusters: int, rng: np.random.Generator, *, min_size: int = 2,
                  max_size: int = 50, skewed: bool = False, forced_large: int = 0,
                  large_size: int = 5000) -> np.ndarray:
    """Cluster sizes: U{min..max}, or the config-4 long tail
    ``n = min(5000, max(2, floor(2 * U**(-1/1.1))))`` plus ``forced_large`` clusters."""
    if skewed:
        u = rng.random(n_clusters)
        sizes = np.minimum(large_size, np.maximum(2, np.floor(2.0 * u ** (-1.0 / 1.1)))).astype(np.int64)
    else:
        sizes = rng.integers(min_size, max_size + 1, size=n_clusters).astype(np.int64)
    if forced_large:
        sizes = np.concatenate([sizes, np.full(forced_large, large_size, np.int64)])
    return sizes


def make_clusters_np(n_clusters: int, seed: int = 0, *, min_size: int = 2, max_size: int = 50,
                     n_template: int = N_TEMPLATE, skewed: bool = False, forced_large: int = 0,
                     large_size: int = 5000, sizes: np.ndarray | None = None):
    """Build a synthetic batch on the host.  Returns a ``SpectraCSR`` (numpy arrays)."""
    from .csr import SpectraCSR

    rng = np.random.default_rng(seed)
    if sizes is None:
        sizes = cluster_sizes(n_clusters, rng, min_size=min_size, max_size=max_size,
                              skewed=skewed, forced_large=forced_large, large_size=large_size)
    sizes = np.asarray(sizes, np.int64)
    C = len(sizes)
    S = int(sizes.sum())
    templates = np.sort(rng.uniform(MZ_LO, MZ_HI, size=(C, n_template)), axis=1)
    owner = np.repeat(np.arange(C), sizes)

    n_noise_max = max(4, int(round(n_template * NOISE_FRAC * 2)))
    width = n_template + n_noise_max
    # build in chunks of spectra to bound host memory
    mz_parts, int_parts, lens = [], [], np.empty(S, np.int64)
    chunk = 65536
    for s0 in range(0, S, chunk):
        s1 = min(S, s0 + chunk)
        m = s1 - s0
        t = templates[owner[s0:s1]]
        jit = t + rng.normal(0.0, JITTER_SD, size=t.shape)
        keep = rng.random(t.shape) >= DROPOUT
        jit[~keep] = np.inf
        n_noise = np.minimum(rng.binomial(n_template, NOISE_FRAC, size=m), n_noise_max)
        noise = rng.uniform(MZ_LO, MZ_HI, size=(m, n_noise_max))
        noise[np.arange(n_noise_max)[None, :] >= n_noise[:, None]] = np.inf
        block = np.concatenate([jit, noise], axis=1)
        # keep inside [MZ_LO, MZ_HI): jitter can push a template peak just outside
        block[(block < MZ_LO) | (block >= MZ_HI)] = np.inf
        block = np.round(np.sort(block, axis=1), 5)
        valid = np.isfinite(block)
        ln = valid.sum(axis=1)
        lens[s0:s1] = ln
        mz_parts.append(block[valid])
        inten = np.round(rng.lognormal(5.0, 1.5, size=int(ln.sum())), 2)
        int_parts.append(np.maximum(inten, 0.01))
    mz = np.concatenate(mz_parts) if mz_parts else np.zeros(0)
    inten = np.concatenate(int_parts) if int_parts else np.zeros(0)

    spec_off = np.zeros(S + 1, np.int64)
    np.cumsum(lens, out=spec_off[1:])
    cluster_off = np.zeros(C + 1, np.int64)
    np.cumsum(sizes, out=cluster_off[1:])
    base_prec = rng.uniform(400.0, 1200.0, size=C)
    prec = np.round(base_prec[owner] + rng.normal(0.0, 0.002, size=S), 5)
    charge = rng.integers(2, 4, size=C).astype(np.int32)[owner]
    rt = np.round(rng.uniform(0.0, 3600.0, size=S), 2)
    return SpectraCSR(cluster_off=cluster_off, spec_off=spec_off, mz=mz, inten=inten,
                      prec_mz=prec, charge=charge, rt=rt,
                      cluster_ids=[f"cluster-{k}" for k in range(C)])


def make_clusters_torch(n_clusters: int, seed: int = 0, *, device="cuda", min_size: int = 2,
                        max_size: int = 50, n_template: int = N_TEMPLATE, skewed: bool = False,
                        forced_large: int = 0, large_size: int = 5000, chunk_spectra: int = 1 << 20):
    """Same law as :func:`make_clusters_np`, generated with torch directly on ``device``.

    Returns a dict of device tensors with the CSR layout (no cluster-id strings:
    benchmark batches are never written to MGF)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rng = np.random.default_rng(seed)
    sizes = cluster_sizes(n_clusters, rng, min_size=min_size, max_size=max_size, skewed=skewed,
                          forced_large=forced_large, large_size=large_size)
    C = len(sizes)
    S = int(sizes.sum())
    f64 = torch.float64
    sizes_t = torch.as_tensor(sizes, device=device)
    templates = torch.sort(MZ_LO + (MZ_HI - MZ_LO) * torch.rand((C, n_template), generator=g,
                                                                  device=device, dtype=f64), dim=1).values
    owner = torch.repeat_interleave(torch.arange(C, device=device), sizes_t)
    n_noise_max = max(4, int(round(n_template * NOISE_FRAC * 2)))
    mz_parts, lens_parts = [], []
    for s0 in range(0, S, chunk_spectra):
        s1 = min(S, s0 + chunk_spectra)
        m = s1 - s0
        t = templates[owner[s0:s1]]
        jit = t + JITTER_SD * torch.randn(t.shape, generator=g, device=device, dtype=f64)
        keep = torch.rand(t.shape, generator=g, device=device) >= DROPOUT
        jit = torch.where(keep, jit, torch.full_like(jit, float("inf")))
        n_noise = torch.binomial(torch.full((m,), float(n_template), device=device),
                                 torch.full((m,), NOISE_FRAC, device=device), generator=g).to(torch.int64)
        n_noise = torch.clamp(n_noise, max=n_noise_max)
        noise = MZ_LO + (MZ_HI - MZ_LO) * torch.rand((m, n_noise_max), generator=g, device=device, dtype=f64)
        col = torch.arange(n_noise_max, device=device)[None, :]
        noise = torch.where(col < n_noise[:, None], noise, torch.full_like(noise, float("inf")))
        block = torch.cat([jit, noise], dim=1)
        block = torch.where((block < MZ_LO) | (block >= MZ_HI), torch.full_like(block, float("inf")), block)
        block = torch.sort(block, dim=1).values
        # the double nearest each 5-decimal value, as an MGF parse gives it: a true
        # division (dividing by a Python scalar may multiply by its reciprocal on
        # the device, which is 1 ulp off for some values)
        block = torch.round(block * 1e5) / torch.full_like(block, 1e5)
        valid = torch.isfinite(block)
        lens_parts.append(valid.sum(dim=1))
        mz_parts.append(block[valid])
        del t, jit, keep, noise, block, valid
    lens = torch.cat(lens_parts)
    P = int(sum(p.numel() for p in mz_parts))
    # fill preallocated arrays chunk by chunk: peak memory ~ one copy of the peaks
    # plus one chunk (a 1M-cluster batch is 5.2G peaks = 42 GB per array)
    mz = torch.empty(P, dtype=f64, device=device)
    o = 0
    while mz_parts:
        part = mz_parts.pop(0)
        mz[o:o + part.numel()] = part
        o += part.numel()
        del part
    inten = torch.empty(P, dtype=f64, device=device)
    step = 1 << 28
    for a in range(0, P, step):
        b = min(P, a + step)
        x = torch.exp(5.0 + 1.5 * torch.randn(b - a, generator=g, device=device, dtype=f64))
        inten[a:b] = torch.clamp(torch.round(x * 100.0) / 100.0, min=0.01)
        del x
    spec_off = torch.zeros(S + 1, dtype=torch.int64, device=device)
    spec_off[1:] = torch.cumsum(lens, 0)
    cluster_off = torch.zeros(C + 1, dtype=torch.int64, device=device)
    cluster_off[1:] = torch.cumsum(sizes_t, 0)
    base_prec = 400.0 + 800.0 * torch.rand(C, generator=g, device=device, dtype=f64)
    prec = torch.round((base_prec[owner] + 0.002 * torch.randn(S, generator=g, device=device, dtype=f64)) * 1e5) / 1e5
    charge = (2 + torch.randint(0, 2, (C,), generator=g, device=device)).to(torch.int32)[owner]
    rt = torch.round(3600.0 * torch.rand(S, generator=g, device=device, dtype=f64) * 100.0) / 100.0
    return dict(cluster_off=cluster_off, spec_off=spec_off, mz=mz, inten=inten, prec_mz=prec,
                charge=charge.contiguous(), rt=rt, n_clusters=C, n_spectra=S, n_peaks=P)


def write_clustered_mgf(path: str, n_clusters: int, seed: int = 0, device="cuda") -> tuple:
    """Write a clustered MGF of this law (the reference's title convention,
    file_formats.md: ``TITLE=cluster-<c>;mzspec:PXDSYN:synthetic:scan:<s>``, PEPMASS,
    CHARGE, RTINSECONDS, repr floats) with the native batched writer; the batch is
    generated by :func:`make_clusters_torch` on ``device``.  Returns (spectra, peaks).
    The tier-3 benchmarks' input (bench.py, tools/bench_tiers.py)."""
    import torch

    from . import engine, mgf_native

    t = make_clusters_torch(n_clusters, seed=seed, device=device)
    h = {k: engine.to_host_array(t[k]) for k in ("cluster_off", "spec_off", "mz", "inten", "prec_mz", "charge", "rt")}
    del t
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    owner = np.repeat(np.arange(n_clusters), np.diff(h["cluster_off"]))
    titles = [f"cluster-{c};mzspec:PXDSYN:synthetic:scan:{s}" for s, c in enumerate(owner.tolist())]
    mgf_native.write_records(path, mgf_native.STYLE_MEDOID, titles, h["spec_off"], h["mz"], h["inten"],
                             h["prec_mz"], h["charge"], h["rt"])
    return int(len(owner)), int(h["spec_off"][-1])
