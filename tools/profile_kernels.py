#!/usr/bin/env python3
"""Kernel timing / diagnostics driver (profiling aid, not the product bench).

    python tools/profile_kernels.py [--clusters 100000] [--reps 5] [--which bm,md,ga] [--stamps]

Times each entry point on a synthetic configs[4]-law batch with HIP events and
prints one JSON line.  Under ``rocprofv3 --pmc`` it is the program the counter
passes run (tools/gpu/pmc.sh).  With --stamps it loads the diagnostic build
(specpride_amd/lib/libspecpride_hip_stamps.so, -DSPX_STAMPS: build it with
``python tools/profile_kernels.py --build-stamps`` on the CPU) and reports the
mean shader-clock cycles per bin-mean phase (SPX_STAMP(k) in the kernels),
overall and per cluster-size band.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
STAMPS_LIB = os.environ.get("SPX_STAMPS_LIB") or os.path.join(REPO, "specpride_amd", "lib", "libspecpride_hip_stamps.so")


def build_stamps():
    from specpride_amd import _lib

    cmd = [_lib.HIPCC, *_lib.HIP_FLAGS, "-DSPX_STAMPS", "-o", STAMPS_LIB, os.path.join(_lib.CSRC, "spx_api.hip")]
    subprocess.run(cmd, check=True)
    print(STAMPS_LIB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--which", default="bm,md,ga")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--stamps-kernel", default="bm", choices=["bm", "md", "ga", "fu"])
    ap.add_argument("--build-stamps", action="store_true")
    ap.add_argument("--shape", default=None, help="an off-shape batch of tools/run_shape.py (skewed_config3, long_spectra_600)")
    a = ap.parse_args()
    if a.build_stamps:
        build_stamps()
        return
    if a.stamps:
        os.environ["SPX_LIB"] = STAMPS_LIB
    import ctypes

    import numpy as np
    import torch

    from specpride_amd import _lib, engine
    from specpride_amd.synthetic import make_clusters_torch

    if a.shape:
        sys.argv = sys.argv[:1]  # run_shape parses argv at import: only its SHAPES table is used
        shapes = {"skewed_config3": dict(n_clusters=20000, seed=4, skewed=True, forced_large=4, large_size=5000),
                  "long_spectra_600": dict(n_clusters=20000, seed=6, n_template=600)}
        t = make_clusters_torch(**shapes[a.shape])
    else:
        t = make_clusters_torch(a.clusters, seed=a.seed)
    b = engine.DeviceBatch.from_device(t)
    which = a.which.split(",")
    res = {"clusters": b.n_clusters, "spectra": b.n_spectra, "peaks": b.n_peaks}
    st = torch.cuda.current_stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / a.reps, 4)

    def digest(*arrays):  # order-sensitive checksum of result arrays (variants must agree)
        import hashlib

        h = hashlib.sha1()
        for x in arrays:
            h.update(x.detach().cpu().numpy().tobytes())
        return h.hexdigest()[:16]

    if "bm" in which:
        bm = engine.bin_mean(b)
        res["bin_mean_ms"] = timed(lambda: engine.bin_mean(b, out=bm))
        off, mz, it = bm.compact()
        res["bin_mean_digest"] = digest(off, mz, it, bm.status, bm.prec, bm.charge)
    if "md" in which:
        md = engine.medoid(b)
        res["medoid_ms"] = timed(lambda: engine.medoid(b, out=md, check=False))
        res["medoid_digest"] = digest(md.rep)
    if "cc" in which:  # the step as two concurrent streams: bin-mean on this one, medoid on a second
        cbm, cmd = engine.bin_mean(b), engine.medoid(b)
        s2 = torch.cuda.Stream()

        def both():
            ev = torch.cuda.Event()
            ev.record(st)
            s2.wait_event(ev)
            engine.bin_mean(b, out=cbm)
            engine.medoid(b, out=cmd, check=False, stream=s2)
            ev2 = torch.cuda.Event()
            ev2.record(s2)
            st.wait_event(ev2)
        res["concurrent_ms"] = timed(both)
        off, mz, it = cbm.compact()
        res["concurrent_digests"] = [digest(off, mz, it, cbm.status, cbm.prec, cbm.charge), digest(cmd.rep)]
    if "fu" in which:  # the fused step (spx_bin_mean_medoid): digests must equal bm's and md's
        fbm, fmd = engine.bin_mean_medoid(b)
        res["fused_ms"] = timed(lambda: engine.bin_mean_medoid(b, out_bm=fbm, out_md=fmd, check=False))
        off, mz, it = fbm.compact()
        res["fused_bin_mean_digest"] = digest(off, mz, it, fbm.status, fbm.prec, fbm.charge)
        res["fused_medoid_digest"] = digest(fmd.rep)
    if "ga" in which:
        ga = engine.gap_average(b)
        res["gap_average_ms"] = timed(lambda: engine.gap_average(b, out=ga))
        off, mz, it = ga.compact()
        res["gap_average_digest"] = digest(off, mz, it, ga.status, ga.prec, ga.charge)
    if a.stamps:
        L = _lib.lib()
        L.spx_debug_stamps.argtypes = [ctypes.c_void_p]
        buf = torch.zeros(b.n_clusters * 8, dtype=torch.int64, device="cuda")
        assert L.spx_debug_stamps(buf.data_ptr()) == 0
        if a.stamps_kernel == "bm":
            engine.bin_mean(b, out=bm)
        elif a.stamps_kernel == "fu":  # a -DSPX_STAMPS_FU build: 0 start, 1-3 after A/B/C, 4 bin-mean end,
            engine.bin_mean_medoid(b, out_bm=fbm, out_md=fmd, check=False)  # 5 rows, 6 after P4, 7 end
        elif a.stamps_kernel == "ga":
            engine.gap_average(b, out=ga)
        else:
            engine.medoid(b, out=md, check=False)
        torch.cuda.synchronize()
        L.spx_debug_stamps(None)
        s = buf.view(-1, 8).cpu().numpy().astype(np.float64)
        sizes = np.diff(b.host_cluster_off)
        ph = {}
        last = 6 if a.stamps_kernel == "bm" else 7
        # phases between consecutive stamps that the build records (a path may skip an index)
        present = [k for k in range(last + 1) if (s[:, k] > 0).any()]
        last = present[-1]
        ph = {}
        for k0, k1 in zip(present[:-1], present[1:]):
            ok = (s[:, k1] > 0) & (s[:, k0] > 0)
            if ok.any():
                ph[f"p{k0}->p{k1}"] = round(float(np.mean(s[ok, k1] - s[ok, k0])), 1)
        first = present[0]  # the gap-average build records no stamp 0 (-DSPX_GA_STAMP_MASK=0xFE)
        ok = (s[:, last] > 0) & (s[:, first] > 0)
        ph["lifetime"] = round(float(np.mean(s[ok, last] - s[ok, first])), 1)
        bands = {}
        for lo, hi in ((2, 10), (11, 25), (26, 40), (41, 50)):
            m = ok & (sizes >= lo) & (sizes <= hi)
            for k in present:
                m &= s[:, k] > 0
            if m.any():
                bands[f"n{lo}-{hi}"] = {f"p{k0}->p{k1}": round(float(np.mean(s[m, k1] - s[m, k0])), 1)
                                        for k0, k1 in zip(present[:-1], present[1:])}
        span = (s[ok, last].max() - s[ok, first].min())
        res["stamps"] = {"phases_cycles": ph, "by_size": bands, "span_cycles": span,
                         "cycles_per_cluster_per_cu": round(span * 256 / ok.sum(), 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
