#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value
per dispatch for each kernel, plus per-wave figures (profiling aid).

    python tools/pmc_summary.py gpurun_out/pmc [--json out.json]

FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3; `hbm_bytes` converts
(x1024) and applies the gfx950 read correction of MI355X_MICROARCH.md (HBM
section): FETCH_SIZE counts half the bytes of a coalesced streaming read, so it
is doubled.  Calibrated on our own access pattern: bin_mean_stream_kernel reads
every m/z and intensity exactly once (8-B lanes, 8.31 GB algorithmic) and
FETCH_SIZE x 2 = 8.45 GB.  With --json, writes {kernel_short_name: bytes_per_launch} for the
FETCH_SIZE + WRITE_SIZE pair (profiles/pmc_traffic.json format read by bench.py).
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    return name.split("(")[0].replace("spx::", "").replace("void ", "")


def load(root, only=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        if only and not os.path.basename(f).startswith(only):
            continue
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Kernel_Name"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (_d, k), cs in per.items():
            for c, v in cs.items():
                acc[short(k)][c].append(v)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--only", help="only counter files whose name starts with this prefix")
    ap.add_argument("--peaks-from", help="log whose last JSON line holds the profiled batch's 'peaks' "
                                         "(stored as '_peaks' so bench.py can rescale)")
    a = ap.parse_args()
    acc = load(a.root, a.only)
    traffic = {}
    for k, cs in sorted(acc.items()):
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}")
        waves = mean.get("SQ_WAVES")
        for c in sorted(mean):
            extra = ""
            if waves and c.startswith("SQ_INSTS"):
                extra = f"   ({mean[c] / waves:.1f} / wave)"
            print(f"   {c:28s} {mean[c]:16.1f}{extra}")
        if "SQ_WAVE_CYCLES" in mean:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in mean:
                    print(f"   {c} / WAVE_CYCLES = {mean[c] / mean['SQ_WAVE_CYCLES']:.3f}")
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            traffic[k] = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
            print(f"   hbm_bytes (fetch+write)      {traffic[k]:16.0f}")
    if a.json:
        if a.peaks_from:
            for line in reversed(open(a.peaks_from).read().splitlines()):
                if line.startswith("{"):
                    traffic["_peaks"] = json.loads(line)["peaks"]
                    break
        with open(a.json, "w") as fh:
            json.dump(traffic, fh, indent=1)


if __name__ == "__main__":
    main()
