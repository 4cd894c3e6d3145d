#!/usr/bin/env python3
"""Per-call HBM traffic and kernel times of the off-shape runs (tools/gpu/shapes_pmc.sh):

    python tools/shapes_traffic.py gpurun_out/shapes_pmc

Each <which>_<shape>/ directory holds a FETCH_SIZE pass (f/), a WRITE_SIZE pass (w/)
and a kernel trace (kt/) of tools/run_shape.py (one checked call + 3 timed calls).
Bytes per call = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 summed over every spx::
dispatch, divided by the calls (the gfx950 read correction of tools/pmc_summary.py).
Prints a table and writes <root>/pmc_traffic_shapes.json ({"bm_skewed_config3": bytes, ...}),
the format bench.py reads from profiles/pmc_traffic_shapes.json."""
import collections
import csv
import glob
import json
import os
import sys

CALLS = 4  # tools/run_shape.py: the first call + 3 reps


def counter_sum(d, name):
    tot = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"][5:] if r["Kernel_Name"].startswith("void ") else r["Kernel_Name"]  # templates
            if kn.startswith("spx::") and r["Counter_Name"] == name:
                tot[kn.split("(")[0][5:]] += float(r["Counter_Value"])
    return tot


def main(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*_*"))):
        if not os.path.isdir(d):
            continue
        key = os.path.basename(d)
        f, w = counter_sum(os.path.join(d, "f"), "FETCH_SIZE"), counter_sum(os.path.join(d, "w"), "WRITE_SIZE")
        per_k = {k: (2.0 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024.0 / CALLS for k in set(f) | set(w)}
        out[key] = sum(per_k.values())
        times = {}
        for s in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(s)):
                kn = r["Name"][5:] if r["Name"].startswith("void ") else r["Name"]  # templates
                if kn.startswith("spx::"):
                    times[kn.split("(")[0][5:]] = (float(r["TotalDurationNs"]) / CALLS / 1e3)
        print(f"== {key}: {out[key] / 1e9:.3f} GB per call")
        for k in sorted(set(per_k) | set(times), key=lambda k: -times.get(k, 0.0)):
            if per_k.get(k, 0.0) > 1e6 or times.get(k, 0.0) > 5.0:
                print(f"   {k:36s} {times.get(k, 0.0):9.1f} us  {per_k.get(k, 0.0) / 1e9:8.3f} GB")
    with open(os.path.join(root, "pmc_traffic_shapes.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
