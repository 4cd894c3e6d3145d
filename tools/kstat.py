"""Average duration (us) of named kernels in rocprofv3 kernel_stats / counter CSVs:
python tools/kstat.py <dir> [<dir> ...]."""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    out = []
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith("spx::") and float(r["AverageNs"]) > 20000:
                out.append(f'{r["Name"].split("(")[0][5:]}={float(r["AverageNs"]) / 1e3:.1f}')
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        agg = {}
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("spx::"):
                k = (r["Kernel_Name"].split("(")[0][5:], r["Counter_Name"])
                agg.setdefault(k, []).append(float(r["Counter_Value"]))
        for (k, c), vals in sorted(agg.items()):
            if max(vals) > 1e5:
                out.append(f"{k}.{c}={sum(vals) / len(vals):.4g}")
    print(os.path.basename(d.rstrip("/")), " ".join(out))
