#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: spx:: kernels (and the top others)."""
import csv
import sys


def main(path, top=8):
    rows = list(csv.DictReader(open(path)))
    def short(n):
        return n.split("(")[0].replace("void ", "")[:70]
    spx = [r for r in rows if "spx::" in r["Name"]]
    other = [r for r in rows if "spx::" not in r["Name"]][:top]
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for group in (spx, other):
        for r in group:
            print(f"{short(r['Name']):70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.2f} "
                  f"{float(r['MinNs'])/1e3:9.2f} {float(r['MaxNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}")
        print("-" * 116)


if __name__ == "__main__":
    main(sys.argv[1])
