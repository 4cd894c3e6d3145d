#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (or a rocpd results .db): spx:: kernels
(and the top others).

    python tools/kstats.py <kernel_stats.csv | run_results.db> [--csv out.csv]"""
import csv
import sys


def rows_of(path):
    if path.endswith(".db"):  # rocprofv3's default rocpd output: its top_kernels view
        import sqlite3

        con = sqlite3.connect(path)
        out = []
        # top_kernels reports microseconds; the kernels view's start/end are nanoseconds
        for name, calls, total, avg in con.execute("select name, total_calls, total_duration * 1000.0, "
                                                   "average * 1000.0 from top_kernels"):
            mn, mx = con.execute("select min(end - start), max(end - start) from kernels where name = ?",
                                 (name,)).fetchone() or (avg, avg)
            out.append({"Name": name, "Calls": calls, "TotalDurationNs": total, "AverageNs": avg,
                        "MinNs": mn if mn is not None else avg, "MaxNs": mx if mx is not None else avg})
        tot = sum(float(r["TotalDurationNs"]) for r in out) or 1.0
        for r in out:
            r["Percentage"] = 100.0 * float(r["TotalDurationNs"]) / tot
        return out
    return list(csv.DictReader(open(path)))


def main(path, top=8, csv_out=None):
    rows = rows_of(path)
    if csv_out:
        with open(csv_out, "w", newline="") as fh:
            w = csv.DictWriter(fh, ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            w.writeheader()
            for r in rows:
                w.writerow({k: r[k] for k in w.fieldnames})
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
    main(sys.argv[1], csv_out=sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None)
