"""Timeline of one call from a rocprofv3 kernel trace: every spx:: kernel between the
nth launch of <first kernel> and the next, with its start / end relative to that launch
and its queue (stream), so overlap between streams shows:
python tools/kt_timeline.py <trace.csv> <first kernel substring> <nth>."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
spx = [r for r in rows if "spx::" in r["Kernel_Name"]]
idx = [i for i, r in enumerate(spx) if sys.argv[2] in r["Kernel_Name"]]
n = int(sys.argv[3])
t0 = int(spx[idx[n]]["Start_Timestamp"])
t1 = int(spx[idx[n + 1]]["Start_Timestamp"]) if n + 1 < len(idx) else None
qk = "Queue_Id" if "Queue_Id" in spx[0] else ("Stream_Id" if "Stream_Id" in spx[0] else None)
last = t0
for r in spx:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 - 200_000 or (t1 is not None and s >= t1):
        continue
    last = max(last, e)
    q = r[qk] if qk else "?"
    print(f'q{q:>3} {r["Kernel_Name"][5:48]:44s} {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f} us  ({(e - s) / 1e3:7.1f})')
print(f"span {(last - t0) / 1e3:.1f} us")
