"""Print the spx:: kernel sequence of one bin-mean call from a rocprofv3 kernel trace:
python tools/kt_seq.py <trace.csv> <nth bin_mean_reg_kernel launch> [count]."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
spx = [r for r in rows if r["Kernel_Name"].startswith("spx::")]
idx = [i for i, r in enumerate(spx) if "bin_mean_reg_kernel" in r["Kernel_Name"]]
g = idx[int(sys.argv[2])]
end = idx[int(sys.argv[2]) + 1] if int(sys.argv[2]) + 1 < len(idx) else len(spx)
t0 = int(spx[g]["Start_Timestamp"])
for r in spx[g:end][:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f'{r["Kernel_Name"][5:42]:38s} {d:8.1f} us  at +{(int(r["Start_Timestamp"]) - t0) / 1e3:8.1f}')
