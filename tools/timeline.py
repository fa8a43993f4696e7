"""Print the kernel timeline of the last complete invert in a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/r01_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "freq_scale_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:8.1f} q{r.get('Queue_Id','')} {r['Kernel_Name'][:60]}")
    prev = max(prev or 0, e)
print(f"total {(prev - t0) / 1e3:.1f} us")
