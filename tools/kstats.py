"""Average duration per kernel (us) from a rocprofv3 --stats directory: kstats.py <name> <dir>"""
import csv
import sys
from pathlib import Path

name, d = sys.argv[1], sys.argv[2]
rows = []
for f in Path(d).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        rows.append((r["Name"].split("(")[0][:60], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
rows.sort(key=lambda t: -t[3])
print(f"== {name}")
for n, c, a, t in rows[:14]:
    print(f"  {n:60s} calls {c:5d} avg {a:9.1f} us")
