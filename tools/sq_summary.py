"""Per-kernel averages of rocprofv3 --pmc SQ counter runs: python tools/sq_summary.py <dir>..."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].split("(")[0][:70]
            vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    if not any(s in k for s in ("scatter_kernel", "scatter_pair", "lds_pattern", "order_kernel", "plan_place", "fft_", "radix")):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")
