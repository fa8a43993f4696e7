"""Time overlap between kernel classes in a rocprofv3 kernel trace:
overlap.py <kernel_trace.csv> <substrA> <substrB> -> fraction of A's busy time
during which some B kernel also runs."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
a_key, b_key = sys.argv[2], sys.argv[3]
A = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if a_key in r["Kernel_Name"])
B = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if b_key in r["Kernel_Name"])
tot = sum(e - s for s, e in A)
ov = 0
j = 0
for s, e in A:
    for bs, be in B:
        if be <= s or bs >= e:
            continue
        ov += min(e, be) - max(s, bs)
print(f"{a_key}: {len(A)} kernels, busy {tot / 1e6:.2f} ms, overlapped by {b_key}: {ov / 1e6:.2f} ms ({ov / max(tot, 1):.1%})")
