"""Concurrent kernel timeline of the pipelined steps in a rocprofv3 kernel trace: per step (scatter start
to the next scatter start on the caller's queue) the kernels >= MIN_US on every queue, and the
period statistics.  Usage: python tools/pipe_timeline.py TRACE.csv [SCATTER_SUBSTR] [MIN_US] [STEPS]"""
import csv
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "scatter_kernel"
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 15.0
nsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# pipelined steps: scatters whose call's planner ran on another queue
plan_q = {r["Queue_Id"] for r in rows if "plan_place_kernel" in r["Kernel_Name"]}
sc = [r for r in rows if pat in r["Kernel_Name"]]
caller_q = sc[-1]["Queue_Id"]
piped = []
for i in range(len(sc) - 1):
    a, b = int(sc[i]["Start_Timestamp"]), int(sc[i + 1]["Start_Timestamp"])
    places = [r for r in rows if "plan_place_kernel" in r["Kernel_Name"] and a <= int(r["Start_Timestamp"]) < b]
    if places and all(p["Queue_Id"] != sc[i]["Queue_Id"] for p in places):
        piped.append((a, b))
print(f"plan queues {sorted(plan_q)}, pipelined steps {len(piped)}")
if piped:
    per = sorted((b - a) / 1e3 for a, b in piped)
    print(f"period us: min {per[0]:.1f} median {per[len(per) // 2]:.1f} max {per[-1]:.1f}")
for a, b in piped[-nsteps:]:
    print(f"--- step {(b - a) / 1e3:.1f} us")
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e > a and s < b and (e - s) / 1e3 >= min_us:
            print(f"{(s - a) / 1e3:9.1f} {(e - a) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:58]}")
