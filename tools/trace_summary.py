"""
Per-kernel average durations over the LAST n invert calls of a rocprofv3
kernel trace (the bench's timed steps; its warm-up calls, which run while the
GPU clocks ramp, are excluded), so the figures compare with bench.py's own
hipEvent timings of the same run.
Usage: python tools/trace_summary.py <kernel_trace.csv> <n_calls> [out.md]
"""
import csv
import sys
from collections import defaultdict


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # one invert call starts with freq_scale_kernel
    starts = [i for i, r in enumerate(rows) if "freq_scale_kernel" in r["Kernel_Name"]]
    first = starts[-n]
    dur = defaultdict(list)
    for r in rows[first:]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"# rocprofv3 kernel trace, last {n} invert calls of `{path}`", "",
             "| kernel | launches | avg us | min us | max us | total us / call |", "|---|---|---|---|---|---|"]
    for name, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{name[:70]}` | {len(d)} | {sum(d) / len(d):.1f} | {min(d):.1f} | {max(d):.1f} | "
                     f"{sum(d) / n:.1f} |")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
