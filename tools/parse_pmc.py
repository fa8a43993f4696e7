"""
Summarise rocprofv3 --pmc runs (one counter per pass) into per-kernel
averages and write profiles/traffic_<config>.json for bench.py's
roofline.traffic. gfx950 corrections (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE (KB) counts exactly half the bytes of wide coalesced reads -> x2;
WRITE_SIZE (KB) reads the bytes exactly for 16-B stores and float atomics.
Usage: python tools/parse_pmc.py <round> <config> <dir>...
Only full-size dispatches are averaged: a dispatch whose counter is below a
quarter of the kernel's largest (a max|err| sample call on 1/50 of the rows,
say) is dropped and counted. Rounds 3 and 4 averaged such a sample into the
per-launch figures (10 dispatches, one of them 2M visibilities): their
scatter / order / place reads read 10 % low (profiles/r06_pmc_delta.md).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    """The kernel's unqualified identifier ("cip::radix_scatter_kernel(...)" ->
    "radix_scatter_kernel"; template arguments dropped). Exact names: a
    substring match would lump radix_scatter_kernel into scatter_kernel."""
    base = name.split("(")[0].split("<")[0].strip().split()[-1]
    return base.split("::")[-1]


def main():
    rnd, config, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in Path(d).glob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    lines = [f"# PMC summary {rnd} ({config}); per-dispatch averages", "",
             "| kernel | dispatches | FETCH_SIZE KB (raw) | HBM read bytes (x2) | WRITE_SIZE KB | TCC_EA0_ATOMIC |",
             "|---|---|---|---|---|---|"]
    dropped = {}
    for k, cs in list(vals.items()):
        for c, v in cs.items():
            top = max(v) if v else 0.0
            keep = [x for x in v if x >= 0.25 * top] if top > 0 else v
            if len(keep) < len(v):
                dropped[f"{k}/{c}"] = len(v) - len(keep)
            cs[c] = keep
    for k, cs in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("FETCH_SIZE", [0]))):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        rd = 2 * avg.get("FETCH_SIZE", 0.0) * 1024
        wr = avg.get("WRITE_SIZE", 0.0) * 1024
        out[k] = {"dispatches": n, "fetch_kb_raw": avg.get("FETCH_SIZE"), "hbm_read_bytes": rd,
                  "write_kb": avg.get("WRITE_SIZE"), "hbm_write_bytes": wr,
                  "atomic_requests": avg.get("TCC_EA0_ATOMIC_sum")}
        lines.append(f"| {k} | {n} | {avg.get('FETCH_SIZE', 0):.0f} | {rd:.3e} | {avg.get('WRITE_SIZE', 0):.0f} | "
                     f"{avg.get('TCC_EA0_ATOMIC_sum', 0):.3e} |")
    sc = out.get("scatter_kernel")
    if sc:
        traffic = {"kernel": "cip::scatter_kernel", "round": rnd,
                   "hbm_bytes_per_launch": int(sc["hbm_read_bytes"] + sc["hbm_write_bytes"]),
                   "hbm_read_bytes_per_launch": int(sc["hbm_read_bytes"]),
                   "hbm_write_bytes_per_launch": int(sc["hbm_write_bytes"]),
                   "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads); WRITE_SIZE as reported",
                   "source": f"profiles/{rnd}_pmc_summary.md"}
        Path("profiles").mkdir(exist_ok=True)
        Path(f"profiles/traffic_{config}.json").write_text(json.dumps(traffic, indent=1))
    if dropped:
        lines += ["", "Dropped small dispatches (below 1/4 of the kernel's largest): " +
                  ", ".join(f"{k} x{n}" for k, n in sorted(dropped.items()))]
    Path(f"profiles/{rnd}_pmc_summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
