#!/usr/bin/env python3
"""
Experiment: S inverts in flight on ONE GPU (S host threads, each with its own
HIP stream and its own libcip_hip workspace), C3 workload. The planner of one
call is latency-bound and the scatter of another LDS-bound, so the GPU can
overlap them. Prints one JSON line (whole-job throughput of steps*S inverts).
"""

import argparse
import json
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20, help="inverts per stream")
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import torch

    from ska_sdp_cip_amd import gridder
    from ska_sdp_cip_amd.distributed import image_buffer

    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    cfg = bench.CONFIGS["c3"]
    npix = cfg["npix"]
    nvis = cfg["rows"] * cfg["nchan"]
    uvw_d, freq_d, vis_d, wgt_d, px, _, _ = bench.make_inputs(cfg, 0, 1, device)
    bufs = [image_buffer(npix, npix, device) for _ in range(args.streams)]
    start = threading.Barrier(args.streams + 1)
    errors = []

    def worker(k):
        try:
            torch.cuda.set_device(device)
            st = torch.cuda.Stream(device=device)
            dirty, sumw = bufs[k]
            with torch.cuda.stream(st):
                def one():
                    gridder.device_ms2dirty(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, support=8,
                                            out=dirty, sum_weights=sumw)
                    dirty.div_(sumw)
                for _ in range(args.warmup):
                    one()
                st.synchronize()
                start.wait()
                for _ in range(args.steps):
                    one()
                st.synchronize()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))
            start.abort()

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(args.streams)]
    for t in threads:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if errors:
        raise RuntimeError(errors)
    n = args.steps * args.streams
    print(json.dumps({"metric": "Mvis/s gridded (invert), concurrent inverts on one GPU", "streams": args.streams,
                      "value": round(nvis * n / dt / 1e6, 1), "unit": "Mvis/s", "inverts": n,
                      "ms_per_invert": round(dt / n * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
