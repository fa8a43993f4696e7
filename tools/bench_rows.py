#!/usr/bin/env python3
"""
Secondary measurements of the SURVEY.md 8(f) rows built beside the hot path
(bench.py keeps the contract's one JSON line for the headline metric):

  --mode stream     invert_measurement_set_streamed: raw (rows, chans, 4)
                    columns in HOST memory, staged through pinned buffers to
                    HBM on a copy stream while the previous chunk grids
                    (PCIe-inclusive; row 2, config C5's host->HBM streaming)
  --mode continuum  continuum_invert: Stokes I, Q, U, V dirty images + PSF on
                    a mosaic of facets (row 4, config C5's products) from
                    device-resident raw columns

Each prints one JSON line (synthetic data: real uvw tracks, random values).
"""

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("stream", "continuum"), required=True)
    ap.add_argument("--rows", type=int, default=156_250)
    ap.add_argument("--nchan", type=int, default=64)
    ap.add_argument("--npix", type=int, default=2048)
    ap.add_argument("--rows-per-chunk", type=int, default=32_768)
    ap.add_argument("--facets", type=int, default=2, help="facets per axis (continuum)")
    ap.add_argument("--facets-xy", type=int, nargs=2, default=None, help="continuum: facets along x and y")
    ap.add_argument("--world", type=int, default=1,
                    help="continuum: time rank 0's share of the facets of a `world`-GPU run (k %% world == 0)")
    ap.add_argument("--refcall", action="store_true",
                    help="continuum: the reference's gridder call (epsilon 1e-4, w-stacking, float class) "
                         "instead of 2-D support 8 fp64")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--no-reuse", action="store_true", help="continuum: plan every product (no CIP_REUSE_PLAN)")
    args = ap.parse_args()

    import torch

    from ska_sdp_cip_amd import synthetic as syn

    ms = syn.make_measurement_set(args.rows, args.nchan, n_ant=64, array_radius_m=4000.0, cheap_visibilities=True)
    uvw, freq = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, freq, args.npix, support=8)
    asec = float(np.degrees(np.arcsin(px)) * 3600.0)
    nvis = args.rows * args.nchan
    out = {"data": "synthetic (real uvw tracks, random complex64 values, 4 pols, 5% flagged)",
           "rows": args.rows, "channels": args.nchan, "npix": args.npix, "visibilities": nvis}
    if args.mode == "stream":
        from ska_sdp_cip_amd.streaming import invert_measurement_set_streamed

        run = lambda: invert_measurement_set_streamed(ms, args.npix, asec,  # noqa: E731
                                                      rows_per_chunk=args.rows_per_chunk, support=8)
        run()  # warm-up: workspace, pinned slots, FFT tables
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.repeat):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.repeat
        host_bytes = nvis * (8 * 4 + 1 * 4 + 4 * 4) + args.rows * 24
        out.update(metric="Mvis/s streamed host->HBM + invert (2-D, support 8)", value=round(nvis / dt / 1e6, 1),
                   unit="Mvis/s", ms_per_call=round(dt * 1e3, 2), host_bytes=host_bytes,
                   host_to_device_GBs=round(host_bytes / dt / 1e9, 1), rows_per_chunk=args.rows_per_chunk)
    else:
        from ska_sdp_cip_amd.continuum import continuum_invert, facet_centres

        dev = torch.device("cuda", 0)
        t = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a if dt is None else a.astype(dt))).to(dev)  # noqa
        cols = (t(ms.visibilities()), t(ms.flags(), np.uint8), t(ms.weights()), t(uvw), t(freq))
        fx, fy = args.facets_xy or (args.facets, args.facets)
        facets = facet_centres(fx, fy, args.npix, px)
        call = (dict(epsilon=1e-4, do_wstacking=True, single_precision_accumulation=True) if args.refcall else
                dict(support=8, do_wstacking=False))
        run = lambda: continuum_invert(*cols, args.npix, asec, facets=facets, stokes="IQUV",  # noqa: E731
                                       psf=True, rank=0, world=args.world, reuse_plans=not args.no_reuse, **call)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.repeat):
            res = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.repeat
        nimg = len(res)
        mode = ("the reference's call: epsilon 1e-4, w-stacking, float class" if args.refcall else
                "2-D, support 8, fp64")
        out.update(metric=f"continuum products: Stokes IQUV + PSF per facet ({mode})", world=args.world,
                   value=round(nimg / dt, 2), unit="images/s", images=nimg, facets=len(facets),
                   facets_this_rank=nimg // 5,
                   ms_per_call=round(dt * 1e3, 2), mvis_per_s_per_image=round(nvis * nimg / dt / 1e6, 1),
                   reuse_plans=not args.no_reuse)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
