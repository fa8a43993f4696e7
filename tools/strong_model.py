#!/usr/bin/env python3
"""
Predicted N-GPU strong scaling of ONE image from a one-GPU run of every
rank's stages (the 8-GPU node is the driver's, not ours):

* `--mode strips` (default): the north star's C4 split - 1G
  visibilities on ONE 16384^2 grid. `strips.invert_strips_local` runs all N
  ranks' stages on one GPU, in the distributed order, each on its own strip +
  halo buffer; every stage is synchronised and timed per rank. A rank owns a
  whole MI355X in the real run, so its stage times are its times there.
* `--mode wplanes`: the reference's w-stacking call on C3 (100M visibilities,
  8192^2 grid, epsilon 1e-4 -> W = 6) split by w-plane groups
  (`wplanes.invert_wplanes_local`): per-rank share times.
* `--mode wstrips`: the same call split by uv strips (every rank grids all w
  planes of its strip rows; per plane pass A, all-to-all, pass B with the w
  screen; `strips.invert_strips_local` with w-stacking parameters).

The exchanges are modelled at a per-link xGMI rate (MI355X: 7 links per GPU,
~153 GB/s each per direction, the prompt's figure; RCCL reaches a fraction of
it, so the model is given at --link-gbs values): strips - halo (W - 1 rows),
all-to-all of pass-A blocks (each rank sends (N - 1)/N of its H, one link per
peer), gather of image rows on rank 0 (N - 1 peers, one link each), with the run's
dependencies (a rank's pass A waits for its neighbours' grids and the halo,
the all-to-all for every pass A, the gather for every pass B);
wplanes - one reduce of the npix^2 fp64 image (a ring: 2 (N - 1)/N of it
per link, pipelined). Speed-up = the one-rank run's time / the predicted
step (step_ms_stage_max_sum: the looser bound summing each stage's max).

Writes one JSON line (stdout); run on the GPU box:
    python tools/strong_model.py --ranks 8 > profiles/r04_strong_model_c4.json
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"), str(ROOT)]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _avg(stage_lists):
    keys = sorted({k for st in stage_lists[0] for k in st})
    n = len(stage_lists)
    return [{k: sum(sl[r].get(k, 0.0) for sl in stage_lists) / n * 1e3 for k in keys}
            for r in range(len(stage_lists[0]))]


def strips_model(args):
    import torch

    from ska_sdp_cip_amd import _lib, strips
    from ska_sdp_cip_amd import synthetic as syn

    dev = torch.device("cuda", 0)
    rows, nchan, npix, seed = args.rows, 256, 8192, 20241008
    uvw_h = syn.uvw_tracks(rows, 64, array_radius_m=4000.0, seed=seed)
    freq_h = syn.channel_frequencies(nchan)
    px = syn.pixel_size_for_grid(uvw_h, freq_h, npix, support=8)
    uvw = torch.from_numpy(uvw_h).to(dev)
    freq = torch.from_numpy(freq_h).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    vis = torch.randn((rows, nchan), dtype=torch.complex64, device=dev, generator=g)
    wgt = torch.rand((rows, nchan), dtype=torch.float32, device=dev, generator=g) + 0.5
    params = _lib.choose_params(npix, npix, px, px, 1e-4, 8)
    out = {}
    for world in sorted({1, args.ranks}):
        layout = strips.plan_strips(uvw, freq, params, px, npix, npix, world,
                                    link_gbs=args.balance_link if args.balance_link > 0 else None)
        datas = []
        for r in range(world):
            rw, c0, c1 = strips.strip_slices(uvw, freq, params, px, *layout.rows(r))
            datas.append(strips.gather_strip(uvw, vis, wgt, rw, c0, c1))
        be = strips.HipStripBackend(params, px, px, npix, npix, device=dev, rows=strips.strip_buffer_rows(layout, 0))
        strips.invert_strips_local(datas, freq, layout, be)  # warm-up (workspaces, plans)
        torch.cuda.synchronize()
        runs, walls = [], []
        for _ in range(args.steps):
            st = []
            t0 = time.perf_counter()
            strips.invert_strips_local(datas, freq, layout, be, stages=st)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            runs.append(st)
        per_rank = _avg(runs)
        out[world] = {"per_rank_ms": [{k: round(v, 3) for k, v in pr.items()} for pr in per_rank],
                      "strip_rows": [layout.rows(r) for r in range(world)],
                      "strip_vis": [d.nvis for d in datas],
                      "buffer_rows": [strips.strip_buffer_rows(layout, r)[1] for r in range(world)],
                      "wall_ms_one_gpu": round(1e3 * sum(walls) / len(walls), 3)}
        log(f"[strips] world {world}: {out[world]['per_rank_ms']}")
        del datas, be
        torch.cuda.empty_cache()
    N = args.ranks
    pr = out[N]["per_rank_ms"]
    # pack / assemble: a sender's live-row compaction before the all-to-all and
    # a receiver's row scatter after it (the distributed run pays both; on the
    # critical path)
    stage_max = {k: max(p.get(k, 0.0) for p in pr) for k in ("grid", "halo", "rows", "pack", "assemble", "cols")}
    t1 = sum(out[1]["per_rank_ms"][0].get(k, 0.0) for k in ("grid", "rows", "cols"))
    H_bytes = [(npix // 4) * (b - a) * 4 * 16 for a, b in out[N]["strip_rows"]]  # each rank's pass-A output
    # what each rank sends in the (sparse) all-to-all: its live pass-A rows'
    # blocks for the other N - 1 ranks (invert_strips_local's count)
    send_bytes = [int(p.get("a2a_send_bytes", 0.0) * 1e-3) for p in out[N]["per_rank_ms"]]
    img_rows = npix // N
    models = {}
    for link in args.link_gbs:
        bw = link * 1e9
        halo_ms = 7 * params.nu * 16 / bw * 1e3
        # one link per peer: a rank's send bytes / (N - 1) per link
        a2a_ms = max(b / (N - 1) for b in send_bytes) / bw * 1e3 if N > 1 else 0.0
        gather_ms = img_rows * npix * 8 / bw * 1e3 if N > 1 else 0.0
        # the dependencies of the distributed run: rank r's pass A starts once
        # it and both neighbours have gridded (their halo rows) and the halo
        # is across; the all-to-all waits for every rank's pass A, pass B for
        # the all-to-all, the gather for every pass B
        g = [p.get("grid", 0.0) for p in pr]
        rows_end = [max(g[max(r - 1, 0):r + 2]) + (halo_ms if N > 1 else 0.0) + pr[r].get("rows", 0.0) +
                    pr[r].get("pack", 0.0) for r in range(N)]
        step = max(rows_end) + a2a_ms + stage_max["assemble"] + stage_max["cols"] + gather_ms
        # bench.py --strong's pipelined steps: step k's gather on the
        # communicator's stream during step k + 1's gridding (hidden while it is
        # shorter than the grid stage)
        step_ov = max(rows_end) + a2a_ms + stage_max["assemble"] + stage_max["cols"] + max(0.0, gather_ms - min(g))
        bound = (stage_max["grid"] + stage_max["rows"] + stage_max["pack"] + stage_max["assemble"] + stage_max["cols"] +
                 halo_ms + a2a_ms + gather_ms)
        models[f"{link:g}GB/s"] = {"halo_ms": round(halo_ms, 3), "alltoall_ms": round(a2a_ms, 3),
                                   "gather_ms": round(gather_ms, 3), "step_ms": round(step, 3),
                                   "step_ms_stage_max_sum": round(bound, 3),
                                   "speedup_vs_1": round(t1 / step, 2),
                                   "gvis_per_s": round(rows * nchan / step / 1e6, 1),
                                   "step_ms_gather_overlapped": round(step_ov, 3),
                                   "speedup_vs_1_gather_overlapped": round(t1 / step_ov, 2)}
    return {"mode": "strips", "balance_link_gbs": args.balance_link, "workload": f"C4: {rows:,} rows x {nchan} ch = {rows * nchan:,} vis, ONE "
                                          f"{params.nu}^2 grid, W = 8, 2-D, fp64",
            "ranks": N, "one_rank_ms": round(t1, 3), "stage_max_ms": {k: round(v, 3) for k, v in stage_max.items()},
            "model": models, "runs": out,
            "alltoall_bytes_per_rank_dense": H_bytes, "alltoall_send_bytes_per_rank": send_bytes,
            "gather_bytes_per_rank": img_rows * npix * 8}


def wplanes_model(args):
    import torch

    sys.path.insert(0, str(ROOT))
    import bench
    from ska_sdp_cip_amd import wplanes

    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    uvw, freq, vis, wgt, px, _, _ = bench.make_inputs(cfg, 0, 1, dev)
    npix = cfg["npix"]
    be = wplanes.HipWPlaneBackend(uvw, freq, vis, wgt, npix, npix, px, px, epsilon=1e-4,
                                  single_precision_accumulation=args.single)
    params = be.params()
    cost = wplanes.plane_cost(wplanes.plane_feeds(uvw, freq, params), params)
    out = {}
    for world in sorted({1, args.ranks}):
        split = wplanes.split_planes(cost, world, group=be.plane_group(params))
        wplanes.invert_wplanes_local(be, split)
        torch.cuda.synchronize()
        runs = []
        for _ in range(args.steps):
            st = []
            wplanes.invert_wplanes_local(be, split, stages=st)
            runs.append(st)
        out[world] = {"per_rank_ms": [{k: round(v, 3) for k, v in pr.items()} for pr in _avg(runs)],
                      "split": split, "share_cost": [round(float(cost[a:b].sum() / cost.sum()), 4)
                                                     for a, b in split]}
        log(f"[wplanes] world {world}: {out[world]}")
    N = args.ranks
    worst = max(p["grid"] for p in out[N]["per_rank_ms"])
    t1 = out[1]["per_rank_ms"][0]["grid"]
    models = {}
    for link in args.link_gbs:
        red_ms = 2 * (N - 1) / N * npix * npix * 8 / (link * 1e9) * 1e3 if N > 1 else 0.0
        step = worst + red_ms
        models[f"{link:g}GB/s"] = {"reduce_ms": round(red_ms, 3), "step_ms": round(step, 3),
                                   "speedup_vs_1": round(t1 / step, 2),
                                   "gvis_per_s": round(cfg["rows"] * cfg["nchan"] / step / 1e6, 1)}
    return {"mode": "wplanes", "workload": f"C3 reference call (epsilon 1e-4 -> W = {params.support}, "
                                           f"{params.nplanes} w planes, "
                                           f"{'packed single' if args.single else 'fp64'} class)",
            "ranks": N, "one_rank_ms": round(t1, 3), "worst_rank_ms": round(worst, 3), "model": models, "runs": out}


def wstrips_model(args):
    import torch

    sys.path.insert(0, str(ROOT))
    import bench
    from ska_sdp_cip_amd import strips, wplanes
    from ska_sdp_cip_amd.gridder import device_ms2dirty

    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    uvw, freq, vis, wgt, px, _, _ = bench.make_inputs(cfg, 0, 1, dev)
    npix = cfg["npix"]
    params = wplanes.HipWPlaneBackend(uvw, freq, vis, wgt, npix, npix, px, px, epsilon=1e-4,
                                      single_precision_accumulation=args.single).params()
    # the one-shot reference call on one GPU (synchronous calls)
    one = []
    for k in range(args.steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        device_ms2dirty(uvw, freq, vis, wgt, npix, npix, px, px, epsilon=1e-4, do_wstacking=True, normalise=True,
                        single_precision_accumulation=args.single)
        torch.cuda.synchronize()
        if k:
            one.append(time.perf_counter() - t0)
    one_ms = 1e3 * sum(one) / len(one)
    log(f"[wstrips] one-shot reference call {one_ms:.2f} ms")
    out = {}
    for world in sorted({1, args.ranks}):
        layout = strips.plan_strips(uvw, freq, params, px, npix, npix, world,
                                    link_gbs=args.balance_link if args.balance_link > 0 else None)
        datas = []
        for r in range(world):
            rw, c0, c1 = strips.strip_slices(uvw, freq, params, px, *layout.rows(r))
            datas.append(strips.gather_strip(uvw, vis, wgt, rw, c0, c1))
        be = strips.HipStripBackend(params, px, px, npix, npix, device=dev,
                                    rows=strips.strip_buffer_rows(layout, 0),
                                    single_precision_accumulation=args.single)
        strips.invert_strips_local(datas, freq, layout, be)
        torch.cuda.synchronize()
        runs = []
        for _ in range(args.steps):
            st = []
            strips.invert_strips_local(datas, freq, layout, be, stages=st)
            runs.append(st)
        out[world] = {"per_rank_ms": [{k: round(v, 3) for k, v in pr.items()} for pr in _avg(runs)],
                      "strip_rows": [layout.rows(r) for r in range(world)],
                      "strip_vis": [d.nvis for d in datas]}
        log(f"[wstrips] world {world}: {out[world]['per_rank_ms']}")
        del datas, be
        torch.cuda.empty_cache()
    N = args.ranks
    pr = out[N]["per_rank_ms"]
    stage_max = {k: max(p.get(k, 0.0) for p in pr) for k in ("grid", "rows", "pack", "assemble", "cols", "final")}
    t1 = sum(out[1]["per_rank_ms"][0].get(k, 0.0) for k in ("grid", "rows", "cols", "final"))
    nplanes, W, nu = int(params.nplanes), int(params.support), int(params.nu)
    # one plane's pass-A output as it crosses the all-to-all (complex64 for the packed class, strips._wire)
    H_bytes = [(npix // 4) * (b - a) * 4 * (8 if args.single else 16) for a, b in out[N]["strip_rows"]]
    # the sparse all-to-all's bytes per rank, summed over the planes (measured)
    send_bytes = [int(p.get("a2a_send_bytes", 0.0) * 1e-3) for p in out[N]["per_rank_ms"]]
    models = {}
    for link in args.link_gbs:
        bw = link * 1e9
        halo_ms = nplanes * (W - 1) * nu * 16 / bw * 1e3
        a2a_ms = max(b / (N - 1) for b in send_bytes) / bw * 1e3 if N > 1 else 0.0
        gather_ms = (npix // N) * npix * 8 / bw * 1e3 if N > 1 else 0.0
        # grid (+ halo) then the plane loop: each plane's pass A, all-to-all and
        # pass B in turn (the slowest rank's summed pass-A and pass-B times),
        # the final correction, the gather
        step = (stage_max["grid"] + halo_ms + stage_max["rows"] + stage_max["pack"] + a2a_ms + stage_max["assemble"] +
                stage_max["cols"] + stage_max["final"] + gather_ms)
        models[f"{link:g}GB/s"] = {"halo_ms": round(halo_ms, 3), "alltoall_ms": round(a2a_ms, 3),
                                   "gather_ms": round(gather_ms, 3), "step_ms": round(step, 3),
                                   "speedup_vs_one_shot": round(one_ms / step, 2),
                                   "speedup_vs_1_strip": round(t1 / step, 2),
                                   "gvis_per_s": round(cfg["rows"] * cfg["nchan"] / step / 1e6, 1)}
    return {"mode": "wstrips", "workload": f"C3 reference call by uv strips (epsilon 1e-4 -> W = {W}, {nplanes} "
                                           f"w planes, {'packed single' if args.single else 'fp64'} class)",
            "ranks": N, "one_shot_ms": round(one_ms, 3), "one_strip_ms": round(t1, 3),
            "stage_max_ms": {k: round(v, 3) for k, v in stage_max.items()}, "model": models, "runs": out,
            "alltoall_bytes_per_rank_dense": [nplanes * h for h in H_bytes], "alltoall_send_bytes_per_rank": send_bytes}


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[1])
    ap.add_argument("--mode", choices=("strips", "wplanes", "wstrips"), default="strips")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rows", type=int, default=3_906_250)
    ap.add_argument("--single", action="store_true")
    ap.add_argument("--link-gbs", type=float, nargs="+", default=[153.0, 64.0])
    ap.add_argument("--balance-link", type=float, default=0.0,
                    help="strips: the per-link rate plan_strips prices the all-to-all at (0: not priced)")
    args = ap.parse_args()
    res = {"strips": strips_model, "wplanes": wplanes_model, "wstrips": wstrips_model}[args.mode](args)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
