#!/usr/bin/env python3
"""
Benchmark of the invert hot path (BASELINE.json metric): Mvis/s gridded
(invert) on an 8k^2 grid with kernel support 8, fp64 accumulation.

Workload (default `--config c3`; `--config c4` is one
GPU's shard of C4, 125M visibilities -> 16384^2 grid): 390,625 rows x 256
channels = 100M synthetic visibilities per GPU (MeerKAT-like 64-antenna
earth-rotation uvw tracks, 856-1712 MHz; complex64 visibilities and float32
weights with 5 % zero (flagged) weights, as the reference passes them to the
gridder, invert.py:170-183) -> 8192 x 8192 grid (4096^2 image, sigma = 2),
2-D mode. One step = one full `cip_ms2dirty` call on device-resident inputs:
sum-of-weights / scale reduction, device tile plan (bucket + sort + chunking),
fp64-accumulating scatter, 8192^2 c2c FFT, grid correction + crop; with
N > 1 GPUs each rank inverts its own 100M-visibility shard of a longer
observation (weak scaling) and the partial dirty images and weight sums are
reduced to rank 0 over RCCL (no other collective exists on this path).

Prints ONE JSON line (rank 0). `roofline` is for the dominant kernel (the
scatter), timed with hipEvents recorded by libcip_hip on the stream it launches
on; `cpu_baseline` times a tiled fp64 CPU restatement of ducc0's gridder
(oracle/cpu_baseline.c) on the whole workload (plus C1, C2 and the numpy
Stokes-I prep); `max_err` is the dirty image's max |GPU - CPU oracle| / sum w
on a row subset at the full grid (the metric's second half).
"""

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT / "ska-sdp-continuum-imaging-pipeline_amd", ROOT / "oracle"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402

CONFIGS = {
    # name: rows, channels, image pixels (grid = 2x), antennas, array radius (m)
    "c1": dict(rows=10_000, nchan=1, npix=128, n_ant=16, radius=1000.0),
    "c2": dict(rows=156_250, nchan=64, npix=2048, n_ant=64, radius=4000.0),
    "c3": dict(rows=390_625, nchan=256, npix=4096, n_ant=64, radius=4000.0),
    # C4's per-GPU shard (BASELINE configs[3]: 1G vis -> 16k^2 grid on 8 GPUs):
    # 3,906,250 / 8 rows x 256 ch = 125M vis/GPU -> 16384^2 grid (8192^2 image)
    "c4": dict(rows=488_282, nchan=256, npix=8192, n_ant=64, radius=4000.0),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_raw_columns(cfg, rank, device, seed=20241008):
    """Device-resident raw linear-feed columns of this rank's shard for
    `--raw`: vis4 (rows, nchan, 4) complex64 XX, XY, YX, YY, wgt4 float32 in
    [0.5, 1.5) and flags4 uint8 with 5 % of the XX and YY entries flagged (as
    an MS holds them; the gridder forms Stokes I on load)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed + 1000 + rank)
    shape = (cfg["rows"], cfg["nchan"], 4)
    vis4 = torch.randn(shape, dtype=torch.complex64, device=device, generator=g)
    wgt4 = torch.rand(shape, dtype=torch.float32, device=device, generator=g) + 0.5
    flags4 = (torch.rand(shape, dtype=torch.float32, device=device, generator=g) < 0.025).to(torch.uint8)
    return vis4, flags4, wgt4


def make_inputs(cfg, rank, world, device, seed=20241008):
    """Device-resident gridder inputs of this rank's shard."""
    import torch

    from ska_sdp_cip_amd import synthetic as syn

    rows = cfg["rows"]
    uvw_all = syn.uvw_tracks(rows * world, cfg["n_ant"], array_radius_m=cfg["radius"], seed=seed)
    freq = syn.channel_frequencies(cfg["nchan"])
    px = syn.pixel_size_for_grid(uvw_all, freq, cfg["npix"], support=8)
    uvw = np.ascontiguousarray(uvw_all[rank * rows:(rank + 1) * rows])
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    vis = torch.randn((rows, cfg["nchan"]), dtype=torch.complex64, device=device, generator=g)
    wgt = torch.rand((rows, cfg["nchan"]), dtype=torch.float32, device=device, generator=g) + 0.5
    flags = torch.rand((rows, cfg["nchan"]), dtype=torch.float32, device=device, generator=g) < 0.05
    wgt = torch.where(flags, torch.zeros_like(wgt), wgt).contiguous()
    t = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
    return t(uvw), t(freq), vis, wgt, px, uvw, freq


def traffic_from_profiles(config):
    """Per-launch HBM bytes of the scatter from committed PMC summaries, if any."""
    p = ROOT / "profiles" / f"traffic_{config}.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())
    except (OSError, ValueError):
        return None


def _cpu_info():
    """CPU model, os.cpu_count() and the affinity set of this process."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo", encoding="ascii", errors="replace") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}


def _cgroup_cpu_max():
    """The process's cgroup-v2 CPU quota ("max 100000" = none), if readable."""
    try:
        return Path("/sys/fs/cgroup/cpu.max").read_text().strip()
    except OSError:
        return None


def cpu_baseline(cfg_name, uvw_h, freq_h, vis_h, wgt_h, px, support, nthreads):
    """
    CPU baseline (BASELINE.md "CPU baseline plan"), timed on this host in this
    run: oracle/cpu_baseline.c - the tiled fp64 restatement of ducc0's CPU
    design (ducc0 itself is not importable on the box) - + threaded scipy FFT
    + crop + correction, i.e. one whole 2-D invert:
    * C1 and C2 in full on their own synthetic inputs (same generator as the
      GPU configs), and the benchmark's own workload in full on exactly the
      GPU run's visibilities (copied to the host);
    * the reference's numpy Stokes-I / effective-weight prep
      (StokesIGridderInput, invert.py:78-116, restated in oracle.stokes_i) on
      C2's (rows, 64, 4) polarisation columns.
    `value` is the benchmark workload's full-size rate (no extrapolation).
    """
    import oracle
    from ska_sdp_cip_amd import synthetic as syn

    def run_threads(uvw, freq, vis, wgt, npix, pxx, nth):
        oracle.baseline_ms2dirty(uvw[:64], freq, vis[:64], wgt[:64], npix, npix, pxx, pxx, support, nth)
        t0 = time.perf_counter()
        oracle.baseline_ms2dirty(uvw, freq, vis, wgt, npix, npix, pxx, pxx, support, nth)
        return time.perf_counter() - t0

    def run(uvw, freq, vis, wgt, npix, pxx):
        return run_threads(uvw, freq, vis, wgt, npix, pxx, nthreads)

    def synth(name):
        c = CONFIGS[name]
        uvw = syn.uvw_tracks(c["rows"], c["n_ant"], array_radius_m=c["radius"])
        freq = syn.channel_frequencies(c["nchan"])
        pxx = syn.pixel_size_for_grid(uvw, freq, c["npix"], support=8)
        rng = np.random.default_rng(1)
        shape = (c["rows"], c["nchan"])
        vis = (rng.standard_normal(shape, dtype=np.float32)
               + 1j * rng.standard_normal(shape, dtype=np.float32)).astype(np.complex64)
        wgt = rng.uniform(0.5, 1.5, shape).astype(np.float32)
        wgt[rng.uniform(size=shape) < 0.05] = 0.0
        return uvw, freq, vis, wgt, pxx

    per = {}
    for name in ("c1", "c2"):
        if name == cfg_name:
            continue
        uvw, freq, vis, wgt, pxx = synth(name)
        t = run(uvw, freq, vis, wgt, CONFIGS[name]["npix"], pxx)
        per[name] = {"mvis_per_s": round(vis.size / t / 1e6, 2), "seconds": round(t, 3), "nvis": int(vis.size)}
    t = run(uvw_h, freq_h, vis_h, wgt_h, CONFIGS[cfg_name]["npix"], px)
    per[cfg_name] = {"mvis_per_s": round(vis_h.size / t / 1e6, 2), "seconds": round(t, 3),
                     "nvis": int(vis_h.size), "inputs": "the GPU run's own visibilities"}
    # BASELINE.md's plan: threads = os.cpu_count(); the headline above uses
    # the box's CPU share for one GPU (16), this is the same full workload
    # with every core the OS reports (the cgroup quota, if any, still applies)
    all_threads = os.cpu_count() or nthreads
    all_cores = None
    if all_threads != nthreads:
        t_all = run_threads(uvw_h, freq_h, vis_h, wgt_h, CONFIGS[cfg_name]["npix"], px, all_threads)
        all_cores = {"threads": all_threads, "mvis_per_s": round(vis_h.size / t_all / 1e6, 2),
                     "seconds": round(t_all, 3), "cgroup_cpu_max": _cgroup_cpu_max(),
                     "what": f"the same full {cfg_name.upper()} invert with os.cpu_count() threads"}
    # the reference's Stokes-I prep in numpy on C2-shaped polarisation columns
    c2 = CONFIGS["c2"]
    rng = np.random.default_rng(2)
    shape4 = (c2["rows"], c2["nchan"], 4)
    vis4 = (rng.standard_normal(shape4, dtype=np.float32)
            + 1j * rng.standard_normal(shape4, dtype=np.float32)).astype(np.complex64)
    w4 = rng.uniform(0.5, 1.5, shape4).astype(np.float32)
    f4 = rng.uniform(size=shape4) < 0.05
    t0 = time.perf_counter()
    oracle.stokes_i(vis4, f4, w4)
    t_st = time.perf_counter() - t0
    n_st = c2["rows"] * c2["nchan"]
    del vis4, w4, f4
    return {
        "value": per[cfg_name]["mvis_per_s"],
        "unit": "Mvis/s",
        "cores": nthreads,
        "kind": "port",
        "sample": (f"full {cfg_name.upper()} invert ({vis_h.size:,} vis, 2-D, support {support}) by "
                   "oracle/cpu_baseline.c: tiled fp64 restatement of ducc0's CPU gridder (ducc0 absent on the box) "
                   f"+ scipy.fft ({nthreads} workers) + correction; C1/C2 in full on their own inputs"),
        "configs": per,
        "stokes_i_prep": {"mvis_per_s": round(n_st / t_st / 1e6, 2), "seconds": round(t_st, 3),
                          "nvis": n_st, "what": "numpy StokesIGridderInput + effective_weights "
                                                "(invert.py:78-116) on C2 (rows, 64, 4) columns, 1 thread"},
        "all_cores": all_cores,
        **_cpu_info(),
        "threads_note": ("value: threads = the box's CPU share for one GPU (OMP_NUM_THREADS); all_cores: the same "
                         "workload with os.cpu_count() threads (BASELINE.md's plan)"),
    }


def max_err_vs_oracle(uvw_h, freq_h, vis_h, wgt_h, npix, px, support, wstacking, single, nthreads, row_step,
                      device):
    """
    Dirty-image max |GPU - CPU oracle| / sum w (BASELINE.json metric, second
    half) on every `row_step`-th row of the benchmark's own inputs at its full
    grid: the GPU through the product path (device_ms2dirty), the CPU through
    the fp64 oracle (oracle/, the parity checker). Outside the timed region.
    """
    import torch

    import oracle
    from ska_sdp_cip_amd import gridder

    uvw = np.ascontiguousarray(uvw_h[::row_step])
    vis = np.ascontiguousarray(vis_h[::row_step])
    wgt = np.ascontiguousarray(wgt_h[::row_step])
    t = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
    img, _ = gridder.device_ms2dirty(t(uvw), t(freq_h), t(vis), t(wgt), npix, npix, px, px, support=support,
                                     do_wstacking=wstacking, single_precision_accumulation=single)
    got = img.cpu().numpy()
    del img
    ref = oracle.ms2dirty(uvw, freq_h, vis, wgt, npix, npix, px, px, support=support, do_wstacking=wstacking,
                          nthreads=nthreads)
    err = float(np.abs(got - ref).max() / wgt.astype(np.float64).sum())
    return {"max_err": err, "gate": 1e-6,
            "sample": f"rows [::{row_step}] of the benchmark inputs ({vis.size:,} vis) at the full "
                      f"{npix}^2 image, GPU (cip_ms2dirty) vs fp64 CPU oracle, both / sum w"}


def run_strong(args, world, rank, device, steps=None, warmup=None):
    """
    `--strong`: the north star's C4 split (BASELINE configs[3]) - ONE dirty
    image of 3,906,250 rows x 256 channels = 1,000,000,000 visibilities on a
    16384^2 grid (8192^2 image) shared by all ranks (strong scaling: the total
    work is fixed). Rank r grids the visibilities whose footprints start in
    its balanced uv strip of grid rows, sends its W - 1 halo rows to rank
    r + 1 (RCCL point-to-point), runs pass A of the FFT on its rows, one
    all-to-all hands every rank its image rows' columns, pass B + correction
    run per image-row strip and the rows are gathered on rank 0
    (ska_sdp_cip_amd.strips). One step = that whole distributed
    invert on HBM-resident strip data; value = 1G vis x steps / time.
    """
    import torch
    import torch.distributed as dist

    from ska_sdp_cip_amd import _lib, strips
    from ska_sdp_cip_amd import synthetic as syn

    seed = 20241008
    rows, nchan, npix = 3_906_250, 256, 8192
    uvw_h = syn.uvw_tracks(rows, 64, array_radius_m=4000.0, seed=seed)
    freq_h = syn.channel_frequencies(nchan)
    px = syn.pixel_size_for_grid(uvw_h, freq_h, npix, support=8)
    uvw = torch.from_numpy(uvw_h).to(device)
    freq = torch.from_numpy(freq_h).to(device)
    params = _lib.choose_params(npix, npix, px, px, 1e-4, args.support)
    # the MS's dense (rows, nchan) columns, resident: counter-based values -
    # every visibility's value and weight are a pure function of its global
    # (row, channel) index, so every rank count grids the SAME 1G visibilities
    # into the same image (parity across N)
    r_all = torch.arange(rows, device=device)
    vis_all, wgt_all = syn.counter_columns_slices(r_all, torch.zeros_like(r_all), torch.full_like(r_all, nchan), nchan,
                                                  seed)
    del r_all
    # the strip split on the device (cip_strips.hip): the per-row cost
    # histogram -> balanced strip bounds, then this rank's row slices with its
    # visibilities and weights gathered into the Tile layout (the reference's
    # offline reorder_by_uvw_tile step, cut by strip) - once per data set,
    # timed and reported as plan_ms
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    layout = strips.plan_strips(uvw, freq, params, px, npix, npix, world)
    data = strips.split_strip(uvw, freq, vis_all, wgt_all, params, px, *layout.rows(rank))
    torch.cuda.synchronize()
    t_plan = time.perf_counter() - t0
    del vis_all, wgt_all, uvw
    torch.cuda.empty_cache()
    vis, wgt = data.vis, data.wgt
    nvis = data.nvis
    # this rank's strip + W - 1 halo rows only (1/N of the grid per rank)
    backend = strips.HipStripBackend(params, px, px, npix, npix, device=device,
                                     rows=strips.strip_buffer_rows(layout, rank))
    y0, y1 = layout.rows(rank)
    log(f"[bench --strong] rank {rank}/{world}: strip rows [{y0}, {y1}) of {params.nv}, {nvis:,} vis "
        f"({data.slice_uvw.shape[0]:,} slices), strip plan + split {t_plan * 1e3:.1f} ms")

    # step k's image-row gather runs on the communicator's stream while step
    # k + 1 grids (its buffers are not touched by the next step); it is waited
    # for before step k + 2 and after the last step, inside the timed region
    pending = [None]

    def step(stages=None):
        if stages is not None:  # profiled steps: every stage synchronised
            return strips.invert_strips(data, freq, layout, backend, dst=0, stages=stages)
        prev = pending[0]
        pending[0] = strips.invert_strips(data, freq, layout, backend, dst=0, gather_async=True)
        if prev is not None:
            prev.wait()
        return None

    def drain():
        img_last = pending[0].wait() if pending[0] is not None else None
        pending[0] = None
        return img_last

    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    for _ in range(warmup):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = {}
    nprof = max(2, min(steps, 5))
    for _ in range(nprof):
        img = step(stages)
    # parity at EVERY rank count, outside the timed region: each rank sums the
    # fp64 DFT of its own visibilities at 8 fixed pixels, the sums are
    # all-reduced and rank 0 compares them with the gathered image
    parity = strong_parity(data, freq, img, npix, px, world, rank, device)
    if world == 1 and data.slice_uvw.shape[0] == rows and nvis == rows * nchan:
        # one strip holding every row whole: the same visibilities as a dense
        # MS - the strip path against the one-shot cip_ms2dirty (fp64 classes,
        # fixed-point quanta of the two calls differ)
        from ska_sdp_cip_amd import gridder

        ref, _ = gridder.device_ms2dirty(data.slice_uvw, freq, vis.view(rows, nchan), wgt.view(rows, nchan), npix,
                                         npix, px, px, support=args.support, normalise=True)
        parity.update({"max_abs_diff_vs_one_shot": float((img - ref).abs().max()),
                       "one_shot_what": "normalised images: invert_strips (1 strip) vs cip_ms2dirty on the same "
                                        "visibilities"})
        del ref
    nv_all = torch.tensor([float(nvis)], dtype=torch.float64, device=device)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [torch.zeros_like(nv_all) for _ in range(world)]
        dist.all_gather(per_rank, nv_all)
        per_rank = [int(x.item()) for x in per_rank]
    else:
        per_rank = [nvis]
    total = sum(per_rank)
    ms_per_step = elapsed / steps * 1e3
    result = {
        "metric": f"Mvis/s gridded (invert) on {params.nu // 1024}k^2 grid, support={params.support}",
        "value": round(total * steps / elapsed / 1e6, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded MeerKAT-like uvw tracks, random complex64 vis, float32 weights, 5% flagged)",
        "config": {
            "workload": (f"C4 (BASELINE configs[3]): {rows:,} rows x {nchan} ch = {rows * nchan:,} vis, ONE "
                         f"{params.nu}x{params.nv} grid ({npix}^2 image), support {params.support}, 2-D, fp64 "
                         "accumulate"),
            "parallelism": (f"uv strips x{world}: balanced grid-row strips + {params.support - 1}-row halo "
                            "send/recv, strip pass A, sparse all-to-all of the live pass-A rows, pass B per "
                            "image-row strip, gather of image rows (step k's gather in flight during step k + 1's "
                            "gridding)" if world > 1 else "uv strips x1 (whole C4 on one GPU)"),
            "strip_rows": [layout.rows(r) for r in range(world)],
            "strip_vis": per_rank,
            "grid_rows_per_rank": [strips.strip_buffer_rows(layout, r)[1] for r in range(world)],
        },
        "stages_ms_rank0": {k: round(v / nprof * 1e3, 3) for k, v in stages.items()},
        # the strip split (cip_strip_histogram + plan_strips' bounds +
        # cip_strip_split with the gather), once per data set, rank 0; the rate
        # if every step re-split its data beside it
        "plan_ms": round(t_plan * 1e3, 3),
        "value_with_plan_per_step": round(total * steps / (elapsed + steps * t_plan) / 1e6, 2),
        "parity": parity,
        "roofline": None,
        "cpu_baseline": None,
    }
    del backend, data, vis, wgt
    torch.cuda.empty_cache()
    return result


def strong_parity(data, freq, img, npix, px, world, rank, device):
    """DFT-pixel parity of a distributed image (every rank calls it; `img` is
    the gathered image on rank 0, None elsewhere): each rank's partial fp64
    DFT sums over its own strip's visibilities at 8 fixed pixels
    (oracle/dft_torch.py), all-reduced with the weight sums; rank 0 reports
    max |image - DFT / sum w| (gate 1e-6, the north star's) and a checksum of
    the image (fp64 sum and sum of squares, equal across rank counts to the
    fixed-point quanta, ~1e-12 relative)."""
    import torch
    import torch.distributed as dist

    import dft_torch

    pix = dft_torch.check_pixels(npix, npix)
    sums, sw = dft_torch.dft_pixels_slices(data.slice_uvw, data.chan_start, data.chan_stop, freq, data.vis,
                                           data.wgt, pix, npix, npix, px, px)
    buf = torch.tensor(list(sums) + [sw], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(buf)
    if rank != 0:
        return None
    vals = buf.cpu().numpy()
    ref = vals[:-1] / vals[-1]
    got = np.array([float(img[i, j].item()) for i, j in pix])
    err = float(np.abs(got - ref).max())
    return {"max_err_dft_pixels": err, "gate": 1e-6, "ok": bool(err < 1e-6),
            "pixels": pix, "sum_weights": float(vals[-1]),
            "image_checksum": {"sum": float(img.sum().item()), "sum_sq": float((img * img).sum().item())},
            "peak": float(img.abs().max().item()),
            "what": (f"the gathered {npix}^2 image at 8 fixed pixels vs the fp64 DFT of all ranks' visibilities "
                     f"(partial sums per rank, all-reduced over {world} rank(s)), normalised by sum w; the "
                     "visibilities are counter-based (global row, channel), the same at every N")}


def weak_parity(uvw, freq, vis, wgt, img, npix, px, wstacking, world, rank, device):
    """The weak headline's reduced image against the definition: each rank's
    partial fp64 DFT sums over its own row shard at 8 fixed pixels
    (oracle/dft_torch.py), all-reduced with the weight sums; rank 0 compares
    them with `img` (the RCCL-reduced, normalised image; None elsewhere)."""
    import torch
    import torch.distributed as dist

    import dft_torch

    pix = dft_torch.check_pixels(npix, npix)
    sums, sw = dft_torch.dft_pixels_dense(uvw, freq, vis, wgt, pix, npix, npix, px, px, apply_w=wstacking)
    buf = torch.tensor(list(sums) + [sw], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(buf)
    if rank != 0:
        return None
    vals = buf.cpu().numpy()
    ref = vals[:-1] / vals[-1]
    got = np.array([float(img[i, j].item()) for i, j in pix])
    err = float(np.abs(got - ref).max())
    return {"max_err_dft_pixels": err, "gate": 1e-6, "ok": bool(err < 1e-6), "pixels": pix,
            "sum_weights": float(vals[-1]),
            "what": (f"rank 0's {'RCCL-reduced ' if world > 1 else ''}normalised {npix}^2 image of the last step "
                     f"at 8 fixed pixels vs the fp64 DFT of all {world} rank(s)' visibilities (partial sums per "
                     "rank, all-reduced), / sum w")}


def run_strong_wplanes(args, world, rank, device):
    """
    `--strong --wstacking`: strong scaling of ONE w-stacking image - the
    reference's gridding mode (invert.py:170-183: epsilon 1e-4 -> W = 6,
    do_wstacking=True) on the C3 workload (100M visibilities, 8192^2 grid) -
    by w-plane groups (SURVEY.md 8(e) option 2, ska_sdp_cip_amd.wplanes):
    every rank holds the visibilities, takes a contiguous range of the plane
    stack balanced by the plane cost model, grids + FFTs + screens only those
    planes (cip_ms2dirty_wplanes) and one RCCL reduce of the 4096^2 partial
    images makes the image on rank 0. value = 100M vis x steps / time.
    """
    import torch
    import torch.distributed as dist

    from ska_sdp_cip_amd import wplanes

    cfg = CONFIGS["c3"]
    uvw_d, freq_d, vis_d, wgt_d, px, _, _ = make_inputs(cfg, 0, 1, device)  # the same data on every rank
    npix = cfg["npix"]
    support = None if args.epsilon_call else args.support
    be = wplanes.HipWPlaneBackend(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, epsilon=1e-4, support=support,
                                  single_precision_accumulation=args.single)
    params = be.params()
    feeds = wplanes.plane_feeds(uvw_d, freq_d, params)
    split = wplanes.split_planes(wplanes.plane_cost(feeds, params), world, group=be.plane_group(params))
    out = torch.zeros((npix, npix), dtype=torch.float64, device=device)
    log(f"[bench --strong --wstacking] rank {rank}/{world}: planes {split[rank]} of {params.nplanes}, "
        f"support {params.support}")

    def step(stages=None):
        return wplanes.invert_wplanes(be, split, dst=0, stages=stages, out=out)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = {}
    nprof = max(2, min(args.steps, 5))
    for _ in range(nprof):
        img = step(stages)
    parity = None
    if world == 1:
        ref, _ = gridder_ms2dirty_ref(uvw_d, freq_d, vis_d, wgt_d, npix, px, params.support, args.single)
        parity = {"max_abs_diff_vs_one_shot": float((img - ref).abs().max()), "peak": float(ref.abs().max()),
                  "what": "normalised images: invert_wplanes (1 rank) vs cip_ms2dirty"}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    nvis = cfg["rows"] * cfg["nchan"]
    return {
        "metric": f"Mvis/s gridded (invert) on {params.nu // 1024}k^2 grid, support={params.support}, w-stacking",
        "value": round(nvis * args.steps / elapsed / 1e6, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32-class (packed 2x32-bit)" if args.single else "f64",
        "data": "synthetic (seeded MeerKAT-like uvw tracks, random complex64 vis, float32 weights, 5% flagged)",
        "config": {
            "workload": (f"C3 reference call: {nvis:,} vis -> {params.nu}^2 grid ({npix}^2 image), support "
                         f"{params.support}, w-stacking {params.nplanes} planes, "
                         f"{'packed single-precision' if args.single else 'fp64'} accumulate"),
            "parallelism": f"w-plane groups x{world} + RCCL image reduce (SURVEY 8(e) option 2)",
            "plane_split": split,
        },
        "stages_ms_rank0": {k: round(v / nprof * 1e3, 3) for k, v in stages.items()},
        "parity": parity,
        "roofline": None,
        "cpu_baseline": None,
    }


def run_strong_wstrips(args, world, rank, device):
    """
    `--strong --wstacking --split strips`: the same w-stacking image (the
    reference call on C3) split by uv strips (SURVEY.md 8(e) option 1, DESIGN.md
    7): rank r grids every w plane's rows of its balanced strip (buffers of
    strip + W - 1 halo rows per plane), the halos of all planes go to rank
    r + 1, then per plane: pass A on its rows, one all-to-all, pass B with the
    plane's w screen into its image rows; the final w correction per rank and
    one gather. value = 100M vis x steps / time.
    """
    import torch
    import torch.distributed as dist

    from ska_sdp_cip_amd import strips, wplanes

    cfg = CONFIGS["c3"]
    uvw_d, freq_d, vis_d, wgt_d, px, _, _ = make_inputs(cfg, 0, 1, device)  # the same data on every rank
    npix = cfg["npix"]
    support = None if args.epsilon_call else args.support
    params = wplanes.HipWPlaneBackend(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, epsilon=1e-4,
                                      support=support, single_precision_accumulation=args.single).params()
    layout = strips.plan_strips(uvw_d, freq_d, params, px, npix, npix, world)
    data = strips.split_strip(uvw_d, freq_d, vis_d, wgt_d, params, px, *layout.rows(rank))
    backend = strips.HipStripBackend(params, px, px, npix, npix, device=device,
                                     rows=strips.strip_buffer_rows(layout, rank),
                                     single_precision_accumulation=args.single)
    y0, y1 = layout.rows(rank)
    log(f"[bench --strong --wstacking] rank {rank}/{world}: strip rows [{y0}, {y1}) of {params.nv}, "
        f"{data.nvis:,} vis, {params.nplanes} planes, support {params.support}")

    def step(stages=None):
        return strips.invert_strips(data, freq_d, layout, backend, dst=0, stages=stages)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = {}
    nprof = max(2, min(args.steps, 5))
    for _ in range(nprof):
        img = step(stages)
    parity = None
    if world == 1:
        ref, _ = gridder_ms2dirty_ref(uvw_d, freq_d, vis_d, wgt_d, npix, px, params.support, args.single)
        parity = {"max_abs_diff_vs_one_shot": float((img - ref).abs().max()), "peak": float(ref.abs().max()),
                  "what": "normalised images: w-stacking invert_strips (1 strip) vs cip_ms2dirty"}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    nvis = cfg["rows"] * cfg["nchan"]
    return {
        "metric": f"Mvis/s gridded (invert) on {params.nu // 1024}k^2 grid, support={params.support}, w-stacking",
        "value": round(nvis * args.steps / elapsed / 1e6, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32-class (packed 2x32-bit)" if args.single else "f64",
        "data": "synthetic (seeded MeerKAT-like uvw tracks, random complex64 vis, float32 weights, 5% flagged)",
        "config": {
            "workload": (f"C3 reference call: {nvis:,} vis -> {params.nu}^2 grid ({npix}^2 image), support "
                         f"{params.support}, w-stacking {params.nplanes} planes, "
                         f"{'packed single-precision' if args.single else 'fp64'} accumulate"),
            "parallelism": f"uv strips x{world} + per-plane all-to-all (SURVEY 8(e) option 1)",
            "strip_rows": [layout.rows(r) for r in range(world)],
        },
        "stages_ms_rank0": {k: round(v / nprof * 1e3, 3) for k, v in stages.items()},
        "parity": parity,
        "roofline": None,
        "cpu_baseline": None,
    }


def gridder_ms2dirty_ref(uvw, freq, vis, wgt, npix, px, support, single):
    from ska_sdp_cip_amd import gridder

    return gridder.device_ms2dirty(uvw, freq, vis, wgt, npix, npix, px, px, support=support, do_wstacking=True,
                                   single_precision_accumulation=single, normalise=True)


def reference_call_rate(invert, buf, steps, warmup=3):
    """Pipelined rate of the reference's ms2dirty call (epsilon = 1e-4 ->
    support 6, w-stacking, packed single-precision class) on the bench's
    resident inputs, plus its synchronous per-phase times."""
    import torch

    from ska_sdp_cip_amd import _lib

    dirty, sumw = buf
    kw = dict(epsilon=1e-4, do_wstacking=True, single_precision_accumulation=True, out=dirty, sum_weights=sumw,
              normalise=True)
    for _ in range(warmup):
        invert(synchronize=False, resident_inputs=True, **kw)
    torch.cuda.synchronize()
    nsteps = max(3, min(steps, 10))
    t0 = time.perf_counter()
    for _ in range(nsteps):
        invert(synchronize=False, resident_inputs=True, **kw)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _lib.profile_enable(True)
    phases = []
    for _ in range(3):
        _, params = invert(**kw)
        phases.append(_lib.profile_last())
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    nvis = int(phases[0]["visibilities"])
    avg = {k: float(np.mean([p[k] for p in phases])) for k in phases[0] if k.endswith("_ms")}
    return {
        "what": "invert.py:170-183 ms2dirty(epsilon=1e-4, do_wstacking=True) on complex64 vis + float32 weights: "
                f"support {params.support}, {params.nplanes} w planes, packed single-precision accumulation "
                "(ducc0's float class for complex64 input), pipelined calls on the same resident inputs",
        "value": round(nvis * nsteps / elapsed / 1e6, 2),
        "unit": "Mvis/s",
        "ms_per_step": round(elapsed / nsteps * 1e3, 3),
        "steps": nsteps,
        "support": params.support,
        "nplanes": params.nplanes,
        "phases_ms_sync": {k.replace("_ms", ""): round(v, 3) for k, v in avg.items()},
    }


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[1])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--support", type=int, default=8)
    ap.add_argument("--wstacking", action="store_true", help="w-stacking mode (secondary measurement)")
    ap.add_argument("--single", action="store_true",
                    help="packed single-precision accumulation class (CIP_ACC_SINGLE; the precision class of the "
                         "reference's float32 ducc0 call) - secondary measurement, not the f64 metric")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync", action="store_true",
                    help="synchronous steps (diagnostic: per-kernel times without the pipelined overlap)")
    ap.add_argument("--no-max-err", action="store_true", help="skip the GPU-vs-oracle max|err| check")
    ap.add_argument("--err-row-step", type=int, default=0,
                    help="max|err| on every k-th row (default: 50 in 2-D, 200 with w-stacking)")
    ap.add_argument("--raw", action="store_true",
                    help="raw linear-feed columns (rows, nchan, 4) resident in HBM: Stokes I and effective weights "
                         "formed inside the planner and scatter (cip_ms2dirty_stokes_i) - the reference's whole "
                         "invert_measurement_set input (secondary measurement)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the reference-call secondary figure of the default run")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling of ONE C4 image (1G vis, 16k^2 grid) over the ranks: uv strips + halo "
                         "exchange + distributed FFT (DESIGN.md 7); with --wstacking: ONE C3 w-stacking image split "
                         "by w-plane groups + one image reduce (SURVEY 8(e) option 2); --config is ignored")
    ap.add_argument("--epsilon-call", action="store_true",
                    help="epsilon = 1e-4 picks the support (the reference's call, W = 6) instead of --support "
                         "(with --wstacking --single: the reference's whole ms2dirty call as the main line)")
    ap.add_argument("--split", choices=("strips", "wplanes"), default="strips",
                    help="with --strong --wstacking: split the w-stacking image by uv strips (default; modelled "
                         "2.83x at 8 ranks on the C3 reference call against 2.49x for w-plane groups) or by "
                         "w-plane groups")
    ap.add_argument("--no-strong-secondary", action="store_true",
                    help="skip the strong-scaling C4 secondary (secondary.strong_c4) of the default run")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside a launcher: start N rank processes (one
        # per GPU) through torch.distributed.run BEFORE anything touches the
        # GPU here, and exit with their status
        import socket
        import subprocess

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
        log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
        return subprocess.call(cmd)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        log(f"[bench] WORLD_SIZE={env_world} but --gpus {args.gpus}: refusing to report a mismatched run")
        return 2

    import torch
    import torch.distributed as dist

    from ska_sdp_cip_amd import _lib, gridder
    from ska_sdp_cip_amd.distributed import image_buffer, reduce_images

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    comm = {"backend": None, "world_size": 1}
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        # what the communicator reports (RCCL is torch's "nccl" backend on ROCm)
        comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                "rccl_version": ".".join(str(x) for x in torch.cuda.nccl.version())}
        if comm["world_size"] != args.gpus:
            raise SystemExit(f"communicator world size {comm['world_size']} != --gpus {args.gpus}")
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    if args.strong:
        result = ((run_strong_wstrips if args.split == "strips" else run_strong_wplanes)(args, world, rank, device)
                  if args.wstacking
                  else run_strong(args, world, rank, device))
        result["communicator"] = comm
        if rank == 0:
            print(json.dumps(result), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return 0
    cfg = CONFIGS[args.config]
    nvis = cfg["rows"] * cfg["nchan"]
    npix = cfg["npix"]
    uvw_d, freq_d, vis_d, wgt_d, px, uvw_h, freq_h = make_inputs(cfg, rank, world, device)
    raw = None
    if args.raw:
        del vis_d, wgt_d
        raw = make_raw_columns(cfg, rank, device)
        vis_d = wgt_d = None

    def invert(**kw):
        if raw is not None:
            return gridder.device_ms2dirty_stokes_i(uvw_d, freq_d, raw[0], raw[1], raw[2], npix, npix, px, px, **kw)
        return gridder.device_ms2dirty(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, **kw)
    # two image buffers (image + weight sum adjacent: one RCCL reduce each):
    # step k's reduce runs on the communicator's stream while step k + 1
    # inverts into the other buffer; a buffer is rewritten only after its
    # previous reduce (and the normalisation on rank 0) completed
    bufs = [image_buffer(npix, npix, device) for _ in range(2)]
    pending = [None, None]
    nstep = [0]

    # --epsilon-call: epsilon = 1e-4 picks the support (invert.py:170-183)
    sup_kw = {"epsilon": 1e-4} if args.epsilon_call else {"support": args.support}

    def step(sync=False):
        k = nstep[0] % 2
        nstep[0] += 1
        if pending[k] is not None:
            pending[k].wait()
        dirty, sumw = bufs[k]
        # sync=False (CIP_ASYNC): the call returns once its work is queued, so
        # the host prepares step k + 1 while the GPU finishes step k; the
        # inputs are resident and unchanged (CIP_PIPELINE), so step k + 1's
        # planner runs beside step k's scatter and FFT
        invert(**sup_kw, do_wstacking=args.wstacking, out=dirty, sum_weights=sumw,
               single_precision_accumulation=args.single, normalise=world == 1, synchronize=sync,
               resident_inputs=not sync)
        # RCCL reduce of the partial images + weights to rank 0, normalised there
        # (one GPU: the image is already normalised in the FFT epilogue)
        pending[k] = reduce_images(dirty, sumw, dst=0, async_op=True, normalise=world > 1)

    def drain():
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    log(f"[bench] rank {rank}/{world} config {args.config}: {nvis:,} vis/GPU, {npix}^2 image, "
        f"pixsize {px:.3e} rad, support {args.support}, wstacking={args.wstacking}")
    for _ in range(args.warmup):
        step(sync=args.sync)
    drain()
    dirty, sumw = bufs[0]
    _, params = invert(**sup_kw, do_wstacking=args.wstacking, out=dirty, sum_weights=sumw,
                       single_precision_accumulation=args.single)
    args.support = params.support
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(sync=args.sync)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the same steps synchronous (each call returns when its image is done; no
    # planner overlap with the previous call): the single-call rate next to
    # the pipelined headline
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step(sync=True)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed_sync = time.perf_counter() - t1
    # phase breakdown (hipEvents on the launching stream) from separate
    # profiled steps after the timed region: profiling synchronises each call
    _lib.profile_enable(True)
    phases = []
    for _ in range(max(3, min(args.steps, 10))):
        step(sync=True)
        phases.append(_lib.profile_last())
    drain()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    # parity of the REDUCED image at every N (outside the timed region): the
    # last step's buffer holds, on rank 0, the RCCL-reduced image / total sum w;
    # each rank sums the fp64 DFT of its own shard at 8 fixed pixels, the sums
    # are all-reduced and rank 0 compares them with that image
    if raw is None:
        last = bufs[(nstep[0] - 1) % 2][0]
        reduced_parity = weak_parity(uvw_d, freq_d, vis_d, wgt_d, last if rank == 0 else None, npix, px,
                                     args.wstacking, world, rank, device)
    else:
        reduced_parity = None
    if world > 1:
        t = torch.tensor([elapsed, elapsed_sync], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_sync = float(t[0].item()), float(t[1].item())

    ms_per_step = elapsed / args.steps * 1e3
    value = world * nvis * args.steps / elapsed / 1e6
    avg = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]}
    runs = avg["runs"]
    launches = max(avg["scatter_launches"], 1.0)
    scatter_ms = avg["scatter_ms"] / launches
    P = params.nplanes
    taps = params.support ** (3 if args.wstacking else 2)
    # algorithmic bytes of one scatter launch, design-independent (SURVEY.md
    # 8(d) B_alg): every visibility's value (c64, 8 B) and weight (f32, 4 B)
    # once per plane it feeds, 32 B per row slice (uvw + channel range) and the
    # plane's grid written once (its read-back belongs to the FFT). The
    # ordered-stream record this design adds (8 B/vis) is not counted.
    vis_per_launch = nvis * (params.support if args.wstacking else 1) / (P if args.wstacking else 1)
    vis_bytes = 52 if args.raw else 12  # raw: 4 x c64 + 4 x f32 + 4 x u8 per visibility
    bytes_launch = vis_per_launch * vis_bytes + runs / launches * 32 + params.nu * params.nv * 16
    achieved = bytes_launch / (scatter_ms * 1e-3) / 1e9
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5),
        "traffic": None,
        "kernel": "cip::scatter_kernel",
        # the roof that binds this kernel is LDS atomic bandwidth (lds_atomic
        # below), not HBM: 1 KiB of LDS read-modify-write per visibility at W = 8
        # against ~40 B of HBM (SURVEY.md 8(d) asks for HBM as the reported bound)
        "binding": "lds_atomic",
        "bytes_per_launch_alg": int(bytes_launch),
        "launch_ms": round(scatter_ms, 4),
    }
    # the bound that actually limits the scatter: LDS atomic bytes. Each tap is
    # a 64-bit fixed-point add to the re and the im plane (16 B of LDS RMW).
    # Round 5 (tools/microbench/lds_conflict.hip, profiles/r05_pairs.md): a
    # conflict-free 64-lane ds_add_u64 keeps the LDS 4 cycles busy (128 B per
    # CU-cycle, the LDS width); the round-1 basis of 8.12 CU-cycles was an 8 x 8
    # tap pattern with half its cycles in bank conflicts, as the scatter has
    # (36 % of its LDS-active cycles: the level-major class order's leftovers)
    lds_bytes = vis_per_launch * params.support ** 2 * (8 if args.single else 16)  # packed: one u64 per tap
    lds_peak = 128.0 * 2.4e9 * 256 / 1e9  # GB/s: 128 B / CU-cycle, 256 CUs at 2.4 GHz
    lds_tap_peak = 64 * 8 / 8.12 * 2.4e9 * 256 / 1e9  # the tap pattern's rate (its conflicts included)
    # the fastest rate any kernel here reaches: the conflict-free ("distinct"
    # addresses) microbenchmark, 6.68 CU-cycles per wave-instruction
    # (profiles/r05_lds_conflict_microbench.txt)
    lds_measured_peak = 64 * 8 / 6.68 * 2.4e9 * 256 / 1e9
    lds_achieved = lds_bytes / (scatter_ms * 1e-3) / 1e9
    roofline["lds_atomic"] = {"achieved": round(lds_achieved, 1), "peak": round(lds_peak, 1), "unit": "GB/s",
                              "frac": round(lds_achieved / lds_peak, 4),
                              "peak_measured": round(lds_measured_peak, 1),
                              "frac_of_peak_measured": round(lds_achieved / lds_measured_peak, 4),
                              "frac_of_tap_pattern_rate": round(lds_achieved / lds_tap_peak, 4),
                              "basis": f"{8 if args.single else 16} B of ds_add_u64 per tap; peak = 4 LDS cycles per "
                                       "conflict-free wave-instr (128 B/CU-cycle); the scatter's own bank conflicts "
                                       "(~36 % of its LDS cycles, profiles/r05_sq_c3_pairs.md) are inside 'achieved'"}
    tr = traffic_from_profiles(args.config)
    # the committed PMC pass is of the default workload (support 8, 2-D, fp64 class)
    if tr and not args.wstacking and not args.single and not args.raw and args.support == tr.get("support", 8):
        roofline["traffic"] = tr.get("hbm_bytes_per_launch")

    result = {
        "metric": f"Mvis/s gridded (invert) on {params.nu // 1024}k^2 grid, support={params.support}",
        "value": round(value, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32-class (packed 2x32-bit)" if args.single else "f64",
        "data": ("synthetic (seeded MeerKAT-like uvw tracks, raw (rows, nchan, 4) complex64 correlations, float32 "
                 "weights, uint8 flags 2.5% per XX/YY entry)" if args.raw else
                 "synthetic (seeded MeerKAT-like uvw tracks, random complex64 vis, float32 weights, 5% flagged)"),
        "config": {
            "input": ("raw linear-feed columns, Stokes I formed in the gridder (cip_ms2dirty_stokes_i)" if args.raw
                      else "Stokes-I visibilities + effective weights (cip_ms2dirty)"),
            "workload": (f"{args.config.upper()}: {cfg['rows']:,} rows x {cfg['nchan']} ch = {nvis:,} vis/GPU -> "
                         f"{params.nu}x{params.nv} grid ({npix}^2 image), support {params.support}, "
                         f"{'w-stacking ' + str(P) + ' planes' if args.wstacking else '2-D'}, "
                         f"{'packed single-precision' if args.single else 'fp64'} accumulate"),
            "rows_per_gpu": cfg["rows"],
            "channels": cfg["nchan"],
            "grid": params.nu,
            "image": npix,
            "support": params.support,
            "wstacking": bool(args.wstacking),
            "parallelism": f"uvw-shard dp{world} + RCCL image reduce" if world > 1 else "single GPU",
            "mode": ("sync" if args.sync else
                     "pipelined: back-to-back CIP_ASYNC|CIP_PIPELINE calls on HBM-resident, unchanged inputs "
                     "(call k+1's planner overlaps call k's scatter/FFT); value_sync = one call at a time"),
        },
        "value_sync": round(world * nvis * args.steps / elapsed_sync / 1e6, 2),
        "ms_per_step_sync": round(elapsed_sync / args.steps * 1e3, 3),
        "roofline": roofline,
        "phases_ms": {k.replace("_ms", ""): round(v, 3) for k, v in avg.items() if k.endswith("_ms")},
        "mean_slice_len": round(avg["visibilities"] / max(runs, 1), 2),
        "gtap_per_s": round(world * nvis * taps * args.steps / elapsed / 1e9, 2),
    }
    result["communicator"] = comm
    result["parity_reduced"] = reduced_parity
    default_run = raw is None and not args.wstacking and not args.single and args.config == "c3"
    secondary = {}
    if world == 1 and not args.no_secondary and default_run:
        # the reference's own gridder call on the same resident inputs
        # (invert.py:170-183: epsilon 1e-4 -> W = 6, do_wstacking=True,
        # complex64 input -> ducc0's float accumulation class): a secondary
        # figure beside the f64 metric, so every default run reports it
        secondary["reference_call"] = reference_call_rate(invert, bufs[0], args.steps)
    if not args.no_strong_secondary and default_run and args.support == 8:
        # the north star's strong split beside the weak headline: ONE C4 image
        # (1G visibilities, 16384^2 grid) over the same ranks (uv strips + halo
        # exchange + distributed FFT) - at N = 1 the whole C4 on
        # one GPU, the base of the strong-scaling curve
        torch.cuda.empty_cache()
        st = run_strong(args, world, rank, device, steps=max(3, min(args.steps, 10)), warmup=2)
        secondary["strong_c4"] = {k: st[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "ms_per_step",
                                                     "scaling", "stages_ms_rank0", "plan_ms",
                                                     "value_with_plan_per_step", "parity")}
        secondary["strong_c4"]["workload"] = st["config"]["workload"]
        secondary["strong_c4"]["parallelism"] = st["config"]["parallelism"]
        secondary["strong_c4"]["grid_rows_per_rank"] = st["config"]["grid_rows_per_rank"]
    if secondary:
        result["secondary"] = secondary
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
    need_host = rank == 0 and ((world == 1 and not args.no_cpu_baseline) or not args.no_max_err)
    vis_h = wgt_h = None
    if need_host and raw is not None:
        # the Stokes-I inputs the gridder formed, restated by the oracle's numpy
        import oracle

        vis_h, _, _, wgt_h = oracle.stokes_i(raw[0].cpu().numpy(), raw[1].cpu().numpy().astype(bool),
                                             raw[2].cpu().numpy())
    elif need_host:
        vis_h = vis_d.cpu().numpy()
        wgt_h = wgt_d.cpu().numpy()
    if rank == 0 and not args.no_max_err:
        step_k = args.err_row_step or (200 if args.wstacking else 50)
        log(f"[bench] max|err| vs the CPU oracle on rows [::{step_k}] ...")
        me = max_err_vs_oracle(uvw_h, freq_h, vis_h, wgt_h, npix, px, args.support, args.wstacking, args.single,
                               nthreads, step_k, device)
        if world == 1:
            result.update(me)
        else:
            # N > 1: the metric's max|err| is the REDUCED image's (DFT pixels,
            # all ranks' visibilities); the oracle check of rank 0's own shard
            # at every pixel stays beside it
            result["max_err_rank0_shard"] = me
            if reduced_parity is not None:
                result.update({"max_err": reduced_parity["max_err_dft_pixels"], "gate": 1e-6,
                               "sample": reduced_parity["what"]})
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.wstacking and args.support <= 16:
        log(f"[bench] cpu baseline with {nthreads} threads ...")
        result["cpu_baseline"] = cpu_baseline(args.config, uvw_h, freq_h, vis_h, wgt_h, px, args.support, nthreads)
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
