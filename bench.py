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
on; `cpu_baseline` times the CPU oracle (oracle/, fp64 OpenMP restatement) on a
bounded sample of the same workload.
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


def cpu_baseline(uvw, freq, npix, px, nvis_full, support, nthreads, sample_rows):
    """
    CPU oracle (oracle/cip_oracle.c, fp64 OpenMP) timed on a bounded sample:
    gridding of `sample_rows` and 2 x `sample_rows` rows (slope = per-vis cost,
    intercept = per-call cost), plus one multi-threaded nu x nv FFT; the full
    workload's time is extrapolated as intercept + slope * N_vis + FFT.
    """
    import scipy.fft

    import oracle

    nchan = freq.size
    rng = np.random.default_rng(1)
    prm = oracle.choose_params(npix, npix, px, px, support=support)

    def grid_time(nr):
        u = np.ascontiguousarray(uvw[:nr])
        vis = (rng.standard_normal((nr, nchan)) + 1j * rng.standard_normal((nr, nchan))).astype(np.complex64)
        w = rng.uniform(0.5, 1.5, (nr, nchan)).astype(np.float32)
        t0 = time.perf_counter()
        oracle.grid_plane(u, freq, vis, w, prm, px, px, 0, nthreads)
        return time.perf_counter() - t0

    t1 = grid_time(sample_rows)
    t2 = grid_time(2 * sample_rows)
    nv1 = sample_rows * nchan
    slope = max((t2 - t1) / nv1, 1e-15)
    intercept = max(t1 - slope * nv1, 0.0)
    grid = np.zeros((prm["nu"], prm["nv"]), dtype=np.complex128)
    grid[::7, ::5] = 1.0
    t0 = time.perf_counter()
    scipy.fft.ifft2(grid, workers=nthreads, overwrite_x=True)
    t_fft = time.perf_counter() - t0
    t_full = intercept + slope * nvis_full + t_fft
    return {
        "value": nvis_full / t_full / 1e6,
        "unit": "Mvis/s",
        "cores": nthreads,
        "kind": "port",
        "sample": (f"oracle fp64 gridding of {nv1:,} and {2 * nv1:,} visibilities of the same workload "
                   f"({t1:.2f} s, {t2:.2f} s -> {slope * 1e9:.1f} ns/vis + {intercept:.2f} s/call) plus one "
                   f"{prm['nu']}^2 c2c FFT ({t_fft:.2f} s, scipy.fft, {nthreads} workers); full "
                   f"{nvis_full:,}-vis time extrapolated"),
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
    ap.add_argument("--cpu-sample-rows", type=int, default=8192)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ska_sdp_cip_amd import _lib, gridder
    from ska_sdp_cip_amd.distributed import image_buffer, reduce_images

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    cfg = CONFIGS[args.config]
    nvis = cfg["rows"] * cfg["nchan"]
    npix = cfg["npix"]
    uvw_d, freq_d, vis_d, wgt_d, px, uvw_h, freq_h = make_inputs(cfg, rank, world, device)
    # two image buffers (image + weight sum adjacent: one RCCL reduce each):
    # step k's reduce runs on the communicator's stream while step k + 1
    # inverts into the other buffer; a buffer is rewritten only after its
    # previous reduce (and the normalisation on rank 0) completed
    bufs = [image_buffer(npix, npix, device) for _ in range(2)]
    pending = [None, None]
    nstep = [0]

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
        gridder.device_ms2dirty(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, support=args.support,
                                do_wstacking=args.wstacking, out=dirty, sum_weights=sumw,
                                single_precision_accumulation=args.single, normalise=world == 1,
                                synchronize=sync, resident_inputs=not sync)
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
    _, params = gridder.device_ms2dirty(uvw_d, freq_d, vis_d, wgt_d, npix, npix, px, px, support=args.support,
                                        do_wstacking=args.wstacking, out=dirty, sum_weights=sumw,
                                        single_precision_accumulation=args.single)
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
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

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
    bytes_launch = vis_per_launch * (8 + 4) + runs / launches * 32 + params.nu * params.nv * 16
    achieved = bytes_launch / (scatter_ms * 1e-3) / 1e9
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5),
        "traffic": None,
        "kernel": "cip::scatter_kernel",
        "bytes_per_launch_alg": int(bytes_launch),
        "launch_ms": round(scatter_ms, 4),
    }
    # the bound that actually limits the scatter: LDS atomic bytes. Each tap is
    # a 64-bit fixed-point add to the re and the im plane (16 B of LDS RMW),
    # and gfx950 sustains one conflict-free 64-lane ds_add_u64 per 8.12
    # CU-cycles (tools/microbench/lds_ops.hip, profiles/microbench_r01.txt).
    lds_bytes = vis_per_launch * params.support ** 2 * (8 if args.single else 16)  # packed: one u64 per tap
    lds_peak = 64 * 8 / 8.12 * 2.4e9 * 256 / 1e9  # GB/s: 256 CUs at 2.4 GHz
    lds_achieved = lds_bytes / (scatter_ms * 1e-3) / 1e9
    roofline["lds_atomic"] = {"achieved": round(lds_achieved, 1), "peak": round(lds_peak, 1), "unit": "GB/s",
                              "frac": round(lds_achieved / lds_peak, 4),
                              "basis": f"{8 if args.single else 16} B of ds_add_u64 per tap; 8.12 CU-cycles per "
                                       "conflict-free wave-instr"}
    tr = traffic_from_profiles(args.config)
    # the committed PMC pass is of the default workload (support 8, 2-D, fp64 class)
    if tr and not args.wstacking and not args.single and args.support == tr.get("support", 8):
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
        "data": "synthetic (seeded MeerKAT-like uvw tracks, random complex64 vis, float32 weights, 5% flagged)",
        "config": {
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
        },
        "roofline": roofline,
        "phases_ms": {k.replace("_ms", ""): round(v, 3) for k, v in avg.items() if k.endswith("_ms")},
        "mean_slice_len": round(avg["visibilities"] / max(runs, 1), 2),
        "gtap_per_s": round(world * nvis * taps * args.steps / elapsed / 1e9, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.wstacking:
        nthreads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
        log(f"[bench] cpu baseline with {nthreads} threads ...")
        result["cpu_baseline"] = cpu_baseline(uvw_h, freq_h, npix, px, nvis, args.support, nthreads,
                                              args.cpu_sample_rows)
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
