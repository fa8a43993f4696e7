#!/usr/bin/env python3
"""
EXPERIMENT driver: the time-track scatter (tools/timetrack/timetrack.hip)
against the lane kernel (libcip_hip.so's scatter_kernel, via cip_grid_ms) on
the bench's C3 data (100M visibilities, 8192^2 grid, W = 8, fp64 class).

The time-track plan is built here with torch on the GPU (not timed, not a
product path): every visibility's footprint tile (the planner's placement
arithmetic), the (baseline, channel) tracks in time order cut into segments
of constant tile, segments grouped by tile into work units of <= CAP samples,
largest first. Both scatters then grid the same visibilities; the grids must
agree to the fp64 flush order. Timing comes from rocprofv3 --kernel-trace
(scatter_kernel vs timetrack_kernel) around this script; it also prints its
own event timing of the two scatter launches sequences.

    python tools/timetrack/run_timetrack.py [--reps 5]
"""
import argparse
import ctypes
import json
import math
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"), str(ROOT)]

CAP = 16384


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_plan(uvw, fx, nrow, nchan, nbl, nu, nv, su, sv, W=8, T=32):
    import torch

    hw = W // 2
    x = (uvw[:, 0:1] * fx[None, :]) * su + float(nu // 2)
    y = (uvw[:, 1:2] * fx[None, :]) * sv + float(nv // 2)
    ix0 = torch.remainder(torch.floor(x - float(hw)).long() + 1, nu)
    iy0 = torch.remainder(torch.floor(y - float(hw)).long() + 1, nv)
    del x, y
    ntx = nu // T
    key = ((iy0 // T) * ntx + ix0 // T).to(torch.int32)
    del ix0, iy0
    ntimes = -(-nrow // nbl)
    pad = ntimes * nbl - nrow
    if pad:
        key = torch.cat([key, torch.full((pad, nchan), -1, dtype=torch.int32, device=key.device)])
    kt = key.view(ntimes, nbl, nchan).permute(1, 2, 0).contiguous().view(-1)  # (b, c, t)
    del key
    total = kt.numel()
    brk = torch.ones(total, dtype=torch.bool, device=kt.device)
    brk[1:] = kt[1:] != kt[:-1]
    brk[torch.arange(0, total, ntimes, device=kt.device)] = True  # a new track starts a segment
    starts = torch.nonzero(brk).squeeze(1)
    ends = torch.cat([starts[1:], torch.tensor([total], device=kt.device)])
    skey = kt[starts]
    keep = skey >= 0
    starts, ends, skey = starts[keep], ends[keep], skey[keep]
    order = torch.sort(skey, stable=True).indices
    starts, ends, skey = starts[order], ends[order], skey[order]
    b = (starts // (nchan * ntimes)).to(torch.int32)
    c = ((starts // ntimes) % nchan).to(torch.int32)
    t0 = (starts % ntimes).to(torch.int32)
    t1 = (t0.long() + (ends - starts)).to(torch.int32)
    n = (ends - starts)
    nseg = n.numel()
    # units: a new unit at a tile change or every CAP samples within a tile
    newtile = torch.ones(nseg, dtype=torch.bool, device=kt.device)
    newtile[1:] = skey[1:] != skey[:-1]
    csum = torch.cumsum(n, 0) - n
    tile_first = torch.nonzero(newtile).squeeze(1)
    tile_rank = torch.cumsum(newtile.long(), 0) - 1
    within = csum - csum[tile_first][tile_rank]
    chunk = within // CAP
    newunit = newtile.clone()
    newunit[1:] |= chunk[1:] != chunk[:-1]
    us0 = torch.nonzero(newunit).squeeze(1)
    us1 = torch.cat([us0[1:], torch.tensor([nseg], device=kt.device)])
    ukey = skey[us0]
    usamp = torch.cumsum(n, 0)
    ucount = usamp[us1 - 1] - (usamp[us0] - n[us0])
    uo = torch.sort(ucount, descending=True, stable=True).indices  # largest units first
    us0, us1, ukey, ucount = us0[uo], us1[uo], ukey[uo], ucount[uo]
    plan = dict(b=b, c=c, t0=t0, t1=t1, us0=us0.contiguous(), us1=us1.contiguous(),
                utx=(ukey % ntx).to(torch.int32), uty=(ukey // ntx).to(torch.int32))
    stats = dict(segments=int(nseg), units=int(us0.numel()), samples=int(n.sum()),
                 mean_segment=float(n.float().mean()), median_segment=float(n.float().median()),
                 max_unit=int(ucount.max()))
    return plan, stats


def main():
    import torch

    import bench
    from ska_sdp_cip_amd import _lib

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    uvw, freq, vis, wgt, px, _, _ = bench.make_inputs(cfg, 0, 1, dev)
    nrow, nchan = vis.shape
    npix = cfg["npix"]
    nbl = cfg["n_ant"] * (cfg["n_ant"] - 1) // 2
    params = _lib.choose_params(npix, npix, px, px, 1e-6, 8)
    nu, nv = params.nu, params.nv
    lib = _lib.lib()
    assert lib.cip_grid_layout(ctypes.byref(params), npix, npix) == 1
    su, sv = float(nu) * px, float(nv) * px
    fx = freq / 299792458.0
    t0 = time.perf_counter()
    plan, stats = build_plan(uvw, fx, nrow, nchan, nbl, nu, nv, su, sv)
    torch.cuda.synchronize()
    stats["plan_s_torch"] = round(time.perf_counter() - t0, 3)
    log("[timetrack] plan", stats)
    maxabs = float((wgt.double().abs() * torch.maximum(vis.real.double().abs(), vis.imag.double().abs())).max())
    fixed_scale = math.ldexp(1.0, 46 - math.frexp(maxabs)[1])
    tt = ctypes.CDLL(str(Path(__file__).resolve().parent / "libtimetrack.so"))
    tt.tt_grid.restype = ctypes.c_int
    vp, i64, f64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    tt.tt_grid.argtypes = [vp, vp, vp, vp, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f64, f64, f64,
                           vp, vp, vp]
    stream = torch.cuda.current_stream().cuda_stream
    grid_tt = torch.zeros(2 * nu * nv, dtype=torch.float64, device=dev)
    grid_ln = torch.zeros_like(grid_tt)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    sumw = torch.zeros(1, dtype=torch.float64, device=dev)
    p = plan

    def run_tt():
        rc = tt.tt_grid(uvw.data_ptr(), fx.data_ptr(), vis.data_ptr(), wgt.data_ptr(), nchan, nbl,
                        p["b"].data_ptr(), p["c"].data_ptr(), p["t0"].data_ptr(), p["t1"].data_ptr(),
                        p["us0"].data_ptr(), p["us1"].data_ptr(), p["utx"].data_ptr(), p["uty"].data_ptr(),
                        p["us0"].numel(), nu, nv, su, sv, fixed_scale, grid_tt.data_ptr(), err.data_ptr(), stream)
        assert rc == 0, rc

    def run_lane():
        _lib.check(lib.cip_grid_ms(uvw.data_ptr(), nrow, freq.data_ptr(), nchan, vis.data_ptr(), _lib.CIP_C64,
                                   wgt.data_ptr(), _lib.CIP_F32, ctypes.byref(params), px, px, npix, npix, 0, stream,
                                   grid_ln.data_ptr(), sumw.data_ptr()))

    run_tt()
    run_lane()
    torch.cuda.synchronize()
    assert int(err.item()) == 0, "a sample fell outside its unit's tile"
    peak = float(grid_ln.abs().max())
    diff = float((grid_tt - grid_ln).abs().max())
    log(f"[timetrack] parity: max|tt - lane| = {diff:.3e}, peak {peak:.3e}, rel {diff / peak:.3e}")
    times = {"timetrack": [], "lane_call": []}
    for _ in range(args.reps):
        for name, fn, g in (("timetrack", run_tt, grid_tt), ("lane_call", run_lane, grid_ln)):
            g.zero_()
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(e))
    res = dict(stats, parity_rel=diff / peak, fixed_scale=fixed_scale,
               ms={k: round(sorted(v)[len(v) // 2], 3) for k, v in times.items()},
               note="lane_call = the whole cip_grid_ms call (planner + lane scatter); the scatter kernels' own "
                    "durations come from the rocprofv3 kernel trace of this run")
    print(json.dumps(res), flush=True)
    assert diff <= 1e-12 * peak


if __name__ == "__main__":
    main()
