"""
Strong scaling of ONE w-stacking image by w-plane groups
(ska_sdp_cip_amd.wplanes; SURVEY.md 8(e) option 2): the plane split covers the
stack exactly once and balances the cost model, the oracle's plane-range
shares sum to its whole image, and a world-size-2 (and 3) gloo run of the real
collective (one reduce of the partial images) gives the single-process image
at 1e-13 - with the CPU oracle standing in for the GPU share
(cip_ms2dirty_wplanes; its GPU form is tests/test_gpu_wplanes.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd import wplanes

NPIX = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case(nrow=600, nchan=8, seed=5):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=12, array_radius_m=1500.0, fov_l=0.05, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = 0.2 / NPIX  # a 0.2 rad field: ~20 w planes (baselines wrap exactly)
    return uvw, f, vis, w, px


class _P:  # the fields wplanes reads from cip_gridder_params
    def __init__(self, prm):
        for k in ("nu", "nv", "support", "nplanes", "w0", "dw"):
            setattr(self, k, prm[k])


class OracleWPlaneBackend:
    """The oracle's share of planes [p0, p1) (unnormalised) + the whole weight sum."""

    def __init__(self, uvw, f, vis, w, px, W):
        self.a = (uvw, f, vis, w)
        self.px, self.W = px, W
        self.sumw = float(w.astype(np.float64).sum())

    def __call__(self, planes, out=None):
        img = oracle.ms2dirty(*self.a, NPIX, NPIX, self.px, self.px, support=self.W, do_wstacking=True,
                              nthreads=1, planes=planes)
        return torch.from_numpy(img), torch.tensor([self.sumw], dtype=torch.float64)


def _params(uvw, f, px, W):
    wmin, wmax = oracle.w_range(uvw, f)
    return oracle.choose_params(NPIX, NPIX, px, px, support=W, do_wstacking=True, wmin=wmin, wmax=wmax)


@pytest.mark.parametrize("world,group", [(1, 3), (2, 3), (3, 3), (4, 2), (8, 3), (40, 3)])
def test_split_partitions_the_stack(world, group):
    uvw, f, vis, w, px = _case()
    prm = _params(uvw, f, px, 6)
    feeds = wplanes.plane_feeds(torch.from_numpy(uvw), torch.from_numpy(f), _P(prm))
    assert feeds.shape == (prm["nplanes"],)
    # every visibility feeds exactly W planes
    assert int(feeds.sum()) == vis.size * prm["support"]
    cost = wplanes.plane_cost(feeds, _P(prm))
    split = wplanes.split_planes(cost, world, group)
    assert len(split) == world and split[0][0] == 0 and split[-1][1] == prm["nplanes"]
    assert all(a <= b for a, b in split) and all(split[r][1] == split[r + 1][0] for r in range(world - 1))
    if prm["nplanes"] >= group * world:
        assert all(a % group == 0 for a, _ in split)
    if world > 1 and prm["nplanes"] >= 4 * group * world:
        share = [cost[a:b].sum() for a, b in split]
        assert max(share) <= cost.sum() / world + group * cost.max() + 1e-9


def test_split_rejects_bad_world():
    with pytest.raises(ValueError):
        wplanes.split_planes(np.ones(10), 0)


@pytest.mark.parametrize("W", [4, 6])
def test_oracle_plane_shares_sum_to_the_image(W):
    uvw, f, vis, w, px = _case()
    full = oracle.ms2dirty(uvw, f, vis, w, NPIX, NPIX, px, px, support=W, do_wstacking=True, nthreads=1)
    prm = _params(uvw, f, px, W)
    split = wplanes.split_planes(np.ones(prm["nplanes"]), 3, 3)
    be = OracleWPlaneBackend(uvw, f, vis, w, px, W)
    img = wplanes.invert_wplanes_local(be, split).numpy()
    assert np.abs(img - full / be.sumw).max() < 1e-13 * np.abs(full / be.sumw).max()
    # an empty range is a zero image
    z, _ = be((2, 2))
    assert float(z.abs().max()) == 0.0


def _worker(rank, world, port, q, W):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "ska-sdp-continuum-imaging-pipeline_amd"), str(root / "oracle"), str(root / "tests")]
    from test_wplanes import OracleWPlaneBackend, _P, _case, _params  # noqa: F811

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uvw, f, vis, w, px = _case()
    prm = _params(uvw, f, px, W)
    feeds = wplanes.plane_feeds(torch.from_numpy(uvw), torch.from_numpy(f), _P(prm))
    split = wplanes.split_planes(wplanes.plane_cost(feeds, _P(prm)), world)
    be = OracleWPlaneBackend(uvw, f, vis, w, px, W)
    img = wplanes.invert_wplanes(be, split, dst=0)
    if rank == 0:
        full = oracle.ms2dirty(uvw, f, vis, w, NPIX, NPIX, px, px, support=W, do_wstacking=True, nthreads=1)
        full /= be.sumw
        q.put((float(np.abs(img.numpy() - full).max()), float(np.abs(full).max()), split))
    else:
        assert img is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W", [(2, 6), (3, 4)])
def test_wplane_split_gloo(world, W):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, W)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    err, peak, split = q.get(timeout=5)
    assert err < 1e-13 * max(1.0, peak)
    assert sum(b > a for a, b in split) >= 2  # the planes really were split
