"""
bench.py's N > 1 correctness checks on CPU (gloo, world size 2): every rank
sums the fp64 DFT of its own share at the fixed pixels, the sums are
all-reduced, and rank 0 compares them with the image it holds - the reduced
image of the weak headline (`weak_parity`, row shards) and the gathered image
of the strong split (`strong_parity`, uv strips). Here the image on rank 0 is
the CPU oracle's image of ALL ranks' visibilities, so both checks must pass
(and flag a wrong image).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from ska_sdp_cip_amd import strips
from ska_sdp_cip_amd import synthetic as syn

NPIX = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case():
    ms = syn.make_measurement_set(600, 8, n_ant=10, array_radius_m=700.0, seed=9)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, NPIX)
    img = oracle.ms2dirty(uvw, f, vis, w, NPIX, NPIX, px, px, support=12) / float(w.astype(np.float64).sum())
    return uvw, f, vis, w, px, img


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        uvw, f, vis, w, px, img = _case()
        dev = torch.device("cpu")
        t = torch.from_numpy
        a, b = [(0, 250), (250, 600)][rank]
        good = t(img) if rank == 0 else None
        weak = bench.weak_parity(t(uvw[a:b]), t(f), t(vis[a:b]), t(w[a:b]), good, NPIX, px, False, world, rank, dev)
        bad = bench.weak_parity(t(uvw[a:b]), t(f), t(vis[a:b]), t(w[a:b]), None if rank else t(img * 1.01), NPIX, px,
                                False, world, rank, dev)
        # strips: the same visibilities in the Tile layout of two uv strips
        prm = oracle.choose_params(NPIX, NPIX, px, px, support=8)

        class P:
            nu, nv, support = prm["nu"], prm["nv"], prm["support"]

        layout = strips.plan_strips(t(uvw), t(f), P, px, NPIX, NPIX, world, balance="vis")
        rws, c0, c1 = strips.strip_slices(t(uvw), t(f), P, px, *layout.rows(rank))
        data = strips.gather_strip(t(uvw), t(vis), t(w), rws, c0, c1)
        strong = bench.strong_parity(data, t(f), good, NPIX, px, world, rank, dev)
        q.put((rank, weak, bad, strong))
    finally:
        dist.destroy_process_group()


def test_reduced_and_gathered_image_parity_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, weak, bad, strong = q.get(timeout=240)
        out[rank] = (weak, bad, strong)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[1] == (None, None, None)
    weak, bad, strong = out[0]
    # W = 12 oracle image vs the DFT: ~5e-11 of sum w
    assert weak["ok"] and weak["max_err_dft_pixels"] < 1e-9
    assert strong["ok"] and strong["max_err_dft_pixels"] < 1e-9
    assert abs(weak["sum_weights"] - strong["sum_weights"]) <= 1e-9 * weak["sum_weights"]
    assert bad["max_err_dft_pixels"] > 1e-4 * float(np.abs(_case()[-1]).max())
    assert strong["image_checksum"]["sum"] == pytest.approx(float(_case()[-1].sum()), rel=1e-12)
