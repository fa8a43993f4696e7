"""
world_size-2 gloo test of the multi-GPU invert decomposition on CPU: each
rank images its row shard (with the CPU oracle standing in for the GPU
pipeline, which is linear), `reduce_images` sums the partial images and
weights onto rank 0, and the result equals the single-process image of the
whole set (reference invert.py:200-209 semantics).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ska_sdp_cip_amd.distributed import image_buffer, reduce_images, shard_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, npix, q, fused=False, async_op=False):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "ska-sdp-continuum-imaging-pipeline_amd"), str(root / "oracle")]
    import oracle
    from ska_sdp_cip_amd import synthetic as syn

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ms = syn.make_measurement_set(801, 3, n_ant=12, array_radius_m=800.0, seed=4)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    a, b = shard_rows(len(uvw), rank, world)
    part = oracle.ms2dirty(uvw[a:b], f, vis[a:b], w[a:b], npix, npix, px, px, support=8, nthreads=1)
    if fused:  # image and weight sum in one buffer: a single collective
        img, sw = image_buffer(npix, npix, "cpu")
        img.copy_(torch.from_numpy(part))
        sw.fill_(float(w[a:b].astype(np.float64).sum()))
    else:
        img = torch.from_numpy(part.copy())
        sw = torch.tensor([w[a:b].astype(np.float64).sum()], dtype=torch.float64)
    if async_op:  # pipelined form (bench.py): the collective in flight, then wait()
        pending = reduce_images(img, sw, dst=0, async_op=True)
        assert pending.wait() is img
    else:
        reduce_images(img, sw, dst=0)
    if rank == 0:
        full = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, nthreads=1)
        q.put(float(np.abs(img.numpy() - full / w.astype(np.float64).sum()).max()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_rows_cover_everything():
    for n, world in [(10, 3), (801, 2), (5, 8), (390_625, 8)]:
        bounds = [shard_rows(n, r, world) for r in range(world)]
        covered = np.zeros(n, dtype=int)
        for a, b in bounds:
            covered[a:b] += 1
        assert (covered == 1).all()
    with pytest.raises(ValueError):
        shard_rows(10, 3, 3)


@pytest.mark.parametrize("fused,async_op", [(False, False), (True, False), (True, True)])
def test_sharded_invert_reduce_world2(fused, async_op):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 64, q, fused, async_op)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) < 1e-13
