"""
The DISTRIBUTED strip invert (strips.invert_strips: halo send/recv, weight-sum
all-reduce, mask all-gather, packed pass A, sparse all-to-all with the unpack
kernel, image gather) with its ranks as threads on ONE GPU: torch.distributed's
collectives are replaced for the test by an in-memory, barrier-synchronised
stand-in (one host thread per rank, each with its own library workspace). The
gloo tests (test_strips.py) run the same function across processes with the
CPU restatement of the kernels; this runs the GPU backend's path - the one an
8-GPU `bench.py --strong` takes - and compares the gathered image with the
one-shot cip_ms2dirty image.
"""
import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import strips
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty
from _thread_dist import run_ranks

pytestmark = pytest.mark.gpu


def _case(nrow, nchan, npix, seed=7):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=1500.0, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    return uvw, f, vis, w, syn.pixel_size_for_grid(uvw, f, npix)


@pytest.mark.parametrize("world,wstack,gather_async", [(2, False, False), (3, False, True), (4, False, False),
                                                       (3, True, False)])
def test_distributed_strips_as_threads_equal_one_shot(gpu_device, monkeypatch, world, wstack, gather_async):
    npix = 512
    uvw, f, vis, w, px = _case(12000 if wstack else 30000, 16 if wstack else 32, npix)
    if wstack:
        uvw = uvw * np.array([1.0, 1.0, 20.0])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu_device)  # noqa: E731
    tu, tf, tv, tw = t(uvw), t(f), t(vis.astype(np.complex64)), t(w.astype(np.float32))
    ref, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=8, do_wstacking=wstack, normalise=True)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
    datas = []
    for r in range(world):
        datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
    torch.cuda.synchronize()
    stages = [dict() for _ in range(world)]

    def rank_fn(r):
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
        out = strips.invert_strips(datas[r], tf, layout, be, stages=stages[r], gather_async=gather_async)
        if gather_async:
            out = out.wait()
        torch.cuda.synchronize()
        # the rank's buffer is left clean for its next invert
        assert float(be.grid.abs().max()) == 0.0 and not be.dirty
        return out

    results, errors = run_ranks(monkeypatch, world, rank_fn)
    assert not errors, errors
    assert all(r is None for r in results[1:])
    img = results[0]
    peak = float(ref.abs().max())
    assert float((img - ref).abs().max()) < 1e-12 * peak
    # the sparse exchange ran (pass A wrote the packed send buffers)
    assert all(st.get("a2a_send_bytes", 0) > 0 for st in stages)


@pytest.mark.parametrize("world", [2, 4])
def test_back_to_back_async_gathers_equal_one_shot(gpu_device, monkeypatch, world):
    """bench.py --strong's step pattern with real stream ordering: each rank
    queues invert k + 1 (gridding into the same strip buffer, halo and
    all-to-all collectives) while invert k's image-row gather is still in
    flight on its communicator stream (tests/_thread_dist.py: asynchronous
    collectives, a stream per rank, no device synchronisation), then waits
    for both. Two different data sets alternate, so a gather that read a
    later step's rows, or a buffer reused too early, gives a wrong image."""
    npix = 512
    uvw, f, vis, w, px = _case(30000, 32, npix)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu_device)  # noqa: E731
    tu, tf, tw = t(uvw), t(f), t(w.astype(np.float32))
    tvs = [t(vis.astype(np.complex64)), t((vis * (0.25 - 1.5j)).astype(np.complex64))]
    refs, prm = [], None
    for tv in tvs:
        ref, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=8, normalise=True)
        refs.append(ref)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
    datas = [[strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)) for r in range(world)] for tv in tvs]
    torch.cuda.synchronize()
    nsteps = 4

    def rank_fn(r):
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
        pend, imgs = None, []
        for k in range(nsteps):
            nxt = strips.invert_strips(datas[k % 2][r], tf, layout, be, gather_async=True)
            if pend is not None:
                imgs.append(pend.wait())
            pend = nxt
        imgs.append(pend.wait())
        torch.cuda.current_stream().synchronize()
        assert float(be.grid.abs().max()) == 0.0 and not be.dirty
        return imgs

    results, errors = run_ranks(monkeypatch, world, rank_fn)
    assert not errors, errors
    assert all(img is None for res in results[1:] for img in res)
    imgs = results[0]
    assert len(imgs) == nsteps
    for k, img in enumerate(imgs):
        ref = refs[k % 2]
        assert float((img - ref).abs().max()) < 1e-12 * float(ref.abs().max()), k
    # every collective went through the asynchronous stand-in
    from _thread_dist import run_ranks as rr
    assert min(rr.last.calls) >= nsteps * 4
