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
import threading

import numpy as np
import pytest
import torch
import torch.distributed as tdist

import oracle
from ska_sdp_cip_amd import strips
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


class _Work:
    def wait(self):
        return True


class _ThreadDist:
    """torch.distributed's calls used by strips.py, for ranks that are threads."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=120)
        self.slots = [None] * world
        self.local = threading.local()

    def rank(self):
        return self.local.rank

    def _exchange(self, obj):
        self.slots[self.rank()] = obj
        torch.cuda.synchronize()
        self.barrier.wait()
        vals = list(self.slots)
        self.barrier.wait()
        return vals

    # -- the API surface
    def is_available(self):
        return True

    def is_initialized(self):
        return True

    def get_world_size(self, group=None):
        return self.world

    def get_rank(self, group=None):
        return self.rank()

    def isend(self, *a, **k):
        raise AssertionError("only through batch_isend_irecv")

    def irecv(self, *a, **k):
        raise AssertionError("only through batch_isend_irecv")

    def P2POp(self, op, tensor, peer, group=None):  # noqa: N802
        return (op, tensor, peer)

    def batch_isend_irecv(self, ops):
        sends = {peer: t.clone() for op, t, peer in ops if op == self.isend}
        vals = self._exchange(sends)
        for op, t, peer in ops:
            if op == self.irecv:
                t.copy_(vals[peer][self.rank()])
        torch.cuda.synchronize()
        return [_Work()]

    def all_reduce(self, t, group=None, op=None):
        vals = self._exchange(t.clone())
        acc = vals[0].clone()
        for v in vals[1:]:
            acc += v
        t.copy_(acc)

    def all_gather(self, out, t, group=None):
        vals = self._exchange(t.clone())
        for o, v in zip(out, vals):
            o.copy_(v)

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None):
        vals = self._exchange([c.clone() for c in torch.split(inp, input_split_sizes)])
        out.copy_(torch.cat([vals[s][self.rank()] for s in range(self.world)]))

    def gather(self, t, gather_list=None, dst=0, group=None, async_op=False):
        vals = self._exchange(t.clone())
        if self.rank() == dst:
            for o, v in zip(gather_list, vals):
                o.copy_(v)
        return _Work() if async_op else None


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
        rows, c0, c1 = strips.strip_slices(tu, tf, prm, px, *layout.rows(r))
        datas.append(strips.gather_strip(tu, tv, tw, rows, c0, c1))
    torch.cuda.synchronize()
    fake = _ThreadDist(world)
    for name in ("is_available", "is_initialized", "get_world_size", "get_rank", "isend", "irecv", "P2POp",
                 "batch_isend_irecv", "all_reduce", "all_gather", "all_to_all_single", "gather"):
        monkeypatch.setattr(tdist, name, getattr(fake, name))
    results, errors, stages = [None] * world, [], [dict() for _ in range(world)]

    def run(r):
        try:
            fake.local.rank = r
            be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
            out = strips.invert_strips(datas[r], tf, layout, be, stages=stages[r], gather_async=gather_async)
            if gather_async:
                out = out.wait()
            torch.cuda.synchronize()
            results[r] = out
            # the rank's buffer is left clean for its next invert
            assert float(be.grid.abs().max()) == 0.0 and not be.dirty
        except Exception as e:  # pylint: disable=broad-except
            errors.append((r, repr(e)))
            fake.barrier.abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
    assert not errors, errors
    assert all(r is None for r in results[1:])
    img = results[0]
    peak = float(ref.abs().max())
    assert float((img - ref).abs().max()) < 1e-12 * peak
    # the sparse exchange ran (pass A wrote the packed send buffers)
    assert all(st.get("a2a_send_bytes", 0) > 0 for st in stages)
