"""
In-memory stand-in for the torch.distributed calls strips.py makes, for ranks
that are host threads on one GPU (test infrastructure: tests/
test_gpu_strips_threads.py, tests/test_gpu_c4.py).
"""
import threading

import torch
import torch.distributed as tdist

NAMES = ("is_available", "is_initialized", "get_world_size", "get_rank", "isend", "irecv", "P2POp",
         "batch_isend_irecv", "all_reduce", "all_gather", "all_to_all_single", "gather")


class _Work:
    def wait(self):
        return True


class ThreadDist:
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



def run_ranks(monkeypatch, world, fn):
    """fn(rank) on `world` threads with torch.distributed replaced -> (results, errors)."""
    fake = ThreadDist(world)
    for name in NAMES:
        monkeypatch.setattr(tdist, name, getattr(fake, name))
    results, errors = [None] * world, []

    def run(r):
        try:
            fake.local.rank = r
            results[r] = fn(r)
        except Exception as e:  # pylint: disable=broad-except
            errors.append((r, repr(e)))
            fake.barrier.abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=600)
    return results, errors
