"""
In-memory stand-in for the torch.distributed calls strips.py makes, for ranks
that are host threads on one GPU (test infrastructure: tests/
test_gpu_strips_threads.py, tests/test_gpu_c4.py).

Asynchronous like RCCL (round 6): every rank thread runs on its own current
stream, and a collective neither synchronises the device nor blocks the host
beyond the ranks' host rendezvous. Each rank stages its input on its own
communicator stream after the work already queued on its current stream (an
event), the ranks exchange the staged tensors and their events on the host,
and each rank's communicator stream waits for every peer's staging event and
copies the peers' data into its outputs. A collective returns a work object
whose wait() makes the caller's CURRENT STREAM wait for that copy (a device
wait, as `Work.wait()` does for NCCL/RCCL); the blocking forms wait at once.
So an asynchronous gather (`invert_strips(..., gather_async=True)`) really is
still in flight while the caller queues its next invert, and buffer reuse or
stream ordering mistakes show up as wrong images.
"""
import threading

import torch
import torch.distributed as tdist

NAMES = ("is_available", "is_initialized", "get_world_size", "get_rank", "isend", "irecv", "P2POp",
         "batch_isend_irecv", "all_reduce", "all_gather", "all_to_all_single", "gather")


class _Work:
    """A collective in flight on the rank's communicator stream."""

    def __init__(self, done):
        self._done = done

    def wait(self):
        torch.cuda.current_stream().wait_event(self._done)
        return True

    def is_completed(self):
        return self._done.query()


class ThreadDist:
    """torch.distributed's calls used by strips.py, for ranks that are threads."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=300)
        self.slots = [None] * world
        self.local = threading.local()
        self.keep = []  # staged tensors: alive until the ranks finish (peers' streams read them)
        self.lock = threading.Lock()
        self.calls = [0] * world  # collectives per rank (the tests check they ran)

    def rank(self):
        return self.local.rank

    def _comm(self):
        if getattr(self.local, "comm", None) is None:
            self.local.comm = torch.cuda.Stream()
        return self.local.comm

    def _collective(self, stage, deliver):
        """stage(): this rank's payload (tensors cloned on the communicator
        stream after the caller's queued work); deliver(vals): copy the peers'
        staged payloads into this rank's outputs (on the communicator stream,
        after every peer's staging). Returns the work object."""
        cur, comm = torch.cuda.current_stream(), self._comm()
        ready = torch.cuda.Event()
        ready.record(cur)
        comm.wait_event(ready)
        with torch.cuda.stream(comm):
            payload = stage()
            staged = torch.cuda.Event()
            staged.record(comm)
        with self.lock:
            self.keep.append(payload)
            self.calls[self.rank()] += 1
        self.slots[self.rank()] = (payload, staged)
        self.barrier.wait()
        vals = list(self.slots)
        self.barrier.wait()
        for _, ev in vals:
            comm.wait_event(ev)
        with torch.cuda.stream(comm):
            deliver([v for v, _ in vals])
            done = torch.cuda.Event()
            done.record(comm)
        return _Work(done)

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
        def stage():
            return {peer: t.clone() for op, t, peer in ops if op == self.isend}

        def deliver(vals):
            for op, t, peer in ops:
                if op == self.irecv:
                    t.copy_(vals[peer][self.rank()], non_blocking=True)

        return [self._collective(stage, deliver)]

    def all_reduce(self, t, group=None, op=None, async_op=False):
        def deliver(vals):
            acc = vals[0].clone()
            for v in vals[1:]:
                acc += v
            t.copy_(acc)

        w = self._collective(lambda: t.clone(), deliver)
        if async_op:
            return w
        w.wait()
        return None

    def all_gather(self, out, t, group=None, async_op=False):
        def deliver(vals):
            for o, v in zip(out, vals):
                o.copy_(v, non_blocking=True)

        w = self._collective(lambda: t.clone(), deliver)
        if async_op:
            return w
        w.wait()
        return None

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None,
                          async_op=False):
        def deliver(vals):
            out.copy_(torch.cat([vals[s][self.rank()] for s in range(self.world)]), non_blocking=True)

        w = self._collective(lambda: [c.clone() for c in torch.split(inp, input_split_sizes)], deliver)
        if async_op:
            return w
        w.wait()
        return None

    def gather(self, t, gather_list=None, dst=0, group=None, async_op=False):
        me = self.rank()

        def deliver(vals):
            if me == dst:
                for o, v in zip(gather_list, vals):
                    o.copy_(v, non_blocking=True)

        w = self._collective(lambda: t.clone(), deliver)
        if async_op:
            return w
        w.wait()
        return None


def run_ranks(monkeypatch, world, fn):
    """fn(rank) on `world` threads with torch.distributed replaced, each rank
    on its own current stream -> (results, errors)."""
    fake = ThreadDist(world)
    for name in NAMES:
        monkeypatch.setattr(tdist, name, getattr(fake, name))
    results, errors = [None] * world, []

    def run(r):
        try:
            fake.local.rank = r
            with torch.cuda.stream(torch.cuda.Stream()):
                results[r] = fn(r)
                torch.cuda.current_stream().synchronize()
        except Exception as e:  # pylint: disable=broad-except
            errors.append((r, repr(e)))
            fake.barrier.abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=900)
    torch.cuda.synchronize()
    run_ranks.last = fake
    return results, errors
