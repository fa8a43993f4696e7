"""
Task dispatch for the dask-shaped API (`dask_invert_measurement_set`,
`reorder_by_uvw_tile`).

dask is not installed in this image; the reference's tasks
(`client.submit(..., resources={"processing_slots": 1})`, invert.py:256-267,
reorder.py:68-82) are duck-typed against any client with `submit` and
`scheduler_info`. `LocalGPUClient` is the single-node form of the
"dask-task -> HIP-stream" dispatch: every local GPU has one
worker thread (the reference's `processing_slots=1`: one in-flight invert per
device), GPU tasks (`resources={"gpu": 1}`) go to the devices in round robin
and run concurrently across devices, each on its device's current stream with
the library's per-(device, thread) workspace; other tasks run on a host thread
pool. Futures passed as arguments are resolved inside the task, so `submit`
never blocks. `concurrent=False` runs every task at submission instead. With
a real dask `Client`, give each GPU worker a `{"gpu": 1}` resource and pin it
to one device with HIP_VISIBLE_DEVICES.
"""

from __future__ import annotations

import concurrent.futures as cf
import contextlib
import itertools
import threading
import time
from typing import Any, Iterable, Optional


class LocalFuture:
    """A task's result with the `Future.result()` interface (computed already,
    or running on one of the client's threads)."""

    def __init__(self, value: Any = None, future: Optional[cf.Future] = None) -> None:
        self._value = value
        self._future = future

    def result(self, timeout: Optional[float] = None) -> Any:
        """The task's return value (waits for it; re-raises its exception)."""
        return self._future.result(timeout) if self._future is not None else self._value

    def done(self) -> bool:
        """True once the result is available."""
        return self._future is None or self._future.done()


def _resolve(obj):
    if isinstance(obj, LocalFuture):
        return obj.result()
    if isinstance(obj, list):
        return [_resolve(o) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_resolve(o) for o in obj)
    return obj


def _has_cuda() -> bool:
    try:
        import torch  # pylint: disable=import-outside-toplevel
    except ModuleNotFoundError:  # pragma: no cover - torch is in the image
        return False
    return torch.cuda.is_available()


class LocalGPUClient:
    """Client that runs GPU tasks on one worker thread per local GPU (round
    robin, concurrent across devices) and other tasks on a host thread pool."""

    def __init__(self, devices: Optional[Iterable[int]] = None, *, concurrent: bool = True,
                 host_threads: int = 8) -> None:
        if devices is None:
            n = 0
            if _has_cuda():
                import torch  # pylint: disable=import-outside-toplevel

                n = torch.cuda.device_count()
            devices = range(max(n, 1))
        self.devices = list(devices)
        self.concurrent = concurrent
        # load the HIP library here, on the constructing (main) thread: the
        # library treats the thread that loaded it as the process's main thread
        # (its workspaces are left to process teardown), so a GPU worker thread
        # must never be the first caller (its workspace would outlive it)
        if _has_cuda():
            from . import _lib  # pylint: disable=import-outside-toplevel

            _lib.lib()
        self._next = 0
        self._lock = threading.Lock()
        self._streams = []  # active task-stream recorders (get_task_stream)
        self._ids = itertools.count()
        self._gpu_pools = {}
        self._host_pool = None
        if concurrent:
            self._gpu_pools = {d: cf.ThreadPoolExecutor(1, thread_name_prefix=f"cip-gpu{d}",
                                                        initializer=self._bind, initargs=(d,))
                               for d in self.devices}
            self._host_pool = cf.ThreadPoolExecutor(max(host_threads, 1), thread_name_prefix="cip-host")

    @staticmethod
    def _bind(device: int) -> None:
        # the worker thread's current device: the library's workspace and the
        # stream the task's kernels go to
        if _has_cuda():
            import torch  # pylint: disable=import-outside-toplevel

            torch.cuda.set_device(device)

    def scheduler_info(self) -> dict:
        """Mimics dask's `Client.scheduler_info()` worker listing."""
        return {"workers": {f"gpu-{d}": {"resources": {"gpu": 1}} for d in self.devices}}

    def _pick_device(self) -> int:
        with self._lock:
            dev = self.devices[self._next % len(self.devices)]
            self._next += 1
        return dev

    def submit(self, fn, *args, resources=None, pure=None, **kwargs):  # noqa: ARG002
        """Queue `fn(*args, **kwargs)`; GPU tasks (resources={'gpu': 1}) go to
        the next device's worker. Returns a LocalFuture."""
        gpu = bool(resources and "gpu" in resources)
        dev = self._pick_device() if gpu else None

        key = f"{getattr(fn, '__name__', 'task')}-{next(self._ids):08x}"

        def run():
            a = _resolve(args)
            kw = {k: _resolve(v) for k, v in kwargs.items()}
            if dev is not None and _has_cuda():
                import torch  # pylint: disable=import-outside-toplevel

                with torch.cuda.device(dev):
                    out = fn(*a, **kw)
                    torch.cuda.current_stream(dev).synchronize()  # the task ends when its GPU work does
                    return out
            return fn(*a, **kw)

        def task():
            t0 = time.time()
            status = "OK"
            try:
                return run()
            except BaseException:
                status = "error"
                raise
            finally:
                self._record(key, dev, status, t0, time.time())

        if not self.concurrent:
            return LocalFuture(task())
        pool = self._gpu_pools[dev] if gpu else self._host_pool
        return LocalFuture(future=pool.submit(task))

    def _record(self, key: str, dev: Optional[int], status: str, start: float, stop: float) -> None:
        if not self._streams:
            return
        entry = {"key": key, "worker": f"gpu-{dev}" if dev is not None else "host", "status": status,
                 "startstops": ({"action": "compute", "start": start, "stop": stop},)}
        if dev is not None:
            entry["device"] = dev
        with self._lock:
            for rec in self._streams:
                rec.data.append(entry)

    @contextlib.contextmanager
    def get_task_stream(self):
        """Record the tasks that finish inside the block, in dask's
        `get_task_stream()` format (`.data`: {key, worker, status,
        startstops[, device]} per task), for `task_metrics.TaskMetrics`."""
        rec = _TaskStream()
        with self._lock:
            self._streams.append(rec)
        try:
            yield rec
        finally:
            with self._lock:
                self._streams.remove(rec)

    def close(self) -> None:
        """Wait for the queued tasks and stop the worker threads."""
        for pool in list(self._gpu_pools.values()) + ([self._host_pool] if self._host_pool else []):
            pool.shutdown(wait=True)
        self._gpu_pools = {}
        self._host_pool = None
        self.concurrent = False

    def __enter__(self) -> "LocalGPUClient":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


class _TaskStream:
    """Recorded task stream (`data`: list of dask-format entries)."""

    def __init__(self) -> None:
        self.data = []


def as_completed(futures: Iterable[LocalFuture]):
    """dask.distributed.as_completed for LocalFutures: in completion order."""
    futures = list(futures)
    done = [f for f in futures if f._future is None]  # pylint: disable=protected-access
    yield from done
    pending = {f._future: f for f in futures if f._future is not None}  # pylint: disable=protected-access
    for fut in cf.as_completed(pending):
        yield pending[fut]


def get_worker_threads() -> int:
    """Threads of the current dask worker, else the host CPU count."""
    import os  # pylint: disable=import-outside-toplevel

    try:
        from dask.distributed import get_worker  # pylint: disable=import-outside-toplevel

        return get_worker().state.nthreads
    except (ImportError, ValueError):
        return os.cpu_count() or 1
