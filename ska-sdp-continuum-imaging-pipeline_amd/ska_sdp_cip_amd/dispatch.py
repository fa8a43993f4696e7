"""
Task dispatch for the dask-shaped API (`dask_invert_measurement_set`,
`reorder_by_uvw_tile`).

dask is not installed in this image; the reference's tasks
(`client.submit(..., resources={"processing_slots": 1})`, invert.py:256-267,
reorder.py:68-82) are duck-typed against any client with `submit` and
`scheduler_info`. `LocalGPUClient` runs each task immediately on one of the
local GPUs (round robin), which is the single-node form of the
"dask-task -> HIP-stream" dispatch: a task owns one device and
enqueues its kernels on that device's current stream. With a real dask
`Client`, give each GPU worker a `{"gpu": 1}` resource and pin it to one
device with HIP_VISIBLE_DEVICES.
"""

from __future__ import annotations

from typing import Any, Iterable, Optional


class LocalFuture:
    """An already-computed result with the `Future.result()` interface."""

    def __init__(self, value: Any) -> None:
        self._value = value

    def result(self) -> Any:
        """The task's return value."""
        return self._value


def _resolve(obj):
    if isinstance(obj, LocalFuture):
        return obj.result()
    if isinstance(obj, list):
        return [_resolve(o) for o in obj]
    if isinstance(obj, tuple):
        return tuple(_resolve(o) for o in obj)
    return obj


class LocalGPUClient:
    """Synchronous client that runs tasks on local GPUs in round robin."""

    def __init__(self, devices: Optional[Iterable[int]] = None) -> None:
        import torch  # pylint: disable=import-outside-toplevel

        if devices is None:
            n = torch.cuda.device_count() if torch.cuda.is_available() else 0
            devices = range(max(n, 1))
        self.devices = list(devices)
        self._next = 0

    def scheduler_info(self) -> dict:
        """Mimics dask's `Client.scheduler_info()` worker listing."""
        return {"workers": {f"gpu-{d}": {"resources": {"gpu": 1}} for d in self.devices}}

    def submit(self, fn, *args, resources=None, pure=None, **kwargs):  # noqa: ARG002
        """Run `fn` now; GPU tasks (resources={'gpu': 1}) go to the next device."""
        args = _resolve(args)
        kwargs = {k: _resolve(v) for k, v in kwargs.items()}
        if resources and "gpu" in resources:
            import torch  # pylint: disable=import-outside-toplevel

            dev = self.devices[self._next % len(self.devices)]
            self._next += 1
            if torch.cuda.is_available():
                with torch.cuda.device(dev):
                    return LocalFuture(fn(*args, **kwargs))
        return LocalFuture(fn(*args, **kwargs))


def as_completed(futures: Iterable[LocalFuture]):
    """dask.distributed.as_completed for LocalFutures (submission order)."""
    yield from futures


def get_worker_threads() -> int:
    """Threads of the current dask worker, else the host CPU count."""
    import os  # pylint: disable=import-outside-toplevel

    try:
        from dask.distributed import get_worker  # pylint: disable=import-outside-toplevel

        return get_worker().state.nthreads
    except (ImportError, ValueError):
        return os.cpu_count() or 1
