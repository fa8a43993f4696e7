"""
Task metrics of a distributed invert as JSON (reference
src/ska_sdp_cip/task_metrics.py:1-135, same API and output): `TaskMetrics`
parses a dask-style task stream - the `data` of `get_task_stream()`, or of
`LocalGPUClient.get_task_stream()` for the GPU tasks of the local dispatch
(dispatch.py) - into `Task` records {key, worker, status, start, stop, name,
duration} and saves them with `save_json` (loadable with `pandas.read_json`).
Entries of GPU tasks carry the device they ran on; it is kept as an extra
`device` field of their records.
"""

from __future__ import annotations

import collections.abc
import json
import os
from dataclasses import dataclass, field
from typing import Optional, Union

_KEYS = ("key", "worker", "status", "start", "stop", "name", "duration")


@dataclass
class Task:
    """One task of the stream: `start` / `stop` are UNIX timestamps spanning
    all its start-stop intervals (transfer and compute); `name` is the key up
    to its last "-" (the function name); `duration` = stop - start
    (reference task_metrics.py:10-85)."""

    key: str
    worker: str
    status: str
    start: float
    stop: float
    device: Optional[int] = None
    name: str = field(init=False)
    duration: float = field(init=False)

    def __post_init__(self) -> None:
        self.name = self.key.rsplit("-", maxsplit=1)[0]
        self.duration = self.stop - self.start

    def as_dict(self) -> dict:
        """The record as a dict (the reference's seven keys, plus `device` for
        GPU tasks)."""
        out = {k: getattr(self, k) for k in _KEYS}
        if self.device is not None:
            out["device"] = self.device
        return out

    @classmethod
    def from_task_stream_entry(cls, entry: dict) -> "Task":
        """From one entry of a task stream: {key, worker, status, startstops:
        ({action, start, stop}, ...)[, device]}."""
        startstops = entry["startstops"]
        return cls(key=entry["key"], worker=entry["worker"], status=entry["status"],
                   start=min(s["start"] for s in startstops), stop=max(s["stop"] for s in startstops),
                   device=entry.get("device"))


class TaskMetrics(collections.abc.Sequence):
    """Sequence of `Task` parsed from task stream data (reference
    task_metrics.py:88-135)."""

    def __init__(self, task_stream_data: list) -> None:
        self._task_list = [Task.from_task_stream_entry(e) for e in task_stream_data]

    def __len__(self) -> int:
        return len(self._task_list)

    def __getitem__(self, index):
        return self._task_list[index]

    def to_json(self, **kwargs) -> str:
        """JSON list of the task records; kwargs go to `json.dumps`."""
        return json.dumps([t.as_dict() for t in self._task_list], **kwargs)

    def save_json(self, path: Union[str, os.PathLike], **kwargs) -> None:
        """Write `to_json(**kwargs)` to `path`."""
        with open(path, "w", encoding="utf-8") as fh:
            fh.write(self.to_json(**kwargs))


__all__ = ["Task", "TaskMetrics"]
