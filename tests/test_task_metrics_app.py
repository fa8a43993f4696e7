"""
TaskMetrics (reference task_metrics.py:1-135 semantics: key/worker/status,
start/stop spanning all start-stops, name = key up to its last "-",
duration) on hand-made dask-format task streams and on the task stream the
local dispatch records; the pipeline app's command line matches the
reference's (pipeline_app.py:17-78). CPU only.
"""
import json

import pytest

from ska_sdp_cip_amd.apps.pipeline_app import get_parser
from ska_sdp_cip_amd.dispatch import LocalGPUClient
from ska_sdp_cip_amd.task_metrics import Task, TaskMetrics

STREAM = [
    {"key": "from_measurement_set_reader-5f1c", "worker": "tcp://10.0.0.1:4001", "status": "OK",
     "startstops": ({"action": "transfer", "start": 100.0, "stop": 100.5},
                    {"action": "compute", "start": 100.5, "stop": 103.25})},
    {"key": "worker_ducc_invert-a-b-99", "worker": "tcp://10.0.0.2:4001", "status": "error",
     "startstops": ({"action": "compute", "start": 104.0, "stop": 110.0},)},
    {"key": "integrate_weighted_images-0", "worker": "gpu-3", "status": "OK", "device": 3,
     "startstops": ({"action": "compute", "start": 111.0, "stop": 111.125},)},
]


def test_task_records():
    tm = TaskMetrics(STREAM)
    assert len(tm) == 3 and isinstance(tm[0], Task)
    assert tm[0].as_dict() == {"key": "from_measurement_set_reader-5f1c", "worker": "tcp://10.0.0.1:4001",
                               "status": "OK", "start": 100.0, "stop": 103.25,
                               "name": "from_measurement_set_reader", "duration": 3.25}
    assert tm[1].name == "worker_ducc_invert-a-b" and tm[1].duration == 6.0 and tm[1].status == "error"
    assert tm[2].as_dict()["device"] == 3
    assert json.loads(tm.to_json()) == [t.as_dict() for t in tm]


def test_save_json(tmp_path):
    p = tmp_path / "task-list.json"
    TaskMetrics(STREAM).save_json(p, indent=4, sort_keys=True)
    assert json.loads(p.read_text())[1]["stop"] == 110.0


def test_local_client_task_stream():
    def add(a, b):
        return a + b

    def boom():
        raise RuntimeError("x")

    with LocalGPUClient(devices=[0]) as client:
        with client.get_task_stream() as ts:
            f1 = client.submit(add, 1, 2)
            f2 = client.submit(add, f1, 4)
            f3 = client.submit(boom)
            assert f2.result() == 7
            with pytest.raises(RuntimeError):
                f3.result()
        after = client.submit(add, 0, 0)
        after.result()
    tm = TaskMetrics(ts.data)
    assert sorted(t.name for t in tm) == ["add", "add", "boom"]
    assert {t.status for t in tm if t.name == "boom"} == {"error"}
    assert all(t.worker == "host" and t.duration >= 0.0 for t in tm)


def test_pipeline_cli_matches_reference():
    p = get_parser()
    a = p.parse_args(["ms", "out", "-n", "512", "-p", "2.5"])
    assert (a.num_pixels, a.pixel_size, a.dask_scheduler, a.row_chunks, a.freq_chunks) == (512, 2.5, None, 1, None)
    a = p.parse_args(["ms", "out", "--num-pixels", "64", "--pixel-size", "1", "-d", "local", "-rc", "3", "-fc", "2"])
    assert (a.dask_scheduler, a.row_chunks, a.freq_chunks) == ("local", 3, 2)
    with pytest.raises(SystemExit):
        p.parse_args(["ms", "out", "-p", "1"])  # -n is required
