"""
The pipeline app end to end on the GPU (reference apps/pipeline_app.py
flow): serial invert and the distributed form over the local GPU dispatch
(`-d local`) give the same image; the distributed run writes task-list.json
with its GPU tasks (TaskMetrics); `--stokes-on-device` (Stokes I inside the
gridder) agrees with the host Stokes path.
"""
import json

import numpy as np
import pytest

from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.apps.pipeline_app import run_program

pytestmark = pytest.mark.gpu


@pytest.fixture()
def ms_file(tmp_path):
    ms = syn.make_measurement_set(2000, 8, n_ant=16, array_radius_m=1000.0, seed=11)
    path = tmp_path / "set.npz"
    ms.save_npz(path)
    return path


def test_pipeline_app_serial_and_local_dask(gpu_device, ms_file, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    run_program([str(ms_file), "serial", "-n", "64", "-p", "20"])
    serial = np.load(tmp_path / "serial.npy")
    assert serial.shape == (64, 64) and serial.dtype == np.float32
    run_program([str(ms_file), "dist", "-n", "64", "-p", "20", "-d", "local", "-rc", "2", "-fc", "2"])
    dist = np.load(tmp_path / "dist.npy")
    # chunked == serial (linearity; the reference checks 1e-5, tests/test_dask_invert_measurement_set.py)
    assert np.abs(dist - serial).max() <= 1e-5 * np.abs(serial).max()
    tasks = json.loads((tmp_path / "task-list.json").read_text())
    gpu = [t for t in tasks if t["name"] == "worker_ducc_invert"]
    assert len(gpu) == 4 and all(t["device"] == 0 and t["worker"] == "gpu-0" and t["status"] == "OK" for t in gpu)
    assert {t["name"] for t in tasks} == {"from_measurement_set_reader", "worker_ducc_invert",
                                          "integrate_weighted_images"}
    run_program([str(ms_file), "dev", "-n", "64", "-p", "20", "-d", "local", "-rc", "2", "-fc", "2",
                 "--stokes-on-device"])
    dev = np.load(tmp_path / "dev.npy")
    assert np.abs(dev - serial).max() <= 1e-5 * np.abs(serial).max()
    tasks = json.loads((tmp_path / "task-list.json").read_text())
    assert sorted({t["name"] for t in tasks}) == ["integrate_weighted_images", "worker_device_invert"]
