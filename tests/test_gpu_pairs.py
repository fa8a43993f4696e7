"""
Time pairs of the 2-D fp64-class scatter (cip_plan.hip
pair_stride_kernel + place pass, cip_grid.hip order_kernel<.., PAIRS>,
cip_scatter.h scatter_pair_kernel): rows of a time-major MS pair with the same
baseline one dump later (row + D, D detected on the device) when both
footprints start on the same cell, and one 64-bit atomic per tap grids both.

* the stride is detected (profile counter `pair_stride` = the baselines per
  dump) and the image equals the CPU oracle at the fp64 gate;
* the same call with CIP_PAIRS=0 (time pairs are opt-in: CIP_PAIRS=1, read
  per call; here in child processes) gives the same image to the fixed-point
  quantum (a pair's integer is within one quantum of its two separately
  rounded contributions);
* NaN visibilities under zero weights - in leaders and in absorbed partners -
  stay out of the image; complex128 input, no weights, the PSF, W = 4 / 16;
* rows that are not time-major (shuffled) find no stride and grid as before.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import _lib
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _pairs_on(monkeypatch):
    # time pairs are opt-in (CIP_PAIRS=1, read per call)
    monkeypatch.setenv("CIP_PAIRS", "1")


ROOT = Path(__file__).resolve().parents[1]
N_ANT = 20
NBL = N_ANT * (N_ANT - 1) // 2  # 190 baselines per dump


def _case(nrow=190 * 24, nchan=24, npix=512, seed=5):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=N_ANT, array_radius_m=1200.0, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    return uvw, f, vis, w, px


def _t(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _invert(dev, uvw, f, vis, w, npix, px, **kw):
    _lib.profile_enable(True)
    try:
        img, _ = device_ms2dirty(_t(dev, uvw), _t(dev, f), None if vis is None else _t(dev, vis),
                                 None if w is None else _t(dev, w), npix, npix, px, px, **kw)
        prof = _lib.profile_last()
    finally:
        _lib.profile_enable(False)
    return img.cpu().numpy(), prof


@pytest.mark.parametrize("W,vdt,weighted", [(8, np.complex64, True), (4, np.complex64, True),
                                            (16, np.complex128, True), (8, np.complex128, False)])
def test_pairs_detected_and_equal_oracle(gpu_device, W, vdt, weighted):
    npix = 512
    uvw, f, vis, w, px = _case(npix=npix)
    wt = w.astype(np.float32) if weighted else None
    img, prof = _invert(gpu_device, uvw, f, vis.astype(vdt), wt, npix, px, support=W)
    assert prof["pair_stride"] == NBL
    ref = oracle.ms2dirty(uvw, f, vis.astype(vdt), wt, npix, npix, px, px, support=W)
    sw = float(w.astype(np.float64).sum()) if weighted else float(vis.size)
    assert float(np.abs(img - ref).max()) / sw < 1e-10


def test_psf_with_pairs(gpu_device):
    npix = 512
    uvw, f, vis, w, px = _case(npix=npix)
    img, prof = _invert(gpu_device, uvw, f, None, w.astype(np.float32), npix, px, support=8, psf=True)
    assert prof["pair_stride"] == NBL
    ref = oracle.ms2dirty(uvw, f, np.ones_like(vis), w.astype(np.float32), npix, npix, px, px, support=8)
    assert float(np.abs(img - ref).max()) / float(w.astype(np.float64).sum()) < 1e-10


def test_nan_under_zero_weights_in_pairs(gpu_device):
    npix = 512
    uvw, f, vis, w, px = _case(npix=npix)
    vis = vis.astype(np.complex64)
    w = w.astype(np.float32)
    rng = np.random.default_rng(3)
    bad = rng.uniform(size=vis.shape) < 0.1  # leaders and absorbed partners alike
    vis[bad] = np.nan
    w[bad] = 0.0
    img, prof = _invert(gpu_device, uvw, f, vis, w, npix, px, support=8)
    assert prof["pair_stride"] == NBL
    assert np.isfinite(img).all()
    clean = np.where(bad, 0, vis)
    ref = oracle.ms2dirty(uvw, f, clean, w, npix, npix, px, px, support=8)
    assert float(np.abs(img - ref).max()) / float(w.astype(np.float64).sum()) < 1e-10


def test_shuffled_rows_find_no_stride(gpu_device):
    npix = 512
    uvw, f, vis, w, px = _case(npix=npix)
    perm = np.random.default_rng(1).permutation(uvw.shape[0])
    uvw, vis, w = uvw[perm], vis[perm], w[perm]
    img, prof = _invert(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32), npix, px, support=8)
    assert prof["pair_stride"] == 0
    ref = oracle.ms2dirty(uvw, f, vis.astype(np.complex64), w.astype(np.float32), npix, npix, px, px, support=8)
    assert float(np.abs(img - ref).max()) / float(w.astype(np.float64).sum()) < 1e-10


CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/ska-sdp-continuum-imaging-pipeline_amd"]
from ska_sdp_cip_amd import synthetic as syn, _lib
from ska_sdp_cip_amd.gridder import device_ms2dirty
out = sys.argv[2]
ms = syn.make_measurement_set(190 * 40, 32, n_ant=20, array_radius_m=2500.0, seed=21)
vis = np.ascontiguousarray(ms.visibilities()[..., 0], dtype=np.complex64)
w = np.ascontiguousarray(ms.weights()[..., 0], dtype=np.float32)
uvw, f = ms.uvw(), ms.channel_frequencies()
npix = 1024
px = syn.pixel_size_for_grid(uvw, f, npix)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
_lib.profile_enable(True)
img, _ = device_ms2dirty(t(uvw), t(f), t(vis), t(w), npix, npix, px, px, support=8)
stride = _lib.profile_last()["pair_stride"]
np.savez(out, img=img.cpu().numpy(), stride=stride)
"""


def _child(tmp_path, **env_over):
    out = tmp_path / ("pairs_" + "_".join(f"{k}{v}" for k, v in env_over.items()) + ".npz")
    env = dict(os.environ)
    env["CIP_PAIRS"] = "1"
    env.update(env_over)
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(out)], env=env, check=True, timeout=180)
    return np.load(out)


def test_pairs_equal_unpaired_to_the_quantum(gpu_device, tmp_path):
    on = _child(tmp_path)
    off = _child(tmp_path, CIP_PAIRS="0")
    assert int(on["stride"]) == 190 and int(off["stride"]) == 0
    peak = float(np.abs(off["img"]).max())
    assert float(np.abs(on["img"] - off["img"]).max()) <= 1e-12 * peak
    again = _child(tmp_path)
    assert np.array_equal(again["img"], on["img"])
