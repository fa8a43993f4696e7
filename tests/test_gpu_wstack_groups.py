"""
w-stacking plane groups (G = 2..3 planes per scatter work unit, up to 5 in the
packed single class: each visibility placed and its u, v, w kernels evaluated
once for all of them) against one plane per
unit (CIP_WSTACK_GROUP=1, in a child process since the switch is read once):
the same images up to the fp64 flush order of differently cut work units, for
W = 4..16, odd plane counts, the packed single class, repeated calls (the
plane pair left clean by the masked FFT pass A), the accumulating path, and a
2-D call after a w-stacking call on the same workspace.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.accumulate import GridAccumulator
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

CASES = [dict(support=6, npix=512), dict(support=8, npix=512), dict(support=4, npix=256),
         dict(support=16, npix=512), dict(support=6, npix=512, single=True), dict(support=12, npix=384),
         # the packed class's larger groups (round 4): 5 planes per unit up to W = 8, 4 at W = 10
         dict(support=8, npix=512, single=True), dict(support=10, npix=384, single=True),
         dict(support=4, npix=256, single=True), dict(support=16, npix=512, single=True)]

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/ska-sdp-continuum-imaging-pipeline_amd"]
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty
W, npix, single, out = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1", sys.argv[5]
ms = syn.make_measurement_set(4000, 16, n_ant=24, array_radius_m=2500.0, seed=8)
vis = np.ascontiguousarray(ms.visibilities()[..., 0], dtype=np.complex64)
w = np.ascontiguousarray(ms.weights()[..., 0], dtype=np.float32)
uvw, f = ms.uvw(), ms.channel_frequencies()
px = syn.pixel_size_for_grid(uvw, f, npix)
t = lambda a: torch.from_numpy(a).cuda()
img, _ = device_ms2dirty(t(uvw), t(f), t(vis), t(w), npix, npix, px, px, support=W, do_wstacking=True,
                         single_precision_accumulation=single)
np.save(out, img.cpu().numpy())
"""


def _inputs(npix):
    ms = syn.make_measurement_set(4000, 16, n_ant=24, array_radius_m=2500.0, seed=8)
    vis = np.ascontiguousarray(ms.visibilities()[..., 0], dtype=np.complex64)
    w = np.ascontiguousarray(ms.weights()[..., 0], dtype=np.float32)
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    return t(uvw), t(f), t(vis), t(w), px


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_groups_equal_single_plane_units(gpu_device, case, tmp_path):
    W, npix, single = case["support"], case["npix"], case.get("single", False)
    out = tmp_path / "per_plane.npy"
    env = dict(os.environ, CIP_WSTACK_GROUP="1")
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(W), str(npix), "1" if single else "0", str(out)],
                   env=env, check=True, timeout=120)
    ref = np.load(out)
    uvw, f, vis, w, px = _inputs(npix)
    for _ in range(2):  # the second call finds its plane pair clean (zeroed by the masked pass A)
        img, prm = device_ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=True,
                                   single_precision_accumulation=single)
        got = img.cpu().numpy()
        tol = (1e-6 if single else 1e-12) * np.abs(ref).max()
        assert np.abs(got - ref).max() <= tol
    assert prm.nplanes > W


def test_groups_accumulate_chunks(gpu_device):
    npix, W = 512, 6
    uvw, f, vis, w, px = _inputs(npix)
    wmin = float(torch.minimum(uvw[:, 2].min() * f.min(), uvw[:, 2].min() * f.max()) / 299792458.0)
    wmax = float(torch.maximum(uvw[:, 2].max() * f.max(), uvw[:, 2].max() * f.min()) / 299792458.0)
    acc = GridAccumulator(npix, npix, px, px, support=W, do_wstacking=True, w_range=(wmin, wmax))
    h = uvw.shape[0] // 3
    for a, b in ((0, h), (h, 2 * h), (2 * h, uvw.shape[0])):
        acc.add_ms(uvw[a:b].contiguous(), f, vis[a:b].contiguous(), w[a:b].contiguous())
    img, sw = acc.dirty()
    one, _ = device_ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=True)
    assert float((img - one).abs().max()) <= 1e-11 * float(one.abs().max())


def test_2d_after_wstacking_same_workspace(gpu_device):
    # the grid buffer holds two planes after a w-stacking call; a 2-D call
    # then reuses its first plane (and its clean mark) correctly
    npix = 512
    uvw, f, vis, w, px = _inputs(npix)
    a, _ = device_ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8)
    device_ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=True)
    b, _ = device_ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8)
    assert torch.equal(a, b)
