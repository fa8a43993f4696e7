"""
The bank-class order's three class sources give the same images: the default
gathers the place pass's per-visibility class bytes, CIP_ORDER_CLASS=runs
recomputes each class in fp32 from its run's (u, v) carried through the radix
sort, and =compute recomputes from a uvw gather per slice. The class only decides the order of a window's
visibilities (which LDS banks a wave's atomics hit); the fixed-point sums are
exact and order-independent, so the images agree to the fp64 flush order
(~1e-16 relative). The split place pass (CIP_PLACE_SPLIT=1: placement and the
weight reduction in separate workgroups) must give the same images too. Each mode runs in a child process (the switch is read once
per process): 2-D and w-stacking, dense rows and ragged tiles (cip_grid_tiles).
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/ska-sdp-continuum-imaging-pipeline_amd"]
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty
from ska_sdp_cip_amd.accumulate import GridAccumulator
out = sys.argv[2]
ms = syn.make_measurement_set(6000, 32, n_ant=24, array_radius_m=2500.0, seed=21)
vis = np.ascontiguousarray(ms.visibilities()[..., 0], dtype=np.complex64)
w = np.ascontiguousarray(ms.weights()[..., 0], dtype=np.float32)
uvw, f = ms.uvw(), ms.channel_frequencies()
npix = 512
px = syn.pixel_size_for_grid(uvw, f, npix)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
res = {}
for ws in (False, True):
    img, _ = device_ms2dirty(t(uvw), t(f), t(vis), t(w), npix, npix, px, px, support=8, do_wstacking=ws)
    res["ws%d" % ws] = img.cpu().numpy()
# ragged row slices (the Tile layout): every row's channels [r % 7, 32 - r % 5)
c0 = (np.arange(uvw.shape[0]) % 7).astype(np.int32)
c1 = (32 - np.arange(uvw.shape[0]) % 5).astype(np.int32)
vv = np.concatenate([vis[r, c0[r]:c1[r]] for r in range(uvw.shape[0])])
ww = np.concatenate([w[r, c0[r]:c1[r]] for r in range(uvw.shape[0])])
acc = GridAccumulator(npix, npix, px, px, support=8)
acc.add_tile(t(uvw), t(c0), t(c1), t(f), t(vv), t(ww))
dirty, _ = acc.dirty()
res["tiles"] = dirty.cpu().numpy()
np.savez(out, **res)
"""


def _run(tmp_path, **switches):
    out = tmp_path / ("order_" + "_".join(f"{k}{v}" for k, v in switches.items()) + ".npz")
    env = dict(os.environ)
    for k in ("CIP_ORDER_CLASS", "CIP_PLACE_SPLIT"):
        env.pop(k, None)
    env.update(switches)
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(out)], env=env, check=True, timeout=180)
    return np.load(out)


def test_class_sources_give_the_same_images(gpu_device, tmp_path):
    base = _run(tmp_path)
    for sw in (dict(CIP_ORDER_CLASS="runs"), dict(CIP_ORDER_CLASS="compute"), dict(CIP_PLACE_SPLIT="1")):
        other = _run(tmp_path, **sw)
        for k in base.files:
            peak = float(np.abs(base[k]).max())
            assert peak > 0.0
            assert float(np.abs(base[k] - other[k]).max()) <= 1e-13 * peak, (sw, k)
