"""
The scatter's in-unit bank-class sort (csrc/cip_scatter.h
scatter_sorted_windows, PERM = 3: 2-D plans over dense rows, the default)
against the planner's order pass (CIP_SCATTER_SORT=0 in a child process - the
switch is read once per process). Both grid the same visibilities of the same
work units into 64-bit fixed-point sub-grids, only in another order within a
window, so the integer sums are equal and the images differ only by the order
of the flush's global adds (1e-13 of sum |w V| for the fp64 class, 1e-6 for
the packed class's float atomics); the weight sums are bit-identical.

Cases: the fp64 class on complex64 / complex128 input, the packed class
(complex64, single-precision accumulation, 2-D), the PSF, 64 and 24 channels
(24: the general place pass), hot tiles of several windows and work units
(a coarse grid under many visibilities: > kChunkVis per tile), a non-square
image, and the accumulating dense gridder (cip_grid_ms).
"""

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _cases():
    import torch

    from ska_sdp_cip_amd import _lib, gridder, synthetic as syn
    from ska_sdp_cip_amd.accumulate import GridAccumulator, w_range_rows

    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = {}
    _lib.profile_enable(True)
    for nchan, nrow, npix, fill in [(64, 3_001, 512, 0.5), (24, 4_000, 384, 0.5), (64, 6_000, 64, 0.9)]:
        ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=2500.0, seed=nchan + npix)
        uvw, f = ms.uvw(), ms.channel_frequencies()
        rng = np.random.default_rng(nchan)
        vis = (rng.standard_normal((nrow, nchan)) + 1j * rng.standard_normal((nrow, nchan)))
        w = np.where(rng.random((nrow, nchan)) < 0.05, 0.0, rng.uniform(0.5, 2.0, (nrow, nchan)))
        px = syn.pixel_size_for_grid(uvw, f, npix, fill=fill)
        tu, tf = t(uvw), t(f)
        runs = [("c64", t(vis.astype(np.complex64)), t(w.astype(np.float32)), dict(support=8)),
                ("c128", t(vis), t(w), dict(support=6)),
                ("packed", t(vis.astype(np.complex64)), t(w.astype(np.float32)),
                 dict(support=8, single_precision_accumulation=True)),
                ("psf", None, t(w.astype(np.float32)), dict(support=8, psf=True))]
        for name, tv, tw, kw in runs:
            sw = torch.empty(1, dtype=torch.float64, device=dev)
            img, _ = gridder.device_ms2dirty(tu, tf, tv, tw, npix, npix - 2, px, px, sum_weights=sw, **kw)
            prof = _lib.profile_last()
            key = f"{name}_{nchan}_{npix}"
            out[f"img_{key}"] = img.cpu().numpy()
            out[f"sw_{key}"] = np.array([sw.item()])
            out[f"cnt_{key}"] = np.array([prof["runs"], prof["chunks"]], dtype=np.int64)
            scale = w.sum() if tv is None else float((np.abs(w) * np.abs(vis)).sum())
            out[f"scale_{key}"] = np.array([scale])
        if npix == 512:
            acc = GridAccumulator(npix, npix, px, px, support=8, do_wstacking=False, w_range=w_range_rows(uvw, f))
            tv, tw = t(vis.astype(np.complex64)), t(w.astype(np.float32))
            for a, b in [(0, 1_000), (1_000, 1_001), (1_001, nrow)]:
                acc.add_ms(tu[a:b], tf, tv[a:b], tw[a:b])
            out[f"img_acc_{nchan}"] = acc.dirty()[0].cpu().numpy()
            out[f"scale_acc_{nchan}"] = np.array([float((np.abs(w) * np.abs(vis)).sum())])
    torch.cuda.synchronize()
    return out


CHILD = """
import sys
sys.path[:0] = [{root!r}, {pkg!r}, {orc!r}, {tests!r}]
import numpy as np
import test_gpu_scatter_sort as t
np.savez({out!r}, **t._cases())
"""


def test_scatter_sort_equals_order_pass(gpu_device, tmp_path):
    mine = _cases()
    out = tmp_path / "order_pass.npz"
    code = CHILD.format(root=str(ROOT), pkg=str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"),
                        orc=str(ROOT / "oracle"), tests=str(ROOT / "tests"), out=str(out))
    env = dict(os.environ, CIP_SCATTER_SORT="0")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    ref = np.load(out)
    assert sorted(ref.files) == sorted(mine)
    # the hot-tile case really has several work units per tile
    assert mine["cnt_c64_64_64"][1] > 6_000 * 64 // 16_384
    for k in mine:
        if k.startswith("sw_") or k.startswith("cnt_"):
            assert np.array_equal(mine[k], ref[k]), (k, mine[k], ref[k])
        elif k.startswith("img_"):
            scale = float(mine["scale_" + k[4:]][0])
            assert float(np.abs(ref[k]).max()) > 0, k
            err = float(np.abs(mine[k] - ref[k]).max()) / scale
            assert err <= (1e-6 if k.startswith("img_packed") else 1e-13), (k, err)
