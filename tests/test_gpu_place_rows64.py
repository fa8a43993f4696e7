"""
The dense-row place pass (csrc/cip_plan.hip place_rows64_body: rows of a
multiple of 64 channels, one row per wave, scalar row / load bases, 32-bit key
arithmetic) against the general place pass (place_body, CIP_PLACE_ROWS64=0 in
a child process - the switch is read once per process). The planner's outputs
must be the same: the weight sum bit for bit (the fused reduction's order is
unchanged), the same run and work-unit counts (the same runs), and the images
equal up to the order of the flush's global adds (asserted at 1e-13 of
sum |w V| for the fp64 class; 1e-6 for the packed class, whose complex64
planes take float atomics). Cases: the fp64 class on complex64 / complex128
input, 64 / 192 / 256 channels (192: the row advance carries a channel
remainder), a partial last place block, the reference's w-stacking call
(packed class), the PSF, and a non-finite counted visibility (an error in
both).
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

    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = {}
    _lib.profile_enable(True)
    for nchan, nrow, npix in [(64, 3_001, 512), (192, 1_500, 384), (256, 2_003, 512)]:
        ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=2500.0, seed=nchan)
        uvw, f = ms.uvw(), ms.channel_frequencies()
        rng = np.random.default_rng(nchan)
        vis = (rng.standard_normal((nrow, nchan)) + 1j * rng.standard_normal((nrow, nchan)))
        w = np.where(rng.random((nrow, nchan)) < 0.05, 0.0, rng.uniform(0.5, 2.0, (nrow, nchan)))
        px = syn.pixel_size_for_grid(uvw, f, npix)
        tu, tf = t(uvw), t(f)
        runs = [("c64", t(vis.astype(np.complex64)), t(w.astype(np.float32)), dict(support=8)),
                ("c128", t(vis), t(w), dict(support=6)),
                ("refcall", t(vis.astype(np.complex64)), t(w.astype(np.float32)),
                 dict(epsilon=1e-4, do_wstacking=True, single_precision_accumulation=True)),
                ("psf", None, t(w.astype(np.float32)), dict(support=8, psf=True))]
        for name, tv, tw, kw in runs:
            sw = torch.empty(1, dtype=torch.float64, device=dev)
            img, _ = gridder.device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, sum_weights=sw, **kw)
            prof = _lib.profile_last()
            key = f"{name}_{nchan}"
            out[f"img_{key}"] = img.cpu().numpy()
            out[f"sw_{key}"] = np.array([sw.item()])
            out[f"cnt_{key}"] = np.array([prof["runs"], prof["chunks"]], dtype=np.int64)
            scale = w.sum() if tv is None else float((np.abs(w) * np.abs(vis)).sum())
            out[f"scale_{key}"] = np.array([scale])
    # the error path: a counted NaN visibility
    ms = syn.make_measurement_set(500, 64, n_ant=16, array_radius_m=1500.0, seed=3)
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, 256)
    vis = np.ones((500, 64), np.complex64)
    vis[7, 9] = np.nan
    w = np.ones((500, 64), np.float32)
    errs = []
    try:
        gridder.device_ms2dirty(t(uvw), t(f), t(vis), t(w), 256, 256, px, px, support=8)
        errs.append("none")
    except ValueError as e:
        errs.append(type(e).__name__)
    out["errs"] = np.array(errs)
    torch.cuda.synchronize()
    return out


CHILD = """
import sys
sys.path[:0] = [{root!r}, {pkg!r}, {orc!r}, {tests!r}]
import numpy as np
import test_gpu_place_rows64 as t
np.savez({out!r}, **t._cases())
"""


def test_rows64_place_equals_general_place(gpu_device, tmp_path):
    mine = _cases()
    out = tmp_path / "general.npz"
    code = CHILD.format(root=str(ROOT), pkg=str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"),
                        orc=str(ROOT / "oracle"), tests=str(ROOT / "tests"), out=str(out))
    env = dict(os.environ, CIP_PLACE_ROWS64="0")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    ref = np.load(out)
    assert sorted(ref.files) == sorted(mine)
    assert list(mine["errs"]) == ["ValueError"] and list(ref["errs"]) == ["ValueError"]
    for k in mine:
        if k.startswith("sw_") or k.startswith("cnt_"):
            assert np.array_equal(mine[k], ref[k]), (k, mine[k], ref[k])
        elif k.startswith("img_"):
            scale = float(mine["scale_" + k[4:]][0])
            assert float(np.abs(ref[k]).max()) > 0, k
            err = float(np.abs(mine[k] - ref[k]).max()) / scale
            assert err <= (1e-6 if k.startswith("img_refcall") else 1e-13), (k, err)
