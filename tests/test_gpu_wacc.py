"""
The packed class's w-stacking float plane accumulator (CIP_WACC_F32, default
on; cip_api.hip ms2dirty_impl, cip_fft.hip fft_cols_kernel<.., float>) against
the fp64-accumulated image, and the fp64 transforms (CIP_FFT_F32=0), with
which the float accumulator must stay off (the fp64-output pass B
would write doubles across the float buffer). Each mode runs in a child
process (the switches are read once per process).
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
out = sys.argv[2]
ms = syn.make_measurement_set(8000, 32, n_ant=24, array_radius_m=2500.0, seed=31)
vis = np.ascontiguousarray(ms.visibilities()[..., 0], dtype=np.complex64)
w = np.ascontiguousarray(ms.weights()[..., 0], dtype=np.float32)
uvw, f = ms.uvw(), ms.channel_frequencies()
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
res = {}
for npix, wscale in ((1024, 20.0), (2048, 35.0)):
    px = syn.pixel_size_for_grid(uvw, f, npix)
    u = uvw * np.array([1.0, 1.0, wscale])
    img, prm = device_ms2dirty(t(u), t(f), t(vis), t(w), npix, npix, px, px, epsilon=1e-4, do_wstacking=True,
                               single_precision_accumulation=True)
    res["n%d" % npix] = img.cpu().numpy()
    res["planes%d" % npix] = prm.nplanes
    img2, _ = device_ms2dirty(t(u), t(f), t(vis), t(w), npix, npix, px, px, epsilon=1e-4, do_wstacking=True,
                              single_precision_accumulation=True, planes=(1, prm.nplanes - 2))
    res["r%d" % npix] = img2.cpu().numpy()
np.savez(out, **res)
"""


def _run(tmp_path, wacc_f32="1", fft_f32="1"):
    out = tmp_path / f"wacc{wacc_f32}{fft_f32}.npz"
    env = dict(os.environ, CIP_WACC_F32=wacc_f32, CIP_FFT_F32=fft_f32)
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(out)], env=env, check=True, timeout=180)
    return np.load(out)


def test_float_plane_accumulator_within_the_class_precision(gpu_device, tmp_path):
    """The packed class's w planes accumulate in a float image by default
    (one rounding per plane, then the fp64 final correction): within 1e-6 of
    the peak of the fp64-accumulated image (the class's own fp32 taps already
    differ from fp64 at ~1e-7), w-plane ranges included."""
    f64, f32 = _run(tmp_path, "0"), _run(tmp_path, "1")
    for k in f64.files:
        if k.startswith("planes"):
            continue
        peak = float(np.abs(f64[k]).max())
        err = float(np.abs(f32[k] - f64[k]).max())
        print(k, err / peak)
        assert 0.0 < err < 1e-6 * peak, k


def test_fp64_transforms_keep_the_fp64_accumulator(gpu_device, tmp_path):
    """CIP_FFT_F32=0 with the float accumulator switch left on: the packed
    w-stacking call must fall back to the fp64 image accumulator (not write
    fp64 pass-B output into the float buffer) - the image agrees with the
    fp32-transform images to the class's precision."""
    ref, f64fft = _run(tmp_path, "0"), _run(tmp_path, "1", "0")
    for k in ref.files:
        if k.startswith("planes"):
            assert int(ref[k]) == int(f64fft[k])
            continue
        peak = float(np.abs(ref[k]).max())
        err = float(np.abs(f64fft[k] - ref[k]).max())
        print(k, err / peak)
        assert np.isfinite(f64fft[k]).all(), k
        assert err < 1e-6 * peak, k
