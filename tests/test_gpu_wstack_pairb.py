"""
w-stacking pass B over plane pairs (CIP_WSTACK_PAIRB=1, cip_fft.hip
fft_cols_wstack_kernel): the packed class's two planes' screened
contributions summed in registers and the image written once per pair, in the
per-plane path's order of additions - the same image bit for bit, for odd and
even plane counts and a w-plane range (cip_ms2dirty_wplanes). Each mode runs
in a child process.
CIP_WSTACK_GROUPB=1 does the same for a whole plane group into the float
accumulator.
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


def _run(tmp_path, on, wacc_f32="0", group_b="0"):
    out = tmp_path / f"pairb{on}{wacc_f32}{group_b}.npz"
    # both forms accumulate the planes in the fp64 image (the pair kernel's
    # form; the default packed-class path accumulates in float: CIP_WACC_F32)
    env = dict(os.environ, CIP_WSTACK_PAIRB="1" if on else "0", CIP_WACC_F32=wacc_f32, CIP_WSTACK_GROUPB=group_b)
    subprocess.run([sys.executable, "-c", CHILD, str(ROOT), str(out)], env=env, check=True, timeout=180)
    return np.load(out)


def test_plane_pair_pass_b_is_bit_identical(gpu_device, tmp_path):
    off, on = _run(tmp_path, False), _run(tmp_path, True)
    counts = {int(off["planes1024"]) % 2, int(off["planes2048"]) % 2}
    print("plane counts", int(off["planes1024"]), int(off["planes2048"]))
    for k in off.files:
        assert np.array_equal(off[k], on[k]), k
    assert counts  # (odd and even counts both exercised when the two differ in parity)


def test_float_plane_accumulator_within_the_class_precision(gpu_device, tmp_path):
    """The packed class's w planes accumulate in a float image by default
    (CIP_WACC_F32; one rounding per plane, then the fp64 final correction):
    within 1e-6 of the peak of the fp64-accumulated image (the class's own
    fp32 taps already differ from fp64 at ~1e-7), w-plane ranges included."""
    f64, f32 = _run(tmp_path, False, "0"), _run(tmp_path, False, "1")
    for k in f64.files:
        if k.startswith("planes"):
            continue
        peak = float(np.abs(f64[k]).max())
        err = float(np.abs(f32[k] - f64[k]).max())
        print(k, err / peak)
        assert 0.0 < err < 1e-6 * peak, k


@pytest.mark.parametrize("group", ["3", "7"])
def test_plane_group_pass_b_is_bit_identical(gpu_device, tmp_path, group):
    """CIP_WSTACK_GROUPB=1 (cip_fft.hip fft_cols_wacc_kernel): a plane group's
    planes through one pass B into an LDS copy of the float accumulator row -
    the per-plane float accumulation bit for bit, whole stacks and w-plane
    ranges that start and end inside a group."""
    os.environ["CIP_WSTACK_GROUP"] = group
    try:
        per_plane = _run(tmp_path, False, "1", "0")
        grouped = _run(tmp_path, False, "1", "1")
    finally:
        del os.environ["CIP_WSTACK_GROUP"]
    for k in per_plane.files:
        assert np.array_equal(per_plane[k], grouped[k]), k
