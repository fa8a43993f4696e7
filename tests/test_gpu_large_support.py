"""
GPU parity of the large kernel supports W = 24, 32, 48, 64 (BASELINE.json
configs[2]: "support = 64, LDS-tile stress"), gridded by the
wave-per-visibility scatter (csrc/cip_scatter_large.hip), against the CPU
oracle (same piecewise-polynomial kernel, plain fp64 accumulation) and the
direct fp64 DFT. Covers 2-D and w-stacking, the hipFFT path (npix 128) and the
pruned FFT path whose dirty-tile mask must follow the two-tile halo of a
W = 64 sub-grid (npix 512), the dtype / weight variants, unit visibilities
(PSF), the plain tile-order stream (bank-class order off, in a child process)
and the argument errors. W = 64 with w-stacking (the reference's gridding
mode, invert.py:180, at configs[2]'s support) is supported since round 4.
"""
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, synthetic as syn
from ska_sdp_cip_amd.invert import StokesIGridderInput

pytestmark = pytest.mark.gpu

TIGHT = 1e-10
GATE = 1e-6  # north star: dirty image / sum w, max |GPU - CPU|
# GPU vs oracle bounds (max |diff| / sum w). Both implement the same kernel and
# grid correction; the correction multiplies the GPU's fixed-point quantum
# (2^-46 of max |w V| per contribution, vs fp64's relative rounding in the
# oracle) by up to 1/F^2 at the image corners (1/F^3 with w-stacking). The
# large supports' shape beta keeps F(1/4)/F(0) >= 0.03 (tools/gen_es_kernels.py;
# at beta = 2.3 W it was 1.6e-4 at W = 64: 3.8e-5 measured with w-stacking, which
# the library then refused), so every support holds the tight bound in 2-D and
# 1e-9 with w-stacking (the VERDICT r03 target for W = 64).
TOL = {(False, 24): TIGHT, (False, 32): TIGHT, (False, 48): TIGHT, (False, 64): TIGHT,
       (True, 24): 1e-9, (True, 32): 1e-9, (True, 48): 1e-9, (True, 64): 1e-9}
ROOT = Path(__file__).resolve().parents[1]


def _case(n_rows, nchan, *, n_ant=16, radius=1000.0, fov=0.01, seed=3):
    ms = syn.make_measurement_set(n_rows, nchan, n_ant=n_ant, array_radius_m=radius, fov_l=fov, seed=seed)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    return gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)


def _dev(*arrays):
    import torch

    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrays]


def _err(gpu, ref, sumw):
    g = gpu.cpu().numpy() if hasattr(gpu, "cpu") else gpu
    return float(np.abs(g - ref).max() / sumw)


@pytest.mark.parametrize("support", [24, 32, 48, 64])
def test_large_support_2d_parity(gpu_device, support):
    uvw, f, vis, w = _case(3_000, 4)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix, support=support)
    gpu, prm = gridder.device_ms2dirty(*_dev(uvw, f, vis.astype(np.complex128), w.astype(np.float64)), npix, npix,
                                       px, px, support=support)
    assert prm.support == support and prm.nu == 256
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=support)
    sumw = float(w.astype(np.float64).sum())
    assert _err(gpu, ref, sumw) < TOL[(False, support)]
    if support == 24:  # the large kernels reproduce the DFT to fp64 rounding
        dft = oracle.dft_dirty(uvw, f, vis, w, npix, npix, px, px, apply_w=False)
        assert _err(gpu, dft, sumw) < 1e-11


@pytest.mark.parametrize("support", [24, 32, 48, 64])
def test_large_support_wstacking_parity(gpu_device, support):
    uvw, f, vis, w = _case(1_500, 4, n_ant=24, radius=2000.0, fov=0.05)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.3)
    gpu, prm = gridder.device_ms2dirty(*_dev(uvw, f, vis, w), npix, npix, px, px, support=support,
                                       do_wstacking=True)
    assert prm.nplanes > support
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=support, do_wstacking=True)
    err = _err(gpu, ref, float(w.astype(np.float64).sum()))
    print(f"W={support} w-stacking ({prm.nplanes} planes): max|GPU - oracle| / sum w = {err:.2e}")
    assert err < TOL[(True, support)]


@pytest.mark.parametrize("wstack", [False, True])
def test_large_support_pruned_fft_halo(gpu_device, wstack):
    # npix 512 -> 1024^2 grid: pruned FFT whose pass A reads only the masked
    # tiles; W = 48 and 64 sub-grids reach two tiles past their own
    W = 64
    uvw, f, vis, w = _case(2_000, 4, n_ant=24, radius=2000.0, fov=0.05 if wstack else 0.01)
    npix = 512
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.3 if wstack else 0.4)
    gpu, prm = gridder.device_ms2dirty(*_dev(uvw, f, vis, w), npix, npix, px, px, support=W, do_wstacking=wstack)
    assert prm.nu == 1024
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=wstack)
    sumw = float(w.astype(np.float64).sum())
    assert _err(gpu, ref, sumw) < TOL[(wstack, W)]
    # the grid is clean again after the masked pass A: a second call is identical
    again, _ = gridder.device_ms2dirty(*_dev(uvw, f, vis, w), npix, npix, px, px, support=W, do_wstacking=wstack)
    assert _err(again, gpu.cpu().numpy(), sumw) < 1e-12


@pytest.mark.parametrize("vis_dtype,wgt_kind", [(np.complex64, "f32"), (np.complex64, "none"),
                                                (np.complex128, "f32")])
def test_large_support_dtypes(gpu_device, vis_dtype, wgt_kind):
    uvw, f, vis, w = _case(1_000, 16, n_ant=24, radius=2000.0)
    vis = vis.astype(vis_dtype)
    wg = None if wgt_kind == "none" else w
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    gpu, _ = gridder.device_ms2dirty(*_dev(uvw, f, vis, wg), npix, npix, px, px, support=48)
    ref = oracle.ms2dirty(uvw, f, vis, wg, npix, npix, px, px, support=48)
    sumw = float(vis.size) if wg is None else float(wg.astype(np.float64).sum())
    assert _err(gpu, ref, sumw) < TOL[(False, 48)]


def test_large_support_psf(gpu_device):
    uvw, f, vis, w = _case(1_000, 4)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    psf, _ = gridder.device_ms2dirty(*_dev(uvw, f, vis, w), npix, npix, px, px, support=32, psf=True,
                                     normalise=True)
    ones = np.ones_like(vis)
    ref = oracle.ms2dirty(uvw, f, ones, w, npix, npix, px, px, support=32) / float(w.astype(np.float64).sum())
    assert _err(psf, ref, 1.0) < TIGHT
    assert abs(float(psf[npix // 2, npix // 2].item()) - 1.0) < 1e-6


def test_large_support_tile_order_stream(gpu_device):
    # CIP_SCATTER_ORDER=0 (read once per process): the scatter locates each
    # visibility through its tile's row slices instead of the ordered stream
    code = textwrap.dedent(f"""
        import sys
        sys.path[:0] = [{str(ROOT / 'ska-sdp-continuum-imaging-pipeline_amd')!r}, {str(ROOT / 'oracle')!r}]
        import numpy as np, torch, oracle
        from ska_sdp_cip_amd import gridder, synthetic as syn
        from ska_sdp_cip_amd.invert import StokesIGridderInput
        ms = syn.make_measurement_set(2000, 8, n_ant=16, array_radius_m=1000.0, fov_l=0.01, seed=9)
        gi = StokesIGridderInput.from_measurement_set_reader(ms)
        w = gi.effective_weights().astype(np.float32)
        px = syn.pixel_size_for_grid(gi.uvw, gi.channel_frequencies, 256)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
        for W in (32, 64):
            img, _ = gridder.device_ms2dirty(t(gi.uvw), t(gi.channel_frequencies), t(gi.visibilities), t(w),
                                             256, 256, px, px, support=W)
            ref = oracle.ms2dirty(gi.uvw, gi.channel_frequencies, gi.visibilities, w, 256, 256, px, px, support=W)
            print(W, float(np.abs(img.cpu().numpy() - ref).max() / w.astype(np.float64).sum()))
    """)
    env = dict(os.environ, CIP_SCATTER_ORDER="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    errs = [float(line.split()[1]) for line in out.stdout.strip().splitlines()]
    assert len(errs) == 2 and errs[0] < TOL[(False, 32)] and errs[1] < TOL[(False, 64)], out.stdout


def test_large_support_argument_errors(gpu_device):
    uvw, f, vis, w = _case(200, 2)
    args = _dev(uvw, f, vis, w)
    px = syn.pixel_size_for_grid(uvw, f, 64)
    with pytest.raises(ValueError):
        gridder.device_ms2dirty(*args, 64, 64, px, px, support=20)
    with pytest.raises(ValueError):
        gridder.device_ms2dirty(*args, 64, 64, px, px, support=32, single_precision_accumulation=True)
    with pytest.raises(ValueError):  # 16 x 16 grid < W = 24
        gridder.device_ms2dirty(*args, 8, 8, px, px, support=24)
