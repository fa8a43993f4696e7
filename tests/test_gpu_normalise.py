"""
GPU tests of CIP_NORMALISE (include/cip.h): cip_ms2dirty returning the image
divided by the call's weight sum (the reference's (1 / total_weight) * image,
src/ska_sdp_cip/invert.py:119-149), fused into the pruned FFT's pass-B
epilogue in 2-D mode and a separate pass otherwise. The normalised image must
equal the unnormalised one divided by the returned weight sum (tolerance 1e-15
of the image maximum: the fused form divides the correction factor, not the
pixel), and the unnormalised one must still match the CPU oracle.
"""
import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, synthetic as syn

pytestmark = pytest.mark.gpu


def _t(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


# grids of 1024..8192 cells per axis (npix 512..4096, power of two) take the
# pruned FFT, whose pass-B epilogue divides by the weight sum (2-D); the other
# sizes, and w-stacking on any size, take the separate scale pass
@pytest.mark.parametrize("npix,wstack,psf,fused", [
    (256, False, False, False), (256, True, False, False), (250, False, False, False), (256, False, True, False),
    (512, False, False, True), (1024, False, False, True), ((512, 1024), False, False, True),
    ((1024, 512), False, True, True), (512, True, False, False)])
def test_normalise_equals_divide(gpu_device, npix, wstack, psf, fused):
    import torch

    from ska_sdp_cip_amd import _lib

    nx, ny = (npix, npix) if isinstance(npix, int) else npix

    uvw = syn.uvw_tracks(1_500, 16, array_radius_m=900.0, seed=11)
    f = syn.channel_frequencies(8)
    rng = np.random.default_rng(3)
    vis = (rng.standard_normal((uvw.shape[0], f.size)) + 1j * rng.standard_normal((uvw.shape[0], f.size)))
    vis = vis.astype(np.complex64)
    w = rng.uniform(0.5, 2.0, vis.shape).astype(np.float32)
    px = syn.pixel_size_for_grid(uvw, f, max(nx, ny))
    args = (_t(uvw), _t(f), None if psf else _t(vis), _t(w), nx, ny, px, px)
    kw = dict(support=8, do_wstacking=wstack, psf=psf)
    s0 = torch.zeros(1, dtype=torch.float64, device="cuda")
    s1 = torch.zeros(1, dtype=torch.float64, device="cuda")
    raw, _ = gridder.device_ms2dirty(*args, sum_weights=s0, **kw)
    raw = raw.clone()
    nrm, params = gridder.device_ms2dirty(*args, sum_weights=s1, normalise=True, **kw)
    torch.cuda.synchronize()
    # the layout the library chose: 1 = pruned FFT (pass-B epilogue divides)
    pruned = bool(_lib.lib().cip_grid_layout(params, nx, ny))
    pow2 = all(n >= 512 and n & (n - 1) == 0 for n in (nx, ny))
    assert pruned == pow2
    assert fused == (pruned and not wstack)
    sw = float(s0.item())
    assert float(s1.item()) == sw  # the raw weight sum is still returned
    assert sw == pytest.approx(float(w.astype(np.float64).sum()), rel=1e-12)
    r = raw.cpu().numpy()
    n = nrm.cpu().numpy()
    assert np.abs(n - r / sw).max() <= 1e-15 * np.abs(r / sw).max() * 4
    if psf:
        assert abs(n[nx // 2, ny // 2] - 1.0) < 1e-6  # gridding accuracy, as test_gpu_continuum
    else:
        ref = oracle.ms2dirty(uvw, f, vis, w, nx, ny, px, px, support=8, do_wstacking=wstack)
        assert np.abs(n - ref / sw).max() < 1e-6 * np.abs(ref / sw).max() + 1e-12


def test_normalise_empty_input_is_nan_like_divide(gpu_device):
    import torch

    uvw = np.zeros((0, 3))
    f = syn.channel_frequencies(4)
    vis = np.zeros((0, 4), np.complex64)
    w = np.zeros((0, 4), np.float32)
    s = torch.zeros(1, dtype=torch.float64, device="cuda")
    out, _ = gridder.device_ms2dirty(_t(uvw), _t(f), _t(vis), _t(w), 64, 64, 1e-5, 1e-5, support=8,
                                     sum_weights=s, normalise=True)
    torch.cuda.synchronize()
    assert float(s.item()) == 0.0
    # 0 / 0, the same as dividing the empty image by its zero weight sum
    assert np.isnan(out.cpu().numpy()).all()
