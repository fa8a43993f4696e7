"""
GPU tests of the continuum products (config C5; beyond
the reference, which makes Stokes I only): Stokes I/Q/U/V conversion
(bit-exact vs numpy float32 arithmetic), facets (rephase + baseline rotation:
each facet image equals the direct DFT at the facet pixels' absolute
directions, 2-D and w-stacking), and the PSF (unit visibilities: peak 1 at
the centre, point symmetric).
"""
import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, synthetic as syn
from ska_sdp_cip_amd.continuum import continuum_invert, continuum_invert_measurement_set, facet_centres

pytestmark = pytest.mark.gpu


def _t(a, dt=None):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a if dt is None else a.astype(dt))).cuda()


@pytest.mark.parametrize("which", ["I", "Q", "U", "V"])
def test_stokes_bit_exact(gpu_device, which):
    rng = np.random.default_rng(4)
    shape = (300, 5, 4)
    vis4 = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    flags4 = rng.random(shape) < 0.1
    wgt4 = rng.uniform(0.0, 2.0, shape).astype(np.float32)
    wgt4[rng.random(shape) < 0.05] = 0.0
    v, eff = gridder.device_stokes(_t(vis4), _t(flags4, np.uint8), _t(wgt4), which)
    rv, reff = oracle.stokes(vis4, flags4, wgt4, which)
    assert np.array_equal(v.cpu().numpy(), rv)
    assert np.array_equal(eff.cpu().numpy(), reff)


@pytest.mark.parametrize("wstack", [False, True])
def test_facet_equals_dft_at_absolute_directions(gpu_device, wstack):
    ms = syn.make_measurement_set(600, 4, n_ant=12, array_radius_m=600.0, fov_l=0.08, seed=8)
    from ska_sdp_cip_amd.invert import StokesIGridderInput

    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    uvw, f, vis, w = gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights()
    npix = 32
    px = syn.pixel_size_for_grid(uvw, f, 4 * npix, support=16)  # a small facet of a larger field
    l0, m0 = 0.6 * npix * px, -1.1 * npix * px
    uvw_f, vis_f = gridder.device_facet_rephase(_t(uvw), _t(f), _t(vis), l0, m0)
    img, _ = gridder.device_ms2dirty(uvw_f, _t(f), vis_f, _t(w), npix, npix, px, px, support=16,
                                     do_wstacking=wstack)
    # facet pixel (i, j) <-> (l', m') of the facet plane <-> direction Q (l', m', n')
    lp = (np.arange(npix) - npix // 2) * px
    L, M = np.meshgrid(lp, lp, indexing="ij")
    N = np.sqrt(1.0 - L ** 2 - M ** 2)
    s = oracle.facet_rotation(l0, m0) @ np.stack([L.ravel(), M.ravel(), N.ravel()])
    sw = float(w.astype(np.float64).sum())
    got = img.cpu().numpy()
    # the gridder on the facet data: the oracle's fp64 restatement, same algorithm
    ora = oracle.ms2dirty(uvw_f.cpu().numpy(), f, vis_f.cpu().numpy(), w, npix, npix, px, px, support=16,
                          do_wstacking=wstack)
    assert float(np.abs(got - ora).max()) / sw < 1e-10
    if wstack:
        # the facet image IS the dirty image at the facet pixels' absolute directions
        # (w-stacking reaches ~3e-7 of the DFT here; north-star gate 1e-6)
        ref = oracle.dft_directions(uvw, f, vis, w, s[0], s[1]).reshape(npix, npix)
        tol = 1e-6
    else:  # 2-D: n := 1 in the facet frame; the DFT of the facet data itself
        ref = oracle.dft_dirty(uvw_f.cpu().numpy(), f, vis_f.cpu().numpy(), w, npix, npix, px, px, apply_w=False)
        tol = 1e-9
    err = float(np.abs(got - ref).max()) / sw
    assert err < tol, err


def test_point_source_at_facet_centre_and_psf(gpu_device):
    import torch

    rows, nchan = 1_200, 4
    uvw = syn.uvw_tracks(rows, 16, array_radius_m=800.0, seed=6)
    f = syn.channel_frequencies(nchan)
    npix = 64
    px = syn.pixel_size_for_grid(uvw, f, 4 * npix)
    fac = facet_centres(2, 2, npix, px)
    l0, m0 = fac[3]
    n0m1 = np.sqrt(1.0 - l0 * l0 - m0 * m0) - 1.0
    fx = f / 299792458.0
    # a 1 Jy source at the facet centre, same on XX and YY; XY = YX = 0
    ph = -2.0 * np.pi * fx[None, :] * (uvw[:, 0:1] * l0 + uvw[:, 1:2] * m0 - uvw[:, 2:3] * n0m1)
    v = np.exp(1j * ph)
    vis4 = np.zeros((rows, nchan, 4), np.complex64)
    vis4[..., 0] = v
    vis4[..., 3] = v
    flags4 = np.zeros(vis4.shape, bool)
    wgt4 = np.ones(vis4.shape, np.float32)
    out = continuum_invert(_t(vis4), _t(flags4, np.uint8), _t(wgt4), _t(uvw), _t(f), npix,
                           np.degrees(np.arcsin(px)) * 3600.0, facets=fac, stokes="IQ", psf=True,
                           support=8, do_wstacking=True)
    assert set(out) == {(s, k) for s in ("I", "Q", "PSF") for k in range(4)}
    img = out[("I", 3)].cpu().numpy()
    assert abs(img[npix // 2, npix // 2] - 1.0) < 1e-6
    assert np.unravel_index(np.argmax(img), img.shape) == (npix // 2, npix // 2)
    assert float(out[("Q", 3)].abs().max().item()) < 1e-6  # XX == YY: no Stokes Q
    for k in range(4):
        p = out[("PSF", k)].cpu().numpy()
        # sum w Re{1} / sum w at the centre, to the W = 8 gridding accuracy
        assert abs(p[npix // 2, npix // 2] - 1.0) < 1e-6 and p.max() <= 1.0 + 1e-6
    # rank split: facets k % world == rank
    out1 = continuum_invert(_t(vis4), _t(flags4, np.uint8), _t(wgt4), _t(uvw), _t(f), npix,
                            np.degrees(np.arcsin(px)) * 3600.0, facets=fac, stokes="I", psf=False, support=8,
                            do_wstacking=True, rank=1, world=2)
    assert set(out1) == {("I", 1), ("I", 3)}
    assert torch.equal(out1[("I", 3)], out[("I", 3)])


def test_continuum_measurement_set_all_stokes(gpu_device):
    ms = syn.make_measurement_set(400, 3, n_ant=10, array_radius_m=500.0, seed=3)
    res = continuum_invert_measurement_set(ms, 32, 30.0, stokes="IQUV", psf=True)
    assert set(res) == {(s, 0) for s in ("I", "Q", "U", "V", "PSF")}
    from ska_sdp_cip_amd import invert_measurement_set

    ref = invert_measurement_set(ms, 32, 30.0)  # the reference path: Stokes I, centre facet
    assert np.abs(res[("I", 0)] - ref).max() <= 2e-6 * np.abs(ref).max()
