"""
BASELINE.json configs[4] (C5, the full continuum invert: PSF + dirty images,
4 Stokes, 32 facets x 4096^2) at its image size, through
`continuum.continuum_invert` (cip_stokes -> cip_facet_rephase ->
cip_ms2dirty, one tile plan per facet), against the CPU oracle:

* two facets of C5's 8 x 4 mosaic of 4096^2 facets (a corner facet and an
  inner one) x (I, Q, U, V, PSF) from C3's uvw tracks (every 100th row:
  3,907 rows x 256 channels = 1.0M visibilities of raw (rows, chan, 4)
  complex64 / uint8 / float32 columns), 2-D, support 8, each image against
  oracle.stokes -> oracle.facet_rephase -> oracle.ms2dirty at the full
  8192^2 grid (10 images);
* the same facet in the reference's w-stacking mode (Stokes I, every 1000th
  row) against the oracle;
* the rank split (facet k on rank k mod world, no exchange): the union of the
  world = 2 ranks' images equals the one-rank run bit for bit.

Images are normalised by each Stokes parameter's fp64 weight sum on both
sides; the fp64 class agrees with the oracle to ~1e-13 (asserted 1e-10,
north-star gate 1e-6).
"""
import os

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.continuum import continuum_invert, facet_centres
from ska_sdp_cip_amd.invert import pixel_size_lm

pytestmark = pytest.mark.gpu

SEED = 20241008
NPIX = 4096
FACETS = (0, 13)  # of the 8 x 4 mosaic: a corner facet and an inner one
NTHREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
BOUND = 1e-10


def _raw(row_step):
    uvw_all = syn.uvw_tracks(390_625, 64, array_radius_m=4000.0, seed=SEED)
    freq = syn.channel_frequencies(256)
    px = syn.pixel_size_for_grid(uvw_all, freq, NPIX, support=8)
    uvw = np.ascontiguousarray(uvw_all[::row_step])
    n = uvw.shape[0]
    rng = np.random.default_rng(SEED + row_step)
    shape = (n, 256, 4)
    vis4 = (rng.standard_normal(shape, dtype=np.float32)
            + 1j * rng.standard_normal(shape, dtype=np.float32)).astype(np.complex64)
    wgt4 = rng.uniform(0.5, 1.5, shape).astype(np.float32)
    flags4 = rng.uniform(size=shape) < 0.025
    asec = float(np.degrees(np.arcsin(px)) * 3600.0)
    return uvw, freq, vis4, flags4, wgt4, asec


def _dev(*arrs):
    import torch

    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _oracle_image(uvw, freq, vis4, flags4, wgt4, pix, centre, name, wstack):
    which = "I" if name == "PSF" else name
    vis, eff = oracle.stokes(vis4, flags4, wgt4, which)
    uvw_f, vis_f = oracle.facet_rephase(uvw, freq, None if name == "PSF" else vis, *centre)
    if name == "PSF":
        vis_f = np.ones(eff.shape, np.complex128)
    else:
        # cip_facet_rephase stores the rephased visibilities in the input's
        # dtype (complex64): the same rounding here (else ~1e-10 of sum w)
        vis_f = vis_f.astype(np.complex64)
    img = oracle.ms2dirty(uvw_f, freq, vis_f, eff, NPIX, NPIX, pix, pix, support=8, do_wstacking=wstack,
                          nthreads=NTHREADS)
    return img / eff.astype(np.float64).sum()


def test_c5_two_4096_facets_iquv_psf_vs_oracle(gpu_device):
    import torch

    uvw, freq, vis4, flags4, wgt4, asec = _raw(100)
    assert vis4.shape[0] * vis4.shape[1] >= 1_000_000
    pix = pixel_size_lm(asec)
    mosaic = facet_centres(8, 4, NPIX, pix)
    centres = [mosaic[k] for k in FACETS]
    d = _dev(vis4, flags4.astype(np.uint8), wgt4, uvw, freq)
    out = continuum_invert(*d, NPIX, asec, facets=centres, stokes="IQUV", psf=True, support=8, do_wstacking=False)
    names = ("I", "Q", "U", "V", "PSF")
    assert set(out) == {(s, k) for s in names for k in range(len(centres))}
    for k, c in enumerate(centres):
        for name in names:
            got = out[(name, k)].cpu().numpy()
            ref = _oracle_image(uvw, freq, vis4, flags4, wgt4, pix, c, name, False)
            err = float(np.abs(got - ref).max())
            print(f"facet {FACETS[k]} ({c[0]:+.4f}, {c[1]:+.4f}) {name}: max|GPU - oracle| = {err:.2e}")
            assert err < BOUND, (k, name, err)
            if name == "PSF":
                assert abs(float(got[NPIX // 2, NPIX // 2]) - 1.0) < 1e-6  # the W = 8 kernel's accuracy
    # rank split over world = 2 (facet k on rank k mod 2): bit-identical images
    for rank in (0, 1):
        part = continuum_invert(*d, NPIX, asec, facets=centres, stokes="IQUV", psf=True, support=8,
                                do_wstacking=False, rank=rank, world=2)
        assert set(part) == {(s, k) for s in names for k in range(len(centres)) if k % 2 == rank}
        for key, img in part.items():
            assert torch.equal(img, out[key]), key
    del out
    torch.cuda.empty_cache()


def test_c5_facet_wstacking_vs_oracle(gpu_device):
    # the reference's gridding mode (w-stacking) on a far facet of the mosaic
    uvw, freq, vis4, flags4, wgt4, asec = _raw(1000)
    pix = pixel_size_lm(asec)
    centre = facet_centres(8, 4, NPIX, pix)[FACETS[0]]
    d = _dev(vis4, flags4.astype(np.uint8), wgt4, uvw, freq)
    out = continuum_invert(*d, NPIX, asec, facets=[centre], stokes="I", psf=False, support=8, do_wstacking=True)
    got = out[("I", 0)].cpu().numpy()
    ref = _oracle_image(uvw, freq, vis4, flags4, wgt4, pix, centre, "I", True)
    err = float(np.abs(got - ref).max())
    print(f"w-stacking facet {FACETS[0]}: max|GPU - oracle| = {err:.2e}")
    assert err < BOUND, err
