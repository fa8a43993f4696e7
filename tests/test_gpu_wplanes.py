"""
GPU parity of the w-plane split (cip_ms2dirty_wplanes; ska_sdp_cip_amd.wplanes,
SURVEY.md 8(e) option 2): each rank's share of the w-stacking stack against
the oracle's share of the same planes, and the whole decomposition - every
rank's share computed separately and summed - against the one-shot device
image, emulated for 1..8 ranks on one GPU. The multi-process form (one RCCL
reduce of the partial images) runs in the gloo test (test_wplanes.py) and in
`bench.py --strong --wstacking`.
"""
import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd import wplanes
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


def _case(nrow, nchan, npix, seed=11):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=2000.0, fov_l=0.05, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = 0.2 / npix  # a 0.2 rad field: ~24 w planes at W = 6 (baselines wrap exactly)
    return uvw, f, vis.astype(np.complex64), w.astype(np.float32), px


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


@pytest.mark.parametrize("W,npix", [(6, 128), (8, 512)])
def test_plane_share_matches_oracle(gpu_device, W, npix):
    uvw, f, vis, w, px = _case(2000, 8, npix)
    be = wplanes.HipWPlaneBackend(*_dev(uvw, f, vis, w), npix, npix, px, px, support=W)
    prm = be.params()
    assert prm.nplanes > 2 * W
    sumw = float(w.astype(np.float64).sum())
    for planes in [(0, 3), (3, prm.nplanes - 2), (prm.nplanes - 2, prm.nplanes), (5, 5)]:
        img, sw = be(planes)
        ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=True, planes=planes)
        assert abs(float(sw.item()) - sumw) <= 1e-12 * sumw  # the whole call's weight sum
        err = float(np.abs(img.cpu().numpy() - ref).max()) / sumw
        assert err < 1e-10, (planes, err)


@pytest.mark.parametrize("world,W,npix,single", [(1, 6, 512, False), (2, 6, 512, False), (3, 8, 512, False),
                                                  (8, 6, 1024, False), (4, 6, 512, True)])
def test_wplane_decomposition_equals_one_shot(gpu_device, world, W, npix, single):
    uvw, f, vis, w, px = _case(20000, 16, npix)
    d = _dev(uvw, f, vis, w)
    ref, prm = device_ms2dirty(*d, npix, npix, px, px, support=W, do_wstacking=True, normalise=True,
                               single_precision_accumulation=single)
    be = wplanes.HipWPlaneBackend(*d, npix, npix, px, px, support=W, single_precision_accumulation=single)
    bprm = be.params()
    assert (bprm.nplanes, bprm.w0, bprm.dw) == (prm.nplanes, prm.w0, prm.dw)
    feeds = wplanes.plane_feeds(d[0], d[1], prm)
    assert int(feeds.sum()) == vis.size * W
    split = wplanes.split_planes(wplanes.plane_cost(feeds, prm), world)
    stages = []
    img = wplanes.invert_wplanes_local(be, split, stages=stages)
    peak = float(ref.abs().max())
    # fp64 class: same integer sums per cell, only the flush's fp64 adds differ;
    # packed class: each share's work units are scaled by their own size
    tol = 1e-5 if single else 1e-12
    assert float((img - ref).abs().max()) < tol * peak
    assert len(stages) == world and all("grid" in s for s in stages)
    # a second round through the same workspace: grid kept clean between shares
    img2 = wplanes.invert_wplanes_local(be, split)
    assert float((img2 - img).abs().max()) <= 1e-13 * peak


def test_wplane_argument_errors(gpu_device):
    uvw, f, vis, w, px = _case(300, 4, 128)
    d = _dev(uvw, f, vis, w)
    with pytest.raises(ValueError):  # a plane range needs w-stacking
        device_ms2dirty(*d, 128, 128, px, px, support=6, planes=(0, 2))
    _, prm = device_ms2dirty(*d, 128, 128, px, px, support=6, do_wstacking=True)
    with pytest.raises(ValueError):  # past the stack
        device_ms2dirty(*d, 128, 128, px, px, support=6, do_wstacking=True, planes=(0, prm.nplanes + 1))
    with pytest.raises(ValueError):
        device_ms2dirty(*d, 128, 128, px, px, support=6, do_wstacking=True, planes=(3, 2))
    z, _ = device_ms2dirty(*d, 128, 128, px, px, support=6, do_wstacking=True, planes=(1, 1))
    assert float(z.abs().max()) == 0.0
