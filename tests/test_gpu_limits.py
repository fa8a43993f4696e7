"""
Hard limits of the C ABI (include/cip.h): nchan <= 65535 (the run record's
16-bit channel fields), and the planner's fallback above 2^32 visibilities
(the bank-class order needs a 32-bit flattened index; larger inputs grid in
plain tile order, cip_api.hip make_plan) - checked by linearity: the image of
4,295,032,830 visibilities (fallback) equals the sum of the images of its two
row halves (each < 2^32, ordered path).
"""
import numpy as np
import pytest
import torch

from ska_sdp_cip_amd import _lib
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


def test_nchan_limit(gpu_device):
    nrow = 4
    uvw = torch.zeros((nrow, 3), dtype=torch.float64, device=gpu_device)
    for nchan, ok in ((65535, True), (65536, False)):
        freq = torch.linspace(1e9, 2e9, nchan, dtype=torch.float64, device=gpu_device)
        vis = torch.ones((nrow, nchan), dtype=torch.complex64, device=gpu_device)
        if ok:
            img, _ = device_ms2dirty(uvw, freq, vis, None, 64, 64, 1e-5, 1e-5, support=8)
            assert float(img.max()) > 0.0
        else:
            with pytest.raises(ValueError, match="nchan"):
                device_ms2dirty(uvw, freq, vis, None, 64, 64, 1e-5, 1e-5, support=8)


def test_above_2_pow_32_visibilities(gpu_device):
    nchan, nrow = 65535, 65538
    nvis = nrow * nchan
    assert nvis >= 1 << 32 and (nrow // 2) * nchan < 1 << 32
    free, _ = torch.cuda.mem_get_info(gpu_device)
    if free < 160 << 30:
        pytest.skip("needs ~160 GiB of free HBM")
    uvw_h = syn.uvw_tracks(nrow, 16, array_radius_m=300.0, seed=5)
    freq_h = syn.channel_frequencies(nchan)
    npix = 512
    px = syn.pixel_size_for_grid(uvw_h, freq_h, npix, support=8)
    uvw = torch.from_numpy(uvw_h).to(gpu_device)
    freq = torch.from_numpy(freq_h).to(gpu_device)
    g = torch.Generator(device=gpu_device)
    g.manual_seed(3)
    vis = torch.randn((nrow, nchan), dtype=torch.complex64, device=gpu_device, generator=g)
    try:
        full, _ = device_ms2dirty(uvw, freq, vis, None, npix, npix, px, px, support=8)
        full = full.cpu()
        h = nrow // 2
        a, _ = device_ms2dirty(uvw[:h].contiguous(), freq, vis[:h], None, npix, npix, px, px, support=8)
        a = a.cpu()
        b, _ = device_ms2dirty(uvw[h:].contiguous(), freq, vis[h:], None, npix, npix, px, px, support=8)
        b = b.cpu()
    finally:
        del vis
        torch.cuda.empty_cache()
        _lib.lib().cip_release_workspace()
    peak = float(full.abs().max())
    assert peak > 0.0
    # three gridding calls with their own fixed-point quanta (2^-46 of max |w V|)
    assert float((full - (a + b)).abs().max()) < 1e-11 * peak
