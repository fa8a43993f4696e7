"""
The per-thread workspace's kept-clean grid across calls of different
geometries (cip_api.hip grid_clean_bytes): a call on a smaller
power-of-two grid zeroes and keeps clean only ITS bytes of the reused grid
buffer, so a later call on a larger grid must not trust the rest. Sequence:
non-power-of-two grid (hipFFT path, leaves the buffer dirty) -> small
power-of-two grid (masked pass A, marks its bytes clean) -> the first
geometry again, which must equal its first image bit for bit.
"""
import numpy as np
import pytest
import torch

from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


def _inputs(dev, nrow, nchan, npix, seed):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=16, array_radius_m=1000.0, seed=seed)
    uvw, f = ms.uvw(), ms.channel_frequencies()
    rng = np.random.default_rng(seed)
    vis = (rng.standard_normal((nrow, nchan)) + 1j * rng.standard_normal((nrow, nchan))).astype(np.complex64)
    w = rng.uniform(0.5, 1.5, (nrow, nchan)).astype(np.float32)
    px = syn.pixel_size_for_grid(uvw, f, npix)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return t(uvw), t(f), t(vis), t(w), px


@pytest.mark.parametrize("wstacking", [False, True])
def test_grid_clean_state_is_per_byte(gpu_device, wstacking):
    big = 600    # nu = 1200: 2/3/5-smooth, not a power of two -> hipFFT path
    small = 512  # nu = 1024: pruned FFT, masked pass A keeps its planes clean
    a = _inputs(gpu_device, 3000, 8, big, 3)
    b = _inputs(gpu_device, 1500, 4, small, 4)
    img_a, prm_a = device_ms2dirty(*a[:4], big, big, a[4], a[4], support=8, do_wstacking=wstacking)
    assert prm_a.nu == 1200
    img_b1, prm_b = device_ms2dirty(*b[:4], small, small, b[4], b[4], support=8, do_wstacking=wstacking)
    assert prm_b.nu == 1024
    img_b2, _ = device_ms2dirty(*b[:4], small, small, b[4], b[4], support=8, do_wstacking=wstacking)
    assert torch.equal(img_b1, img_b2)  # the kept-clean small grid needs no memset
    img_a2, _ = device_ms2dirty(*a[:4], big, big, a[4], a[4], support=8, do_wstacking=wstacking)
    assert torch.equal(img_a, img_a2)


def test_grid_zeroed_flag_ignores_unaligned_planes(gpu_device):
    # CIP_GRID_ZEROED's private-cell stores are 16-byte: planes that are only
    # 8-byte aligned take the atomic path (same values) instead of faulting
    from ska_sdp_cip_amd import _lib
    from ska_sdp_cip_amd.gridder import _codes

    npix = 8192  # a 16384^2 grid: the size where the flush stores are on
    nrow, nchan = 400, 4
    uvw, f, vis, w, px = _inputs(gpu_device, nrow, nchan, 512, 5)
    prm = _lib.choose_params(npix, npix, px / 16, px / 16, 1e-4, 8)
    vc, wc = _codes()
    n = 2 * prm.nu * prm.nv
    out = []
    for off in (0, 1):  # 16-byte aligned, then shifted by one double
        store = torch.zeros(n + 2, dtype=torch.float64, device=gpu_device)
        planes = store[off:off + n]
        assert (planes.data_ptr() % 16 == 0) == (off == 0)
        sw = torch.zeros(1, dtype=torch.float64, device=gpu_device)
        _lib.check(_lib.lib().cip_grid_ms(uvw.data_ptr(), nrow, f.data_ptr(), nchan, vis.data_ptr(), vc[vis.dtype],
                                          w.data_ptr(), wc[w.dtype], prm, px / 16, px / 16, npix, npix,
                                          _lib.CIP_GRID_ZEROED, torch.cuda.current_stream().cuda_stream,
                                          planes.data_ptr(), sw.data_ptr()))
        torch.cuda.synchronize()
        out.append(planes.clone())
        del store, planes
    peak = float(out[0].abs().max())
    assert peak > 0.0
    # halo cells take fp64 atomics from up to four work units in either run
    assert float((out[0] - out[1]).abs().max()) <= 1e-13 * peak
