"""
The pruned FFT fast path (csrc/cip_fft.hip row pass + hipFFT column pass on
the kept half) against the fp64 oracle, at every grid size it serves
(nv = 1024 .. 16384, i.e. npix = 512 .. 8192 at sigma = 2), in 2-D and
w-stacking mode. Other sizes take the full 2-D hipFFT path (covered by
test_gpu_invert_parity.py at npix <= 256). At nv = 16384 (C4's grid) the
oracle's 4 GiB host FFT is replaced by the definition itself: sampled
pixels against the direct fp64 DFT at W = 16 (kernel error ~2e-14).
"""

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, synthetic as syn
from ska_sdp_cip_amd.invert import StokesIGridderInput

pytestmark = pytest.mark.gpu

TIGHT = 1e-10


def _case(n_rows, nchan, seed=11):
    ms = syn.make_measurement_set(n_rows, nchan, n_ant=32, array_radius_m=3000.0, fov_l=0.02, seed=seed)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    return gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)


@pytest.mark.parametrize("npix,wstack", [(512, False), (1024, False), (2048, False), (4096, False),
                                         (512, True)])
def test_pruned_fft_matches_oracle(gpu_device, npix, wstack):
    uvw, f, vis, w = _case(3_000 if npix < 4096 else 1_000, 4)
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.4)
    gpu, prm = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=wstack,
                                return_params=True, double_precision_accumulation=True)
    assert prm.nu == 2 * npix
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=wstack)
    sumw = float(w.astype(np.float64).sum())
    # float32 output for complex64 input: compare at float32 resolution of the peak
    tol = max(TIGHT, 4e-7 * float(np.abs(ref).max()) / sumw)
    assert float(np.abs(gpu - ref).max()) / sumw < tol


def test_pruned_fft_rectangular_image(gpu_device):
    # npix_x != npix_y: the row pass keeps npix_y columns of an nv-point transform
    uvw, f, vis, w = _case(2_000, 2)
    px = syn.pixel_size_for_grid(uvw, f, 1024, fill=0.4)
    import torch

    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis.astype(np.complex128), w.astype(np.float64))]
    gpu, prm = gridder.device_ms2dirty(*args, 768, 1024, px, px, support=8)
    ref = oracle.ms2dirty(uvw, f, vis, w, 768, 1024, px, px, support=8)
    sumw = float(w.astype(np.float64).sum())
    assert prm.nv == 2048
    assert float(np.abs(gpu.cpu().numpy() - ref).max()) / sumw < TIGHT


@pytest.mark.parametrize("wstack", [False, True])
def test_pruned_fft_16k_grid_matches_dft(gpu_device, wstack):
    # 16384-point passes (one 1024-thread workgroup per CU, 136 KiB LDS)
    import torch

    uvw, f, vis, w = _case(400, 4, seed=5)
    npix = 8192
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.4)
    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis.astype(np.complex128), w.astype(np.float64))]
    gpu, prm = gridder.device_ms2dirty(*args, npix, npix, px, px, support=16, do_wstacking=wstack)
    assert (prm.nu, prm.nv) == (16384, 16384)
    rng = np.random.default_rng(8)
    pix = [(npix // 2, npix // 2), (0, 0), (npix - 1, npix - 1), (npix // 2, 17), (3, npix - 2)]
    pix += [tuple(int(x) for x in rng.integers(0, npix, 2)) for _ in range(11)]
    ii = np.array([p[0] for p in pix])
    jj = np.array([p[1] for p in pix])
    l, m = (ii - npix // 2) * px, (jj - npix // 2) * px
    if wstack:
        ref = oracle.dft_directions(uvw, f, vis, w, l, m)
        ref = ref / np.sqrt(1.0 - l * l - m * m)
    else:
        flat = uvw.copy()
        flat[:, 2] = 0.0
        ref = oracle.dft_directions(flat, f, vis, w, l, m)
    got = gpu[torch.from_numpy(ii).cuda(), torch.from_numpy(jj).cuda()].cpu().numpy()
    sumw = float(w.astype(np.float64).sum())
    assert float(np.abs(got - ref).max()) / sumw < 1e-10


def test_pruned_fft_16k_even_odd_pass_b_whole_rows(gpu_device):
    # 2-D at nv = 16384: pass B by even / odd column halves
    # (cip_fft.hip fft_cols_eo_kernel; pass A writes H by row parity). Whole
    # image rows - every output cell of their columns, both halves' k' mapping,
    # the +- combination, the crop's both wrapped ranges and (few
    # visibilities: most tile rows are clean) the skipped H rows - against the
    # direct fp64 DFT.
    import torch

    uvw, f, vis, w = _case(400, 4, seed=9)
    npix = 8192
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.4)
    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis.astype(np.complex128), w.astype(np.float64))]
    gpu, prm = gridder.device_ms2dirty(*args, npix, npix, px, px, support=16)
    assert (prm.nu, prm.nv) == (16384, 16384)
    flat = uvw.copy()
    flat[:, 2] = 0.0
    sumw = float(w.astype(np.float64).sum())
    jj = np.arange(npix)
    for i in (0, 1, npix // 2 - 1, npix // 2, 5001, npix - 1):
        l = np.full(npix, (i - npix // 2) * px)
        m = (jj - npix // 2) * px
        ref = oracle.dft_directions(flat, f, vis, w, l, m)
        got = gpu[i].cpu().numpy()
        assert float(np.abs(got - ref).max()) / sumw < 1e-10, i


def test_pruned_fft_16k_even_odd_rectangular(gpu_device):
    # the even / odd pass B beside an 8192-point pass A (npix_x = 4096: nu =
    # 8192, nv = 16384), i.e. nx != ny: whole image rows against the direct DFT
    import torch

    uvw, f, vis, w = _case(300, 3, seed=13)
    npix_x, npix_y = 4096, 8192
    px = syn.pixel_size_for_grid(uvw, f, npix_y, fill=0.4)
    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis.astype(np.complex128), w.astype(np.float64))]
    gpu, prm = gridder.device_ms2dirty(*args, npix_x, npix_y, px, px, support=16)
    assert (prm.nu, prm.nv) == (8192, 16384) and tuple(gpu.shape) == (npix_x, npix_y)
    flat = uvw.copy()
    flat[:, 2] = 0.0
    sumw = float(w.astype(np.float64).sum())
    jj = np.arange(npix_y)
    for i in (0, npix_x // 2, npix_x - 1):
        l = np.full(npix_y, (i - npix_x // 2) * px)
        m = (jj - npix_y // 2) * px
        ref = oracle.dft_directions(flat, f, vis, w, l, m)
        assert float(np.abs(gpu[i].cpu().numpy() - ref).max()) / sumw < 1e-10, i
