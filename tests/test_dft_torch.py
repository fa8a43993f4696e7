"""
CPU tests of the full-size checkers used by bench.py's parity fields and the
large GPU tests: the torch fp64 DFT at sampled pixels (oracle/dft_torch.py)
equals the C oracle's DFT (oracle.dft_directions) on dense and ragged layouts,
its partial sums over a split of the visibilities add up to the whole, and the
counter-based synthetic columns are a pure function of the global index (so a
strong-scaling run grids the same visibilities at every rank count).
"""
import numpy as np
import torch

import dft_torch
import oracle
from ska_sdp_cip_amd import strips
from ska_sdp_cip_amd import synthetic as syn


def _case(nrow=400, nchan=8, npix=64):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=10, array_radius_m=600.0, seed=3)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    return uvw * np.array([1.0, 1.0, 30.0]), f, vis, w, px


def test_dft_pixels_dense_and_slices_equal_oracle():
    npix = 64
    uvw, f, vis, w, px = _case(npix=npix)
    pix = dft_torch.check_pixels(npix, npix)
    l = np.array([(i - npix // 2) * px for i, _ in pix])  # noqa: E741
    m = np.array([(j - npix // 2) * px for _, j in pix])
    nm1 = -(l * l + m * m) / (np.sqrt(1.0 - l * l - m * m) + 1.0)
    t = torch.from_numpy
    for apply_w in (False, True):
        ref = oracle.dft_directions(uvw if apply_w else uvw * np.array([1.0, 1.0, 0.0]), f, vis, w, l, m)
        if apply_w:
            ref = ref / (nm1 + 1.0)
        got, sw = dft_torch.dft_pixels_dense(t(uvw), t(f), t(vis), t(w), pix, npix, npix, px, px, apply_w=apply_w,
                                             row_chunk=97)
        assert np.abs(got - ref).max() <= 1e-10 * np.abs(ref).max()
        assert abs(sw - float(w.astype(np.float64).sum())) <= 1e-9 * sw
        # ragged layout: rows split into two slices each, in another order
        nchan = vis.shape[1]
        rows = torch.arange(uvw.shape[0]).repeat_interleave(2)
        c0 = torch.tensor([0, 3] * uvw.shape[0])
        c1 = torch.tensor([3, nchan] * uvw.shape[0])
        data = strips.gather_strip(t(uvw), t(vis), t(w), rows, c0, c1)
        got2, sw2 = dft_torch.dft_pixels_slices(data.slice_uvw, data.chan_start, data.chan_stop, t(f), data.vis,
                                                data.wgt, pix, npix, npix, px, px, apply_w=apply_w, vis_chunk=333)
        assert np.abs(got2 - ref).max() <= 1e-10 * np.abs(ref).max()
        assert abs(sw2 - sw) <= 1e-9 * sw


def test_dft_partial_sums_add_up():
    npix = 64
    uvw, f, vis, w, px = _case(npix=npix)
    pix = dft_torch.check_pixels(npix, npix)
    t = torch.from_numpy
    whole, sw = dft_torch.dft_pixels_dense(t(uvw), t(f), t(vis), t(w), pix, npix, npix, px, px)
    parts = [dft_torch.dft_pixels_dense(t(uvw[a:b]), t(f), t(vis[a:b]), t(w[a:b]), pix, npix, npix, px, px)
             for a, b in [(0, 150), (150, 151), (151, 400)]]
    assert np.abs(sum(p[0] for p in parts) - whole).max() <= 1e-11 * np.abs(whole).max()
    assert abs(sum(p[1] for p in parts) - sw) <= 1e-12 * sw


def test_counter_columns_are_a_function_of_the_global_index():
    idx = torch.arange(0, 300_000, dtype=torch.int64)
    vis, wgt = syn.counter_columns(idx, seed=11)
    assert vis.dtype == torch.complex64 and wgt.dtype == torch.float32
    # any subset / order of indices draws the same values
    perm = torch.randperm(idx.numel(), generator=torch.Generator().manual_seed(0))[:5000]
    v2, w2 = syn.counter_columns(idx[perm], seed=11)
    assert torch.equal(v2, vis[perm]) and torch.equal(w2, wgt[perm])
    # another seed, other values; statistics of the bench's columns
    v3, _ = syn.counter_columns(idx[:1000], seed=12)
    assert not torch.equal(v3, vis[:1000])
    assert abs(float(vis.real.mean())) < 0.01 and abs(float(vis.real.std()) - 1.0) < 0.01
    assert abs(float(vis.imag.std()) - 1.0) < 0.01
    flagged = float((wgt == 0).double().mean())
    assert 0.045 < flagged < 0.055
    live = wgt[wgt > 0]
    assert float(live.min()) >= 0.5 and float(live.max()) <= 1.5
