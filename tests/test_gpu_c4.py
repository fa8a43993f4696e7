"""
GPU test at one GPU's share of C4 (BASELINE.json configs[3]: 1G visibilities
-> 16384^2 grid on 8 GPUs; one rank inverts 488,282 rows x 256 channels =
125M visibilities onto the full 16384^2 grid, 8192^2 image, W = 8, 2-D, the
`bench.py --config c4` workload): the 16384-point pruned FFT, 4 GiB grid and
2 GiB pass-A buffer at full size, checked through properties that need no CPU
oracle run at that size (the oracle's host FFT alone would be 4 GiB):

* sampled pixels equal the direct fp64 DFT (the definition, evaluated on the
  GPU in torch fp64 - TEST CODE) within the W = 8 kernel's accuracy
  (~3e-7 of the weight sum);
* the normalised image is the raw image divided by the device weight sum,
  which equals torch's fp64 sum.
"""
import math

import numpy as np
import pytest

from ska_sdp_cip_amd import gridder, synthetic as syn

pytestmark = pytest.mark.gpu

ROWS, NCHAN, NPIX, N_ANT, RADIUS, SEED = 488_282, 256, 8192, 64, 4000.0, 20241008
SPEED_OF_LIGHT = 299792458.0


@pytest.fixture(scope="module")
def c4(gpu_device):
    import torch

    dev = torch.device("cuda", 0)
    uvw = syn.uvw_tracks(ROWS, N_ANT, array_radius_m=RADIUS, seed=SEED)
    freq = syn.channel_frequencies(NCHAN)
    px = syn.pixel_size_for_grid(uvw, freq, NPIX, support=8)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED)
    vis = torch.randn((ROWS, NCHAN), dtype=torch.complex64, device=dev, generator=g)
    wgt = torch.rand((ROWS, NCHAN), dtype=torch.float32, device=dev, generator=g) + 0.5
    flags = torch.rand((ROWS, NCHAN), dtype=torch.float32, device=dev, generator=g) < 0.05
    wgt = torch.where(flags, torch.zeros_like(wgt), wgt).contiguous()
    yield torch.from_numpy(uvw).to(dev), torch.from_numpy(freq).to(dev), vis, wgt, px
    torch.cuda.empty_cache()


def _dft_pixels(c, pix):
    """sum_{r,c} w Re{V exp(2 pi i (f/c) (u l + v m))} at pixels (i, j) (2-D)."""
    import torch

    uvw, f, vis, wgt, px = c
    fx = f / SPEED_OF_LIGHT
    out = []
    for i, j in pix:
        l, m = (i - NPIX // 2) * px, (j - NPIX // 2) * px
        acc = torch.zeros((), dtype=torch.float64, device=vis.device)
        for r0 in range(0, ROWS, 65_536):
            r1 = min(r0 + 65_536, ROWS)
            ph = (2.0 * math.pi) * (uvw[r0:r1, 0] * l + uvw[r0:r1, 1] * m)[:, None] * fx[None, :]
            v = vis[r0:r1].to(torch.complex128)
            acc += (wgt[r0:r1].double() * (v.real * torch.cos(ph) - v.imag * torch.sin(ph))).sum()
        out.append(float(acc.item()))
    return np.array(out)


def test_c4_shard_sampled_pixels_equal_dft(c4):
    import torch

    uvw, f, vis, wgt, px = c4
    img, prm = gridder.device_ms2dirty(uvw, f, vis, wgt, NPIX, NPIX, px, px, support=8)
    assert (prm.nu, prm.nv, prm.nplanes) == (2 * NPIX, 2 * NPIX, 1)
    rng = np.random.default_rng(4)
    pix = [(NPIX // 2, NPIX // 2), (0, 0), (NPIX - 1, NPIX - 1), (NPIX // 2, 0)]
    pix += [tuple(int(x) for x in rng.integers(0, NPIX, 2)) for _ in range(4)]
    ref = _dft_pixels(c4, pix)
    got = np.array([float(img[i, j].item()) for i, j in pix])
    sumw = float(wgt.double().sum().item())
    err = np.abs(got - ref).max() / sumw
    print(f"max |GPU - DFT| / sum w = {err:.3e}")
    # the north-star gate (1e-6); W = 8 measures ~1e-8 on these random visibilities
    assert err < 1e-6, (err, got, ref)

    # normalised in the pass-B epilogue == raw / device weight sum
    raw = img.clone()
    out = torch.empty_like(raw)
    sw = torch.empty(1, dtype=torch.float64, device=raw.device)
    gridder.device_ms2dirty(uvw, f, vis, wgt, NPIX, NPIX, px, px, support=8, normalise=True, out=out,
                            sum_weights=sw)
    assert abs(float(sw.item()) - sumw) <= 1e-12 * sumw
    scale = float(raw.abs().max().item()) / sumw
    assert float((out - raw / sw).abs().max().item()) <= 1e-12 * max(scale, 1e-300)
    torch.cuda.synchronize()


def test_c4_full_eight_strips_equal_one_shot(gpu_device):
    """The north star's strong split at C4's full size (BASELINE configs[3]:
    1G visibilities, ONE 16384^2 grid, 8192^2 image, W = 8), 8 ranks emulated
    on one GPU (strips.invert_strips_local: each rank grids its cost-balanced
    uv strip into a strip + W - 1 halo buffer, halos move to the next rank,
    pass A per strip, the pass-A blocks regroup per image-row strip (the
    all-to-all), pass B per image-row strip), against the one-shot
    cip_ms2dirty of the same visibilities (1e-12 of the peak: only the
    fixed-point quantum of each gridding call differs) and against the fp64
    DFT at sampled pixels. The visibilities are bench.py --strong's
    counter-based columns, the same at every rank count."""
    import torch

    import dft_torch
    from ska_sdp_cip_amd import strips

    dev = torch.device("cuda", 0)
    rows, world = 3_906_250, 8
    uvw_h = syn.uvw_tracks(rows, N_ANT, array_radius_m=RADIUS, seed=SEED)
    freq_h = syn.channel_frequencies(NCHAN)
    px = syn.pixel_size_for_grid(uvw_h, freq_h, NPIX, support=8)
    uvw, f = torch.from_numpy(uvw_h).to(dev), torch.from_numpy(freq_h).to(dev)
    r = torch.arange(rows, device=dev)
    vis, wgt = syn.counter_columns_slices(r, torch.zeros_like(r), torch.full_like(r, NCHAN), NCHAN, SEED)
    vis, wgt = vis.view(rows, NCHAN), wgt.view(rows, NCHAN)
    ref, prm = gridder.device_ms2dirty(uvw, f, vis, wgt, NPIX, NPIX, px, px, support=8, normalise=True)
    assert (prm.nu, prm.nv) == (2 * NPIX, 2 * NPIX)
    layout = strips.plan_strips(uvw, f, prm, px, NPIX, NPIX, world)
    datas = []
    for k in range(world):
        datas.append(strips.split_strip(uvw, f, vis, wgt, prm, px, *layout.rows(k)))
    assert sum(d.nvis for d in datas) == rows * NCHAN
    del vis, wgt
    torch.cuda.empty_cache()
    be = strips.HipStripBackend(prm, px, px, NPIX, NPIX, device=dev)
    img = strips.invert_strips_local(datas, f, layout, be)
    torch.cuda.synchronize()
    peak = float(ref.abs().max())
    diff = float((img - ref).abs().max())
    print(f"C4 8 strips vs one-shot: max |diff| = {diff:.3e} (peak {peak:.3e}); strips {layout.y_bounds}")
    assert diff < 1e-12 * peak
    for k, b in enumerate(be.ranks):
        assert b.rows == strips.strip_buffer_rows(layout, k)
        assert float(b.grid.abs().max()) == 0.0 and not b.dirty
    # the definition at sampled pixels, summed over the ranks' visibilities
    pix = dft_torch.check_pixels(NPIX, NPIX)[:4]
    sums, sw = np.zeros(len(pix)), 0.0
    for d in datas:
        s, w = dft_torch.dft_pixels_slices(d.slice_uvw, d.chan_start, d.chan_stop, f, d.vis, d.wgt, pix, NPIX, NPIX,
                                           px, px)
        sums, sw = sums + s, sw + w
    got = np.array([float(img[i, j].item()) for i, j in pix])
    err = float(np.abs(got - sums / sw).max())
    print(f"C4 8 strips vs DFT pixels: {err:.3e} of sum w")
    assert err < 1e-6
    del be, img
    torch.cuda.empty_cache()
    _distributed_as_threads(datas, f, layout, prm, px, ref, world)
    del datas, ref
    torch.cuda.empty_cache()


def _distributed_as_threads(datas, f, layout, prm, px, ref, world):
    """The same split through the DISTRIBUTED function (strips.invert_strips:
    halo send/recv, mask all-gather, packed pass A, sparse all-to-all, unpack
    kernel, image gather) with the 8 ranks as host threads on this GPU and
    torch.distributed's calls replaced by an in-memory stand-in
    (tests/_thread_dist.py): the configs[3] 8-GPU leg's code path at its size."""
    import torch

    from _thread_dist import run_ranks
    from ska_sdp_cip_amd import strips

    mp = pytest.MonkeyPatch()
    try:
        def rank_fn(r):
            be = strips.HipStripBackend(prm, px, px, NPIX, NPIX, device=torch.device("cuda", 0))
            out = strips.invert_strips(datas[r], f, layout, be)
            torch.cuda.synchronize()
            assert float(be.grid.abs().max()) == 0.0 and not be.dirty
            return out

        results, errors = run_ranks(mp, world, rank_fn)
    finally:
        mp.undo()
    assert not errors, errors
    img = results[0]
    peak = float(ref.abs().max())
    diff = float((img - ref).abs().max())
    print(f"C4 8 distributed ranks (threads) vs one-shot: max |diff| = {diff:.3e} (peak {peak:.3e})")
    assert diff < 1e-12 * peak
