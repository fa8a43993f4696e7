"""
GPU parity of the strong-scaling uv-strip path (ska_sdp_cip_amd.strips,
cip_strip_rows / cip_strip_cols): the strip passes against their CPU
restatement (tests/_strip_np.py) on the same grid, and the whole
decomposition - strips gridded separately, halos exchanged, pass A per strip,
blocks exchanged, pass B per image-row strip - against the one-shot device
image, emulated for 1..8 ranks on one GPU. The multi-process form runs in the
world-size-2/3 gloo test (test_strips.py) and in `bench.py --strong`.
"""

import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import _lib, strips
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty

pytestmark = pytest.mark.gpu


def _case(nrow, nchan, npix, seed=7):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=1500.0, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    return uvw, f, vis, w, px


def _to(dev, *arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in arrs]


@pytest.mark.parametrize("W", [4, 8])
def test_strip_passes_match_cpu_restatement(gpu_device, W):
    from _strip_np import NumpyStripBackend

    npix = 512  # the pruned FFT covers grids of 1024 .. 16384
    uvw, f, vis, w, px = _case(2000, 8, npix)
    prm = _lib.choose_params(npix, npix, px, px, 1e-4, W)
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
    nb = NumpyStripBackend(oracle.choose_params(npix, npix, px, px, support=W), px, px, npix, npix)
    rng = np.random.default_rng(1)
    g = rng.standard_normal((prm.nv, prm.nu, 2))
    for y0, y1 in [(0, 17), (17, prm.nv), (100, 101), (prm.nv - 9, prm.nv)]:
        be.grid[y0:y1] = torch.from_numpy(g[y0:y1]).to(gpu_device)
        nb.grid[y0:y1] = torch.from_numpy(g[y0:y1])
        H = be.pass_rows(be.grid, y0, y1)
        Hn = nb.pass_rows(nb.grid, y0, y1)
        assert float(be.grid.abs().max()) == 0.0  # rows read are zeroed
        scale = float(Hn.abs().max())
        assert float((H.cpu() - Hn).abs().max()) < 1e-13 * scale
    Hfull = torch.from_numpy(rng.standard_normal((npix // 4, prm.nv, 4, 2)))
    norm = torch.tensor([3.5], dtype=torch.float64)
    for i0, i1 in [(0, npix), (0, 4), (60, 128), (npix - 4, npix)]:
        Hs = Hfull[i0 // 4:i1 // 4].contiguous()
        out = be.pass_cols(Hs.to(gpu_device), i0, i1, norm=norm.to(gpu_device))
        ref = nb.pass_cols(Hs, i0, i1, norm=norm)
        assert float((out.cpu() - ref).abs().max()) < 1e-12 * float(ref.abs().max())


@pytest.mark.parametrize("world,W,npix", [(1, 8, 512), (2, 8, 512), (3, 6, 512), (4, 8, 1024), (8, 4, 1024)])
def test_strip_decomposition_equals_one_shot(gpu_device, world, W, npix):
    uvw, f, vis, w, px = _case(30000, 32, npix)
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    ref, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=W, normalise=True)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
    datas = []
    for r in range(world):
        datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
    assert sum(d.nvis for d in datas) == vis.size
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
    stages = []
    img = strips.invert_strips_local(datas, tf, layout, be, stages=stages)
    torch.cuda.synchronize()
    # same visibilities and weights; only the fixed-point quantum of each
    # gridding call differs (2^-46 of each strip's max |w V|)
    peak = float(ref.abs().max())
    assert float((img - ref).abs().max()) < 1e-12 * peak
    # each rank holds only its strip + W - 1 halo rows, left clean
    for r, b in enumerate(be.ranks):
        assert b.rows == strips.strip_buffer_rows(layout, r)
        assert tuple(b.grid.shape) == (b.rows[1], prm.nu, 2)
        assert float(b.grid.abs().max()) == 0.0 and not b.dirty
    assert len(stages) == world and all("grid" in st and "rows" in st and "cols" in st for st in stages)
    # a second call through the same rank buffers gives the same image
    img2 = strips.invert_strips_local(datas, tf, layout, be)
    assert torch.equal(img, img2)


@pytest.mark.parametrize("world,W,single", [(1, 6, False), (2, 6, False), (3, 8, False), (8, 6, False),
                                             (4, 6, True)])
def test_wstacking_strip_decomposition_equals_one_shot(gpu_device, world, W, single):
    # the reference's gridding mode split by uv strips: each rank grids every
    # w plane's strip rows, the halos of all planes move at once, then per
    # plane pass A / regrouping / pass B with the w screen into the rank's
    # image rows, and the final w correction per rank
    npix = 512
    uvw, f, vis, w, px = _case(12000, 16, npix)
    uvw = uvw * np.array([1.0, 1.0, 20.0])  # a deep w range: many planes
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    ref, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=W, do_wstacking=True, normalise=True,
                               single_precision_accumulation=single)
    assert prm.nplanes > W
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
    datas = []
    for r in range(world):
        datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device, single_precision_accumulation=single)
    stages = []
    img = strips.invert_strips_local(datas, tf, layout, be, stages=stages)
    torch.cuda.synchronize()
    peak = float(ref.abs().max())
    # fp64 class: only the fixed-point quantum per gridding call differs; the
    # packed class: the one-shot call's complex64 planes and pass-A output
    # against the strips' complex128 planes (the class's own rounding)
    assert float((img - ref).abs().max()) < (1e-5 if single else 1e-12) * peak
    for r, b in enumerate(be.ranks):
        assert tuple(b.grid.shape) == (prm.nplanes, b.rows[1], prm.nu, 2)
        assert float(b.grid.abs().max()) == 0.0 and not b.dirty
    assert all("final" in st for st in stages)
    img2 = strips.invert_strips_local(datas, tf, layout, be)
    assert torch.equal(img, img2)


def test_strip_buffer_rejects_footprints_outside_its_rows(gpu_device):
    # cip_grid_tiles_strip: a visibility whose footprint leaves the buffer's
    # row window is an error (CIP_ERANGE), not an out-of-bounds write
    npix = 512
    uvw, f, vis, w, px = _case(3000, 8, npix)
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    prm = _lib.choose_params(npix, npix, px, px, 1e-4, 8)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, 4)
    data = strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(2))
    assert data.nvis > 0
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
    be.bind(layout, 1)  # another rank's rows
    with pytest.raises(ValueError, match="strip"):
        be.grid_strip(data, tf)
    assert be.dirty  # the failed call leaves the buffer marked dirty ...
    be.bind(layout, 2)  # (rebinding reallocates a clean buffer)
    buf, sw = be.grid_strip(data, tf)
    assert float(buf.abs().max()) > 0.0
    H = be.pass_rows(buf, 0, layout.rows(2)[1] - layout.rows(2)[0])
    buf[layout.rows(2)[1] - layout.rows(2)[0]:].zero_()
    be.mark_clean()
    assert float(buf.abs().max()) == 0.0 and H.shape[1] == layout.rows(2)[1] - layout.rows(2)[0]


def test_strip_backend_recovers_from_an_interrupted_invert(gpu_device):
    # a dirty buffer (an invert that stopped between gridding and pass A) is
    # zeroed by the next grid_strip instead of being trusted as CIP_GRID_ZEROED
    npix = 512
    uvw, f, vis, w, px = _case(3000, 8, npix)
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    ref, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=8, normalise=True)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, 1)
    data = strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(0))
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
    be.grid_strip(data, tf)  # interrupted: no pass A
    assert be.dirty
    img = strips.invert_strips_local([data], tf, layout, be)
    assert float((img - ref).abs().max()) < 1e-12 * float(ref.abs().max())


def test_allreduce_grids_multi_gpu():
    # cip_allreduce_grid with ndev >= 2 (single process, one RCCL clique over
    # the node's GPUs): needs a multi-GPU box, skipped on the 1-GPU test box
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs")
    from ska_sdp_cip_amd.distributed import allreduce_grids

    ndev = torch.cuda.device_count()
    n = 1 << 20
    ts = [torch.full((n,), float(k + 1), dtype=torch.float64, device=f"cuda:{k}") for k in range(ndev)]
    allreduce_grids(ts)
    want = ndev * (ndev + 1) / 2
    for t in ts:
        assert bool(torch.all(t == want))
    ts = [torch.arange(n, dtype=torch.float64, device=f"cuda:{k}") * (k + 1) for k in range(ndev)]
    allreduce_grids(ts, root=0)
    assert torch.equal(ts[0].cpu(), want * torch.arange(n, dtype=torch.float64))


@pytest.mark.parametrize("wstack,support", [(False, 6), (True, 6), (False, 48), (False, 64)])
def test_masked_strip_pass_a_equals_dense(gpu_device, monkeypatch, wstack, support):
    # cip_strip_rows_masked reads only the strip's dirty tiles; every other
    # cell is zero, so the images equal the dense pass A's bit for bit and
    # both leave the buffers clean
    npix = 512
    uvw, f, vis, w, px = _case(12000, 16, npix)
    if wstack:
        uvw = uvw * np.array([1.0, 1.0, 20.0])
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    _, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=support, do_wstacking=wstack,
                             normalise=True)
    world = 4
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
    datas = []
    for r in range(world):
        datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
    imgs = {}
    for masked in ("1", "0"):
        monkeypatch.setenv("CIP_STRIP_MASK", masked)
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
        assert be.masked == (masked == "1")
        imgs[masked] = strips.invert_strips_local(datas, tf, layout, be)
        torch.cuda.synchronize()
        for b in be.ranks:
            assert float(b.grid.abs().max()) == 0.0
    assert torch.equal(imgs["1"], imgs["0"])


def test_strip_mask_follows_the_frequencies(gpu_device):
    # the masked pass A's dirty-tile mask depends on the frequencies as well as
    # on the strip data: gridding the same StripData with other frequencies
    # must recompute it (a stale mask would skip tiles that are now dirty).
    # One strip (the whole grid: no strip window for the moved footprints to
    # leave), the band shifted by 3 % on the second call.
    npix, W = 512, 6
    uvw, f, vis, w, px = _case(12000, 16, npix)
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    _, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=W, normalise=True)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, 1)
    datas = [strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(0))]
    be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
    assert be.masked
    strips.invert_strips_local(datas, tf, layout, be)
    tf2 = tf * 1.03
    img = strips.invert_strips_local(datas, tf2, layout, be)
    torch.cuda.synchronize()
    assert float(be.grid.abs().max()) == 0.0
    ref, _ = device_ms2dirty(tu, tf2, tv, tw, npix, npix, px, px, support=W, normalise=True)
    assert float((img - ref).abs().max()) <= 1e-12 * float(ref.abs().max())


@pytest.mark.parametrize("wstack,W", [(False, 8), (False, 16), (True, 6)])
def test_ragged_stream_forms_are_bit_identical(gpu_device, monkeypatch, wstack, W):
    """The strips' ragged row slices grid through three forms of the planner's
    ordered stream: packed runs (the default: a run record is its first
    stream entry, its length rides in the sort key), packed entries built from
    (row, channel) run records with the delta[row] gather (CIP_PACKED_RUNS=0),
    and the (row << 16) | channel entries of inputs too large to pack
    (CIP_RAGGED_PACK=0; both switches are read per call). Fixed-point integer
    sums: the same image bit for bit, at W = 8 / 16 and in w-stacking."""
    npix = 512
    uvw, f, vis, w, px = _case(20000, 24, npix)
    if wstack:
        uvw = uvw * np.array([1.0, 1.0, 20.0])
    tu, tf, tv, tw = _to(gpu_device, uvw, f, vis.astype(np.complex64), w.astype(np.float32))
    _, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=W, do_wstacking=wstack)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, 3)
    datas = []
    for r in range(3):
        datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
    imgs = []
    for env in ({}, {"CIP_PACKED_RUNS": "0"}, {"CIP_RAGGED_PACK": "0"}):
        for k in ("CIP_PACKED_RUNS", "CIP_RAGGED_PACK"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
        imgs.append(strips.invert_strips_local(datas, tf, layout, be).clone())
    torch.cuda.synchronize()
    assert float(imgs[0].abs().max()) > 0.0
    assert torch.equal(imgs[0], imgs[1])
    assert torch.equal(imgs[0], imgs[2])
