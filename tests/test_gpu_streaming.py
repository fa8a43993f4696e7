"""
GPU tests of the accumulating gridder and the chunked host -> HBM streaming
invert: gridding a data set chunk by chunk onto one
set of resident planes equals the one-shot cip_ms2dirty (linearity; each
chunk has its own fixed-point scale, so they agree to rounding, < 1e-10 of
the weight sum), tile-layout (ragged row slice) chunks equal the MS they were
cut from, and the file-streaming paths equal invert_measurement_set.
"""
import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, invert_measurement_set, synthetic as syn
from ska_sdp_cip_amd.accumulate import GridAccumulator, w_range_rows
from ska_sdp_cip_amd.dispatch import LocalGPUClient
from ska_sdp_cip_amd.invert import StokesIGridderInput
from ska_sdp_cip_amd.measurement_set import InMemoryMeasurementSet
from ska_sdp_cip_amd.streaming import invert_measurement_set_streamed, invert_tile_files
from ska_sdp_cip_amd.uvw_tiling import Tile, create_uvw_tile_mapping_sequential, reorder_by_uvw_tile

pytestmark = pytest.mark.gpu
TIGHT = 1e-10


def _case(n_rows, nchan, seed=5):
    ms = syn.make_measurement_set(n_rows, nchan, n_ant=16, array_radius_m=1500.0, fov_l=0.01, seed=seed)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    return ms, gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)


def _t(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("wstack", [False, True])
def test_grid_ms_chunks_equal_one_shot(gpu_device, wstack):
    _, uvw, f, vis, w = _case(3_000, 16)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    one, prm = gridder.device_ms2dirty(_t(uvw), _t(f), _t(vis), _t(w), npix, npix, px, px, support=8,
                                       do_wstacking=wstack)
    acc = GridAccumulator(npix, npix, px, px, support=8, do_wstacking=wstack, w_range=w_range_rows(uvw, f))
    assert (acc.params.nplanes, acc.params.nu) == (prm.nplanes, prm.nu)
    if wstack:
        assert prm.nplanes > 1 and acc.params.w0 == prm.w0 and acc.params.dw == prm.dw
    for a, b in [(0, 700), (700, 701), (701, 2_200), (2_200, 3_000)]:
        acc.add_ms(_t(uvw[a:b]), _t(f), _t(vis[a:b]), _t(w[a:b]))
    dirty, sumw = acc.dirty()
    sw = float(w.astype(np.float64).sum())
    assert abs(float(sumw.item()) - sw) < 1e-9 * sw
    err = float((dirty - one).abs().max().item()) / sw
    assert err < TIGHT, err


def _tiles_of(uvw, f, vis, w, tile_size=(300.0, 300.0, 10_000.0)):
    mapping = create_uvw_tile_mapping_sequential(uvw, tile_size, f)
    return [Tile._from_jagged_visibilities_slice(vis, uvw, k, v, weights=w)  # pylint: disable=protected-access
            for k, v in mapping.items()]


@pytest.mark.parametrize("wstack,support", [(False, 8), (True, 8), (False, 32), (True, 24)])
def test_grid_tiles_equal_dense(gpu_device, wstack, support):
    # ragged row slices (the Tile layout) vs the dense MS they were cut from
    # (W = 24 / 32: the wave-per-visibility scatter on the ragged row map)
    _, uvw, f, vis, w = _case(2_000, 24, seed=9)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    tiles = _tiles_of(uvw, f, vis, w)
    assert len(tiles) > 10 and sum(t.num_visibilities for t in tiles) == vis.size
    acc = GridAccumulator(npix, npix, px, px, support=support, do_wstacking=wstack, w_range=w_range_rows(uvw, f))
    fd = _t(f)
    for t in tiles:
        acc.add_tile(_t(t.uvw), _t(t.channel_start_indices.astype(np.int32)),
                     _t(t.channel_stop_indices.astype(np.int32)), fd, _t(t.visibilities), _t(t.weights))
    dirty, sumw = acc.dirty()
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=support, do_wstacking=wstack)
    sw = float(w.astype(np.float64).sum())
    err = float(np.abs(dirty.cpu().numpy() - ref).max()) / sw
    # large supports: conditioning of the grid correction (test_gpu_large_support.py TOL)
    assert err < (TIGHT if support <= 16 else 1e-9), err


def test_grid_tiles_edge_cases(gpu_device):
    _, uvw, f, vis, w = _case(200, 8, seed=2)
    npix = 64
    px = syn.pixel_size_for_grid(uvw, f, npix)
    acc = GridAccumulator(npix, npix, px, px, support=6)
    fd = _t(f)
    # empty slices (c0 == c1) between real ones, and an empty tile
    c0 = np.array([0, 3, 3, 5], dtype=np.int32)
    c1 = np.array([2, 3, 8, 5], dtype=np.int32)
    rows = [0, 1, 2, 3]
    v = np.concatenate([vis[r, a:b] for r, a, b in zip(rows, c0, c1)])
    ww = np.concatenate([w[r, a:b] for r, a, b in zip(rows, c0, c1)])
    acc.add_tile(_t(uvw[rows]), _t(c0), _t(c1), fd, _t(v), _t(ww))
    acc.add_tile(_t(uvw[:0]), _t(c0[:0]), _t(c1[:0]), fd, _t(v[:0]), _t(ww[:0]))
    with pytest.raises(ValueError):  # visibility count differs from the slices' total
        acc.add_tile(_t(uvw[rows]), _t(c0), _t(c1), fd, _t(v[:-1]), _t(ww[:-1]))
    with pytest.raises(ValueError):  # channel range beyond nchan
        acc.add_tile(_t(uvw[:1]), _t(np.array([6], np.int32)), _t(np.array([9], np.int32)), fd, _t(v[:3]),
                     _t(ww[:3]))
    dirty, sumw = acc.dirty()
    # the same visibilities as a dense (masked-weight) MS
    wd = np.zeros((4, 8), np.float32)
    for r, a, b in zip(range(4), c0, c1):
        wd[r, a:b] = w[rows[r], a:b]
    ref = oracle.ms2dirty(uvw[rows], f, vis[rows], wd, npix, npix, px, px, support=6, do_wstacking=False)
    sw = float(wd.astype(np.float64).sum())
    assert abs(float(sumw.item()) - sw) < 1e-9 * sw
    assert float(np.abs(dirty.cpu().numpy() - ref).max()) / sw < TIGHT


@pytest.mark.parametrize("wstack", [False, True])
def test_grid_tiles_ragged_slices_stress(gpu_device, wstack):
    # the place pass finds each lane's slice from its 64-visibility segment's
    # first slice (cip_common.h ragged_row_of): slices of 0 .. nchan channels
    # cross segment starts, several start inside one segment, and a run of 200
    # empty slices (more than one wave of repeated starts) sits between two
    # segments; against the same visibilities as a dense masked-weight MS
    nrow, nchan = 3000, 40
    _, uvw, f, vis, w = _case(nrow, nchan, seed=6)
    npix = 256
    px = syn.pixel_size_for_grid(uvw, f, npix)
    rng = np.random.default_rng(4)
    c0 = rng.integers(0, nchan, nrow).astype(np.int32)
    ln = np.where(rng.uniform(size=nrow) < 0.5, rng.integers(0, 4, nrow), rng.integers(0, nchan + 1, nrow))
    c1 = np.minimum(c0 + ln, nchan).astype(np.int32)
    c1[1000:1200] = c0[1000:1200]
    rows = np.arange(nrow)
    v = np.concatenate([vis[r, a:b] for r, a, b in zip(rows, c0, c1)])
    ww = np.concatenate([w[r, a:b] for r, a, b in zip(rows, c0, c1)])
    acc = GridAccumulator(npix, npix, px, px, support=8, do_wstacking=wstack, w_range=w_range_rows(uvw, f))
    acc.add_tile(_t(uvw), _t(c0), _t(c1), _t(f), _t(v), _t(ww))
    dirty, sumw = acc.dirty()
    wd = np.zeros((nrow, nchan), np.float32)
    for r, a, b in zip(rows, c0, c1):
        wd[r, a:b] = w[r, a:b]
    ref = oracle.ms2dirty(uvw, f, vis, wd, npix, npix, px, px, support=8, do_wstacking=wstack)
    sw = float(wd.astype(np.float64).sum())
    assert abs(float(sumw.item()) - sw) < 1e-9 * sw
    assert float(np.abs(dirty.cpu().numpy() - ref).max()) / sw < TIGHT


def _golden_like_ms(seed=11):
    ms = syn.make_measurement_set(1_500, 8, n_ant=20, array_radius_m=2000.0, fov_l=0.01, seed=seed)
    return InMemoryMeasurementSet(ms.uvw(), ms.visibilities(), ms.flags(), ms.weights(),
                                  ms.channel_frequencies())


@pytest.mark.parametrize("wstack", [False, True])
def test_invert_tile_files_streamed(gpu_device, tmp_path, wstack):
    ms = _golden_like_ms()
    pix_asec = 20.0
    paths = reorder_by_uvw_tile(ms, (2000.0, 2000.0, 8000.0), tmp_path, LocalGPUClient(), num_time_intervals=3,
                                max_vis_per_chunk=800, with_weights=True)
    assert len(paths) > 4
    img = invert_tile_files(paths, ms.channel_frequencies(), 64, pix_asec, support=8, do_wstacking=wstack)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    w = gi.effective_weights()
    px = float(np.sin(np.radians(pix_asec / 3600.0)))
    ref = oracle.ms2dirty(gi.uvw, gi.channel_frequencies, gi.visibilities, w, 64, 64, px, px, support=8,
                          do_wstacking=wstack)
    ref = ref / float(w.astype(np.float64).sum())
    assert np.abs(img - ref).max() < TIGHT * max(1.0, np.abs(ref).max())
    # the reference's own files (no weights key): unit weights
    img1 = invert_tile_files(paths, ms.channel_frequencies(), 64, pix_asec, support=8, use_weights=False)
    ones = np.ones_like(w)
    ref1 = oracle.ms2dirty(gi.uvw, gi.channel_frequencies, gi.visibilities, ones, 64, 64, px, px, support=8,
                           do_wstacking=False) / ones.size
    assert np.abs(img1 - ref1).max() < TIGHT * max(1.0, np.abs(ref1).max())


def test_invert_measurement_set_streamed_equals_one_shot(gpu_device):
    ms = _golden_like_ms(seed=12)
    one = invert_measurement_set(ms, 64, 20.0)  # reference arguments: epsilon 1e-4, w-stacking
    for rows_per_chunk in (256, 1_000_000):
        img = invert_measurement_set_streamed(ms, 64, 20.0, rows_per_chunk=rows_per_chunk, do_wstacking=True)
        assert img.dtype == np.float32 and img.shape == one.shape
        # same gridding; the reference sums the total weight in float32 numpy
        assert np.abs(img - one).max() <= 2e-6 * np.abs(one).max()


def test_allreduce_grids_native_rccl(gpu_device):
    # cip_allreduce_grid (single process, RCCL): on the one-GPU test box the
    # clique has one device (sum of one); with more devices every one holds
    # the sum of all
    import torch

    from ska_sdp_cip_amd.distributed import allreduce_grids

    ndev = torch.cuda.device_count()
    ts = [torch.full((1000,), float(k + 1), dtype=torch.float64, device=f"cuda:{k}") for k in range(ndev)]
    allreduce_grids(ts)
    want = ndev * (ndev + 1) / 2
    for t in ts:
        assert torch.all(t == want)
    ts = [torch.arange(10, dtype=torch.float64, device=f"cuda:{k}") for k in range(ndev)]
    allreduce_grids(ts, root=0)
    assert torch.equal(ts[0].cpu(), ndev * torch.arange(10, dtype=torch.float64))
