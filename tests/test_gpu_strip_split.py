"""
The uv-strip split on the device (cip_strips.hip; cip_strip_histogram,
cip_strip_split, cip_grid_tiles_strip_mask) against the torch restatement of
the same arithmetic on CPU tensors (strips.strip_histogram / strip_slices /
gather_strip, the gloo tests' path): histograms, row slices and gathered
visibilities bit for bit, for channel counts below, at and above a 64-channel
wave, wrapped (long) baselines and empty strips; and the planner-made strip
dirty-tile mask covering every cell the strip's gridding writes (supports 8,
48, 64 and w-stacking; the masked pass A reads only marked tiles).
"""
import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import _lib, strips
from ska_sdp_cip_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _case(nrow, nchan, npix, seed=11, radius=1500.0, px_scale=1.0):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=radius, seed=seed)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix) * px_scale
    return uvw, f, vis, w, px


@pytest.mark.parametrize("nchan,px_scale", [(37, 1.0), (64, 1.0), (130, 1.0), (48, 3.0)])
def test_histogram_and_split_equal_torch(gpu_device, nchan, px_scale):
    # px_scale 3: baselines past the grid edge wrap (the origin rows modulo nv)
    npix = 1024
    uvw, f, vis, w, px = _case(3000, nchan, npix, px_scale=px_scale)
    prm = _lib.choose_params(npix, npix, px, px, 1e-4, 8)
    tu, tf = torch.from_numpy(uvw), torch.from_numpy(f)
    tv, tw = torch.from_numpy(vis.astype(np.complex64)), torch.from_numpy(w.astype(np.float32))
    du, df, dv, dw = (t.to(gpu_device) for t in (tu, tf, tv, tw))
    hv, hr = strips.strip_histogram(du, df, prm, px, px)
    cv, cr = strips.strip_histogram(tu, tf, prm, px, px)
    assert torch.equal(hv.cpu(), cv) and torch.equal(hr.cpu(), cr)
    assert int(hv.sum()) == vis.size
    layout = strips.plan_strips(du, df, prm, px, npix, npix, 5)
    layout_cpu = strips.plan_strips(tu, tf, prm, px, npix, npix, 5)
    assert layout.y_bounds == layout_cpu.y_bounds
    total = 0
    for k in range(layout.world):
        y0, y1 = layout.rows(k)
        dev = strips.split_strip(du, df, dv, dw, prm, px, y0, y1)
        ref = strips.gather_strip(tu, tv, tw, *strips.strip_slices(tu, tf, prm, px, y0, y1))
        assert torch.equal(dev.rows.cpu(), ref.rows)
        assert torch.equal(dev.chan_start.cpu(), ref.chan_start) and torch.equal(dev.chan_stop.cpu(), ref.chan_stop)
        assert torch.equal(dev.slice_uvw.cpu(), ref.slice_uvw)
        assert torch.equal(dev.vis.cpu(), ref.vis) and torch.equal(dev.wgt.cpu(), ref.wgt)
        total += dev.nvis
    assert total == vis.size  # every visibility in exactly one strip
    # an empty strip (a row band no footprint starts in, far outside the tracks)
    hv_np = hv.cpu().numpy()
    empty = int(np.flatnonzero(hv_np == 0)[0]) if (hv_np == 0).any() else None
    if empty is not None:
        d = strips.split_strip(du, df, dv, dw, prm, px, empty, empty + 1)
        assert d.nvis == 0 and d.slice_uvw.shape[0] == 0
    rows, c0, c1 = strips.strip_slices(du, df, prm, px, 0, prm.nv)
    assert int((c1 - c0).sum()) == vis.size


@pytest.mark.parametrize("wstack,support", [(False, 8), (True, 6), (False, 48), (False, 64)])
def test_planner_strip_mask_covers_every_gridded_cell(gpu_device, wstack, support):
    # cip_strip_rows_masked reads only the marked tiles: every non-zero cell of
    # a rank's gridded strip buffer (and the halo rows it receives) must lie in
    # a marked tile of its plane, and the mask must be sparse. W = 48 / 64
    # footprints cross three 32-cell tiles per axis.
    npix = 512
    uvw, f, vis, w, px = _case(900, 12, npix, seed=4, radius=800.0)
    if wstack:
        uvw = uvw * np.array([1.0, 1.0, 40.0])
        wmin, wmax = oracle.w_range(uvw, f)
        prm = _lib.choose_params(npix, npix, px, px, 1e-4, support, True, wmin, wmax)
    else:
        prm = _lib.choose_params(npix, npix, px, px, 1e-4, support)
    du, df = torch.from_numpy(uvw).to(gpu_device), torch.from_numpy(f).to(gpu_device)
    dv = torch.from_numpy(vis.astype(np.complex128)).to(gpu_device)
    dw = torch.from_numpy(w.astype(np.float64)).to(gpu_device)
    world = 3
    layout = strips.plan_strips(du, df, prm, px, npix, npix, world)
    nu, nv = prm.nu, prm.nv
    for r in range(world):
        y0, y1 = layout.rows(r)
        data = strips.split_strip(du, df, dv, dw, prm, px, y0, y1)
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device).bind(layout, r)
        grid, _ = be.grid_strip(data, df)
        torch.cuda.synchronize()
        assert be._bits_valid  # pylint: disable=protected-access
        bits = be._bits.cpu().numpy()  # pylint: disable=protected-access
        planes = grid.cpu().numpy() if grid.dim() == 4 else grid.cpu().numpy()[None]
        assert bits.shape == (planes.shape[0], nv // 32, nu // 1024)
        marked = 0
        for p in range(planes.shape[0]):
            k, x = np.nonzero(np.abs(planes[p]).sum(-1))
            gy = (be.rows[0] + k) % nv
            words = bits[p][gy // 32, x // 1024].astype(np.int64) & 0xFFFFFFFF
            assert np.all((words >> ((x // 32) % 32)) & 1), (r, p)
            # the halo rows [row0, row0 + W - 1) are marked whole
            for yy in range(be.rows[0], be.rows[0] + support - 1):
                assert np.all(bits[p][(yy % nv) // 32] == -1), (r, p, yy)
            marked += int(np.unpackbits(bits[p].view(np.uint8)).sum())
        assert marked < (0.6 if support <= 16 else 0.85) * planes.shape[0] * (nu // 32) * (nv // 32)
        be.grid.zero_()
        be.mark_clean()
