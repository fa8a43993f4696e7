"""
The uv strips' sparse all-to-all copy kernels (cip_strip_pack_rows /
cip_strip_unpack_rows, strips._pack_live / _unpack_rows): a sender compacts
its live pass-A rows, a receiver scatters every rank's piece into its pass-B
input with zeros for the rows nobody sent - equal, element for element, to the
torch index forms they replace (index_select / advanced-index assignment), for
complex128 and the complex64 wire of the packed class, with empty pieces and
dense (all-live) ranks.
"""
import pytest
import torch

from ska_sdp_cip_amd import strips

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_pack_unpack_equal_index_forms(gpu_device, dtype):
    g = torch.Generator(device="cpu").manual_seed(3)
    nv, world, nb_all = 512, 4, 24
    layout = strips.StripLayout(nu=nv, nv=nv, npix_x=4 * nb_all, npix_y=nv // 2, support=8,
                                y_bounds=[0, 100, 230, 231, nv], x_bounds=[0, 32, 64, 80, 96])
    hs = [layout.rows(r)[1] - layout.rows(r)[0] for r in range(world)]
    Hs = [torch.randn((nb_all, h, 4, 2), generator=g, dtype=torch.float64).to(dtype).to(gpu_device) for h in hs]
    masks = [torch.rand(h, generator=g) < 0.6 for h in hs]
    masks[2][:] = False  # a rank with nothing live
    masks[1][:] = True   # and one with every row live
    masks = [m.to(gpu_device) for m in masks]
    counts = [int(m.sum()) for m in masks]
    sends = [strips._pack_live(H, m, c) for H, m, c in zip(Hs, masks, counts)]  # pylint: disable=protected-access
    for H, m, snd in zip(Hs, masks, sends):
        assert torch.equal(snd, H.index_select(1, torch.nonzero(m).reshape(-1)))
    for s in range(world):
        i0, i1 = layout.image_rows(s)
        b0, b1 = i0 // 4, i1 // 4
        recv = torch.cat([snd[b0:b1].reshape(-1) for snd in sends])
        got = strips._unpack_rows(recv, b1 - b0, layout, masks, dtype)  # pylint: disable=protected-access
        ref = torch.zeros((b1 - b0, nv, 4, 2), dtype=dtype, device=gpu_device)
        for r, H in enumerate(Hs):
            y0, _ = layout.rows(r)
            rows = torch.nonzero(masks[r]).reshape(-1)
            ref[:, y0 + rows] = H[b0:b1].index_select(1, rows)
        assert torch.equal(got, ref)
    # dense ranks (no masks): every row sent
    recv = torch.cat([H[0:2].reshape(-1) for H in Hs])
    got = strips._unpack_rows(recv, 2, layout, [None] * world, dtype)  # pylint: disable=protected-access
    assert torch.equal(got, torch.cat([H[0:2] for H in Hs], dim=1))


@pytest.mark.parametrize("wstack", [False, True])
def test_packed_pass_a_equals_pass_a_then_pack(gpu_device, wstack):
    """cip_strip_rows_packed (pass A writing only the live rows, compacted:
    the send buffer) == the masked pass A followed by the live-row pack, and
    it leaves the strip buffer as clean as the masked pass A does."""
    import numpy as np

    import oracle
    from ska_sdp_cip_amd import _lib
    from ska_sdp_cip_amd import synthetic as syn
    from ska_sdp_cip_amd.gridder import device_ms2dirty

    npix = 512
    ms = syn.make_measurement_set(6000, 16, n_ant=24, array_radius_m=1500.0, seed=9)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    if wstack:
        uvw = uvw * np.array([1.0, 1.0, 20.0])
    px = syn.pixel_size_for_grid(uvw, f, npix)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu_device)  # noqa: E731
    tu, tf, tv, tw = t(uvw), t(f), t(vis.astype(np.complex64)), t(w.astype(np.float32))
    _, prm = device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=8, do_wstacking=wstack)
    layout = strips.plan_strips(tu, tf, prm, px, npix, npix, 2)
    data = strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(1))
    outs = []
    for packed in (False, True):
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=gpu_device)
        be.bind(layout, 1)
        buf, _ = be.grid_strip(data, tf)
        h = layout.rows(1)[1] - layout.rows(1)[0]
        # the halo rows past the strip go to the next rank (sent, then zeroed)
        (buf[:, h:] if wstack else buf[h:]).zero_()
        res = []
        for p in range(int(prm.nplanes) if wstack else 1):
            plane_buf = buf[p] if wstack else buf
            live = be.live_rows(h, p)
            assert live is not None and 0 < int(live.sum()) < h
            cnt = int(live.sum())
            if packed:
                res.append(be.pass_rows_packed(plane_buf, 0, h, live, cnt, plane=p))
            else:
                res.append(strips._pack_live(be.pass_rows(plane_buf, 0, h, plane=p), live, cnt))  # pylint: disable=protected-access
        torch.cuda.synchronize()
        assert float(buf.abs().max()) == 0.0
        outs.append(res)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    del _lib
