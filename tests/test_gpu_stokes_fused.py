"""
Stokes I fused into the gridder (cip_ms2dirty_stokes_i):
the planner and scatter read the raw (nrow, nchan, 4) linear-feed columns and
form Stokes I and the effective weights as they load each visibility. Images,
weight sums and parameters must equal cip_stokes_i + cip_ms2dirty bit for bit
(the same float32 Stokes arithmetic, pinned against the reference's numpy by
tests/golden/stokes_i.npz in test_gpu_tiling_and_api.py), in every mode.
"""
import numpy as np
import pytest
import torch

import oracle
from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.gridder import device_ms2dirty, device_ms2dirty_stokes_i, device_stokes_i
from ska_sdp_cip_amd.invert import device_invert, invert_measurement_set

pytestmark = pytest.mark.gpu


def _raw_case(nrow=3000, nchan=16, npix=256, seed=3):
    ms = syn.make_measurement_set(nrow, nchan, n_ant=24, array_radius_m=1500.0, seed=seed)
    vis4 = np.ascontiguousarray(ms.visibilities(), dtype=np.complex64)
    flags4 = np.ascontiguousarray(ms.flags()).astype(np.uint8)
    wgt4 = np.ascontiguousarray(ms.weights(), dtype=np.float32)
    rng = np.random.default_rng(seed)
    # flagged entries, zero weights on one feed, NaN visibilities under flags
    flags4[rng.uniform(size=flags4.shape) < 0.03] = 1
    wgt4[rng.uniform(size=wgt4.shape) < 0.02] = 0.0
    bad = (flags4[..., 0] != 0) & (rng.uniform(size=flags4.shape[:2]) < 0.3)
    vis4[bad, 0] = np.nan
    uvw, f = ms.uvw(), ms.channel_frequencies()
    px = syn.pixel_size_for_grid(uvw, f, npix)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    return t(uvw), t(f), t(vis4), t(flags4), t(wgt4), px, (vis4, flags4, wgt4)


@pytest.mark.parametrize("kw", [
    dict(support=8),
    dict(support=6, do_wstacking=True),             # the reference's call: epsilon 1e-4 -> W = 6, w-stacking
    dict(epsilon=1e-4, do_wstacking=True),
    dict(support=8, single_precision_accumulation=True),
    dict(support=8, psf=True),
    dict(support=4, normalise=True),
    dict(support=24),                                # wave-per-visibility large-support scatter
])
def test_fused_equals_two_pass_bit_for_bit(gpu_device, kw):
    uvw, f, vis4, flags4, wgt4, px, _ = _raw_case()
    npix = 256
    vis_i, eff = device_stokes_i(vis4, flags4, wgt4)
    sw_a = torch.zeros(1, dtype=torch.float64, device=gpu_device)
    sw_b = torch.zeros(1, dtype=torch.float64, device=gpu_device)
    a, pa = device_ms2dirty(uvw, f, vis_i, eff, npix, npix, px, px, sum_weights=sw_a, **kw)
    b, pb = device_ms2dirty_stokes_i(uvw, f, vis4, flags4, wgt4, npix, npix, px, px, sum_weights=sw_b, **kw)
    torch.cuda.synchronize()
    assert pa.as_dict() == pb.as_dict()
    assert torch.equal(sw_a, sw_b)
    assert torch.equal(a, b)


def test_fused_against_oracle_and_flags_none(gpu_device):
    uvw, f, vis4, flags4, wgt4, px, (v4, f4, w4) = _raw_case(nrow=1500, nchan=8, npix=128)
    npix = 128
    img, _ = device_ms2dirty_stokes_i(uvw, f, vis4, flags4, wgt4, npix, npix, px, px, support=8)
    vis_i, _, _, eff = oracle.stokes_i(v4, f4.astype(bool), w4)
    ref = oracle.ms2dirty(uvw.cpu().numpy(), f.cpu().numpy(), vis_i, eff, npix, npix, px, px, support=8)
    assert float(np.abs(img.cpu().numpy() - ref).max()) < 1e-12 * float(eff.astype(np.float64).sum())
    # flags4=None: nothing flagged (so NaN visibilities must go: zero them)
    v = vis4.clone()
    v[torch.isnan(v.real) | torch.isnan(v.imag)] = 0
    none, _ = device_ms2dirty_stokes_i(uvw, f, v, None, wgt4, npix, npix, px, px, support=8)
    zero, _ = device_ms2dirty_stokes_i(uvw, f, v, torch.zeros_like(flags4), wgt4, npix, npix, px, px, support=8)
    assert torch.equal(none, zero)
    # bool flags are taken as bytes
    b, _ = device_ms2dirty_stokes_i(uvw, f, vis4, flags4.bool(), wgt4, npix, npix, px, px, support=8)
    assert torch.equal(b, img)


def test_fused_pipelined_calls(gpu_device):
    # resident inputs, back-to-back CIP_ASYNC | CIP_PIPELINE calls (the bench's mode)
    uvw, f, vis4, flags4, wgt4, px, _ = _raw_case()
    npix = 256
    one, _ = device_ms2dirty_stokes_i(uvw, f, vis4, flags4, wgt4, npix, npix, px, px, support=8, normalise=True)
    outs = [torch.empty_like(one) for _ in range(3)]
    for o in outs:
        device_ms2dirty_stokes_i(uvw, f, vis4, flags4, wgt4, npix, npix, px, px, support=8, normalise=True,
                                 out=o, synchronize=False, resident_inputs=True)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, one)


def test_fused_rejects_bad_input(gpu_device):
    uvw, f, vis4, flags4, wgt4, px, _ = _raw_case(nrow=200, nchan=4, npix=64)
    with pytest.raises(ValueError):  # misaligned flags (the flag word is read as 32 bits)
        raw = torch.zeros(flags4.numel() + 1, dtype=torch.uint8, device=gpu_device)
        mis = raw[1:].view(flags4.shape)
        device_ms2dirty_stokes_i(uvw, f, vis4, mis, wgt4, 64, 64, px, px, support=8)
    with pytest.raises(ValueError):
        device_ms2dirty_stokes_i(uvw, f, vis4, flags4, wgt4.double(), 64, 64, px, px, support=8)
    with pytest.raises(ValueError):
        device_ms2dirty_stokes_i(uvw, f, vis4[:, :2].contiguous(), flags4, wgt4, 64, 64, px, px, support=8)


def test_device_invert_fused_default(gpu_device):
    uvw, f, vis4, flags4, wgt4, px, _ = _raw_case(nrow=1000, nchan=8, npix=64)
    fused = device_invert(vis4, flags4, wgt4, uvw, f, 64, 20.0)
    two = device_invert(vis4, flags4, wgt4, uvw, f, 64, 20.0, fused=False)
    assert torch.equal(fused, two)
