"""
GPU parity of the invert hot path: libcip_hip.so (through its C ABI, via
`ska_sdp_cip_amd.gridder`) against the CPU oracle (oracle/oracle.py, fp64
restatement) and against the fp64 direct DFT (the definition of ms2dirty).

Tolerance (north star, BASELINE.json): dirty image normalised by the sum of
weights, max |GPU - oracle| < 1e-6. The two implement the identical algorithm,
so the tests also check the much tighter 1e-10 they actually reach.
"""

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import _lib, gridder, synthetic as syn
from ska_sdp_cip_amd.invert import StokesIGridderInput

pytestmark = pytest.mark.gpu

GATE = 1e-6
TIGHT = 1e-10


def _case(n_rows, nchan, *, n_ant=16, radius=1000.0, fov=0.01, seed=3, wspec=True):
    ms = syn.make_measurement_set(n_rows, nchan, n_ant=n_ant, array_radius_m=radius, fov_l=fov,
                                  seed=seed, weight_spectrum=wspec)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    return gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)


def _norm_err(a, b, sumw):
    return float(np.abs(a - b).max() / sumw)


@pytest.mark.parametrize("support", [4, 8, 16])
def test_2d_parity_vs_oracle_and_dft(gpu_device, support):
    uvw, f, vis, w = _case(10_000, 1)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix, support=support)
    gpu, prm = gridder.ms2dirty(uvw, f, vis.astype(np.complex128), w.astype(np.float64), npix, npix, px, px,
                                support=support, do_wstacking=False, return_params=True)
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=support, do_wstacking=False)
    sumw = float(w.astype(np.float64).sum())
    err = _norm_err(gpu, ref, sumw)
    assert prm.support == support and prm.nu == 256
    assert err < GATE
    assert err < TIGHT, err
    if support == 16:  # W=16 reproduces the DFT to ~1e-14
        dft = oracle.dft_dirty(uvw, f, vis, w, npix, npix, px, px, apply_w=False)
        assert _norm_err(gpu, dft, sumw) < 1e-12


@pytest.mark.parametrize("vis_dtype,wgt_kind", [(np.complex64, "f32"), (np.complex128, "f64"),
                                                (np.complex64, "none")])
def test_multichannel_dtypes(gpu_device, vis_dtype, wgt_kind):
    uvw, f, vis, w = _case(3_000, 64, n_ant=32, radius=3000.0)
    vis = vis.astype(vis_dtype)
    wg = {"f32": w, "f64": w.astype(np.float64), "none": None}[wgt_kind]
    npix = 256
    px = syn.pixel_size_for_grid(uvw, f, npix)
    gpu = gridder.ms2dirty(uvw, f, vis, wg, npix, npix, px, px, support=8, do_wstacking=False)
    assert gpu.dtype == (np.float32 if vis_dtype == np.complex64 else np.float64)
    # fp64 result for the parity check
    import torch

    gpu64, _ = gridder.device_ms2dirty(
        torch.from_numpy(uvw).cuda(), torch.from_numpy(f).cuda(), torch.from_numpy(vis).cuda(),
        None if wg is None else torch.from_numpy(wg).cuda(), npix, npix, px, px, support=8)
    ref = oracle.ms2dirty(uvw, f, vis, wg, npix, npix, px, px, support=8)
    sumw = float(np.sum(wg, dtype=np.float64)) if wg is not None else float(vis.size)
    assert _norm_err(gpu64.cpu().numpy(), ref, sumw) < TIGHT


def test_wstacking_parity_vs_oracle_and_dft(gpu_device):
    uvw, f, vis, w = _case(4_000, 4, n_ant=24, radius=2000.0, fov=0.05)
    npix = 192
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.3)  # wide field: several w planes
    gpu, prm = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=10, do_wstacking=True,
                                return_params=True)
    import torch

    g64, _ = gridder.device_ms2dirty(torch.from_numpy(uvw).cuda(), torch.from_numpy(f).cuda(),
                                     torch.from_numpy(vis).cuda(), torch.from_numpy(w).cuda(), npix, npix,
                                     px, px, support=10, do_wstacking=True)
    ref, oprm = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=10, do_wstacking=True,
                                return_params=True)
    assert prm.nplanes == oprm["nplanes"] and prm.nplanes > 10
    sumw = float(w.astype(np.float64).sum())
    assert _norm_err(g64.cpu().numpy(), ref, sumw) < TIGHT
    dft = oracle.dft_dirty(uvw, f, vis, w, npix, npix, px, px, apply_w=True)
    assert _norm_err(g64.cpu().numpy(), dft, sumw) < 1e-7


def test_grid_plane_matches_oracle_grid(gpu_device):
    import torch

    uvw, f, vis, w = _case(2_000, 16, n_ant=24, radius=2000.0)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    prm = _lib.choose_params(npix, npix, px, px, 1e-4, 8, False)
    grid = torch.empty((prm.nu, prm.nv), dtype=torch.complex128, device="cuda")
    # keep the device tensors alive for the whole call
    tu, tf, tv, tw = (torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (uvw, f, vis, w))
    _lib.check(_lib.lib().cip_grid_plane(
        tu.data_ptr(), uvw.shape[0], tf.data_ptr(), f.size, tv.data_ptr(), _lib.CIP_C64,
        tw.data_ptr(), _lib.CIP_F32, prm, px, px, 0, 0, None, grid.data_ptr()))
    torch.cuda.synchronize()
    oprm = oracle.choose_params(npix, npix, px, px, support=8)
    ref = oracle.grid_plane(uvw, f, vis, w, oprm, px, px, 0)
    scale = np.abs(ref).max()
    assert np.abs(grid.cpu().numpy() - ref).max() / scale < 1e-13
    # single-precision class: each contribution quantised to <= 2^-20 of
    # max|w V| (chunks here hold < 2^11 visibilities)
    _lib.check(_lib.lib().cip_grid_plane(
        tu.data_ptr(), uvw.shape[0], tf.data_ptr(), f.size, tv.data_ptr(), _lib.CIP_C64,
        tw.data_ptr(), _lib.CIP_F32, prm, px, px, 0, _lib.CIP_ACC_SINGLE, None, grid.data_ptr()))
    torch.cuda.synchronize()
    maxwv = float(np.abs(w.astype(np.float64) * vis).max())
    per_cell = np.abs(grid.cpu().numpy() - ref).max() / maxwv
    assert 0 < per_cell < 2e-3  # random walk of <= 0.5-unit roundings over a cell's contributions


@pytest.mark.parametrize("wstack", [False, True])
def test_single_precision_class_vs_oracle(gpu_device, wstack):
    # CIP_ACC_SINGLE (ducc0's float class; the reference calls ducc0 with
    # epsilon=1e-4): normalised error well below epsilon, and the default path
    # on the same complex64 input stays at the fp64 class
    import torch

    uvw, f, vis, w = _case(4_000, 16, n_ant=24, radius=2000.0, fov=0.05)
    npix = 192
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.3 if wstack else 0.5)
    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis, w)]
    single, _ = gridder.device_ms2dirty(*args, npix, npix, px, px, support=8, do_wstacking=wstack,
                                        single_precision_accumulation=True)
    double, _ = gridder.device_ms2dirty(*args, npix, npix, px, px, support=8, do_wstacking=wstack)
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=wstack)
    sumw = float(w.astype(np.float64).sum())
    assert _norm_err(double.cpu().numpy(), ref, sumw) < TIGHT
    assert _norm_err(single.cpu().numpy(), ref, sumw) < 1e-5
    np_single = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, do_wstacking=wstack,
                                 double_precision_accumulation=False, support=8)
    assert np_single.dtype == np.float32
    assert np.abs(np_single - single.cpu().numpy()).max() / sumw < 1e-6
    with pytest.raises(ValueError):  # complex128 has no single class
        gridder.device_ms2dirty(args[0], args[1], args[2].to(torch.complex128), args[3], npix, npix, px, px,
                                support=8, single_precision_accumulation=True)


def test_point_source_at_centre_and_off_centre(gpu_device):
    n_rows, nchan, npix = 5_000, 8, 128
    uvw = syn.uvw_tracks(n_rows, 16, array_radius_m=1500.0)
    f = syn.channel_frequencies(nchan)
    px = syn.pixel_size_for_grid(uvw, f, npix)
    for (i, j) in [(npix // 2, npix // 2), (npix // 2 + 17, npix // 2 - 9)]:
        l, m = (i - npix // 2) * px, (j - npix // 2) * px
        src = [syn.PointSource(l, m, 1.0)]
        vis = syn.predict_visibilities(uvw, f, src)
        w = np.ones(vis.shape, dtype=np.float64)
        img = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=12, do_wstacking=True)
        img = img / w.sum()
        assert np.unravel_index(np.argmax(img), img.shape) == (i, j)
        # the definition divides by n: a unit source peaks at 1 / n(l, m)
        n = np.sqrt(1.0 - l * l - m * m)
        assert abs(img[i, j] - 1.0 / n) < 1e-8


@pytest.mark.parametrize("wstack", [False, True])
def test_uv_beyond_grid_wraps_like_the_dft(gpu_device, wstack):
    # the image is sampled at l = k * pixsize, so u is periodic with period
    # 1 / pixsize (the grid extent): baselines longer than the grid wrap exactly
    # (the reference's own test set-up, 2048 px at 5", wraps MeerKAT baselines)
    uvw, f, vis, w = _case(3_000, 2, fov=0.02, seed=1)
    npix = 64
    px = syn.pixel_size_for_grid(uvw, f, npix) * 3.0
    gpu = gridder.ms2dirty(uvw, f, vis.astype(np.complex128), w.astype(np.float64), npix, npix, px, px,
                           support=12, do_wstacking=wstack)
    dft = oracle.dft_dirty(uvw, f, vis, w, npix, npix, px, px, apply_w=wstack)
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=12, do_wstacking=wstack)
    sumw = float(w.astype(np.float64).sum())
    assert _norm_err(gpu, ref, sumw) < TIGHT
    assert _norm_err(gpu, dft, sumw) < 1e-9


def test_non_finite_uvw_raises(gpu_device):
    uvw, f, vis, w = _case(500, 1)
    uvw = uvw.copy()
    uvw[17, 0] = np.nan
    px = syn.pixel_size_for_grid(uvw[:10], f, 64)
    with pytest.raises(ValueError):
        gridder.ms2dirty(uvw, f, vis, w, 64, 64, px, px, support=8, do_wstacking=False)


def test_non_finite_visibility(gpu_device):
    uvw, f, vis, w = _case(500, 4)
    vis, w = vis.copy(), w.copy()
    px = syn.pixel_size_for_grid(uvw, f, 64)
    vis[3, 1] = np.nan
    w[3, 1] = 0.0  # a zero-weight sample is skipped whatever it holds
    img = gridder.ms2dirty(uvw, f, vis, w, 64, 64, px, px, support=8)
    assert np.isfinite(img).all()
    w[3, 1] = 1.0
    with pytest.raises(ValueError):
        gridder.ms2dirty(uvw, f, vis, w, 64, 64, px, px, support=8)


def test_bad_arguments_raise(gpu_device):
    uvw, f, vis, w = _case(100, 1)
    px = syn.pixel_size_for_grid(uvw, f, 64)
    with pytest.raises(ValueError):
        gridder.ms2dirty(uvw, f, vis, w, 63, 64, px, px)  # odd npix
    with pytest.raises(ValueError):
        gridder.ms2dirty(uvw, f, vis, w, 64, 64, px, px, support=7)
    with pytest.raises(ValueError):
        gridder.ms2dirty(uvw, f, vis[:, :0], w[:, :0], 64, 64, px, px)
    # non-positive / non-finite frequencies: caught on the host (w-stacking
    # needs the range there) or by the device check (2-D), the same error
    for bad in (0.0, -1.0e9, np.nan):
        fb = f.copy()
        fb[0] = bad
        for ws in (False, True):
            with pytest.raises(ValueError, match="frequencies"):
                gridder.ms2dirty(uvw, fb, vis, w, 64, 64, px, px, do_wstacking=ws)
    # and a later call with good input is unaffected
    assert np.isfinite(gridder.ms2dirty(uvw, f, vis, w, 64, 64, px, px)).all()


def test_zero_rows_gives_zero_image(gpu_device):
    uvw = np.zeros((0, 3))
    f = syn.channel_frequencies(4)
    vis = np.zeros((0, 4), np.complex64)
    w = np.zeros((0, 4), np.float32)
    img = gridder.ms2dirty(uvw, f, vis, w, 64, 64, 1e-5, 1e-5, support=8, do_wstacking=True)
    assert img.shape == (64, 64) and not np.any(img)


def test_repeatable(gpu_device):
    uvw, f, vis, w = _case(5_000, 16, n_ant=24, radius=2000.0)
    npix = 128
    px = syn.pixel_size_for_grid(uvw, f, npix)
    a = gridder.ms2dirty(uvw, f, vis.astype(np.complex128), w, npix, npix, px, px, support=8)
    b = gridder.ms2dirty(uvw, f, vis.astype(np.complex128), w, npix, npix, px, px, support=8)
    # per-chunk sums are exact (fixed point); only the fp64 order of the
    # global flush adds may differ between runs
    assert np.abs(a - b).max() <= 1e-13 * np.abs(a).max()


def test_dense_single_channel_tiles(gpu_device):
    # one channel, a small grid: every row slice holds one visibility and the
    # tiles hold thousands of them, so bank-ordering windows meet 1024 slices
    uvw, f, vis, w = _case(30_000, 1, n_ant=40, radius=1500.0)
    npix = 64
    px = syn.pixel_size_for_grid(uvw, f, npix) * 2.5
    gpu = gridder.ms2dirty(uvw, f, vis.astype(np.complex128), w.astype(np.float64), npix, npix, px, px,
                           support=8, do_wstacking=False)
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=False)
    sumw = float(w.astype(np.float64).sum())
    assert _norm_err(gpu, ref, sumw) < TIGHT


def test_grid_left_clean_between_calls(gpu_device):
    # the pruned FFT's pass A zeroes the grid tiles the scatter wrote (no
    # whole-grid memset per call): a call after one with different uv coverage,
    # w-stacking planes or an error must not see any residue
    # complex128 visibilities: fp64 output (complex64 returns float32, as ducc0 does)
    a = _case(2_000, 8, n_ant=16, radius=1500.0, seed=21)
    b = _case(1_500, 4, n_ant=10, radius=400.0, seed=22)
    a = (a[0], a[1], a[2].astype(np.complex128), a[3])
    b = (b[0], b[1], b[2].astype(np.complex128), b[3])
    npix = 1024  # grid 2048: power of two -> pruned FFT path
    res = {}
    for name, (uvw, f, vis, w) in (("a", a), ("b", b)):
        px = syn.pixel_size_for_grid(uvw, f, npix, support=8)
        res[name] = (px, oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=False))
    for name, ws in (("a", False), ("b", False), ("a", True), ("a", False), ("b", False)):
        uvw, f, vis, w = a if name == "a" else b
        px, ref = res[name]
        gpu = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=ws)
        if not ws:
            assert _norm_err(gpu, ref, float(w.astype(np.float64).sum())) < TIGHT, name
        if name == "b":  # an error after planning leaves the grid dirty: the next call must still be exact
            bad = vis.copy()
            bad[3, 1] = np.nan
            with pytest.raises(ValueError):
                gridder.ms2dirty(uvw, f, bad, w, npix, npix, px, px, support=8, do_wstacking=False)
