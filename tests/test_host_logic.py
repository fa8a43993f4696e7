"""
CPU-only tests of the product's host side: the reader protocol and its
partitioning, the tile data format (split / concatenate / rechunk / npz), the
parameter choice of libcip_hip.so (host-only entry point) against the oracle,
and the C ABI's exported symbols (no compute calls without a GPU).
"""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import _lib, synthetic as syn
from ska_sdp_cip_amd.invert import integrate_weighted_images, set_env
from ska_sdp_cip_amd.measurement_set import (InMemoryMeasurementSet, MeasurementSetReader,
                                             UnsupportedMeasurementSetLayout, balanced_chunk_bounds,
                                             balanced_chunk_sizes)
from ska_sdp_cip_amd.uvw_tiling import Tile, concatenate_tiles, rechunk_tiles_on_disk, split_tile

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"


def _ms(nrow=74214, nchan=4):
    z = np.zeros
    return InMemoryMeasurementSet(z((nrow, 3)), z((nrow, nchan, 4), np.complex64), z((nrow, nchan, 4), bool),
                                  np.ones((nrow, nchan, 4), np.float32),
                                  np.array([959969726.5625, 960805664.0625, 961641601.5625, 962477539.0625]))


def test_partition_matches_reference_golden():
    g = np.load(GOLD / "partition.npz")
    ms = _ms()
    for key in ("1x1", "2x3", "5x1", "7x4", "3x2"):
        rc, fc = map(int, key.split("x"))
        got = [(c.row_start, c.row_end, c.channel_start, c.channel_end) for c in ms.partition(rc, fc)]
        assert got == [tuple(x) for x in g[key].tolist()]
    ms.set_row_bounds(1000, 5001)
    ms.set_channel_bounds(1, 4)
    got = [(c.row_start, c.row_end, c.channel_start, c.channel_end) for c in ms.partition(3, 2)]
    assert got == [tuple(x) for x in g["sub_3x2"].tolist()]


def test_partition_raises_on_excessive_chunks():
    # reference tests/test_measurement_set_partition_indices.py:87-97
    ms = _ms()
    with pytest.raises(ValueError):
        ms.partition(1_000_000, 1)
    with pytest.raises(ValueError):
        ms.partition(1, 1_000_000)


def test_bounds_clip_and_chunked_reads_equal_full_read():
    ms = syn.make_measurement_set(300, 6, n_ant=8, array_radius_m=500.0, seed=2)
    ms.set_row_bounds(-5, 10_000)
    ms.set_channel_bounds(-1, 99)
    assert (ms.row_start, ms.row_end, ms.channel_start, ms.channel_end) == (0, 300, 0, 6)
    # reference tests/test_measurement_set_chunked_read.py: chunked == slices of full
    for method in ("visibilities", "flags", "weights", "uvw", "channel_frequencies"):
        full = getattr(ms, method)()
        for rc, fc in [(1, 4), (2, 3), (7, 1)]:
            for chunk in ms.partition(rc, fc):
                part = getattr(chunk, method)()
                if method == "uvw":
                    ref = full[chunk.row_start:chunk.row_end]
                elif method == "channel_frequencies":
                    ref = full[chunk.channel_start:chunk.channel_end]
                else:
                    ref = full[chunk.row_start:chunk.row_end, chunk.channel_start:chunk.channel_end]
                assert np.array_equal(part, ref)


def test_weight_column_fallback_repeats_over_channels():
    ms = syn.make_measurement_set(50, 3, n_ant=6, array_radius_m=300.0, weight_spectrum=False)
    w = ms.weights()
    assert w.shape == (50, 3, 4) and w.dtype == np.float32
    assert np.array_equal(w[:, 0], w[:, 2])


def test_reader_errors():
    with pytest.raises(FileNotFoundError):
        MeasurementSetReader("/nonexistent/path.ms")
    with pytest.raises(UnsupportedMeasurementSetLayout):
        InMemoryMeasurementSet(np.zeros((2, 3)), np.zeros((2, 1, 2), np.complex64), np.zeros((2, 1, 4), bool),
                               np.ones((2, 1, 4), np.float32), np.ones(1))
    with pytest.raises(ValueError):
        list(balanced_chunk_sizes(0, 1))
    with pytest.raises(ValueError):
        list(balanced_chunk_sizes(3, 4))


def test_balanced_bounds_match_golden():
    g = np.load(GOLD / "partition.npz")
    for key in g.files:
        if key.startswith("bounds_"):
            _, s, e, k = key.split("_")
            assert list(balanced_chunk_bounds(int(s), int(e), int(k))) == [tuple(x) for x in g[key].tolist()]


def _golden_tile():
    g = np.load(GOLD / "tile_split.npz")
    return g, Tile((1, -2, 0), g["uvw"], g["visibilities"], g["chan_start"], g["chan_stop"])


@pytest.mark.parametrize("mv", [1, 25, 64, 100, 1000, 10_000])
def test_split_tile_matches_reference(mv):
    g, tile = _golden_tile()
    chunks = split_tile(tile, mv)
    assert [c.num_rows for c in chunks] == g[f"split_{mv}__nrows"].tolist()
    assert [c.num_visibilities for c in chunks] == g[f"split_{mv}__nvis"].tolist()
    cat = concatenate_tiles(chunks)
    assert np.array_equal(cat.visibilities, tile.visibilities) and np.array_equal(cat.uvw, tile.uvw)


def test_concatenate_errors():
    _, tile = _golden_tile()
    with pytest.raises(ValueError):
        concatenate_tiles([])
    other = Tile((0, 0, 0), tile.uvw, tile.visibilities, tile.channel_start_indices, tile.channel_stop_indices)
    with pytest.raises(ValueError):
        concatenate_tiles([tile, other])


def test_npz_roundtrip_and_rechunk(tmp_path):
    _, tile = _golden_tile()
    parts = split_tile(tile, 100)
    paths = []
    for i, p in enumerate(parts):
        path = tmp_path / f"in_{i:02d}.npz"
        p.save_npz(path)
        paths.append(path)
    back = Tile.load_npz(paths[0])
    assert back.coords == (1, -2, 0) and np.array_equal(back.visibilities, parts[0].visibilities)
    out = rechunk_tiles_on_disk(paths, tmp_path, "tile_x", max_vis_per_chunk=250)
    assert [p.name for p in out] == [f"tile_x_chunk{i:03d}.npz" for i in range(len(out))]
    tiles = [Tile.load_npz(p) for p in out]
    assert all(t.num_visibilities <= 250 for t in tiles)
    assert np.array_equal(np.concatenate([t.visibilities for t in tiles]), tile.visibilities)


def test_tile_weights_extension_roundtrip(tmp_path):
    _, tile = _golden_tile()
    tile.weights = np.arange(tile.num_visibilities, dtype=np.float32)
    tile.save_npz(tmp_path / "t.npz")
    back = Tile.load_npz(tmp_path / "t.npz")
    assert np.array_equal(back.weights, tile.weights)
    assert all(np.array_equal(c.weights, tile.weights[i:i + c.num_visibilities])
               for c, i in zip(split_tile(tile, 64), np.cumsum([0] + [c.num_visibilities
                                                                      for c in split_tile(tile, 64)])))


def test_from_jagged_slice_gather():
    rng = np.random.default_rng(0)
    vis = (rng.standard_normal((10, 8)) + 1j * rng.standard_normal((10, 8))).astype(np.complex64)
    uvw = rng.standard_normal((10, 3))
    slices = [(1, 2, 5), (4, 0, 1), (9, 3, 8)]
    t = Tile._from_jagged_visibilities_slice(vis, uvw, (0, 1, 2), slices)  # pylint: disable=protected-access
    assert np.array_equal(t.visibilities, np.concatenate([vis[1, 2:5], vis[4, 0:1], vis[9, 3:8]]))
    assert np.array_equal(t.uvw, uvw[[1, 4, 9]])


def test_params_match_oracle():
    for npix, px, eps, sup, ws, wr in [(4096, 1e-5, 1e-4, 8, False, (0, 0)), (128, 8e-5, 1e-4, None, True, (-900.0, 1400.0)),
                                       (1000, 3e-5, 1e-7, None, True, (-50.0, 20000.0)), (250, 1e-4, 1e-3, 4, False, (0, 0))]:
        p = _lib.choose_params(npix, npix, px, px, eps, sup or 0, ws, *wr)
        o = oracle.choose_params(npix, npix, px, px, eps, sup, ws, *wr)
        assert (p.nu, p.nv, p.support, p.nplanes) == (o["nu"], o["nv"], o["support"], o["nplanes"])
        assert p.w0 == pytest.approx(o["w0"], rel=1e-15, abs=1e-12) and p.dw == pytest.approx(o["dw"], rel=1e-15)
    with pytest.raises(ValueError):
        _lib.choose_params(63, 64, 1e-5, 1e-5, 1e-4)
    with pytest.raises(ValueError):
        _lib.choose_params(64, 64, 1e-5, 1e-5, 1e-4, support=18)
    with pytest.raises(ValueError):
        _lib.choose_params(64, 64, 0.1, 0.1, 1e-4, do_wstacking=True)  # beyond the horizon


def test_plane_group_and_wplane_split_on_its_lattice(monkeypatch):
    # cip_plane_group is the scatter's w-plane group (cip_api.hip wstack_group):
    # 1 in 2-D and above W = 16, 7 packed at W = 6 (6 at W = 8), 3 / 2 in the fp64 class;
    # split_planes with that group cuts only on group boundaries
    from ska_sdp_cip_amd import wplanes

    monkeypatch.delenv("CIP_WSTACK_GROUP", raising=False)
    p2d = _lib.choose_params(4096, 4096, 1e-5, 1e-5, 1e-4, 8, False, 0, 0)
    assert _lib.plane_group(p2d) == 1 and _lib.plane_group(p2d, packed=True) == 1
    pw = _lib.choose_params(4096, 4096, 3e-6, 3e-6, 1e-4, 0, True, -60000.0, 60000.0)
    assert pw.support == 6 and pw.nplanes > 10
    assert _lib.plane_group(pw, packed=True) == 7 and _lib.plane_group(pw) == 3
    pw8 = _lib.choose_params(4096, 4096, 3e-6, 3e-6, 1e-4, 8, True, -60000.0, 60000.0)
    assert _lib.plane_group(pw8, packed=True) == 6
    pw12 = _lib.choose_params(4096, 4096, 3e-6, 3e-6, 1e-4, 12, True, -60000.0, 60000.0)
    assert _lib.plane_group(pw12) == 2
    g = _lib.plane_group(pw, packed=True)
    split = wplanes.split_planes(np.ones(pw.nplanes), 3, group=g)
    assert split[0][0] == 0 and split[-1][1] == pw.nplanes
    assert all(a % g == 0 or a == pw.nplanes for a, _ in split[1:])


def test_library_exports_every_declared_symbol():
    header = (ROOT / "include" / "cip.h").read_text()
    declared = set(re.findall(r"^(?:int|const char\*)\s+(cip_\w+)\(", header, flags=re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    so = ctypes.CDLL(str(_lib.LIB_PATH))
    for name in declared:
        assert hasattr(so, name), name
    assert b"gfx950" in _lib.lib().cip_build_info()


def test_integrate_and_set_env(monkeypatch):
    imgs = [(np.ones((2, 2)), 2.0), (3 * np.ones((2, 2)), 6.0)]
    assert np.allclose(integrate_weighted_images(imgs), 0.5)
    monkeypatch.delenv("CIP_TEST_VAR", raising=False)
    with set_env("CIP_TEST_VAR", 3):
        import os

        assert os.environ["CIP_TEST_VAR"] == "3"
    assert "CIP_TEST_VAR" not in os.environ


def test_synthetic_ms_shapes():
    ms = syn.make_measurement_set(500, 4, n_ant=8, array_radius_m=500.0)
    assert ms.visibilities().dtype == np.complex64 and ms.visibilities().shape == (500, 4, 4)
    assert ms.flags().dtype == bool and ms.weights().dtype == np.float32
    assert ms.uvw().shape == (500, 3) and ms.uvw().dtype == np.float64


def test_w_ranges_and_facet_centres():
    # host helpers of the accumulating gridder and the continuum products
    from ska_sdp_cip_amd.accumulate import merge_w_ranges, w_range_rows, w_range_slices
    from ska_sdp_cip_amd.continuum import facet_centres

    rng = np.random.default_rng(0)
    uvw = rng.normal(0.0, 500.0, (200, 3))
    f = np.linspace(0.9e9, 1.7e9, 16)
    lo, hi = w_range_rows(uvw, f)
    w = uvw[:, 2:3] * (f[None, :] / 299792458.0)
    assert np.isclose(lo, w.min()) and np.isclose(hi, w.max())
    # slices of every row: the same range; empty slices are ignored
    c0 = np.zeros(200, np.int32)
    c1 = np.full(200, 16, np.int32)
    c1[::3] = 0
    lo2, hi2 = w_range_slices(uvw, c0, c1, f)
    keep = c1 > c0
    assert (lo2, hi2) == w_range_rows(uvw[keep], f)
    assert w_range_slices(uvw, c0, c0, f) == (np.inf, -np.inf)
    assert merge_w_ranges([(1.0, 2.0), (-3.0, 0.5), (np.inf, -np.inf)]) == (-3.0, 2.0)
    cen = facet_centres(3, 2, 100, 1e-5)
    assert len(cen) == 6 and cen[0] == (-1e-3, -5e-4) and cen[-1] == (1e-3, 5e-4)
    assert np.allclose(np.mean(cen, axis=0), 0.0)


def test_oracle_stokes_and_facet_rotation():
    # the oracle's restatements used by the GPU tests: Stokes I equals the
    # golden-pinned stokes_i; the facet rotation takes the pole to the centre
    g = np.load(GOLD / "stokes_i.npz")
    v, eff = oracle.stokes(g["vis4"], g["flags4"], g["weights4"], "I")
    assert np.array_equal(v, g["vis_i"]) and np.array_equal(eff, g["eff_w"])
    for l0, m0 in [(0.0, 0.0), (0.05, -0.02), (-0.3, 0.4)]:
        q = oracle.facet_rotation(l0, m0)
        assert np.allclose(q @ q.T, np.eye(3), atol=1e-14)
        assert np.allclose(q @ [0.0, 0.0, 1.0], [l0, m0, np.sqrt(1 - l0 * l0 - m0 * m0)], atol=1e-14)


def test_allreduce_rejects_duplicate_devices():
    """cip_allreduce_grid validates its device list before any HIP/RCCL call
    (a repeated device would otherwise reach ncclCommInitAll)."""
    import ctypes

    from ska_sdp_cip_amd import _lib

    L = _lib.lib()
    bufs = (ctypes.c_double * 4)()
    grids = (ctypes.c_void_p * 2)(ctypes.addressof(bufs), ctypes.addressof(bufs))
    devs = (ctypes.c_int * 2)(0, 0)
    assert L.cip_allreduce_grid(grids, devs, 2, 4, -1, None) == _lib.CIP_EINVAL
    assert b"distinct" in L.cip_last_error()
    devs = (ctypes.c_int * 2)(-1, 1)
    assert L.cip_allreduce_grid(grids, devs, 2, 4, -1, None) == _lib.CIP_EINVAL


def test_python_constants_match_c_header():
    # every status / dtype / flag code the ctypes layer passes equals the
    # #define of include/cip.h (the C ABI is the boundary)
    header = (Path(__file__).resolve().parents[1] / "include" / "cip.h").read_text()
    defines = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (CIP_[A-Z0-9_]+) \(?(-?\d+)\)?", header)}
    checked = 0
    for name, value in vars(_lib).items():
        if name.startswith("CIP_") and isinstance(value, int):
            assert defines.get(name) == value, name
            checked += 1
    assert checked >= 16
    assert {v: k for k, v in _lib.STOKES_CODES.items()} == {defines[f"CIP_STOKES_{s}"]: s for s in "IQUV"}


def test_local_gpu_client_runs_devices_concurrently():
    # one worker thread per device: two GPU tasks that wait for each other
    # complete only if they run at the same time (on CPU the device binding is
    # skipped); futures passed as arguments are resolved inside the task
    import threading

    from ska_sdp_cip_amd.dispatch import LocalGPUClient, as_completed

    with LocalGPUClient(devices=[0, 1]) as client:
        assert len(client.scheduler_info()["workers"]) == 2
        barrier = threading.Barrier(2, timeout=30)
        names = []

        def task(x):
            barrier.wait()
            names.append(threading.current_thread().name)
            return x

        futs = [client.submit(task, k, resources={"gpu": 1}) for k in (1, 2)]
        total = client.submit(lambda xs: sum(xs), futs)
        assert sorted(f.result() for f in as_completed(futs)) == [1, 2]
        assert total.result() == 3
        assert sorted(n.split("_")[0] for n in names) == ["cip-gpu0", "cip-gpu1"]
        bad = client.submit(lambda: 1 / 0, resources={"gpu": 1})
        with pytest.raises(ZeroDivisionError):
            bad.result()


def test_local_gpu_client_synchronous_mode():
    from ska_sdp_cip_amd.dispatch import LocalGPUClient, as_completed

    client = LocalGPUClient(devices=[0], concurrent=False)
    a = client.submit(lambda: 2, resources={"gpu": 1})
    b = client.submit(lambda x, y: x * y, a, 5)
    assert a.done() and b.result() == 10
    assert [f.result() for f in as_completed([a, b])] == [2, 10]


def test_bench_refuses_a_world_size_other_than_gpus():
    # bench.py --gpus N under a launcher whose WORLD_SIZE differs: rc != 0
    # before anything touches a GPU (the driver must never get an n_gpus that
    # is not the run's)
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "1"], env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 2, out.stderr[-2000:]
    assert "WORLD_SIZE=2" in out.stderr
