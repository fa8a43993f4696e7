"""
Generate the golden fixtures in tests/golden/ by running the REFERENCE's own
code (read-only at /root/reference) on seeded inputs. Run once in the
development container (the reference does not exist on the GPU box):

    python tests/golden/make_golden.py

The reference package cannot be imported normally (no installed metadata,
dask / casacore / ducc0 absent); its modules are loaded
standalone with `importlib` and minimal stubs for the missing third-party
modules:
  * `ska_sdp_cip` / `ska_sdp_cip.uvw_tiling`: empty package shells so the
    modules' absolute imports resolve to the reference files themselves;
  * `casacore.tables.table`: a fake table serving in-memory columns
    (getcol / getcolslice / nrows) so MeasurementSetReader.partition() and the
    readers run unmodified;
  * `dask.distributed`: a synchronous fake Client (submit -> immediate result);
  * `ducc0.wgridder.ms2dirty`: records its arguments and returns a
    deterministic image (only the wrapper arithmetic around it is pinned; the
    gridding values of ducc0 are not available here - parity unpinned).
Nothing from the reference is copied; the fixtures hold inputs and outputs only.
"""

from __future__ import annotations

import importlib.util
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

REF = Path("/root/reference/src/ska_sdp_cip")
OUT = Path(__file__).resolve().parent
SEED = 20241008


# ------------------------------------------------------------- stubs ----
class _FakeTable:
    """casacore.tables.table over a registry of in-memory measurement sets."""

    registry: dict = {}

    def __init__(self, spec, readonly=True, ack=False):  # noqa: ARG002
        path, _, name = str(spec).partition("::")
        self.cols = _FakeTable.registry[str(Path(path).resolve())][name or "MAIN"]

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def nrows(self):
        return len(next(iter(self.cols.values())))

    def getcol(self, name, startrow=0, nrow=-1):
        data = self.cols[name]
        return data[startrow:] if nrow < 0 else data[startrow:startrow + nrow]

    def getcolslice(self, name, blc, trc, startrow=0, nrow=-1):
        if name not in self.cols:
            raise RuntimeError(f"no column {name}")
        data = self.getcol(name, startrow, nrow)
        blc = np.atleast_1d(blc)
        trc = np.atleast_1d(trc)
        idx = tuple(slice(b, t + 1) for b, t in zip(blc, trc))
        if name == "CHAN_FREQ":  # (nspw, nchan)
            return data[(slice(None),) + idx]
        return data[(slice(None),) + idx]


class _FakeFuture:
    def __init__(self, v):
        self.v = v

    def result(self):
        return self.v


class _FakeClient:
    def __init__(self, nworkers=2):
        self.nworkers = nworkers

    def scheduler_info(self):
        return {"workers": {f"w{i}": {} for i in range(self.nworkers)}, "type": "x", "id": "x"}

    def submit(self, fn, *args, resources=None, **kwargs):  # noqa: ARG002
        res = lambda a: a.result() if isinstance(a, _FakeFuture) else (  # noqa: E731
            [x.result() if isinstance(x, _FakeFuture) else x for x in a] if isinstance(a, list) else a)
        return _FakeFuture(fn(*[res(a) for a in args], **{k: res(v) for k, v in kwargs.items()}))


MS2DIRTY_CALLS = []


def _fake_ms2dirty(uvw, freq, ms, wgt, npix_x, npix_y, pixsize_x, pixsize_y, **kw):
    MS2DIRTY_CALLS.append(dict(uvw_dtype=str(uvw.dtype), freq_dtype=str(freq.dtype), ms_dtype=str(ms.dtype),
                               wgt_dtype=str(wgt.dtype), npix_x=npix_x, npix_y=npix_y, pixsize_x=pixsize_x,
                               pixsize_y=pixsize_y, **{k: (v if v is None or np.isscalar(v) else str(v))
                                                       for k, v in kw.items()}))
    # deterministic stand-in image: linear in (ms * wgt), so chunk sums are exact
    img = np.zeros((npix_x, npix_y), dtype=np.float32)
    img.flat[: ms.size] += (ms.real * wgt).ravel()[: img.size]
    return img


def install_stubs():
    casacore = types.ModuleType("casacore")
    tables = types.ModuleType("casacore.tables")
    tables.table = _FakeTable
    casacore.tables = tables
    dask = types.ModuleType("dask")
    dd = types.ModuleType("dask.distributed")
    dd.Client = _FakeClient
    dd.Future = _FakeFuture
    dd.as_completed = lambda futs: iter(futs)

    def get_worker():
        raise ValueError("not on a worker")

    dd.get_worker = get_worker
    dask.distributed = dd
    ducc0 = types.ModuleType("ducc0")
    wg = types.ModuleType("ducc0.wgridder")
    wg.ms2dirty = _fake_ms2dirty
    ducc0.wgridder = wg
    sys.modules.update({"casacore": casacore, "casacore.tables": tables, "dask": dask,
                        "dask.distributed": dd, "ducc0": ducc0, "ducc0.wgridder": wg})
    pkg = types.ModuleType("ska_sdp_cip")
    pkg.__path__ = [str(REF)]
    sub = types.ModuleType("ska_sdp_cip.uvw_tiling")
    sub.__path__ = [str(REF / "uvw_tiling")]
    sys.modules["ska_sdp_cip"] = pkg
    sys.modules["ska_sdp_cip.uvw_tiling"] = sub


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# ------------------------------------------------------------ inputs ----
def meerkat_uvw(nrow, n_ant=64, seed=SEED):
    """Seeded earth-rotation tracks (same recipe as ska_sdp_cip_amd.synthetic)."""
    rng = np.random.default_rng(seed)
    r = 4000.0 * np.sqrt(rng.uniform(0, 1, n_ant))
    phi = rng.uniform(0, 2 * np.pi, n_ant)
    enu = np.stack([r * np.cos(phi), r * np.sin(phi), rng.normal(0, 2.0, n_ant)], 1)
    a1, a2 = np.triu_indices(n_ant, 1)
    bl = enu[a2] - enu[a1]
    lat, dec = np.radians(-30.7), np.radians(-30.0)
    x = -np.sin(lat) * bl[:, 1] + np.cos(lat) * bl[:, 2]
    y = bl[:, 0]
    z = np.cos(lat) * bl[:, 1] + np.sin(lat) * bl[:, 2]
    nt = -(-nrow // len(bl))
    ha = (np.arange(nt) - (nt - 1) / 2) * 8.0 * 7.292115e-5
    sh, ch = np.sin(ha)[:, None], np.cos(ha)[:, None]
    u = sh * x + ch * y
    v = -np.sin(dec) * ch * x + np.sin(dec) * sh * y + np.cos(dec) * z
    w = np.cos(dec) * ch * x - np.cos(dec) * sh * y + np.sin(dec) * z
    return np.ascontiguousarray(np.stack([u, v, w], -1).reshape(-1, 3)[:nrow])


def boundary_uvw(tile_size, freq, n=200, seed=1):
    """uvw placed so f/c * u / tile + 0.5 sits on (and 1 ulp around) integers."""
    rng = np.random.default_rng(seed)
    ts = np.asarray(tile_size)
    out = []
    for _ in range(n):
        f = freq[rng.integers(len(freq))]
        k = rng.integers(-20, 20, 3) - 0.5
        uvw = k * ts * 299792458.0 / f
        for step in (-1, 0, 1):
            out.append(np.nextafter(uvw, uvw + step * np.inf) if step else uvw)
    return np.asarray(out, dtype=np.float64)


def main():
    install_stubs()
    tp = load("ska_sdp_cip.uvw_tiling.tiling_plan", REF / "uvw_tiling" / "tiling_plan.py")
    tile_mod = load("ska_sdp_cip.uvw_tiling.tile", REF / "uvw_tiling" / "tile.py")
    msmod = load("ska_sdp_cip.measurement_set", REF / "measurement_set.py")
    sys.modules["ska_sdp_cip"].MeasurementSetReader = msmod.MeasurementSetReader
    inv = load("ska_sdp_cip.invert", REF / "invert.py")
    reo = load("ska_sdp_cip.uvw_tiling.reorder", REF / "uvw_tiling" / "reorder.py")

    # 1. tiling plans ------------------------------------------------------
    lband = 856.0e6 + (214.0e6 / 256) * np.arange(256)  # tests/uvw_tiling/test_uvw_tiling_plan.py:17-21
    cases = {
        "meerkat_ts3000_256ch": (meerkat_uvw(3000), (3000.0, 3000.0, 6000.0), lband),
        "meerkat_ts1000_64ch": (meerkat_uvw(2000, seed=5), (1000.0, 1000.0, 2000.0), lband[::4]),
        "meerkat_ts700_4ch": (meerkat_uvw(4000, seed=6),
                              (500.0, 700.0, 1300.0),
                              np.array([959969726.5625, 960805664.0625, 961641601.5625, 962477539.0625])),
        "boundary_ts3000": (boundary_uvw((3000.0, 3000.0, 6000.0), lband), (3000.0, 3000.0, 6000.0), lband),
        "descending_freq": (meerkat_uvw(500, seed=9), (3000.0, 3000.0, 6000.0), lband[::-1].copy()),
    }
    arrays = {}
    for name, (uvw, ts, freq) in cases.items():
        mapping = tp.create_uvw_tile_mapping_sequential(uvw, ts, freq, row_offset=7)
        keys, irow, c0, c1, order = [], [], [], [], []
        for t_i, (k, slices) in enumerate(mapping.items()):
            for s in slices:
                keys.append(k)
                irow.append(s.irow)
                c0.append(s.chan_start)
                c1.append(s.chan_stop)
                order.append(t_i)
        arrays[f"{name}__uvw"] = uvw
        arrays[f"{name}__tile_size"] = np.asarray(ts)
        arrays[f"{name}__freq"] = freq
        arrays[f"{name}__key"] = np.asarray(keys, dtype=np.int64)
        arrays[f"{name}__irow"] = np.asarray(irow, dtype=np.int64)
        arrays[f"{name}__c0"] = np.asarray(c0, dtype=np.int64)
        arrays[f"{name}__c1"] = np.asarray(c1, dtype=np.int64)
        arrays[f"{name}__tile_order"] = np.asarray(order, dtype=np.int64)
    # parallel (Pool) version == sequential with row offsets, in chunk order
    par = tp.create_uvw_tile_mapping(cases["meerkat_ts3000_256ch"][0], (3000.0, 3000.0, 6000.0), lband,
                                     processes=3)
    arrays["parallel3__nslices"] = np.asarray([sum(len(v) for v in par.values())])
    arrays["parallel3__ntiles"] = np.asarray([len(par)])
    np.savez_compressed(OUT / "tiling_plan.npz", **arrays)

    # 2. Stokes I + effective weights ---------------------------------------
    rng = np.random.default_rng(SEED)
    nrow, nchan = 60, 5
    vis = (rng.standard_normal((nrow, nchan, 4)) + 1j * rng.standard_normal((nrow, nchan, 4))).astype(np.complex64)
    flags = rng.uniform(size=(nrow, nchan, 4)) < 0.15
    wts = rng.uniform(0.0, 2.0, (nrow, nchan, 4)).astype(np.float32)
    wts[rng.uniform(size=wts.shape) < 0.1] = 0.0  # zero weights -> 1/0
    uvw = meerkat_uvw(nrow)
    freq = lband[:nchan]
    _FakeTable.registry.clear()
    tmp = Path(tempfile.mkdtemp())
    _FakeTable.registry[str(tmp.resolve())] = {
        "MAIN": {"UVW": uvw, "DATA": vis, "FLAG": flags, "WEIGHT_SPECTRUM": wts, "WEIGHT": wts[:, 0, :]},
        "SPECTRAL_WINDOW": {"CHAN_FREQ": freq[None, :]},
        "FIELD": {"X": np.zeros(1)},
        "POLARIZATION": {"CORR_TYPE": np.array([[9, 10, 11, 12]])},
    }
    reader = msmod.MeasurementSetReader(tmp)
    gi = inv.StokesIGridderInput.from_measurement_set_reader(reader)
    np.savez_compressed(OUT / "stokes_i.npz", vis4=vis, flags4=flags, weights4=wts, uvw=uvw, freq=freq,
                        vis_i=gi.visibilities, flags_i=gi.flags, weights_i=gi.weights,
                        eff_w=gi.effective_weights())

    # 3. partition bounds ---------------------------------------------------
    tmp2 = Path(tempfile.mkdtemp())
    _FakeTable.registry[str(tmp2.resolve())] = {
        "MAIN": {"UVW": np.zeros((74214, 3)), "DATA": np.zeros((74214, 4, 4), np.complex64),
                 "FLAG": np.zeros((74214, 4, 4), bool), "WEIGHT_SPECTRUM": np.ones((74214, 4, 4), np.float32)},
        "SPECTRAL_WINDOW": {"CHAN_FREQ": np.array([[959969726.5625, 960805664.0625, 961641601.5625,
                                                    962477539.0625]])},
        "FIELD": {"X": np.zeros(1)},
        "POLARIZATION": {"CORR_TYPE": np.array([[9, 10, 11, 12]])},
    }
    big = msmod.MeasurementSetReader(tmp2)
    part = {}
    for rc, fc in [(1, 1), (2, 3), (5, 1), (7, 4), (3, 2)]:
        part[f"{rc}x{fc}"] = np.asarray([(c.row_start, c.row_end, c.channel_start, c.channel_end)
                                         for c in big.partition(rc, fc)], dtype=np.int64)
    sub = msmod.MeasurementSetReader(tmp2)
    sub.set_row_bounds(1000, 5001)
    sub.set_channel_bounds(1, 4)
    part["sub_3x2"] = np.asarray([(c.row_start, c.row_end, c.channel_start, c.channel_end)
                                  for c in sub.partition(3, 2)], dtype=np.int64)
    bal = {f"bounds_{s}_{e}_{k}": np.asarray(list(msmod.balanced_chunk_bounds(s, e, k)), dtype=np.int64)
           for s, e, k in [(0, 10, 3), (5, 6, 1), (0, 74214, 5), (17, 1017, 7), (0, 4, 4)]}
    np.savez_compressed(OUT / "partition.npz", **part, **bal)

    # 4. split / concatenate tiles -------------------------------------------
    t_arrays = {}
    sizes = rng.integers(1, 40, size=50)
    ns = len(sizes)
    starts = rng.integers(0, 10, ns)
    tile = tile_mod.Tile(coords=(1, -2, 0), uvw=rng.standard_normal((ns, 3)),
                         visibilities=(rng.standard_normal(sizes.sum()) + 1j).astype(np.complex64),
                         channel_start_indices=starts, channel_stop_indices=starts + sizes)
    t_arrays.update(uvw=tile.uvw, visibilities=tile.visibilities, chan_start=tile.channel_start_indices,
                    chan_stop=tile.channel_stop_indices)
    for mv in (1, 25, 64, 100, 1000, 10_000):
        chunks = tile_mod.split_tile(tile, mv)
        t_arrays[f"split_{mv}__nrows"] = np.asarray([c.num_rows for c in chunks])
        t_arrays[f"split_{mv}__nvis"] = np.asarray([c.num_visibilities for c in chunks])
    cat = tile_mod.concatenate_tiles(tile_mod.split_tile(tile, 64))
    t_arrays["concat_equal"] = np.asarray([np.array_equal(cat.visibilities, tile.visibilities)])
    np.savez_compressed(OUT / "tile_split.npz", **t_arrays)

    # 5. reorder multiset + 6. invert normalisation --------------------------
    nrow, nchan = 400, 16
    vis = (rng.standard_normal((nrow, nchan, 4)) + 1j * rng.standard_normal((nrow, nchan, 4))).astype(np.complex64)
    uvw = meerkat_uvw(nrow, seed=11)
    freq = lband[::16].copy()
    wts = rng.uniform(0.5, 1.5, (nrow, nchan, 4)).astype(np.float32)
    flg = rng.uniform(size=(nrow, nchan, 4)) < 0.05
    tmp3 = Path(tempfile.mkdtemp())
    _FakeTable.registry[str(tmp3.resolve())] = {
        "MAIN": {"UVW": uvw, "DATA": vis, "FLAG": flg, "WEIGHT_SPECTRUM": wts},
        "SPECTRAL_WINDOW": {"CHAN_FREQ": freq[None, :]},
        "FIELD": {"X": np.zeros(1)},
        "POLARIZATION": {"CORR_TYPE": np.array([[9, 10, 11, 12]])},
    }
    r3 = msmod.MeasurementSetReader(tmp3)
    outdir = Path(tempfile.mkdtemp())
    paths = reo.reorder_by_uvw_tile(r3, (3000.0, 3000.0, 6000.0), outdir, _FakeClient(2), num_time_intervals=4,
                                    max_vis_per_chunk=300)
    recs = []
    for p in sorted(paths):
        t = tile_mod.Tile.load_npz(p)
        off = 0
        for i, (s, e) in enumerate(zip(t.channel_start_indices, t.channel_stop_indices)):
            for c in range(s, e):
                recs.append((*t.coords, c, *t.uvw[i], t.visibilities[off].real, t.visibilities[off].imag))
                off += 1
    recs = np.asarray(sorted(recs))
    names = sorted(p.name for p in paths)
    MS2DIRTY_CALLS.clear()
    img = inv.invert_measurement_set(r3, 64, 5.0)
    call = MS2DIRTY_CALLS[0]
    gi3 = inv.StokesIGridderInput.from_measurement_set_reader(r3)
    np.savez_compressed(OUT / "reorder_invert.npz", uvw=uvw, vis4=vis, flags4=flg, weights4=wts, freq=freq,
                        records=recs, n_files=np.asarray([len(paths)]), file_names=np.asarray(names),
                        invert_image=img, invert_total_weight=np.asarray([gi3.effective_weights().sum()]),
                        pixsize=np.asarray([call["pixsize_x"]]),
                        call_dtypes=np.asarray([call["uvw_dtype"], call["freq_dtype"], call["ms_dtype"],
                                                call["wgt_dtype"]]),
                        call_epsilon=np.asarray([call["epsilon"]]),
                        call_wstacking=np.asarray([bool(call["do_wstacking"])]))
    print("wrote", sorted(p.name for p in OUT.glob("*.npz")))


if __name__ == "__main__":
    main()
