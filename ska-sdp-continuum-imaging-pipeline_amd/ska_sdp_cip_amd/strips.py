"""
Strong scaling of ONE dirty image over several GPUs: uv strips with a halo
exchange before the FFT (SURVEY.md 8(e) option 1; the north
star's "UVW tiles shard naturally across the 8 GPUs ... RCCL reduce over xGMI
of overlapping partial-grid halos before the FFT-to-dirty-image step").

The uv grid is stored transposed for the pruned FFT (gT[y][x], y along v).
Rank r owns grid rows [y0_r, y1_r) - contiguous v strips balanced by
visibility count - and grids the visibilities whose footprint origin row lies
in its strip (the UVW tiles of that strip: the data layout the reference's
reorder_by_uvw_tile produces offline, reorder.py:19-111). A footprint reaches
W - 1 rows past the origin, so rank r's partial grid also holds rows
[y1_r, y1_r + W - 1) of its successor (mod nv): that halo goes to rank r + 1
(point-to-point, RCCL over xGMI) and is added there. Then the FFT runs
distributed: pass A (along u) on each rank's own rows, one all-to-all that
hands every rank the pass-A columns of its image rows [i0_r, i1_r) (blocks of
4 kept u frequencies x all v), pass B (along v) + crop + grid correction on
them, and a gather of the image rows onto the destination rank. The weight sum
is all-reduced and divided out in pass B's epilogue. Traffic per rank at C4
(16384^2 grid, 8 ranks): halo 1.8 MB, all-to-all 224 MB, image rows 64 MB -
against a 4 GiB partial-grid reduce for row (weak) sharding.

The per-rank stages are backend-independent (`HipStripBackend` runs them
through libcip_hip.so; tests plug in a CPU restatement); `invert_strips` wires
them with torch.distributed collectives (RCCL, or gloo on CPU tensors), and
`invert_strips_local` runs all ranks' stages in one process (one device),
exchanging in memory - the single-GPU check of the decomposition.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Sequence

import ctypes

import numpy as np

SPEED_OF_LIGHT = 299792458.0
COL_BLOCK = 4  # pass-A output block width (cip_fft.hip kColBlock)
ctypes_i64 = ctypes.c_int64

try:
    import torch
except ModuleNotFoundError:  # pragma: no cover - torch is in the image
    torch = None


@dataclass
class StripLayout:
    """Row strips of the grid and image-row strips of the dirty image.

    y_bounds: world + 1 grid-row bounds (0 .. nv); x_bounds: world + 1 image-
    row bounds (0 .. npix_x, multiples of COL_BLOCK); halo = W - 1 rows.
    """

    nu: int
    nv: int
    npix_x: int
    npix_y: int
    support: int
    y_bounds: list
    x_bounds: list

    @property
    def world(self) -> int:
        return len(self.y_bounds) - 1

    @property
    def halo(self) -> int:
        return self.support - 1

    def rows(self, r: int) -> tuple[int, int]:
        return self.y_bounds[r], self.y_bounds[r + 1]

    def image_rows(self, r: int) -> tuple[int, int]:
        return self.x_bounds[r], self.x_bounds[r + 1]


def origin_rows(v_m, fx, scale_v: float, nv: int, support: int):
    """Footprint origin row of every (row, channel): iy0 = floor(v f/c nv
    pixsize_y + nv/2 - W/2) + 1, wrapped into [0, nv) - the gridder's placement
    arithmetic (cip_common.h place_vis: the same fp64 operations in the same
    order), so the strip a visibility is assigned to is the one its footprint
    starts in. v_m (nrow,), fx (nchan,) tensors -> (nrow, nchan) int64."""
    y = (v_m[:, None] * fx[None, :]) * scale_v + float(nv // 2)
    iy0 = torch.floor(y - float(support // 2)).to(torch.int64) + 1
    return torch.remainder(iy0, nv)


TILE = 32  # the scatter's tile edge (cip_common.h kTile): the dirty-tile mask's unit


def _on_device(t) -> bool:
    """CUDA tensors take the HIP split (cip_strips.hip); CPU tensors (the gloo
    tests' ranks) the torch restatement of the same arithmetic."""
    return t is not None and getattr(t, "is_cuda", False)


def _gridder_params(params):
    """The ctypes cip_gridder_params of `params` (a GridderParams, or any object
    with its fields - the CPU tests' stand-in)."""
    from . import _lib  # pylint: disable=import-outside-toplevel

    if isinstance(params, _lib.GridderParams):
        return params
    out = _lib.GridderParams()
    for name, _ in _lib.GridderParams._fields_:
        setattr(out, name, type(getattr(out, name))(getattr(params, name, 32 if name == "tile" else 0)))
    return out


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def strip_histogram(uvw, freq, params, pixsize_x: float, pixsize_y: float):
    """(visibilities, row slices) per grid row (int64 (nv,) tensors each): by
    footprint-origin row, a slice starting at each row's first channel and
    wherever the origin's 32-cell tile changes along the channels. CUDA
    tensors: one HIP pass (cip_strip_histogram, block-private LDS histograms);
    CPU tensors: the torch restatement below."""
    nu, nv, W = int(params.nu), int(params.nv), int(params.support)
    if _on_device(uvw):
        from . import _lib  # pylint: disable=import-outside-toplevel

        hist = torch.empty(2 * nv, dtype=torch.int64, device=uvw.device)
        uvw_c, f_c = uvw.contiguous().to(torch.float64), freq.contiguous().to(torch.float64)
        _lib.check(_lib.lib().cip_strip_histogram(uvw_c.data_ptr(), int(uvw_c.shape[0]), f_c.data_ptr(),
                                                  int(f_c.shape[0]), _gridder_params(params), float(pixsize_x),
                                                  float(pixsize_y), _stream(uvw_c), hist.data_ptr()))
        return hist[:nv], hist[nv:]
    fx = freq / SPEED_OF_LIGHT
    vis = torch.zeros(nv, dtype=torch.int64, device=uvw.device)
    runs = torch.zeros(nv, dtype=torch.int64, device=uvw.device)
    for a, b in _row_chunks(uvw.shape[0]):
        iy = origin_rows(uvw[a:b, 1], fx, float(params.nv) * pixsize_y, nv, W)
        ix = origin_rows(uvw[a:b, 0], fx, float(params.nu) * pixsize_x, nu, W)
        key = torch.div(iy, 32, rounding_mode="floor") * (nu // 32 + 1) + torch.div(ix, 32, rounding_mode="floor")
        start = torch.ones_like(key, dtype=torch.bool)
        start[:, 1:] = key[:, 1:] != key[:, :-1]
        vis += torch.bincount(iy.reshape(-1), minlength=nv)
        runs += torch.bincount(iy[start], minlength=nv)
    return vis, runs


def _row_chunks(nrow: int, chunk: int = 65536):
    for a in range(0, nrow, chunk):
        yield a, min(nrow, a + chunk)


# Per-rank cost model of a strip (measured on MI355X, profiles/
# r04_strong_model_c4_n8.json: the 8 strips of C4 balanced by visibility count
# took 6.7-9.5 ms to grid, linear in their row slices): gridding costs
# ~36.9 ps per visibility + ~112 ps per row slice (the planner's runs and the
# scatter's per-slice loads), pass A ~8.9 ps per grid cell of the strip's rows.
COST_PS_PER_VIS = 36.9
COST_PS_PER_SLICE = 112.0
COST_PS_PER_CELL = 8.9


def row_costs(uvw, freq, params, pixsize_x: float, pixsize_y: float, a2a_ps_per_row: float = 0.0):
    """Modelled cost (ps) of each grid row as a strip member: its visibilities
    (by footprint-origin row; per tap, W^2 taps per visibility, W^3 with
    w-stacking - the C3 reference call's w-stacking strips measured 0.63 ps
    per tap against 0.58 for C4's W = 8), the row slices starting there (a
    slice starts at each row's first channel and wherever the origin's 32-cell
    tile changes along the channels) and its pass-A cells (one pass per w
    plane), plus `a2a_ps_per_row` per row and plane: the row's pass-A output
    crossing the all-to-all (a rank's exchange time grows with its rows)."""
    nu, W = int(params.nu), int(params.support)
    wstack = bool(int(getattr(params, "do_wstacking", 0)))
    taps = W * W * (W if wstack else 1)
    nplanes = int(params.nplanes) if wstack else 1
    vis, runs = strip_histogram(uvw, freq, params, pixsize_x, pixsize_y)
    cost = (COST_PS_PER_VIS * (taps / 64.0) * vis.double() + COST_PS_PER_SLICE * runs.double() +
            (COST_PS_PER_CELL * nu + a2a_ps_per_row) * nplanes)
    return cost.cpu().numpy()


def plan_strips(uvw, freq, params, pixsize_y: float, npix_x: int, npix_y: int, world: int,
                balance: str = "cost", pixsize_x: Optional[float] = None,
                link_gbs: Optional[float] = None) -> StripLayout:
    """Balanced strips: grid-row bounds splitting a per-row histogram (all
    visibilities, so every rank computes the same bounds without
    communication) into `world` near-equal parts, each at least W rows high
    (the halo then only reaches the next strip); image rows split into
    near-equal multiples of COL_BLOCK. balance="cost": the measured per-rank
    cost model (`row_costs`: visibilities, row slices, pass-A rows; needs
    pixsize_x, default pixsize_y) plus, for world > 1 and `link_gbs` (off by
    default), each row's share of the all-to-all: its pass-A output (npix_x
    complex128) leaves on world - 1 links, 16 npix_x / world bytes per link
    at link_gbs - the tall, sparse edge strips of long baselines get fewer
    rows (C4 at 8 ranks: 5.86x modelled at 64 GB/s against 5.93x unpriced,
    profiles/r05g_strong_model_c4_bal64.json - the grid imbalance costs more
    than the exchange gains); "vis":
    visibility count only. uvw (nrow, 3), freq (nchan) tensors."""
    nv, W = int(params.nv), int(params.support)
    if world < 1:
        raise ValueError("world must be >= 1")
    nb = npix_x // COL_BLOCK
    if npix_x % COL_BLOCK != 0 or nb < world:
        raise ValueError(f"npix_x must be a multiple of {COL_BLOCK} with at least one block of "
                         f"{COL_BLOCK} image rows per rank")
    if nv < W * world:
        raise ValueError("grid too small for this many strips")
    if balance == "cost":
        a2a = 16.0 * npix_x / world / (link_gbs * 1e9) * 1e12 if (world > 1 and link_gbs) else 0.0
        hist = row_costs(uvw, freq, params, pixsize_y if pixsize_x is None else pixsize_x, pixsize_y,
                         a2a_ps_per_row=a2a)
    elif balance == "vis":
        hist = strip_histogram(uvw, freq, params, pixsize_y if pixsize_x is None else pixsize_x,
                               pixsize_y)[0].cpu().numpy()
    else:
        raise ValueError("balance must be 'cost' or 'vis'")
    cum = np.cumsum(hist)
    total = float(cum[-1]) if cum.size else 0.0
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        y = int(np.searchsorted(cum, target, side="left")) + 1
        y = max(y, bounds[-1] + W)
        y = min(y, nv - W * (world - r))
        bounds.append(y)
    bounds.append(nv)
    return StripLayout(int(params.nu), nv, int(npix_x), int(npix_y), W, bounds,
                       [COL_BLOCK * (r * nb // world) for r in range(world + 1)])


@dataclass
class StripData:
    """One strip's visibilities in the Tile layout (reference
    uvw_tiling/tile.py:14-124): row slices with uvw and channel ranges,
    visibilities / weights concatenated in slice order."""

    slice_uvw: "torch.Tensor"   # (ns, 3) f64
    chan_start: "torch.Tensor"  # (ns,) int32
    chan_stop: "torch.Tensor"   # (ns,) int32
    vis: "torch.Tensor"         # (nvis,) complex
    wgt: Optional["torch.Tensor"]  # (nvis,) f32/f64 or None
    rows: "torch.Tensor"        # (ns,) int64: the MS row of each slice

    @property
    def nvis(self) -> int:
        return int(self.vis.shape[0])


def _split_device(uvw, freq, params, pixsize_y: float, y0: int, y1: int, vis=None, wgt=None):
    """cip_strip_split: (slice_uvw, c0, c1 (int32), rows (int64), vis, wgt)
    of the strip [y0, y1) - one count pass + scans, then one emit pass that
    writes the slices and gathers the strip's visibilities (when given)."""
    from . import _lib  # pylint: disable=import-outside-toplevel
    from .gridder import _codes  # pylint: disable=import-outside-toplevel

    dev = uvw.device
    uvw_c, f_c = uvw.contiguous().to(torch.float64), freq.contiguous().to(torch.float64)
    nrow, nchan = int(uvw_c.shape[0]), int(f_c.shape[0])
    prm = _gridder_params(params)
    vis_codes, wgt_codes = _codes()
    if vis is not None:
        vis = vis.reshape(nrow, nchan).contiguous()
        wgt = None if wgt is None else wgt.reshape(nrow, nchan).contiguous()
    vp = vis.data_ptr() if vis is not None else None
    vc = vis_codes[vis.dtype] if vis is not None else _lib.CIP_C64
    wp = wgt.data_ptr() if wgt is not None else None
    wc = wgt_codes[wgt.dtype] if wgt is not None else _lib.CIP_NONE
    counts = (ctypes_i64 * 2)()
    lib = _lib.lib()
    args = (uvw_c.data_ptr(), nrow, f_c.data_ptr(), nchan, vp, vc, wp, wc, prm, float(pixsize_y), int(y0), int(y1),
            _stream(uvw_c), counts)
    _lib.check(lib.cip_strip_split(*args, None, None, None, None, None, None))
    ns, nvis = int(counts[0]), int(counts[1])
    suvw = torch.empty((ns, 3), dtype=torch.float64, device=dev)
    c0 = torch.empty(ns, dtype=torch.int32, device=dev)
    c1 = torch.empty(ns, dtype=torch.int32, device=dev)
    rows = torch.empty(ns, dtype=torch.int64, device=dev)
    vout = torch.empty(nvis, dtype=vis.dtype, device=dev) if vis is not None else None
    wout = torch.empty(nvis, dtype=wgt.dtype, device=dev) if wgt is not None else None
    _lib.check(lib.cip_strip_split(*args, suvw.data_ptr(), c0.data_ptr(), c1.data_ptr(), rows.data_ptr(),
                                   vout.data_ptr() if vout is not None and nvis else None,
                                   wout.data_ptr() if wout is not None and nvis else None))
    return suvw, c0, c1, rows, vout, wout


def split_strip(uvw, freq, vis, wgt, params, pixsize_y: float, y0: int, y1: int) -> "StripData":
    """Rank-local strip data from dense (nrow, nchan) columns: the row slices
    whose footprint-origin rows lie in [y0, y1) and their visibilities /
    weights, in the Tile layout (the reference's reorder_by_uvw_tile output,
    reorder.py:19-111, cut by strip). CUDA tensors: cip_strip_split (one
    count pass, one emit + gather pass); CPU tensors: strip_slices +
    gather_strip (the same slices and order)."""
    if _on_device(uvw):
        suvw, c0, c1, rows, v, w = _split_device(uvw, freq, params, pixsize_y, y0, y1, vis, wgt)
        return StripData(suvw, c0, c1, v, w, rows)
    rows, c0, c1 = strip_slices(uvw, freq, params, pixsize_y, y0, y1)
    return gather_strip(uvw, vis, wgt, rows, c0, c1)


def strip_slices(uvw, freq, params, pixsize_y: float, y0: int, y1: int):
    """(rows, c0, c1) int64 tensors: the maximal channel runs of each row whose
    origin row lies in [y0, y1) (one run per row unless a row's v track wraps
    or leaves and re-enters the strip). CUDA tensors: cip_strip_split."""
    if _on_device(uvw):
        _, c0, c1, rows, _, _ = _split_device(uvw, freq, params, pixsize_y, y0, y1)
        return rows, c0.to(torch.int64), c1.to(torch.int64)
    nv, W = int(params.nv), int(params.support)
    fx = freq / SPEED_OF_LIGHT
    scale_v = float(params.nv) * pixsize_y
    rows_l, c0_l, c1_l = [], [], []
    for a, b in _row_chunks(uvw.shape[0]):
        iy = origin_rows(uvw[a:b, 1], fx, scale_v, nv, W)
        m = (iy >= y0) & (iy < y1)
        pad = torch.zeros((m.shape[0], 1), dtype=torch.bool, device=m.device)
        mp = torch.cat([pad, m, pad], dim=1)
        starts = torch.nonzero(mp[:, 1:] & ~mp[:, :-1])  # (row, channel) of each run start
        stops = torch.nonzero(~mp[:, 1:] & mp[:, :-1])   # (row, channel) one past each run's end
        rows_l.append(starts[:, 0] + a)
        c0_l.append(starts[:, 1])
        c1_l.append(stops[:, 1])
    if not rows_l:
        e = torch.zeros(0, dtype=torch.int64, device=uvw.device)
        return e, e, e
    return torch.cat(rows_l), torch.cat(c0_l), torch.cat(c1_l)


def gather_strip(uvw, vis, wgt, rows, c0, c1) -> StripData:
    """The strip's Tile-layout data from dense (nrow, nchan) columns."""
    nchan = vis.shape[1]
    lengths = (c1 - c0)
    starts = rows * nchan + c0
    idx = torch.repeat_interleave(starts, lengths)
    if idx.numel():
        first = torch.repeat_interleave(torch.cumsum(lengths, 0) - lengths, lengths)
        idx = idx + (torch.arange(idx.numel(), device=idx.device) - first)
    return StripData(uvw[rows].contiguous(), c0.to(torch.int32), c1.to(torch.int32),
                     vis.reshape(-1)[idx].contiguous(), None if wgt is None else wgt.reshape(-1)[idx].contiguous(),
                     rows)


def strip_buffer_rows(layout: StripLayout, r: int) -> tuple[int, int]:
    """(row0, nrows) of rank r's grid buffer: its strip rows [y0, y1) plus the
    W - 1 halo rows after them (buffer row k = grid row (y0 + k) mod nv). One
    strip holding the whole grid: (0, nv), its halo wraps onto its own rows."""
    y0, y1 = layout.rows(r)
    if layout.world == 1:
        return 0, layout.nv
    return y0, y1 - y0 + layout.halo


class HipStripBackend:
    """Per-rank stages on the current GPU through libcip_hip.so:
    cip_grid_tiles_strip (accumulating gridder) onto a buffer holding only the
    rank's strip + halo rows (`bind`: 1/N of the grid plus W - 1 rows instead
    of a full-size grid per rank), cip_strip_rows (pass A), cip_strip_cols
    (pass B + crop + correction). The buffer is kept between calls and left
    clean (pass A zeroes the rows it reads; the halo rows are zeroed after
    they are sent); an invert that fails in between leaves it marked dirty and
    the next `grid_strip` zeroes it first instead of trusting CIP_GRID_ZEROED.
    Unbound (rows=None) the buffer is the whole transposed grid.
    w-stacking parameters (nplanes > 1): the buffer holds the strip's rows of
    every w plane, (nplanes, nrows, nu, 2); pass A runs per plane, pass B per
    plane with the w screen into the rank's image rows (`pass_cols_wplane`),
    then `finish_rows` applies the final w and grid corrections.
    `single_precision_accumulation`: the packed class (complex64 visibilities;
    the reference call's float class), gridded into the same fp64 planes."""

    def __init__(self, params, pixsize_x: float, pixsize_y: float, npix_x: int, npix_y: int, device=None,
                 rows: Optional[tuple] = None, single_precision_accumulation: bool = False):
        from . import _lib  # pylint: disable=import-outside-toplevel
        from .gridder import _require_gpu  # pylint: disable=import-outside-toplevel

        _require_gpu()
        self._lib = _lib
        self.params = params
        self.px, self.py = float(pixsize_x), float(pixsize_y)
        self.npix_x, self.npix_y = int(npix_x), int(npix_y)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if not _lib.lib().cip_grid_layout(params, self.npix_x, self.npix_y):
            raise ValueError("strips need a grid in the pruned-FFT layout (power-of-two grids)")
        self.nplanes = int(params.nplanes) if int(params.do_wstacking) else 1
        self.single = bool(single_precision_accumulation)
        # the gridded strip's dirty-tile bits, written by every grid_strip call
        # (cip_grid_tiles_strip_mask: the call's own planner mask + the halo
        # tile rows); CIP_STRIP_MASK=0 runs pass A over every cell
        self.masked = os.environ.get("CIP_STRIP_MASK", "1") != "0"
        self._bits = None
        self._bits_valid = False
        self.rows = None
        self.grid = None
        self.dirty = False
        self._alloc((0, int(params.nv)) if rows is None else rows)

    def _alloc(self, rows):
        row0, nrows = int(rows[0]), int(rows[1])
        if not (0 <= row0 < int(self.params.nv) and 1 <= nrows <= int(self.params.nv)):
            raise ValueError("strip rows outside the grid")
        if self.rows != (row0, nrows):
            self.grid = None  # free the old buffer first
            shape = (nrows, int(self.params.nu), 2) if self.nplanes == 1 else (self.nplanes, nrows,
                                                                                 int(self.params.nu), 2)
            self.grid = torch.zeros(shape, dtype=torch.float64, device=self.device)
            self.rows = (row0, nrows)
            self.dirty = False

    def spawn(self) -> "HipStripBackend":
        """A backend of the same configuration (another rank's, for the
        single-process emulation)."""
        return HipStripBackend(self.params, self.px, self.py, self.npix_x, self.npix_y, device=self.device,
                               rows=self.rows, single_precision_accumulation=self.single)

    def bind(self, layout: StripLayout, rank: int) -> "HipStripBackend":
        """Hold rank `rank`'s strip + halo rows of `layout` (reallocates when they change)."""
        self._alloc(strip_buffer_rows(layout, rank))
        return self

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def grid_strip(self, data: StripData, freq):
        """Grid the strip's visibilities; returns (strip buffer (nrows, nu, 2) f64 - (nplanes, nrows, nu, 2)
        with w-stacking -, weight sum (1,) f64)."""
        from .gridder import _codes  # pylint: disable=import-outside-toplevel

        if self.dirty:  # a previous invert did not finish: the buffer may hold partial sums
            self.grid.zero_()
        self.dirty = True
        self._bits_valid = False
        vis_codes, wgt_codes = _codes()
        sumw = torch.zeros(1, dtype=torch.float64, device=self.device)
        ns = int(data.slice_uvw.shape[0])
        nu, nv = int(self.params.nu), int(self.params.nv)
        mask = self.masked and nu % 1024 == 0
        if mask:
            shape = (self.nplanes, nv // TILE, nu // TILE // 32)
            if self._bits is None or tuple(self._bits.shape) != shape:
                self._bits = torch.empty(shape, dtype=torch.int32, device=self.device)
        fn = self._lib.lib().cip_grid_tiles_strip_mask if mask else self._lib.lib().cip_grid_tiles_strip
        extra = (self._bits.data_ptr(),) if mask else ()
        if ns or mask:
            # an empty strip still writes its mask (the halo rows it receives)
            self._lib.check(fn(
                data.slice_uvw.data_ptr() if ns else None, data.chan_start.data_ptr() if ns else None,
                data.chan_stop.data_ptr() if ns else None, ns,
                freq.data_ptr(), int(freq.shape[0]), data.vis.data_ptr() if data.nvis else None, data.nvis,
                vis_codes[data.vis.dtype],
                data.wgt.data_ptr() if data.wgt is not None and data.nvis else None,
                wgt_codes[data.wgt.dtype] if data.wgt is not None else self._lib.CIP_NONE,
                self.params, self.px, self.py, self.npix_x, self.npix_y, self.rows[0], self.rows[1],
                self._lib.CIP_GRID_ZEROED | (self._lib.CIP_ACC_SINGLE if self.single else 0), self._stream(),
                self.grid.data_ptr(), sumw.data_ptr(), *extra))
        self._bits_valid = mask
        return self.grid, sumw

    def mark_clean(self) -> None:
        """Pass A consumed the strip rows and the halo rows were zeroed."""
        self.dirty = False

    def pass_rows(self, grid, y0: int, y1: int, plane: int = 0):
        """Pass A over buffer rows [y0, y1) of w plane `plane` -> H (npix_x / 4, y1 - y0, 4, 2); zeroes the
        rows (only the dirty tiles' cells are read when the gridded strip's mask is known)."""
        H = torch.empty((self.npix_x // COL_BLOCK, y1 - y0, COL_BLOCK, 2), dtype=torch.float64, device=self.device)
        if self._bits_valid and self.dirty:
            self._lib.check(self._lib.lib().cip_strip_rows_masked(
                grid.data_ptr(), self.params, self.npix_x, self.npix_y, int(y0), int(y1), int(self.rows[0]),
                self._bits[plane].data_ptr(), self._stream(), H.data_ptr()))
        else:
            self._lib.check(self._lib.lib().cip_strip_rows(grid.data_ptr(), self.params, self.npix_x, self.npix_y,
                                                           int(y0), int(y1), self._stream(), H.data_ptr()))
        return H

    def pass_rows_packed(self, grid, y0: int, y1: int, live, count: int, plane: int = 0):
        """Pass A over buffer rows [y0, y1) keeping only the live rows (`live`:
        bool over them, as live_rows gives; `count` Trues) -> H (npix_x / 4,
        count, 4, 2): the sparse all-to-all's send buffer, written by pass A
        itself (cip_strip_rows_packed) instead of packed after it."""
        if not (self._bits_valid and self.dirty):
            return _pack_live(self.pass_rows(grid, y0, y1, plane), live, count)
        slot = torch.cumsum(live.to(torch.int64), 0).sub_(1)
        slot = torch.where(live, slot, torch.full_like(slot, -1))
        H = torch.empty((self.npix_x // COL_BLOCK, count, COL_BLOCK, 2), dtype=torch.float64, device=self.device)
        self._lib.check(self._lib.lib().cip_strip_rows_packed(
            grid.data_ptr(), self.params, self.npix_x, self.npix_y, int(y0), int(y1), int(self.rows[0]),
            self._bits[plane].data_ptr(), slot.data_ptr(), int(count), self._stream(),
            H.data_ptr() if count else None))
        return H

    def live_rows(self, h: int, plane: int = 0):
        """Buffer rows [0, h) of `plane` that may hold a non-zero cell (their
        tile row has a dirty tile in the gridded strip's mask), or None when
        no mask is known: pass A of every other row is exactly zero."""
        if not self._bits_valid:
            return None
        words = self._bits[plane]  # (nty, ntx / 32) int32
        tile_live = (words != 0).any(dim=1)
        rows = torch.remainder(torch.arange(self.rows[0], self.rows[0] + h, device=words.device), int(self.params.nv))
        return tile_live[rows // TILE]

    def pass_cols(self, H, i0: int, i1: int, norm=None):
        """Pass B for image rows [i0, i1) from H ((i1 - i0) / 4, nv, 4, 2)."""
        out = torch.empty((i1 - i0, self.npix_y), dtype=torch.float64, device=self.device)
        self._lib.check(self._lib.lib().cip_strip_cols(H.data_ptr(), self.params, self.npix_x, self.npix_y,
                                                       int(i0), int(i1), None if norm is None else norm.data_ptr(),
                                                       self._stream(), out.data_ptr()))
        return out

    def pass_cols_wplane(self, H, i0: int, i1: int, plane: int, first: bool, acc):
        """Pass B of w plane `plane` for image rows [i0, i1) with its w screen, into acc ((i1 - i0), npix_y)
        f64 (overwritten when `first`)."""
        self._lib.check(self._lib.lib().cip_strip_cols_wplane(
            H.data_ptr(), self.params, self.npix_x, self.npix_y, self.px, self.py, int(i0), int(i1), int(plane),
            int(bool(first)), self._stream(), acc.data_ptr()))
        return acc

    def finish_rows(self, acc, i0: int, i1: int, norm=None):
        """The final w and grid corrections of image rows [i0, i1) (acc, in place), / norm."""
        self._lib.check(self._lib.lib().cip_strip_wfinal(
            acc.data_ptr(), self.params, self.npix_x, self.npix_y, self.px, self.py, int(i0), int(i1),
            None if norm is None else norm.data_ptr(), self._stream()))
        return acc


def _assemble_H(pieces: Sequence, nb: int, layout: StripLayout, device, dtype, idx=None):
    """Rank s's pass-B input from every rank's pass-A blocks [i0_s / 4, i1_s / 4)
    (piece r: (nb, h_r, 4, 2), or with idx[r] (sparse) only rank r's rows
    idx[r] of its strip: (nb, len(idx[r]), 4, 2), the other rows zero) ->
    (nb, nv, 4, 2). The torch form, for CPU tensors (the gloo tests' backend);
    GPU buffers go through _unpack_rows (one copy kernel)."""
    sparse = idx is not None and any(i is not None for i in idx)
    H = (torch.zeros if sparse else torch.empty)((nb, layout.nv, COL_BLOCK, 2), dtype=dtype, device=device)
    for r, piece in enumerate(pieces):
        y0, y1 = layout.rows(r)
        if idx is None or idx[r] is None:
            H[:, y0:y1] = piece.reshape(nb, y1 - y0, COL_BLOCK, 2)
        elif idx[r].numel():
            H[:, y0 + idx[r]] = piece.reshape(nb, idx[r].numel(), COL_BLOCK, 2)
    return H


def invert_strips(data: StripData, freq, layout: StripLayout, backend, *, dst: int = 0, group=None,
                  stages: Optional[dict] = None, sparse: bool = True, gather_async: bool = False):
    """This rank's share of the strip-distributed invert (torch.distributed
    initialised, one rank per strip). Returns the normalised dirty image
    (npix_x, npix_y) on `dst`, None elsewhere. Collectives: one point-to-point
    halo exchange with the ring neighbours, one all-to-all of the pass-A
    blocks, a scalar all-reduce of the weight sum, a gather of image rows.
    The backend is bound to this rank's strip + halo rows (`strip_buffer_rows`).
    `sparse` (default): the all-to-all carries only the rows of the pass-A
    output that can be non-zero (after an all-gather of the live-row masks).
    `gather_async`: return a `PendingGather` at once (the image-row gather in
    flight on the communicator's stream, e.g. beside the next invert's
    gridding); `.wait()` gives the image.
    `stages` (a dict, diagnostic): each stage is synchronised and its seconds
    added under its name (grid, halo, rows, alltoall, cols, gather), and the
    all-to-all's bytes sent by this rank under a2a_send_bytes."""
    import time  # pylint: disable=import-outside-toplevel

    import torch.distributed as dist  # pylint: disable=import-outside-toplevel

    t_last = [time.perf_counter()]
    single = not dist.is_available() or not dist.is_initialized()
    world = 1 if single else dist.get_world_size(group)
    rank = 0 if single else dist.get_rank(group)
    if world != layout.world:
        raise ValueError("the layout was planned for another number of ranks")
    backend.bind(layout, rank)
    y0, y1 = layout.rows(rank)
    h = y1 - y0
    buf, sumw = backend.grid_strip(data, freq)

    def mark(name):
        if stages is not None:
            if buf.is_cuda:
                torch.cuda.synchronize(buf.device)
            t = time.perf_counter()
            stages[name] = stages.get(name, 0.0) + t - t_last[0]
            t_last[0] = t

    mark("grid")
    # w-stacking buffers hold every plane's rows: rows are the second axis
    nplanes = int(getattr(backend, "nplanes", 1))
    rowsel = (lambda a, b: buf[a:b]) if nplanes == 1 else (lambda a, b: buf[:, a:b])
    if world > 1:
        # halo: buffer rows [h, h + W - 1) = the grid rows past the strip ->
        # the next rank, added to its first rows (every plane's at once)
        send = rowsel(h, h + layout.halo).contiguous()
        recv = torch.empty_like(send)
        ops = [dist.P2POp(dist.isend, send, (rank + 1) % world, group),
               dist.P2POp(dist.irecv, recv, (rank - 1) % world, group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        rowsel(h, h + layout.halo).zero_()
        rowsel(0, layout.halo).add_(recv)
        dist.all_reduce(sumw, group=group)
    mark("halo")
    if nplanes > 1:
        # per w plane: pass A on this rank's rows, the all-to-all, pass B with
        # the plane's w screen added into this rank's image rows
        i0, i1 = layout.image_rows(rank)
        acc = torch.empty((i1 - i0, backend.npix_y), dtype=torch.float64, device=buf.device)
        for p in range(nplanes):
            snd = _packed_send(backend, buf[p], h, p, layout, rank, world, group) if (sparse and world > 1) else None
            if snd is not None:
                mark("rows")
                Hm = _alltoall_rows(snd[0], layout, rank, world, group, snd[1], snd[2], snd[3],
                                    stages).to(torch.float64)
            else:
                H = backend.pass_rows(buf[p], 0, h, plane=p)
                mark("rows")
                Hm = (_alltoall_H(_wire(H, backend), layout, rank, world, group,
                                  live=_live_of(backend, H, h, p) if sparse else None, stats=stages).to(torch.float64)
                      if world > 1 else H)
            mark("alltoall")
            backend.pass_cols_wplane(Hm, i0, i1, p, p == 0, acc)
            mark("cols")
        backend.mark_clean()
        rows_img = backend.finish_rows(acc, i0, i1, norm=sumw)
        mark("final")
        return _gather_rows(rows_img, layout, rank, world, dst, group, mark, async_op=gather_async)
    snd = _packed_send(backend, buf, h, 0, layout, rank, world, group) if (sparse and world > 1) else None
    i0, i1 = layout.image_rows(rank)
    if snd is not None:
        backend.mark_clean()
        mark("rows")
        Hm = _alltoall_rows(snd[0], layout, rank, world, group, snd[1], snd[2], snd[3], stages).to(torch.float64)
    else:
        H = backend.pass_rows(buf, 0, h)
        live = _live_of(backend, H, h) if (sparse and world > 1) else None
        backend.mark_clean()
        mark("rows")
        Hm = (_alltoall_H(_wire(H, backend), layout, rank, world, group, live=live, stats=stages).to(torch.float64)
              if world > 1 else H)
    mark("alltoall")
    rows_img = backend.pass_cols(Hm, i0, i1, norm=sumw)
    mark("cols")
    return _gather_rows(rows_img, layout, rank, world, dst, group, mark, async_op=gather_async)


def _wire(H, backend):
    """The pass-A blocks as they cross the all-to-all: complex64 for the packed
    class (its own precision; half the bytes), complex128 otherwise."""
    return H.to(torch.float32) if getattr(backend, "single", False) else H


def _live_of(backend, H, h: int, plane: int = 0):
    """Rows of this rank's pass-A output H (nb, h, 4, 2) that can be non-zero:
    the backend's dirty-tile rows when it knows them, else a scan of H (a
    row whose grid row was empty transforms to exact zeros either way)."""
    fn = getattr(backend, "live_rows", None)
    live = fn(h, plane) if fn is not None else None
    if live is None:
        live = (H != 0).reshape(H.shape[0], h, -1).any(dim=2).any(dim=0)
    return live.to(torch.bool)


def _elem_bytes(H) -> int:
    """Bytes of one complex element of a (..., 2) real view."""
    return 2 * H.element_size()


def _pack_live(H, live, count: int):
    """This rank's live pass-A rows, compacted: (nb, h, 4, 2) -> (nb, count,
    4, 2) (`live`: bool (h); count = its number of Trues). On the GPU one
    copy kernel (cip_strip_pack_rows); CPU tensors (the gloo tests' backend)
    take the torch form."""
    nb, h = int(H.shape[0]), int(H.shape[1])
    if H.device.type != "cuda":
        return H.index_select(1, torch.nonzero(live).reshape(-1))
    from . import _lib  # pylint: disable=import-outside-toplevel

    H = H.contiguous()
    slot = torch.cumsum(live.to(torch.int64), 0).sub_(1)
    slot = torch.where(live, slot, torch.full_like(slot, -1))
    out = torch.empty((nb, count) + tuple(H.shape[2:]), dtype=H.dtype, device=H.device)
    _lib.check(_lib.lib().cip_strip_pack_rows(H.data_ptr(), nb, h, _elem_bytes(H), slot.data_ptr(), count,
                                              torch.cuda.current_stream(H.device).cuda_stream, out.data_ptr()))
    return out


_ROW_MAPS: dict = {}


def _unpack_rows(recv, nb: int, layout: StripLayout, masks, dtype, stacked=None):
    """A receiver's pass-B input (nb, nv, 4, 2) from the flat received buffer:
    rank r's piece (nb, its live row count, 4, 2) holds its live rows
    (masks[r], bool over its strip rows; None: every row), in order; rows no
    rank sent are zero. One copy kernel (cip_strip_unpack_rows); its row map - the record
    of each grid row's block 0 and its source's row count - in a handful of
    vectorised ops (`stacked`: the ranks' masks as one (world, >= max rows)
    tensor, when the caller has it)."""
    from . import _lib  # pylint: disable=import-outside-toplevel

    dev = recv.device
    nv, world = layout.nv, layout.world
    hs = [layout.rows(r)[1] - layout.rows(r)[0] for r in range(world)]
    if stacked is None:
        stacked = torch.zeros((world, max(hs)), dtype=torch.uint8, device=dev)
        for r, m in enumerate(masks):
            stacked[r, :hs[r]] = 1 if m is None else m.to(torch.uint8)
    M = stacked[:, :max(hs)].to(torch.int64)
    key = (tuple(layout.y_bounds), str(dev))
    maps = _ROW_MAPS.get(key)
    if maps is None:  # grid row -> (its rank, its row in the rank's strip), per layout
        rr = torch.repeat_interleave(torch.arange(world, device=dev), torch.tensor(hs, device=dev))
        y0s = torch.tensor([layout.rows(r)[0] for r in range(world)], device=dev)
        maps = (rr, torch.arange(nv, device=dev) - y0s[rr])
        if len(_ROW_MAPS) > 16:
            _ROW_MAPS.clear()
        _ROW_MAPS[key] = maps
    rr, jj = maps
    cnt = M.sum(dim=1)  # = counts, on the device (no host copies)
    base = (torch.cumsum(cnt, 0) - cnt) * nb
    rec = torch.where(M[rr, jj] != 0, torch.cumsum(M, dim=1).sub_(1)[rr, jj] + base[rr],
                      torch.full((nv,), -1, dtype=torch.int64, device=dev))
    stride = cnt[rr]
    H = torch.empty((nb, nv, COL_BLOCK, 2), dtype=dtype, device=dev)
    _lib.check(_lib.lib().cip_strip_unpack_rows(recv.data_ptr(), nb, nv, 2 * H.element_size(), rec.data_ptr(),
                                                stride.data_ptr(), torch.cuda.current_stream(dev).cuda_stream,
                                                H.data_ptr()))
    return H


def _exchange_masks(live, layout: StripLayout, rank: int, world: int, group):
    """All ranks' live-row masks of their pass-A output (one all-gather) ->
    (stacked (world, max rows) uint8, counts, masks (bool over each rank's
    rows)); the counts are the all-to-all's split sizes (one host wait)."""
    import torch.distributed as dist  # pylint: disable=import-outside-toplevel

    hs = [layout.rows(r)[1] - layout.rows(r)[0] for r in range(world)]
    h = hs[rank]
    mine = torch.zeros(max(hs), dtype=torch.uint8, device=live.device)
    mine[:h] = live.to(torch.uint8)
    allm = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allm, mine, group=group)
    stacked = torch.stack(allm)
    counts = [int(c) for c in stacked.sum(dim=1).tolist()]
    return stacked, counts, [allm[r][:hs[r]].to(torch.bool) for r in range(world)]


def _alltoall_rows(Hsend, layout: StripLayout, rank: int, world: int, group, counts, masks, stacked=None,
                   stats: Optional[dict] = None):
    """The all-to-all of pass-A rows: `Hsend` (nb_all, counts[rank], 4, 2) is
    this rank's send buffer (its live rows, or every row when masks[rank] is
    None); rank s receives blocks [i0_s / 4, i1_s / 4) of every rank's rows ->
    its pass-B input (nb, nv, 4, 2), rows nobody sent zero."""
    import torch.distributed as dist  # pylint: disable=import-outside-toplevel

    i0, i1 = layout.image_rows(rank)
    nb = (i1 - i0) // COL_BLOCK
    splits_in = [(layout.image_rows(s)[1] - layout.image_rows(s)[0]) // COL_BLOCK * counts[rank] * COL_BLOCK * 2
                 for s in range(world)]
    splits_out = [nb * counts[r] * COL_BLOCK * 2 for r in range(world)]
    if stats is not None:
        stats["a2a_send_bytes"] = stats.get("a2a_send_bytes", 0) + sum(splits_in) * Hsend.element_size()
    recv = torch.empty(sum(splits_out), dtype=Hsend.dtype, device=Hsend.device)
    dist.all_to_all_single(recv, Hsend.reshape(-1), splits_out, splits_in, group=group)
    if Hsend.device.type == "cuda":
        return _unpack_rows(recv, nb, layout, masks, Hsend.dtype, stacked)
    pieces = list(torch.split(recv, splits_out))
    idx = [None if m is None else torch.nonzero(m).reshape(-1) for m in masks]
    return _assemble_H(pieces, nb, layout, Hsend.device, Hsend.dtype, idx)


def _alltoall_H(H, layout: StripLayout, rank: int, world: int, group, live=None, stats: Optional[dict] = None):
    """The all-to-all of pass-A blocks: rank s receives blocks [i0_s / 4,
    i1_s / 4) of every rank's rows -> its pass-B input (nb, nv, 4, 2).
    Sparse (`live`, this rank's rows that can be non-zero): the ranks first
    all-gather their live-row masks, then send only live rows; a receiver
    fills the others with zeros. The tall edge strips of C4's cost-balanced
    layout are mostly empty long-baseline rows."""
    if live is None:
        hs = [layout.rows(r)[1] - layout.rows(r)[0] for r in range(world)]
        return _alltoall_rows(H, layout, rank, world, group, hs, [None] * world, stats=stats)
    stacked, counts, masks = _exchange_masks(live, layout, rank, world, group)
    return _alltoall_rows(_pack_live(H, masks[rank], counts[rank]), layout, rank, world, group, counts, masks,
                          stacked, stats)


def _packed_send(backend, buf, h: int, plane: int, layout: StripLayout, rank: int, world: int, group):
    """Sparse exchange with pass A writing the send buffer (the backend knows
    its live rows before pass A): (Hsend on the wire, counts, masks, stacked),
    or None when it does not (then pass A runs dense and _alltoall_H packs)."""
    fn = getattr(backend, "live_rows", None)
    live = fn(h, plane) if fn is not None else None
    if live is None or not hasattr(backend, "pass_rows_packed"):
        return None
    stacked, counts, masks = _exchange_masks(live, layout, rank, world, group)
    Hs = backend.pass_rows_packed(buf, 0, h, masks[rank], counts[rank], plane=plane)
    return _wire(Hs, backend), counts, masks, stacked


class PendingGather:
    """A strip invert whose image-row gather is in flight
    (`invert_strips(..., gather_async=True)`): the collective runs on the
    communicator's stream while the caller goes on - e.g. with the next
    invert's gridding, which touches none of its buffers. `wait()` returns
    the image on `dst` (None elsewhere)."""

    def __init__(self, work, gathered, layout: StripLayout, rank: int, dst: int, image=None):
        self._work, self._gathered, self._layout = work, gathered, layout
        self._rank, self._dst, self._image = rank, dst, image
        self._done = work is None

    def wait(self):
        if not self._done:
            self._work.wait()
            self._done = True
            if self._rank == self._dst:
                lay = self._layout
                self._image = torch.cat([g[:lay.image_rows(r)[1] - lay.image_rows(r)[0]]
                                         for r, g in enumerate(self._gathered)])
            self._gathered = None
        return self._image


def _gather_rows(rows_img, layout: StripLayout, rank: int, world: int, dst: int, group, mark,
                 async_op: bool = False):
    """This rank's image rows -> the whole image on `dst` (None elsewhere);
    async_op: a PendingGather instead."""
    import torch.distributed as dist  # pylint: disable=import-outside-toplevel

    if world == 1:
        return PendingGather(None, None, layout, rank, dst, rows_img) if async_op else rows_img
    # gather the image rows (strips padded to the largest: gather needs equal sizes)
    hmax = max(layout.image_rows(r)[1] - layout.image_rows(r)[0] for r in range(world))
    if rows_img.shape[0] < hmax:
        rows_img = torch.cat([rows_img, rows_img.new_zeros((hmax - rows_img.shape[0], rows_img.shape[1]))])
    gathered = [torch.empty_like(rows_img) for _ in range(world)] if rank == dst else None
    work = dist.gather(rows_img, gathered, dst=dst, group=group, async_op=async_op)
    if async_op:
        return PendingGather(work, gathered, layout, rank, dst)
    mark("gather")
    if rank != dst:
        return None
    return torch.cat([g[:layout.image_rows(r)[1] - layout.image_rows(r)[0]] for r, g in enumerate(gathered)])


def _count_a2a(stages, Hs, lives, layout: StripLayout, backend):
    """Add each rank's all-to-all send bytes (to the other ranks) to its
    stage dict: (N - 1) / N of its (live) pass-A rows on the wire."""
    if stages is None or layout.world == 1:
        return
    esize = _wire(Hs[0][:0], backend).element_size()
    for r, H in enumerate(Hs):
        rows = int(lives[r].sum()) if lives is not None else H.shape[1]
        i0, i1 = layout.image_rows(r)
        own = (i1 - i0) // COL_BLOCK
        stages[r]["a2a_send_bytes"] = stages[r].get("a2a_send_bytes", 0) + \
            (H.shape[0] - own) * rows * COL_BLOCK * 2 * esize


def _local_pieces(Hs, b0: int, b1: int, backend, lives):
    """The emulated all-to-all for one receiver: blocks [b0, b1) of every
    rank's H, only its live rows when `lives` (sparse) - as _alltoall_H
    sends them."""
    if lives is None:
        return [_wire(H[b0:b1], backend) for H in Hs], None
    idx = [torch.nonzero(lv).reshape(-1) for lv in lives]
    return [_wire(H[b0:b1].index_select(1, i), backend) for H, i in zip(Hs, idx)], idx


def _local_sends(Hs, lives, backend, timed):
    """The emulated all-to-all's send side: every rank packs its live rows
    once (timed as its "pack" stage, as _alltoall_H's sender does) ->
    (sends, masks, counts, stacked masks); a receiver's buffer is the concatenation of the
    sends' block ranges (the network: untimed), unpacked by _unpack_rows."""
    wires = [_wire(H, backend) for H in Hs]
    hs = [int(H.shape[1]) for H in Hs]
    if lives is None:
        return wires, [None] * len(Hs), hs, None
    masks = [lv.to(torch.bool) for lv in lives]
    counts = [int(c) for c in torch.stack([m.sum() for m in masks]).tolist()]
    stacked = torch.zeros((len(Hs), max(hs)), dtype=torch.uint8, device=Hs[0].device)
    for r, m in enumerate(masks):
        stacked[r, :hs[r]] = m.to(torch.uint8)
    sends = [timed(r, "pack", lambda r=r: _pack_live(wires[r], masks[r], counts[r])) for r in range(len(Hs))]
    return sends, masks, counts, stacked


def _local_pass_a(ranks, grids, hs, plane, sparse: bool, on_gpu: bool, timed, backend, layout, stages):
    """Every rank's pass A in the emulation -> (Hs, lives, sends): with the
    sparse exchange on the GPU and every rank's live rows known from its mask,
    pass A writes the packed send buffer itself (Hs None; sends = (buffers,
    masks, counts, stacked)), else dense pass A (sends from _local_sends)."""
    world = len(ranks)
    if sparse and world > 1 and on_gpu and all(hasattr(rk, "pass_rows_packed") for rk in ranks):
        lives = [rk.live_rows(h, plane) for rk, h in zip(ranks, hs)]
        if all(lv is not None for lv in lives):
            masks = [lv.to(torch.bool) for lv in lives]
            counts = [int(c) for c in torch.stack([m.sum() for m in masks]).tolist()]
            stacked = torch.zeros((world, max(hs)), dtype=torch.uint8, device=masks[0].device)
            for r, m in enumerate(masks):
                stacked[r, :hs[r]] = m.to(torch.uint8)
            bufs = [timed(r, "rows", lambda r=r: _wire(ranks[r].pass_rows_packed(
                grids[r], 0, hs[r], masks[r], counts[r], plane=plane), backend)) for r in range(world)]
            _count_a2a(stages, bufs, masks, layout, backend)
            return None, masks, (bufs, masks, counts, stacked)
    Hs = [timed(r, "rows", lambda r=r: ranks[r].pass_rows(grids[r], 0, hs[r], plane=plane)) for r in range(world)]
    lives = [_live_of(ranks[r], Hs[r], hs[r], plane) for r in range(world)] if (sparse and world > 1) else None
    _count_a2a(stages, Hs, lives, layout, backend)
    sends = _local_sends(Hs, lives, backend, timed) if (world > 1 and on_gpu) else None
    return Hs, lives, sends


def invert_strips_local(datas: Sequence[StripData], freq, layout: StripLayout, backend,
                        stages: Optional[list] = None, sparse: bool = True):
    """All ranks' stages in ONE process on one device, the exchanges done in
    memory (the single-GPU check of the decomposition and its kernels, and the
    per-rank cost breakdown of the N-GPU split). Rank r's stages run on its
    own strip + halo buffer (`backend.spawn()` per rank, kept as
    `backend.ranks`), in the distributed order: every rank grids its strip,
    the halos move to the next rank, pass A runs per strip, the pass-A blocks
    are regrouped per image-row strip (the all-to-all) and pass B runs per
    image-row strip. `sparse`: the regrouping moves only each rank's live
    rows (as the distributed sparse all-to-all). `stages` (a list,
    diagnostic): filled with one dict per rank of synchronised seconds (grid,
    halo, rows, pack, assemble, cols) and the bytes the rank would send in
    the all-to-all (a2a_send_bytes). Returns the normalised dirty image
    (npix_x, npix_y)."""
    import time  # pylint: disable=import-outside-toplevel

    world = layout.world
    if len(datas) != world:
        raise ValueError("one StripData per strip")
    if stages is not None:
        stages[:] = [{} for _ in range(world)]
    dev = getattr(backend, "device", None)
    on_gpu = dev is not None and torch.device(dev).type == "cuda"

    def timed(r, name, fn):
        if stages is None:
            return fn()
        if on_gpu:
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fn()
        if on_gpu:
            torch.cuda.synchronize(dev)
        stages[r][name] = stages[r].get(name, 0.0) + time.perf_counter() - t0
        return out

    ranks = getattr(backend, "ranks", None)
    if not ranks or len(ranks) != world:
        ranks = [backend] + [backend.spawn() for _ in range(world - 1)]
        backend.ranks = ranks
    for r in range(world):
        ranks[r].bind(layout, r)
    bufs, sums = [None] * world, [None] * world
    for r in range(world):
        bufs[r], sums[r] = timed(r, "grid", lambda r=r: ranks[r].grid_strip(datas[r], freq))
    sumw = sums[0].clone()
    for sw in sums[1:]:
        sumw = sumw + sw
    hs = [layout.rows(r)[1] - layout.rows(r)[0] for r in range(world)]
    nplanes = int(getattr(backend, "nplanes", 1))
    rowsel = (lambda b, lo, hi: b[lo:hi]) if nplanes == 1 else (lambda b, lo, hi: b[:, lo:hi])
    if world > 1:
        halos = []
        for r in range(world):
            halos.append(rowsel(bufs[r], hs[r], hs[r] + layout.halo).clone())
            rowsel(bufs[r], hs[r], hs[r] + layout.halo).zero_()
        for r in range(world):
            timed(r, "halo", lambda r=r: rowsel(bufs[r], 0, layout.halo).add_(halos[(r - 1) % world]))
    if nplanes > 1:
        # per w plane: every rank's pass A, the regrouping, every rank's pass B
        # with the plane's w screen into its image rows; then the corrections
        accs = []
        for s in range(world):
            i0, i1 = layout.image_rows(s)
            accs.append(torch.empty((i1 - i0, backend.npix_y), dtype=torch.float64, device=bufs[0].device))
        for p in range(nplanes):
            Hs, lives, sends = _local_pass_a(ranks, [b[p] for b in bufs], hs, p, sparse, on_gpu, timed, backend,
                                             layout, stages)
            for s in range(world):
                i0, i1 = layout.image_rows(s)
                b0, b1 = i0 // COL_BLOCK, i1 // COL_BLOCK
                if world == 1:
                    Hm = Hs[0]
                elif sends is not None:
                    recv = torch.cat([snd[b0:b1].reshape(-1) for snd in sends[0]])
                    Hm = timed(s, "assemble", lambda b0=b0, b1=b1, recv=recv: _unpack_rows(
                        recv, b1 - b0, layout, sends[1], recv.dtype, sends[3]).to(torch.float64))
                else:
                    def regroup(b0=b0, b1=b1):
                        pieces, idx = _local_pieces(Hs, b0, b1, backend, lives)
                        return _assemble_H(pieces, b1 - b0, layout, Hs[0].device, _wire(Hs[0][:0], backend).dtype,
                                           idx).to(torch.float64)
                    Hm = timed(s, "assemble", regroup)
                timed(s, "cols", lambda s=s, Hm=Hm, i0=i0, i1=i1: ranks[s].pass_cols_wplane(
                    Hm.contiguous(), i0, i1, p, p == 0, accs[s]))
        out = []
        for s in range(world):
            ranks[s].mark_clean()
            i0, i1 = layout.image_rows(s)
            out.append(timed(s, "final", lambda s=s, i0=i0, i1=i1: ranks[s].finish_rows(accs[s], i0, i1, norm=sumw)))
        return torch.cat(out, dim=0)
    Hs, lives, sends = _local_pass_a(ranks, bufs, hs, 0, sparse, on_gpu, timed, backend, layout, stages)
    for r in range(world):
        ranks[r].mark_clean()
    out = []
    for s in range(world):
        i0, i1 = layout.image_rows(s)
        b0, b1 = i0 // COL_BLOCK, i1 // COL_BLOCK
        if world == 1:
            Hm = Hs[0]
        elif sends is not None:
            recv = torch.cat([snd[b0:b1].reshape(-1) for snd in sends[0]])
            Hm = timed(s, "assemble", lambda b0=b0, b1=b1, recv=recv: _unpack_rows(
                recv, b1 - b0, layout, sends[1], recv.dtype, sends[3]).to(torch.float64))
        else:
            def regroup(b0=b0, b1=b1):
                pieces, idx = _local_pieces(Hs, b0, b1, backend, lives)
                return _assemble_H(pieces, b1 - b0, layout, Hs[0].device, _wire(Hs[0][:0], backend).dtype,
                                   idx).to(torch.float64)
            Hm = timed(s, "assemble", regroup)
        out.append(timed(s, "cols", lambda s=s, Hm=Hm, i0=i0, i1=i1: ranks[s].pass_cols(Hm.contiguous(), i0, i1,
                                                                                         norm=sumw)))
    return torch.cat(out, dim=0)
