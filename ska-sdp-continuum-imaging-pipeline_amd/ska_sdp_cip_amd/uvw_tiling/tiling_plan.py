"""
UVW tiling plan - API mirror of
`/root/reference/src/ska_sdp_cip/uvw_tiling/tiling_plan.py`.

The per-(row, channel) tile keys and their constant runs along the channel
axis are computed on the GPU by `cip_tile_runs` (libcip_hip.so), bit-exact with
the reference's `floor(f/c * (uvw / tile_size) + 0.5)` (tiling_plan.py:41-51).
The host only groups the runs into the reference's dict-of-lists shape:
tiles in first-appearance order, row slices ascending in `irow` within a tile
(which is what the reference's row loop and in-order chunk merge produce,
tiling_plan.py:46-61, :137-147).
"""

from __future__ import annotations

import ctypes
import os
from typing import NamedTuple

import numpy as np
from numpy.typing import NDArray

from .. import _lib

TileCoords = tuple[int, int, int]
"""Tile index of the form (iu, iv, iw) (reference :10-13)."""


class RowSliceId(NamedTuple):
    """A slice of one visibility row along the frequency axis (reference :16-23)."""

    irow: int
    chan_start: int
    chan_stop: int


TileMapping = dict[TileCoords, list[RowSliceId]]


def tile_runs(uvw, tile_size, channel_freqs, *, row_offset: int = 0):
    """
    Device computation of all constant-key channel runs, rows in order.
    Returns numpy arrays (keys (n,3) int64, irow (n,) int64, c0, c1 (n,) int32).
    """
    import torch  # pylint: disable=import-outside-toplevel

    if not torch.cuda.is_available():
        raise RuntimeError("create_uvw_tile_mapping needs a ROCm GPU (no CPU fallback)")
    uvw = np.ascontiguousarray(uvw, dtype=np.float64).reshape(-1, 3)
    freqs = np.ascontiguousarray(channel_freqs, dtype=np.float64).ravel()
    if freqs.size == 0:
        raise ValueError("channel_freqs must not be empty")
    ts = (ctypes.c_double * 3)(*[float(t) for t in tile_size])
    nrow, nchan = uvw.shape[0], freqs.size
    dev = torch.device("cuda", torch.cuda.current_device())
    uvw_d = torch.from_numpy(uvw).to(dev)
    f_d = torch.from_numpy(freqs).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    n = ctypes.c_int64(0)
    so = _lib.lib()
    _lib.check(so.cip_tile_runs(uvw_d.data_ptr(), nrow, f_d.data_ptr(), nchan, ts, int(row_offset), stream,
                                ctypes.byref(n), None, None, None, None))
    total = n.value
    key = torch.empty((max(total, 1), 3), dtype=torch.int64, device=dev)
    row = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    c0 = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    c1 = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    if total:
        _lib.check(so.cip_tile_runs(uvw_d.data_ptr(), nrow, f_d.data_ptr(), nchan, ts, int(row_offset), stream,
                                    ctypes.byref(n), key.data_ptr(), row.data_ptr(), c0.data_ptr(),
                                    c1.data_ptr()))
    return (key[:total].cpu().numpy(), row[:total].cpu().numpy(), c0[:total].cpu().numpy(),
            c1[:total].cpu().numpy())


def group_runs(keys: NDArray, irow: NDArray, c0: NDArray, c1: NDArray) -> TileMapping:
    """Runs (rows in order) -> {coords: [RowSliceId, ...]} in first-appearance order."""
    if len(keys) == 0:
        return {}
    uniq, first, inverse = np.unique(keys, axis=0, return_index=True, return_inverse=True)
    inverse = inverse.ravel()
    rank = np.empty(len(first), dtype=np.int64)
    rank[np.argsort(first, kind="stable")] = np.arange(len(first))
    tile_rank = rank[inverse]
    order = np.argsort(tile_rank, kind="stable")  # stable: rows stay ascending
    bounds = np.searchsorted(tile_rank[order], np.arange(len(first) + 1))
    irow_l = irow[order].tolist()
    c0_l = c0[order].tolist()
    c1_l = c1[order].tolist()
    coords_by_rank = uniq[np.argsort(first, kind="stable")].tolist()
    mapping: TileMapping = {}
    for t, coords in enumerate(coords_by_rank):
        lo, hi = bounds[t], bounds[t + 1]
        mapping[tuple(coords)] = [RowSliceId(r, a, b) for r, a, b in
                                  zip(irow_l[lo:hi], c0_l[lo:hi], c1_l[lo:hi])]
    return mapping


def create_uvw_tile_mapping_sequential(
    uvw: NDArray,
    tile_size: tuple[float, float, float],
    channel_freqs: NDArray,
    *,
    row_offset: int = 0,
) -> TileMapping:
    """Bin UVW coordinates by UVW tile (reference :29-61); device-computed."""
    return group_runs(*tile_runs(uvw, tile_size, channel_freqs, row_offset=row_offset))


class TileMappingCreator:
    """Callable over (uvw chunk, row offset) pairs (reference :64-81)."""

    def __init__(self, tile_size: tuple[float, float, float], channel_freqs: NDArray) -> None:
        self.tile_size = tile_size
        self.channel_freqs = channel_freqs

    def __call__(self, chunk_and_offset: tuple[NDArray, int]) -> TileMapping:
        uvw, row_offset = chunk_and_offset
        return create_uvw_tile_mapping_sequential(uvw, self.tile_size, self.channel_freqs,
                                                  row_offset=row_offset)


def create_uvw_tile_mapping(
    uvw: NDArray,
    tile_size: tuple[float, float, float],
    channel_freqs: NDArray,
    *,
    processes: int = os.cpu_count(),  # noqa: ARG001 - one device launch covers every row
) -> TileMapping:
    """
    Bin the UVW coordinates of visibilities by UVW tile (reference :84-134).
    The reference splits rows over a multiprocessing pool; here one device
    launch processes every row and `processes` is accepted for compatibility.
    The tile with coordinates (i, j, k) is centred on (i Du, j Dv, k Dw).
    """
    return create_uvw_tile_mapping_sequential(uvw, tile_size, channel_freqs)


def merge_tile_mappings(tile_mappings: list[TileMapping]) -> TileMapping:
    """Concatenate per-chunk mappings in order (reference :137-147)."""
    result: TileMapping = {}
    for mapping in tile_mappings:
        for coords, row_slices in mapping.items():
            result.setdefault(coords, []).extend(row_slices)
    return result
