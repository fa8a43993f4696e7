"""
Tile container and on-disk chunking - API mirror of
`/root/reference/src/ska_sdp_cip/uvw_tiling/tile.py` (the tile data format on
either side of the hot path).

npz layout (reference :40-65): coords int64 (3,), uvw f64 (nslices, 3),
visibilities complex64 (nvis,), channel_start_indices / channel_stop_indices
int64 (nslices,). Optional extension: `weights`
float32 (nvis,) effective weights, written only when present and ignored by
readers that do not know it (the reference's load_npz reads keys by name).
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path
from typing import Iterable, Optional, Sequence, Union

import numpy as np
from numpy.typing import NDArray

from .tiling_plan import RowSliceId, TileCoords

_ARRAYS = ("uvw", "visibilities", "channel_start_indices", "channel_stop_indices")


@dataclass(repr=False)
class Tile:
    """Visibility data and metadata of one UVW tile (reference :14-124)."""

    coords: TileCoords
    uvw: NDArray
    visibilities: NDArray
    channel_start_indices: NDArray
    channel_stop_indices: NDArray
    weights: Optional[NDArray] = None

    @property
    def num_rows(self) -> int:
        """Number of row slices stored."""
        return len(self.uvw)

    @property
    def num_visibilities(self) -> int:
        """Number of visibilities stored."""
        return len(self.visibilities)

    def slice_sizes(self) -> NDArray:
        """Visibilities per row slice."""
        return np.asarray(self.channel_stop_indices) - np.asarray(self.channel_start_indices)

    def save_npz(self, path: Union[str, os.PathLike]) -> None:
        """Save in numpy's npz format (reference :40-51)."""
        items = {
            "coords": np.asarray(self.coords).astype(int),
            "uvw": self.uvw,
            "visibilities": self.visibilities,
            "channel_start_indices": self.channel_start_indices,
            "channel_stop_indices": self.channel_stop_indices,
        }
        if self.weights is not None:
            items["weights"] = self.weights
        np.savez(path, **items)

    @classmethod
    def load_npz(cls, path: Union[str, os.PathLike]) -> "Tile":
        """Load from an npz file (reference :53-65); plain data only."""
        with np.load(path, allow_pickle=False) as npz:
            return cls(
                coords=tuple(int(c) for c in npz["coords"]),
                uvw=npz["uvw"],
                visibilities=npz["visibilities"],
                channel_start_indices=npz["channel_start_indices"],
                channel_stop_indices=npz["channel_stop_indices"],
                weights=npz["weights"] if "weights" in npz.files else None,
            )

    @classmethod
    def _zeros(cls, coords: TileCoords, num_row_slices: int, num_vis: int) -> "Tile":
        """Zero-filled tile (reference :67-81)."""
        return cls(
            coords=coords,
            uvw=np.zeros((num_row_slices, 3), dtype=float),
            visibilities=np.zeros(num_vis, dtype=np.complex64),
            channel_start_indices=np.zeros(num_row_slices, dtype=int),
            channel_stop_indices=np.zeros(num_row_slices, dtype=int),
        )

    @classmethod
    def _from_jagged_visibilities_slice(
        cls,
        vis: NDArray,
        uvw: NDArray,
        coords: TileCoords,
        row_slices: list[RowSliceId],
        weights: Optional[NDArray] = None,
    ) -> "Tile":
        """
        Gather the row slices of a (row, freq) block into one tile (reference
        :83-115), vectorised: one fancy-index gather instead of a slice loop.
        """
        if not row_slices:
            return cls._zeros(coords, 0, 0)
        rs = np.asarray(row_slices, dtype=np.int64).reshape(-1, 3)
        irow, start, stop = rs[:, 0], rs[:, 1], rs[:, 2]
        sizes = stop - start
        offsets = np.concatenate(([0], np.cumsum(sizes)))
        slice_of = np.repeat(np.arange(len(rs)), sizes)
        chan = start[slice_of] + (np.arange(offsets[-1]) - offsets[slice_of])
        rows = irow[slice_of]
        tile_vis = np.asarray(vis)[rows, chan].astype(np.complex64, copy=False)
        return cls(
            coords=coords,
            uvw=np.asarray(uvw, dtype=float)[irow],
            visibilities=tile_vis,
            channel_start_indices=start.astype(int),
            channel_stop_indices=stop.astype(int),
            weights=None if weights is None else np.asarray(weights, dtype=np.float32)[rows, chan],
        )

    def __str__(self) -> str:
        return f"Tile(coords={self.coords}, nrows={self.num_rows}, nvis={self.num_visibilities})"

    def __repr__(self) -> str:
        return str(self)


def concatenate_tiles(tiles: Sequence[Tile]) -> Tile:
    """Concatenate tiles of identical coordinates (reference :127-152)."""
    if not tiles:
        raise ValueError("Cannot concatenate empty sequence of tiles")
    coords = tiles[0].coords
    if any(t.coords != coords for t in tiles):
        raise ValueError("Cannot merge tiles with different coordinates")
    attrs = {name: np.concatenate([getattr(t, name) for t in tiles]) for name in _ARRAYS}
    weights = None
    if all(t.weights is not None for t in tiles):
        weights = np.concatenate([t.weights for t in tiles])
    return Tile(coords=coords, weights=weights, **attrs)


def _split_points(sizes: NDArray, max_vis: int) -> list[int]:
    """
    Row-slice indices where chunks start, greedily packing at most `max_vis`
    visibilities per chunk, never splitting a row slice and never emitting an
    empty chunk (same chunks as reference split_tile :155-211).
    """
    csum = np.concatenate(([0], np.cumsum(sizes)))
    n = len(sizes)
    points, r0 = [0], 0
    while True:
        # last r1 with csum[r1] - csum[r0] <= max_vis, at least one slice
        r1 = int(np.searchsorted(csum, csum[r0] + max_vis, side="right")) - 1
        r1 = max(r1, r0 + 1)
        if r1 >= n:
            break
        points.append(r1)
        r0 = r1
    return points


def split_tile(tile: Tile, max_vis_per_chunk: int) -> list[Tile]:
    """Split into chunks of at most `max_vis_per_chunk` visibilities (reference :155-211)."""
    sizes = tile.slice_sizes()
    if len(sizes) == 0:
        return []
    points = _split_points(sizes, max_vis_per_chunk)
    voff = np.concatenate(([0], np.cumsum(sizes)))
    out = []
    for a, b in zip(points, points[1:] + [len(sizes)]):
        out.append(Tile(
            coords=tile.coords,
            uvw=tile.uvw[a:b],
            visibilities=tile.visibilities[voff[a]:voff[b]],
            channel_start_indices=tile.channel_start_indices[a:b],
            channel_stop_indices=tile.channel_stop_indices[a:b],
            weights=None if tile.weights is None else tile.weights[voff[a]:voff[b]],
        ))
    return out


def rechunk_tiles_on_disk(
    tile_paths: Iterable[Path],
    outdir: Path,
    basename: str,
    *,
    max_vis_per_chunk: int = 5_000_000,
) -> list[Path]:
    """
    Rewrite same-coordinate tile files as `{basename}_chunk{NNN:03d}.npz` files
    of at most `max_vis_per_chunk` visibilities each (unless a single row slice
    is larger), in input order (reference :214-265).
    """
    outdir = Path(outdir)
    written: list[Path] = []
    pending: list[Tile] = []

    def emit(t: Tile) -> None:
        path = outdir / f"{basename}_chunk{len(written):03d}.npz"
        t.save_npz(path)
        written.append(path)

    for path in tile_paths:
        pending.append(Tile.load_npz(path))
        total = sum(t.num_visibilities for t in pending)
        if total <= max_vis_per_chunk:
            continue
        merged = concatenate_tiles(pending) if len(pending) > 1 else pending[0]
        parts = split_tile(merged, max_vis_per_chunk)
        for part in parts[:-1]:
            emit(part)
        pending = [parts[-1]]
    if len(pending) > 1:
        pending = [concatenate_tiles(pending)]
    for t in pending:
        emit(t)
    return written
