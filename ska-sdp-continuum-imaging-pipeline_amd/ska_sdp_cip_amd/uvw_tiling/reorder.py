"""
Reorder visibilities into UVW tile chunk files - API mirror of
`/root/reference/src/ska_sdp_cip/uvw_tiling/reorder.py`.

Two passes as in the reference (:19-111): (1) per time interval, map rows to
tiles (device `cip_tile_runs`) and write `tile_iu{u:+03d}_iv{v:+03d}_iw{w:+03d}
_interval{NN:02d}.npz`; (2) per tile, concatenate / split those files into
`..._chunk{NNN:03d}.npz` of at most `max_vis_per_chunk` visibilities and delete
the interval files. `client` is a dask Client or
`ska_sdp_cip_amd.dispatch.LocalGPUClient`.
"""

from __future__ import annotations

import itertools
from pathlib import Path
from typing import Optional

from ..dispatch import as_completed as _local_as_completed
from .tile import Tile, rechunk_tiles_on_disk
from .tiling_plan import TileCoords, TileMapping, create_uvw_tile_mapping


def _as_completed(futures):
    try:
        from dask.distributed import as_completed  # pylint: disable=import-outside-toplevel

        if futures and not hasattr(futures[0], "key"):
            raise ImportError
        return as_completed(futures)
    except ImportError:
        return _local_as_completed(futures)


def reorder_by_uvw_tile(  # pylint: disable=too-many-locals
    ms_reader,
    tile_size: TileCoords,
    outdir: Path,
    client,
    *,
    num_time_intervals: Optional[int] = None,
    max_vis_per_chunk: int = 5_000_000,
    with_weights: bool = False,
) -> list[Path]:
    """
    Convert to Stokes I and reorder into UVW tile chunk files (reference
    :19-111). Returns the written chunk paths. `with_weights=True` also stores
    each visibility's Stokes-I effective weight (flags folded in, reference
    invert.py:72-116) under the npz key `weights`; the
    reference's files carry none, and its readers ignore the extra key.
    """
    if num_time_intervals is None:
        num_time_intervals = max(2 * len(client.scheduler_info()["workers"]), 2)
    outdir = Path(outdir).resolve()
    channel_freqs = ms_reader.channel_frequencies()
    futures = []
    for interval_index, interval_reader in enumerate(ms_reader.partition(num_time_intervals, 1)):
        mapping = client.submit(create_time_interval_tile_mapping, interval_reader, tile_size, channel_freqs,
                                resources={"gpu": 1})
        futures.append(client.submit(reorder_time_interval, interval_reader, mapping, outdir,
                                     interval_index=interval_index, with_weights=with_weights))
    coords_set = set()
    for fut in _as_completed(futures):
        coords_set.update(fut.result())
    rechunk = [client.submit(rechunk_tile_chunk_group, coords, outdir, max_vis_per_chunk=max_vis_per_chunk)
               for coords in coords_set]
    return list(itertools.chain.from_iterable(f.result() for f in _as_completed(rechunk)))


def create_time_interval_tile_mapping(ms_reader, tile_size: TileCoords, channel_freqs) -> TileMapping:
    """Tile mapping of one time interval (reference :114-126)."""
    return create_uvw_tile_mapping(ms_reader.uvw(), tile_size, channel_freqs)


def reorder_time_interval(ms_reader, tile_mapping: TileMapping, outdir: Path, *,
                          interval_index: int, with_weights: bool = False) -> list[TileCoords]:
    """Write one interval's tiles; returns their coordinates (reference :129-155)."""
    uvw = ms_reader.uvw()
    vis = ms_reader.visibilities()
    stokes_i_vis = 0.5 * (vis[..., 0] + vis[..., 3])
    eff_w = None
    if with_weights:
        from ..invert import StokesIGridderInput  # pylint: disable=import-outside-toplevel

        eff_w = StokesIGridderInput.from_measurement_set_reader(ms_reader).effective_weights()
    for coords, row_slices in tile_mapping.items():
        tile = Tile._from_jagged_visibilities_slice(  # pylint: disable=protected-access
            stokes_i_vis, uvw, coords, row_slices, weights=eff_w)
        tile.save_npz(Path(outdir) / _tile_filename(coords, interval_index))
    return list(tile_mapping.keys())


def rechunk_tile_chunk_group(tile_coords: TileCoords, outdir: Path, *,
                             max_vis_per_chunk: int = 5_000_000) -> list[Path]:
    """Rechunk the interval files of one tile and delete them (reference :158-183)."""
    outdir = Path(outdir)
    base = _tile_basename(tile_coords)
    inputs = sorted(outdir.glob(f"{base}_interval*.npz"))
    out = rechunk_tiles_on_disk(inputs, outdir, base, max_vis_per_chunk=max_vis_per_chunk)
    for p in inputs:
        p.unlink()
    return out


def _tile_basename(tile_coords: TileCoords) -> str:
    u, v, w = tile_coords
    return f"tile_iu{u:+03d}_iv{v:+03d}_iw{w:+03d}"


def _tile_filename(tile_coords: TileCoords, interval_index: int) -> str:
    """Interval file name (reference :186-192)."""
    return f"{_tile_basename(tile_coords)}_interval{interval_index:02d}.npz"
