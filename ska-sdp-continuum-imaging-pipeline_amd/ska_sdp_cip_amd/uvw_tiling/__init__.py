"""UVW tiling - public surface of `/root/reference/src/ska_sdp_cip/uvw_tiling/__init__.py:1-17`."""

from .reorder import reorder_by_uvw_tile
from .tile import Tile, concatenate_tiles, rechunk_tiles_on_disk, split_tile
from .tiling_plan import (
    RowSliceId,
    TileCoords,
    TileMapping,
    create_uvw_tile_mapping,
    create_uvw_tile_mapping_sequential,
    merge_tile_mappings,
)

__all__ = [
    "create_uvw_tile_mapping",
    "create_uvw_tile_mapping_sequential",
    "merge_tile_mappings",
    "reorder_by_uvw_tile",
    "RowSliceId",
    "TileCoords",
    "TileMapping",
    "Tile",
    "concatenate_tiles",
    "rechunk_tiles_on_disk",
    "split_tile",
]
