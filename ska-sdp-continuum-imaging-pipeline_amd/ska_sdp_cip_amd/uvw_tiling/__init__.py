"""
UVW tiling: tile keys and row slices of a measurement set, the on-disk `Tile`
chunk format and the two-pass reorder.

Exposes the names of the reference package
(`/root/reference/src/ska_sdp_cip/uvw_tiling/__init__.py:1-17`) plus the
helpers the device gridder's streaming path uses (`split_tile`,
`concatenate_tiles`, `rechunk_tiles_on_disk`, the sequential mapping and the
merge), each re-exported from the submodule that defines it.
"""

from importlib import import_module

# submodule -> the public names it provides
_PUBLIC = {
    "tiling_plan": (
        "RowSliceId",
        "TileCoords",
        "TileMapping",
        "create_uvw_tile_mapping",
        "create_uvw_tile_mapping_sequential",
        "merge_tile_mappings",
    ),
    "tile": ("Tile", "concatenate_tiles", "rechunk_tiles_on_disk", "split_tile"),
    "reorder": ("reorder_by_uvw_tile",),
}

for _sub, _names in _PUBLIC.items():
    _module = import_module(f"{__name__}.{_sub}")
    globals().update({_n: getattr(_module, _n) for _n in _names})

__all__ = sorted(_n for _names in _PUBLIC.values() for _n in _names)

del _sub, _names, _module
