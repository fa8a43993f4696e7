"""
ska_sdp_cip_amd - MI355X-native invert hot path of ska_sdp_cip.

Public API mirrors `/root/reference/src/ska_sdp_cip/__init__.py:1-10`
(`MeasurementSetReader`, `invert_measurement_set`,
`dask_invert_measurement_set`, `__version__`) plus the drop-in gridder
`ms2dirty` (replaces `ducc0.wgridder.ms2dirty`) and the `uvw_tiling` package.
"""

__version__ = "0.1.0"

from .gridder import ms2dirty  # noqa: E402
from .invert import (  # noqa: E402
    StokesIGridderInput,
    dask_invert_measurement_set,
    ducc_invert,
    integrate_weighted_images,
    invert_measurement_set,
)
from .measurement_set import (  # noqa: E402
    InMemoryMeasurementSet,
    MeasurementSetReader,
    UnsupportedMeasurementSetLayout,
)

# Load libcip_hip.so at import, on the importing thread, when it is built: the
# library records the thread that loads it as the main thread (whose workspaces
# are left to process teardown, cip_api.hip), so the first call from a worker
# thread must not be the one that loads it. A missing library raises at the
# first call instead (no CPU fallback).
try:
    from . import _lib as _cip_lib

    if _cip_lib.LIB_PATH.exists():
        _cip_lib.lib()
except OSError:  # pragma: no cover - a broken build raises again at first use
    pass

__all__ = [
    "__version__",
    "MeasurementSetReader",
    "InMemoryMeasurementSet",
    "UnsupportedMeasurementSetLayout",
    "StokesIGridderInput",
    "dask_invert_measurement_set",
    "ducc_invert",
    "integrate_weighted_images",
    "invert_measurement_set",
    "ms2dirty",
]
