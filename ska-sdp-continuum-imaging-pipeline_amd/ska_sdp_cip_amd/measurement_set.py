"""
MeasurementSet reader protocol for the invert hot path.

Mirrors the reader interface of the reference
(`/root/reference/src/ska_sdp_cip/measurement_set.py:130-358`): row / channel
reading bounds, `partition()` into (row x freq) chunks with the reference's
balanced bounds (`:234-277`, `:361-391`), and the five data accessors that feed
`StokesIGridderInput` (`uvw`, `visibilities`, `flags`, `weights`,
`channel_frequencies`).

Two back-ends share the bounds/partition logic (`_BoundedReader`):

* `MeasurementSetReader(path)` - the on-disk MSv2 reader. It needs
  python-casacore, which is absent from this image and the GPU box; the casacore
  table I/O is OUT OF SCOPE for this build. Construction
  raises `ModuleNotFoundError` when casacore is missing, `FileNotFoundError` for a
  missing directory (reference `:67-72`).
* `InMemoryMeasurementSet` - numpy-backed columns with the exact shapes and dtypes
  casacore returns (uvw (r,3) f64, DATA (r,c,4) c64, FLAG (r,c,4) bool,
  WEIGHT_SPECTRUM (r,c,4) f32 or WEIGHT (r,4) f32, CHAN_FREQ (c,) f64). The
  synthetic generator (`synthetic.py`) produces these.
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import Iterator, Optional, Union

import numpy as np
from numpy.typing import NDArray


class UnsupportedMeasurementSetLayout(Exception):
    """
    Raised when a MeasurementSet layout deviates from what is supported
    (reference `measurement_set.py:12-16`).
    """


def balanced_chunk_sizes(n: int, k: int) -> Iterator[int]:
    """
    Sizes of `k` chunks of a population of `n`, as balanced as possible; the
    first `n % k` chunks get one extra element
    (reference `measurement_set.py:361-376`).
    """
    if not n > 0:
        raise ValueError("n must be > 0")
    if not 0 < k <= n:
        raise ValueError("k must be > 0 and <= n")
    base, extra = divmod(n, k)
    for i in range(k):
        yield base + (1 if i < extra else 0)


def balanced_chunk_bounds(
    start: int, end: int, k: int
) -> Iterator[tuple[int, int]]:
    """
    (start, end) bounds of `k` balanced chunks of the index range
    [start, end) (reference `measurement_set.py:379-391`).
    """
    lo = start
    for size in balanced_chunk_sizes(end - start, k):
        yield lo, lo + size
        lo += size


class _BoundedReader:
    """
    Row / channel bounds and partitioning shared by every reader back-end.
    Semantics follow reference `measurement_set.py:167-277`: bounds are
    clipped to the data extent, start inclusive, end exclusive.
    """

    _total_rows: int
    _total_channels: int

    def _init_bounds(self) -> None:
        self._row_start = 0
        self._row_end = self._total_rows
        self._channel_start = 0
        self._channel_end = self._total_channels

    @property
    def row_start(self) -> int:
        """Absolute start row index."""
        return self._row_start

    @property
    def row_end(self) -> int:
        """Absolute end row index (exclusive)."""
        return self._row_end

    @property
    def num_data_rows(self) -> int:
        """Number of rows within reading bounds."""
        return self.row_end - self.row_start

    @property
    def channel_start(self) -> int:
        """Absolute start channel index."""
        return self._channel_start

    @property
    def channel_end(self) -> int:
        """Absolute end channel index (exclusive)."""
        return self._channel_end

    @property
    def num_channels(self) -> int:
        """Number of channels within reading bounds (a property, as in
        reference `measurement_set.py:208-213`)."""
        return self.channel_end - self.channel_start

    def set_row_bounds(self, row_start: int, row_end: int) -> None:
        """Clip and set row bounds (reference `:217-223`)."""
        self._row_start = max(row_start, 0)
        self._row_end = min(row_end, self._total_rows)

    def set_channel_bounds(self, channel_start: int, channel_end: int) -> None:
        """Clip and set channel bounds (reference `:225-232`)."""
        self._channel_start = max(channel_start, 0)
        self._channel_end = min(channel_end, self._total_channels)

    def _clone_unbounded(self) -> "_BoundedReader":
        raise NotImplementedError

    def partition(
        self, row_chunks: int, freq_chunks: int
    ) -> list["_BoundedReader"]:
        """
        Partition into `row_chunks` x `freq_chunks` readers, rows outer and
        channels inner (reference `measurement_set.py:234-277`). Raises
        ValueError when a chunk count is outside [1, extent].
        """
        if not 1 <= row_chunks <= self.num_data_rows:
            raise ValueError(
                "Number of row chunks must be within [1, total data rows]"
            )
        if not 1 <= freq_chunks <= self.num_channels:
            raise ValueError(
                "Number of row chunks must be within [1, total freq channels]"
            )
        result = []
        for r0, r1 in balanced_chunk_bounds(
            self.row_start, self.row_end, row_chunks
        ):
            for c0, c1 in balanced_chunk_bounds(
                self.channel_start, self.channel_end, freq_chunks
            ):
                reader = self._clone_unbounded()
                reader.set_row_bounds(r0, r1)
                reader.set_channel_bounds(c0, c1)
                result.append(reader)
        return result


class InMemoryMeasurementSet(_BoundedReader):
    """
    A MeasurementSet held in memory as casacore-shaped numpy columns.

    Parameters
    ----------
    uvw : (nrow, 3) float64, metres
    visibilities : (nrow, nchan, 4) complex64 (XX, XY, YX, YY or RR, RL, LR, LL)
    flags : (nrow, nchan, 4) bool
    weights : (nrow, nchan, 4) float32 (WEIGHT_SPECTRUM) or (nrow, 4) float32
        (WEIGHT only; repeated over channels exactly like the reference's
        fallback, `measurement_set.py:345-358`)
    channel_frequencies : (nchan,) float64, Hz
    """

    def __init__(
        self,
        uvw: NDArray,
        visibilities: NDArray,
        flags: NDArray,
        weights: NDArray,
        channel_frequencies: NDArray,
    ) -> None:
        nrow, nchan = visibilities.shape[:2]
        if uvw.shape != (nrow, 3):
            raise ValueError(f"uvw shape {uvw.shape} != ({nrow}, 3)")
        if visibilities.shape != (nrow, nchan, 4):
            raise UnsupportedMeasurementSetLayout(
                "Visibilities must have 4 correlation products"
            )
        if flags.shape != (nrow, nchan, 4):
            raise ValueError("flags shape mismatch")
        if weights.shape not in ((nrow, nchan, 4), (nrow, 4)):
            raise ValueError("weights shape mismatch")
        if channel_frequencies.shape != (nchan,):
            raise ValueError("channel_frequencies shape mismatch")
        self._uvw = np.ascontiguousarray(uvw, dtype=np.float64)
        self._vis = np.ascontiguousarray(visibilities, dtype=np.complex64)
        self._flags = np.ascontiguousarray(flags, dtype=bool)
        self._weights = np.ascontiguousarray(weights, dtype=np.float32)
        self._freqs = np.ascontiguousarray(channel_frequencies, dtype=np.float64)
        self._total_rows = nrow
        self._total_channels = nchan
        self._init_bounds()

    _NPZ_KEYS = ("uvw", "visibilities", "flags", "weights", "channel_frequencies")

    def save_npz(self, path: Union[str, os.PathLike]) -> None:
        """Write the whole set's columns to an .npz file (a stand-in for an MS
        directory where python-casacore is absent; `open_measurement_set`)."""
        np.savez(path, uvw=self._uvw, visibilities=self._vis, flags=self._flags, weights=self._weights,
                 channel_frequencies=self._freqs)

    @classmethod
    def load_npz(cls, path: Union[str, os.PathLike]) -> "InMemoryMeasurementSet":
        """Read a set written by `save_npz` (plain arrays, no pickles)."""
        with np.load(path, allow_pickle=False) as z:
            return cls(*(z[k] for k in cls._NPZ_KEYS))

    def _clone_unbounded(self) -> "InMemoryMeasurementSet":
        clone = object.__new__(InMemoryMeasurementSet)
        clone.__dict__.update(self.__dict__)
        clone._init_bounds()
        return clone

    @property
    def path(self) -> Optional[Path]:
        """In-memory sets have no path on disk."""
        return None

    def _rows(self) -> slice:
        return slice(self.row_start, self.row_end)

    def _chans(self) -> slice:
        return slice(self.channel_start, self.channel_end)

    def channel_frequencies(self) -> NDArray:
        """Channel frequencies in Hz, shape (nchan,)."""
        return self._freqs[self._chans()].copy()

    def uvw(self) -> NDArray:
        """UVW coordinates in metres, shape (nrows, 3)."""
        return self._uvw[self._rows()].copy()

    def flags(self) -> NDArray:
        """Flags, bool (nrows, nchan, 4)."""
        return self._flags[self._rows(), self._chans()].copy()

    def visibilities(self) -> NDArray:
        """Visibilities, complex64 (nrows, nchan, 4)."""
        return self._vis[self._rows(), self._chans()].copy()

    def weights(self) -> NDArray:
        """
        Weights, float32 (nrows, nchan, 4); a WEIGHT-only set is repeated along
        the frequency axis (reference `measurement_set.py:345-358`).
        """
        if self._weights.ndim == 3:
            return self._weights[self._rows(), self._chans()].copy()
        data = self._weights[self._rows()]
        return np.repeat(data[:, None, :], self.num_channels, axis=1)

    def read_into(self, out: dict, row0: int = 0, row1: Optional[int] = None) -> None:
        """
        Copy rows [row0, row1) of this (bounded) set's columns straight into
        caller-owned arrays - e.g. pinned staging buffers - instead of
        returning fresh ones (the streaming path; a casacore
        reader does the same with `getcolnp(column, out, startrow, nrow)`).
        `out` holds any of "uvw" (n, 3) float64, "vis4" (n, nchan, 4)
        complex64, "flags4" (n, nchan, 4) uint8 or bool, "wgt4" (n, nchan, 4)
        float32 with n = row1 - row0 rows. Called on disjoint row ranges from
        several threads at once (numpy releases the GIL for the copies).
        """
        row1 = self.num_data_rows if row1 is None else row1
        a, b = self.row_start + row0, self.row_start + row1
        ch = self._chans()
        if "uvw" in out:
            np.copyto(out["uvw"], self._uvw[a:b])
        if "vis4" in out:
            np.copyto(out["vis4"], self._vis[a:b, ch])
        if "flags4" in out:
            dst = out["flags4"]
            np.copyto(dst.view(np.bool_) if dst.dtype == np.uint8 else dst, self._flags[a:b, ch])
        if "wgt4" in out:
            if self._weights.ndim == 3:
                np.copyto(out["wgt4"], self._weights[a:b, ch])
            else:
                np.copyto(out["wgt4"], self._weights[a:b, None, :])


def open_measurement_set(path: Union[str, os.PathLike]) -> _BoundedReader:
    """A reader for `path`: an .npz column file (`InMemoryMeasurementSet.
    save_npz`) or a MeasurementSet v2 directory (`MeasurementSetReader`,
    which needs python-casacore)."""
    p = Path(path)
    if p.suffix == ".npz":
        return InMemoryMeasurementSet.load_npz(p)
    return MeasurementSetReader(p)


class MeasurementSetReader(_BoundedReader):
    """
    On-disk MeasurementSet v2 reader (reference `measurement_set.py:130-358`).

    The casacore table back-end is out of scope for this build: this class
    only validates the path and requires python-casacore, which is not installed
    here or on the GPU box. Use `InMemoryMeasurementSet` (or the synthetic
    generator) for the invert path.
    """

    def __init__(
        self, path: Union[str, os.PathLike], *, validate_layout: bool = True
    ) -> None:
        self._path = Path(path).resolve()
        if not self._path.is_dir():
            raise FileNotFoundError(
                "Cannot initialise MeasurementSet: path is not a directory: "
                f"{self._path}"
            )
        try:
            from casacore.tables import table  # noqa: F401  pylint: disable=import-outside-toplevel
        except ModuleNotFoundError as err:
            raise ModuleNotFoundError(
                "python-casacore is required to read MeasurementSets from disk; "
                "it is not part of this build (use InMemoryMeasurementSet)"
            ) from err
        raise NotImplementedError(
            "casacore-backed reading is out of scope for this build"
        )

    @property
    def path(self) -> Path:
        """Absolute path on disk."""
        return self._path
