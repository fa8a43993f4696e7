"""
Chunked host -> HBM streaming invert (config C5's
"chunked-MS host->HBM streaming").

Two sources, one pipeline:

* `invert_tile_files` - uvw_tiling chunk files (`tile_..._chunkNNN.npz`, the
  reorder output of reference uvw_tiling/reorder.py:19-111, optional
  `weights` key), gridded slice-wise by `cip_grid_tiles`;
* `invert_measurement_set_streamed` - row blocks of a measurement set reader
  (raw (rows, chans, 4) columns read straight into pinned slots by the
  reader's `read_into`; Stokes I formed inside the gridder,
  `cip_grid_ms_stokes_i`), `RowStreamer`.

Pipeline: while chunk k is gridded on the compute stream onto the resident
planes of a `GridAccumulator`, later chunks are read into pinned staging
slots and sent to HBM on a dedicated copy stream. One FFT at the end.
"""

from __future__ import annotations

import concurrent.futures as cf
import threading
from pathlib import Path
from typing import Callable, Iterable, Optional, Sequence

import numpy as np

from .accumulate import GridAccumulator, merge_w_ranges, w_range_rows, w_range_slices
from .gridder import _require_gpu
from .invert import EPSILON, pixel_size_lm
from .uvw_tiling.tile import Tile

try:
    import torch
except ModuleNotFoundError:  # pragma: no cover - torch is in the image
    torch = None

_TORCH_DTYPES = {}


def _torch_dtype(dt: np.dtype):
    if not _TORCH_DTYPES:
        _TORCH_DTYPES.update({np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32,
                              np.dtype(np.complex64): torch.complex64, np.dtype(np.complex128): torch.complex128,
                              np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                              np.dtype(np.uint8): torch.uint8, np.dtype(np.bool_): torch.uint8})
    return _TORCH_DTYPES[np.dtype(dt)]


class ChunkStager:
    """
    Pinned host slots + device slots, filled on a copy stream. `stage(slot,
    arrays)` copies numpy arrays into slot `slot`'s pinned buffers and issues
    their host->device copies on the copy stream; `wait(slot)` orders the
    current (compute) stream after them. A slot is reused only after the
    gridding call that read it returned (the gridder calls are synchronous).
    """

    # host copies into the pinned slots are split over threads (one numpy copy
    # runs at ~6 GB/s and capped the pipeline; numpy releases the GIL for them)
    _COPY_PIECE = 8 << 20
    _pool = None

    def __init__(self, device, nslots: int = 2, copy_threads: int = 8):
        self.device = torch.device(device)
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self._host = [dict() for _ in range(nslots)]
        self._dev = [dict() for _ in range(nslots)]
        self._ready = [None] * nslots
        self.bytes_staged = 0
        if ChunkStager._pool is None and copy_threads > 1:
            ChunkStager._pool = cf.ThreadPoolExecutor(max_workers=copy_threads)

    @classmethod
    def _copy(cls, dst: np.ndarray, src: np.ndarray) -> None:
        n = src.size
        if cls._pool is None or n <= cls._COPY_PIECE:
            dst[:] = src
            return
        step = max(cls._COPY_PIECE, -(-n // 32))
        list(cls._pool.map(lambda a: np.copyto(dst[a:a + step], src[a:a + step]), range(0, n, step)))

    @staticmethod
    def _grow(pool: dict, name: str, nbytes: int, **kw):
        t = pool.get(name)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 1) + max(nbytes, 1) // 8, dtype=torch.uint8, **kw)
            pool[name] = t
        return t

    def stage(self, slot: int, arrays: dict) -> dict:
        out = {}
        with torch.cuda.stream(self.copy_stream):
            for name, a in arrays.items():
                a = np.ascontiguousarray(a)
                if a.dtype == np.bool_:
                    a = a.view(np.uint8)
                nb = a.nbytes
                h = self._grow(self._host[slot], name, nb, pin_memory=True)[:nb]
                if nb:
                    self._copy(h.numpy(), a.reshape(-1).view(np.uint8))
                d = self._grow(self._dev[slot], name, nb, device=self.device)[:nb]
                d.copy_(h, non_blocking=True)
                out[name] = d.view(_torch_dtype(a.dtype)).view(a.shape)
                self.bytes_staged += nb
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        self._ready[slot] = ev
        return out

    def wait(self, slot: int) -> None:
        torch.cuda.current_stream(self.device).wait_event(self._ready[slot])


def _pipeline(loaders: Sequence[Callable[[], dict]], stager: ChunkStager, consume: Callable[[dict], None],
              readers: int = 4) -> None:
    """
    Read on `readers` threads (up to that many chunks ahead: a reader's copy
    out of the measurement set or an npz file is single-threaded, ~3-6 GB/s),
    stage in order on one thread (pinned slot -> copy stream), consume on the
    caller's thread (compute stream). Chunk k + 1 is staged while chunk k is
    gridded; chunk k + 2's staging is queued only once chunk k's (synchronous)
    gridding returned, since it reuses chunk k's slot.
    """
    n = len(loaders)
    if n == 0:
        return
    with cf.ThreadPoolExecutor(max_workers=max(1, readers)) as rpool, \
            cf.ThreadPoolExecutor(max_workers=1) as spool:
        reads = {}

        def read_upto(k):
            for j in range(k):
                if j < n and j not in reads:
                    reads[j] = rpool.submit(loaders[j])

        def job(k):
            arrays = reads[k].result()
            with torch.cuda.device(stager.device):
                return stager.stage(k % 2, arrays)

        read_upto(readers + 1)
        pending = {k: spool.submit(job, k) for k in range(min(2, n))}
        for k in range(n):
            staged = pending.pop(k).result()
            reads.pop(k, None)
            read_upto(k + readers + 2)
            stager.wait(k % 2)
            consume(staged)
            if k + 2 < n:
                pending[k + 2] = spool.submit(job, k + 2)


def _npz_w_range(path, freq) -> tuple[float, float]:
    with np.load(path, allow_pickle=False) as z:
        return w_range_slices(z["uvw"], z["channel_start_indices"], z["channel_stop_indices"], freq)


def invert_tile_files(
    paths: Iterable,
    channel_freqs: np.ndarray,
    num_pixels: int,
    pixel_size_asec: float,
    *,
    epsilon: float = EPSILON,
    support: Optional[int] = None,
    do_wstacking: bool = False,
    w_range: Optional[tuple[float, float]] = None,
    use_weights: bool = True,
    device=None,
    return_weight: bool = False,
):
    """
    Dirty image (normalised, float64 numpy (N, N)) of the visibilities held
    in uvw_tiling tile chunk files, streamed through HBM chunk by chunk. Tiles
    without a `weights` key (the reference's format) grid with unit weights;
    `use_weights=False` ignores the key. In w-stacking mode the w range of all
    files is read first (their uvw and channel ranges only) unless given.
    """
    _require_gpu()
    paths = [Path(p) for p in paths]
    freq = np.asarray(channel_freqs, dtype=np.float64)
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if do_wstacking and w_range is None:
        w_range = merge_w_ranges(_npz_w_range(p, freq) for p in paths)
    pix = pixel_size_lm(pixel_size_asec)
    acc = GridAccumulator(num_pixels, num_pixels, pix, pix, epsilon=epsilon, support=support,
                          do_wstacking=do_wstacking, w_range=w_range or (0.0, 0.0), device=dev)
    freq_d = torch.from_numpy(freq).to(dev)

    def loader(path):
        def load():
            t = Tile.load_npz(path)
            arrays = {"uvw": np.asarray(t.uvw, dtype=np.float64).reshape(-1, 3),
                      "c0": np.asarray(t.channel_start_indices, dtype=np.int32),
                      "c1": np.asarray(t.channel_stop_indices, dtype=np.int32),
                      "vis": np.asarray(t.visibilities, dtype=np.complex64)}
            if use_weights and t.weights is not None:
                arrays["wgt"] = np.asarray(t.weights, dtype=np.float32)
            return arrays
        return load

    def consume(c):
        acc.add_tile(c["uvw"], c["c0"], c["c1"], freq_d, c["vis"], c.get("wgt"))

    with torch.cuda.device(dev):
        _pipeline([loader(p) for p in paths], ChunkStager(dev), consume)
        dirty, sumw = acc.dirty()
        image = (dirty / sumw).cpu().numpy()
    if return_weight:
        return image, float(sumw.item())
    return image


class RowStreamer:
    """
    Raw MS rows host -> HBM at link speed: the reader fills
    pinned staging slots directly (`read_into`, several threads on disjoint
    row blocks - no fresh arrays, no second host copy), a copy stream moves
    each filled slot to a device slot, and the caller grids it from there.

    Three pinned slots and two device slots: while chunk k grids on the
    compute stream (synchronous gridder call), chunk k + 1's H2D copy is in
    flight and chunks k + 2, k + 3 are being filled; a pinned slot is refilled
    once its previous H2D copy completed (event waited on by the filling
    thread), a device slot is rewritten only after the gridding call that read
    it returned. The slots persist across calls (pinned allocation is slow).
    """

    # per-thread slots: {device: ((rows, nchan), RowStreamer)} in a
    # threading.local, so a worker thread's pinned slots are released with the
    # thread and a new thread never inherits another's (ids are reused)
    _local = threading.local()
    COLUMNS = (("uvw", np.float64, (3,)), ("vis4", np.complex64, ("c", 4)), ("flags4", np.uint8, ("c", 4)),
               ("wgt4", np.float32, ("c", 4)))

    def __init__(self, device, rows: int, nchan: int, fill_threads: int = 16, nhost: int = 3, ndev: int = 2):
        self.device = torch.device(device)
        self.rows, self.nchan = int(rows), int(nchan)
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.host, self.dev = [], []
        for _ in range(nhost):
            self.host.append({n: torch.empty(self._shape(sh), dtype=_torch_dtype(dt), pin_memory=True)
                              for n, dt, sh in self.COLUMNS})
        for _ in range(ndev):
            self.dev.append({n: torch.empty(self._shape(sh), dtype=_torch_dtype(dt), device=self.device)
                             for n, dt, sh in self.COLUMNS})
        self.h2d_done = [None] * nhost
        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, fill_threads))
        self.fill_threads = max(1, fill_threads)
        self.bytes_staged = 0

    def _shape(self, sh):
        return (self.rows,) + tuple(self.nchan if d == "c" else d for d in sh)

    @classmethod
    def get(cls, device, rows: int, nchan: int) -> "RowStreamer":
        """The calling thread's streamer for `device` (one set of slots per
        (thread, device): concurrent streamed inverts on several GPUs - e.g.
        LocalGPUClient's per-device worker threads - never evict or share each
        other's slots). A new shape replaces only this thread's slots."""
        cache = getattr(cls._local, "slots", None)
        if cache is None:
            cache = cls._local.slots = {}
        owner = str(torch.device(device))
        shape = (int(rows), int(nchan))
        ent = cache.get(owner)
        if ent is not None and ent[0] == shape:
            return ent[1]
        cache.pop(owner, None)  # drop the old slots before pinning new ones
        st = cls(device, rows, nchan)
        cache[owner] = (shape, st)
        return st

    @classmethod
    def release(cls) -> None:
        """Free the calling thread's streamers (pinned and device slots)."""
        cache = getattr(cls._local, "slots", None)
        if cache:
            for _, st in cache.values():
                st.pool.shutdown(wait=True)
            cache.clear()

    def fill(self, slot: int, reader, row0: int, row1: int) -> int:
        """Fill pinned slot `slot` with reader rows [row0, row1) (blocking;
        parallel over row blocks). Waits for the slot's previous H2D copy."""
        ev = self.h2d_done[slot]
        if ev is not None:
            ev.synchronize()
        n = row1 - row0
        views = {name: t.numpy()[:n] for name, t in self.host[slot].items()}
        step = max(256, -(-n // self.fill_threads))
        jobs = [self.pool.submit(reader.read_into, {k: v[a:min(n, a + step)] for k, v in views.items()},
                                 row0 + a, row0 + min(n, a + step)) for a in range(0, n, step)]
        for j in jobs:
            j.result()
        return n

    def send(self, hslot: int, dslot: int, n: int) -> dict:
        """H2D copy of the first n rows of pinned slot hslot into device slot
        dslot on the copy stream; returns the device views (valid for work on
        the current stream once `wait` is called)."""
        out = {}
        with torch.cuda.stream(self.copy_stream):
            for name, h in self.host[hslot].items():
                d = self.dev[dslot][name][:n]
                d.copy_(h[:n], non_blocking=True)
                out[name] = d
                self.bytes_staged += h[:n].numel() * h.element_size()
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        self.h2d_done[hslot] = ev
        return out

    def wait(self, hslot: int) -> None:
        torch.cuda.current_stream(self.device).wait_event(self.h2d_done[hslot])


def invert_measurement_set_streamed(
    ms_reader,
    num_pixels: int,
    pixel_size_asec: float,
    *,
    rows_per_chunk: int = 65536,
    epsilon: float = EPSILON,
    support: Optional[int] = None,
    do_wstacking: bool = False,
    device=None,
):
    """
    `invert_measurement_set` (reference invert.py:119-149) for measurement
    sets larger than one transfer: the raw (rows, chans, 4) columns are read
    `rows_per_chunk` rows at a time straight into pinned staging slots (the
    reader's `read_into`; readers without it are copied from their returned
    arrays), sent to HBM on a copy stream and gridded onto one set of resident
    planes with Stokes I formed inside the gridder (`add_ms_stokes_i`).
    Returns the normalised image as float32 numpy (N, N), like the reference.
    """
    _require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    freq = np.asarray(ms_reader.channel_frequencies(), dtype=np.float64)
    nrow = ms_reader.num_data_rows
    nchan = freq.size
    w_range = w_range_rows(ms_reader.uvw(), freq) if do_wstacking else (0.0, 0.0)
    pix = pixel_size_lm(pixel_size_asec)
    acc = GridAccumulator(num_pixels, num_pixels, pix, pix, epsilon=epsilon, support=support,
                          do_wstacking=do_wstacking, w_range=w_range, device=dev)
    freq_d = torch.from_numpy(freq).to(dev)
    rpc = max(1, min(int(rows_per_chunk), max(nrow, 1)))
    bounds = [(a, min(nrow, a + rpc)) for a in range(0, nrow, rpc)]
    reader = ms_reader if hasattr(ms_reader, "read_into") else _CopyingReader(ms_reader)
    with torch.cuda.device(dev):
        if bounds:
            st = RowStreamer.get(dev, rpc, nchan)
            H, D = len(st.host), len(st.dev)
            fills = {}

            def submit_fill(k):
                if k < len(bounds) and k not in fills:
                    fills[k] = _FILL_POOL.submit(st.fill, k % H, reader, *bounds[k])

            for k in range(min(H, len(bounds))):
                submit_fill(k)
            staged = {0: st.send(0, 0, fills.pop(0).result())}
            for k in range(len(bounds)):
                if k + 1 < len(bounds):
                    # the device slot of chunk k + 1 was last read by chunk k - 1's (returned) call
                    staged[k + 1] = st.send((k + 1) % H, (k + 1) % D, fills.pop(k + 1).result())
                submit_fill(k + H)  # into chunk k's pinned slot, once its H2D copy is done
                c = staged.pop(k)
                st.wait(k % H)
                acc.add_ms_stokes_i(c["uvw"], freq_d, c["vis4"], c["flags4"], c["wgt4"])
        dirty, sumw = acc.dirty()
        image = (dirty / sumw).to(torch.float32).cpu().numpy()
    return image


class _CopyingReader:
    """read_into for readers that only return fresh arrays (the reference's
    reader protocol, measurement_set.py:281-358): one extra host copy."""

    def __init__(self, reader):
        self.reader = reader

    def read_into(self, out: dict, row0: int, row1: int) -> None:
        r = self.reader.partition(1, 1)[0] if hasattr(self.reader, "partition") else self.reader
        r.set_row_bounds(self.reader.row_start + row0, self.reader.row_start + row1)
        cols = {"uvw": r.uvw, "vis4": r.visibilities, "flags4": r.flags, "wgt4": r.weights}
        for name, dst in out.items():
            src = cols[name]()
            np.copyto(dst.view(np.bool_) if name == "flags4" and dst.dtype == np.uint8 else dst, src)


_FILL_POOL = cf.ThreadPoolExecutor(max_workers=4)


__all__ = ["ChunkStager", "RowStreamer", "invert_measurement_set_streamed", "invert_tile_files"]
