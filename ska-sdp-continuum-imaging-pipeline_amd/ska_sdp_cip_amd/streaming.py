"""
Chunked host -> HBM streaming invert (config C5's
"chunked-MS host->HBM streaming").

Two sources, one pipeline:

* `invert_tile_files` - uvw_tiling chunk files (`tile_..._chunkNNN.npz`, the
  reorder output of reference uvw_tiling/reorder.py:19-111, optional
  `weights` key), gridded slice-wise by `cip_grid_tiles`;
* `invert_measurement_set_streamed` - row blocks of a measurement set reader
  (raw (rows, chans, 4) columns; Stokes I formed on the device by
  `cip_stokes_i`), gridded by `cip_grid_ms`.

Pipeline: while chunk k is gridded on the compute stream onto the resident
planes of a `GridAccumulator`, a worker thread reads chunk k + 1 (disk /
reader), copies it into its pinned staging slot and sends it to HBM on a
dedicated copy stream (two slots). One FFT at the end.
"""

from __future__ import annotations

import concurrent.futures as cf
from pathlib import Path
from typing import Callable, Iterable, Optional, Sequence

import numpy as np

from .accumulate import GridAccumulator, merge_w_ranges, w_range_rows, w_range_slices
from .gridder import _require_gpu, device_stokes_i
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
    `rows_per_chunk` rows at a time, staged through pinned memory to HBM on a
    copy stream, turned into Stokes I + effective weights on the device and
    gridded onto one set of resident planes. Returns the normalised image as
    float32 numpy (N, N), like the reference.
    """
    _require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    freq = np.asarray(ms_reader.channel_frequencies(), dtype=np.float64)
    nrow = ms_reader.num_data_rows
    nchunks = max(1, -(-nrow // max(int(rows_per_chunk), 1)))
    w_range = w_range_rows(ms_reader.uvw(), freq) if do_wstacking else (0.0, 0.0)
    pix = pixel_size_lm(pixel_size_asec)
    acc = GridAccumulator(num_pixels, num_pixels, pix, pix, epsilon=epsilon, support=support,
                          do_wstacking=do_wstacking, w_range=w_range, device=dev)
    freq_d = torch.from_numpy(freq).to(dev)
    chunks = list(ms_reader.partition(nchunks, 1)) if nrow > 0 else []

    def loader(chunk):
        def load():
            return {"uvw": np.asarray(chunk.uvw(), dtype=np.float64),
                    "vis4": np.asarray(chunk.visibilities(), dtype=np.complex64),
                    "flags4": np.asarray(chunk.flags(), dtype=np.bool_),
                    "wgt4": np.asarray(chunk.weights(), dtype=np.float32)}
        return load

    def consume(c):
        vis_i, eff = device_stokes_i(c["vis4"], c["flags4"], c["wgt4"])
        acc.add_ms(c["uvw"], freq_d, vis_i, eff)

    with torch.cuda.device(dev):
        _pipeline([loader(ch) for ch in chunks], ChunkStager(dev), consume)
        dirty, sumw = acc.dirty()
        image = (dirty / sumw).to(torch.float32).cpu().numpy()
    return image


__all__ = ["ChunkStager", "invert_measurement_set_streamed", "invert_tile_files"]
