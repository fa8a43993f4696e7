"""
Strong scaling of ONE w-stacking dirty image over several GPUs by w-plane
groups (SURVEY.md 8(e) option 2): the reference's own gridding mode
(invert.py:170-183, `do_wstacking=True`) split by planes instead of rows.

The w-stacking image is a sum over the planes of the stack (each plane:
scatter of the visibilities feeding it, 2-D FFT, w screen), followed by a
per-pixel correction - all linear. Rank r takes a contiguous range of planes
[p0_r, p1_r) (`split_planes`, balanced by a cost model of the planes' scatter
and FFT work), grids + FFTs + screens only those (`cip_ms2dirty_wplanes`: its
planner keeps only the visibilities feeding the range), and one RCCL reduce
of the npix^2 fp64 partial images onto the destination rank makes the image.
Every rank holds the same visibilities (the weight sum and the stack's
parameters are those of the whole call, so the shares are consistent) - the
exchange is one image reduce, and both the scatter and the FFTs split.

`invert_wplanes` wires the per-rank share with torch.distributed (RCCL, or
gloo for CPU tests); `invert_wplanes_local` runs every rank's share in one
process (the single-GPU check of the decomposition and its per-rank times).
The per-rank computation is a backend callable, `planes -> (partial image,
weight sum)`: `HipWPlaneBackend` (libcip_hip.so) or, in tests, the oracle.
"""

from __future__ import annotations

import math
from typing import Callable, Optional, Sequence

import numpy as np

SPEED_OF_LIGHT = 299792458.0
# FFT work of one plane in units of "visibility feeds" (one visibility gridded
# onto one plane) per grid cell, measured at C3 with the reference's call
# (profiles r03: scatter 9.52 ms for 6.0e8 feeds, FFT 0.476 ms per 8192^2
# plane -> 3.0e7 feeds per plane = 0.45 per cell)
FFT_FEEDS_PER_CELL = 0.45

try:
    import torch
except ModuleNotFoundError:  # pragma: no cover - torch is in the image
    torch = None


def plane_feeds(uvw, freq, params) -> np.ndarray:
    """Visibilities feeding each w plane (nplanes,): a visibility at w layer
    iw0 = floor((w f/c - w0)/dw - W/2) + 1 feeds planes iw0 .. iw0 + W - 1
    (the gridder's w footprint, cip_common.h place_vis). uvw (nrow, 3) and
    freq (nchan,) tensors on any device."""
    W, P = int(params.support), int(params.nplanes)
    ntw = max(P - W + 1, 1)
    fx = freq / SPEED_OF_LIGHT
    hist = torch.zeros(ntw, dtype=torch.int64, device=uvw.device)
    for a in range(0, uvw.shape[0], 65536):
        b = min(uvw.shape[0], a + 65536)
        xw = ((uvw[a:b, 2:3] * fx[None, :]) - float(params.w0)) / float(params.dw)
        iw0 = torch.floor(xw - float(W // 2)).to(torch.int64) + 1
        hist += torch.bincount(iw0.clamp(0, ntw - 1).reshape(-1), minlength=ntw)
    h = np.concatenate([[0], np.cumsum(hist.cpu().numpy())])
    p = np.arange(P)
    lo = np.clip(p - W + 1, 0, ntw)
    hi = np.clip(p + 1, 0, ntw)
    return (h[hi] - h[lo]).astype(np.int64)


def plane_cost(feeds: np.ndarray, params, fft_feeds_per_cell: float = FFT_FEEDS_PER_CELL) -> np.ndarray:
    """Relative cost of each plane: its feeds (scatter) + one FFT."""
    return np.asarray(feeds, dtype=np.float64) + fft_feeds_per_cell * float(params.nu) * float(params.nv)


def split_planes(cost: Sequence[float], world: int, group: int = 3) -> list:
    """Contiguous plane ranges [(p0, p1)] for `world` ranks with near-equal
    summed cost; cuts on multiples of `group` (the gridder's plane groups:
    three planes share one scatter pass) where the stack allows it. Ranges
    may be empty when there are fewer planes than ranks."""
    cost = np.asarray(cost, dtype=np.float64)
    P = cost.size
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.concatenate([[0.0], np.cumsum(cost)])
    total = cum[-1]
    g = group if P >= group * world else 1
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(cum, target))
        # nearest cut on the group lattice, not before the previous cut
        cand = sorted({max(cuts[-1], min(P, g * (k // g))), max(cuts[-1], min(P, g * -(-k // g)))})
        best = min(cand, key=lambda c: abs(cum[c] - target))
        cuts.append(best)
    cuts.append(P)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


class HipWPlaneBackend:
    """A rank's share through libcip_hip.so (cip_ms2dirty_wplanes) on
    device-resident inputs: returns (unnormalised partial image, weight sum)."""

    def __init__(self, uvw, freq, vis, wgt, npix_x: int, npix_y: int, pixsize_x: float, pixsize_y: float, *,
                 epsilon: float = 1e-4, support: Optional[int] = None, single_precision_accumulation: bool = False):
        from .gridder import _require_gpu  # pylint: disable=import-outside-toplevel

        _require_gpu()
        self.args = (uvw, freq, vis, wgt, int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y))
        self.kw = dict(epsilon=epsilon, support=support, do_wstacking=True,
                       single_precision_accumulation=single_precision_accumulation)
        self.device = uvw.device

    def params(self):
        """The whole stack's parameters (the w range of all visibilities)."""
        from . import _lib  # pylint: disable=import-outside-toplevel
        from .accumulate import w_range_rows  # pylint: disable=import-outside-toplevel

        uvw, freq, _, _, nx, ny, px, py = self.args
        wmin, wmax = w_range_rows(uvw.cpu().numpy(), freq.cpu().numpy())
        return _lib.choose_params(nx, ny, px, py, self.kw["epsilon"], self.kw["support"] or 0, True, wmin, wmax)

    def plane_group(self, params=None) -> int:
        """The library's w-plane group for these parameters (cip_plane_group):
        pass it to `split_planes` so no rank boundary falls inside a group."""
        from . import _lib  # pylint: disable=import-outside-toplevel

        return _lib.plane_group(self.params() if params is None else params,
                                bool(self.kw["single_precision_accumulation"]))

    def __call__(self, planes, out=None, sum_weights=None):
        from .gridder import device_ms2dirty  # pylint: disable=import-outside-toplevel

        if sum_weights is None:
            sum_weights = torch.zeros(1, dtype=torch.float64, device=self.device)
        img, _ = device_ms2dirty(*self.args, out=out, sum_weights=sum_weights, planes=tuple(planes), **self.kw)
        return img, sum_weights


def invert_wplanes(backend: Callable, split: Sequence[tuple], *, dst: int = 0, group=None,
                   stages: Optional[dict] = None, out=None):
    """This rank's share of the plane-split invert (torch.distributed
    initialised, one rank per entry of `split`): the partial image of planes
    split[rank], reduced (sum) onto `dst` and divided there by the weight sum
    (every rank's call reduces the same, whole weight sum). Returns the
    normalised image on `dst`, None elsewhere. `stages` (diagnostic): seconds
    of the synchronised "grid" (the share: scatter + FFTs) and "reduce"."""
    import time  # pylint: disable=import-outside-toplevel

    import torch.distributed as dist  # pylint: disable=import-outside-toplevel

    single = not dist.is_available() or not dist.is_initialized()
    world = 1 if single else dist.get_world_size(group)
    rank = 0 if single else dist.get_rank(group)
    if len(split) != world:
        raise ValueError("one plane range per rank")

    def sync(t):
        if t.is_cuda:
            torch.cuda.synchronize(t.device)

    t0 = time.perf_counter()
    img, sumw = backend(split[rank], out=out)
    if stages is not None:
        sync(img)
        stages["grid"] = stages.get("grid", 0.0) + time.perf_counter() - t0
    t1 = time.perf_counter()
    if world > 1:
        dist.reduce(img, dst, group=group)
    if stages is not None:
        sync(img)
        stages["reduce"] = stages.get("reduce", 0.0) + time.perf_counter() - t1
    if rank != dst:
        return None
    return img.div_(sumw)


def invert_wplanes_local(backend: Callable, split: Sequence[tuple], stages: Optional[list] = None):
    """Every rank's share in ONE process (one device), summed in memory - the
    single-GPU check of the decomposition and the per-rank breakdown of the
    N-GPU split (`stages`: filled with one {"grid": seconds} per rank).
    Returns the normalised image."""
    import time  # pylint: disable=import-outside-toplevel

    if stages is not None:
        stages[:] = [{} for _ in split]
    acc, sumw = None, None
    for r, planes in enumerate(split):
        t0 = time.perf_counter()
        img, sw = backend(planes)
        if stages is not None:
            if img.is_cuda:
                torch.cuda.synchronize(img.device)
            stages[r]["grid"] = time.perf_counter() - t0
        acc = img.clone() if acc is None else acc.add_(img)
        sumw = sw
    return acc.div_(sumw)


def predicted_speedup(rank_seconds: Sequence[float], one_rank_seconds: float, reduce_seconds: float = 0.0) -> float:
    """Strong-scaling speed-up of the slowest rank's share (+ the reduce)
    against the one-rank time."""
    worst = max(rank_seconds) if rank_seconds else 0.0
    return one_rank_seconds / (worst + reduce_seconds) if worst + reduce_seconds > 0 else math.inf


__all__ = ["plane_feeds", "plane_cost", "split_planes", "HipWPlaneBackend", "invert_wplanes",
           "invert_wplanes_local", "predicted_speedup"]
