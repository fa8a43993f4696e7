"""
TEST INFRASTRUCTURE ONLY - the ms2dirty definition (the direct fp64 DFT) at a
few pixels, evaluated with torch in fp64 on whatever device holds the inputs.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s checks (outside its
timed region) use it; the product never does. It is the same definition as
`oracle.dft_dirty` / `oracle.dft_directions` (the C restatement), cheap enough
to run at full workload size because it evaluates only the requested pixels:

    dirty[i, j] = sum_{r,c} wgt Re{ vis exp(2 pi i f_c/c (u_r l + v_r m - w_r (n - 1))) }  [/ n]
    l = (i - npix_x/2) px, m = (j - npix_y/2) py, n = sqrt(1 - l^2 - m^2)

with the w term and the 1/n only when `apply_w` (w-stacking images; 2-D
images use n := 1). The sums are PARTIAL: each rank of a distributed run
evaluates them over its own visibilities and the ranks' results are summed
(all-reduce), so the check sees the reduced / gathered image.
"""

from __future__ import annotations

import math

import numpy as np

SPEED_OF_LIGHT = 299792458.0


def _directions(pixels, npix_x, npix_y, px, py):
    l = np.array([(i - npix_x // 2) * px for i, _ in pixels], dtype=np.float64)  # noqa: E741
    m = np.array([(j - npix_y // 2) * py for _, j in pixels], dtype=np.float64)
    nm1 = -(l * l + m * m) / (np.sqrt(1.0 - l * l - m * m) + 1.0)
    return l, m, nm1


def _accumulate(acc, u, v, w, fx, vis, wgt, l, m, nm1, apply_w):
    """acc (P,) += sum over the visibilities of wgt Re{vis e^{i phase}};
    u, v, w, fx: (K,) per visibility; vis (K,) complex; wgt (K,) or None."""
    import torch  # pylint: disable=import-outside-toplevel

    vr = vis.real.to(torch.float64)
    vi = vis.imag.to(torch.float64)
    if wgt is not None:
        wd = wgt.to(torch.float64)
        vr, vi = vr * wd, vi * wd
    for p in range(l.size):
        path = u * float(l[p]) + v * float(m[p])
        if apply_w:
            path = path - w * float(nm1[p])
        ph = (2.0 * math.pi) * (path * fx)
        acc[p] += (vr * torch.cos(ph) - vi * torch.sin(ph)).sum()


def dft_pixels_dense(uvw, freq, vis, wgt, pixels, npix_x, npix_y, px, py, apply_w=False, row_chunk=32768):
    """Partial DFT sums at `pixels` [(i, j), ...] over dense MS columns:
    uvw (nrow, 3) f64, freq (nchan,) f64, vis (nrow, nchan) complex, wgt
    (nrow, nchan) or None (tensors on one device). Returns (sums (P,) f64
    numpy, weight sum float)."""
    import torch  # pylint: disable=import-outside-toplevel

    l, m, nm1 = _directions(pixels, npix_x, npix_y, px, py)
    dev = vis.device
    acc = torch.zeros(len(pixels), dtype=torch.float64, device=dev)
    sw = torch.zeros((), dtype=torch.float64, device=dev)
    fx = (freq.to(torch.float64) / SPEED_OF_LIGHT)[None, :]
    nrow = int(uvw.shape[0])
    for a in range(0, nrow, row_chunk):
        b = min(nrow, a + row_chunk)
        u, v, w = (uvw[a:b, k].to(torch.float64)[:, None] for k in range(3))
        wg = None if wgt is None else wgt[a:b]
        _accumulate(acc, u, v, w, fx, vis[a:b], wg, l, m, nm1, apply_w)
        sw += wg.to(torch.float64).sum() if wg is not None else float((b - a) * vis.shape[1])
    out = acc.cpu().numpy()
    if apply_w:
        out = out / (nm1 + 1.0)
    return out, float(sw.item())


def dft_pixels_slices(slice_uvw, chan_start, chan_stop, freq, vis, wgt, pixels, npix_x, npix_y, px, py,
                      apply_w=False, vis_chunk=1 << 23):
    """The same over Tile-layout data (ragged row slices: slice s holds
    channels [chan_start[s], chan_stop[s]) of a row with uvw slice_uvw[s];
    vis / wgt concatenated in slice order)."""
    import torch  # pylint: disable=import-outside-toplevel

    l, m, nm1 = _directions(pixels, npix_x, npix_y, px, py)
    dev = vis.device
    acc = torch.zeros(len(pixels), dtype=torch.float64, device=dev)
    sw = torch.zeros((), dtype=torch.float64, device=dev)
    fx_all = freq.to(torch.float64) / SPEED_OF_LIGHT
    c0 = chan_start.to(torch.int64)
    lengths = chan_stop.to(torch.int64) - c0
    ends = torch.cumsum(lengths, 0)
    total = int(ends[-1]) if ends.numel() else 0
    for a in range(0, total, vis_chunk):
        b = min(total, a + vis_chunk)
        k = torch.arange(a, b, device=dev)
        sl = torch.searchsorted(ends, k, right=True)
        ch = c0[sl] + (k - (ends[sl] - lengths[sl]))
        uvw = slice_uvw[sl].to(torch.float64)
        wg = None if wgt is None else wgt[a:b]
        _accumulate(acc, uvw[:, 0], uvw[:, 1], uvw[:, 2], fx_all[ch], vis[a:b], wg, l, m, nm1, apply_w)
        sw += wg.to(torch.float64).sum() if wg is not None else float(b - a)
    out = acc.cpu().numpy()
    if apply_w:
        out = out / (nm1 + 1.0)
    return out, float(sw.item())


def check_pixels(npix_x, npix_y, seed=4, n_random=4):
    """The fixed pixel set of the full-size checks: centre, corners, an edge
    midpoint and `n_random` seeded random pixels."""
    rng = np.random.default_rng(seed)
    pix = [(npix_x // 2, npix_y // 2), (0, 0), (npix_x - 1, npix_y - 1), (npix_x // 2, 0)]
    pix += [(int(rng.integers(0, npix_x)), int(rng.integers(0, npix_y))) for _ in range(n_random)]
    return pix
