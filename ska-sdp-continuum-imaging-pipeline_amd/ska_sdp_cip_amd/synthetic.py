"""
Seeded synthetic MeerKAT-like measurement sets.

The reference's test MS (`tests/data/mkt_ecdfs25_nano.zip`) is missing from the
mount and casacore is absent, so every invert test and benchmark of this build
runs on synthetic data with the same column shapes and dtypes:

* array: `n_ant` antennas uniform in a disc of radius `array_radius_m` (ENU),
  no autocorrelations; rows are ordered time-major, baseline-minor as in an MS;
* tracks: latitude -30.7 deg, declination -30 deg, 8 s dumps, hour angles
  centred on transit;
* channels: f_k = f0 + k * bandwidth / nchan (default 856 MHz + k 856/nchan MHz);
* visibilities: point sources through the forward model that is the adjoint of
  the imaging convention of `oracle/` and the gridder
  (V = sum_s F_s exp(-2 pi i (u l_s + v m_s - w (n_s - 1))), uvw in wavelengths)
  plus complex Gaussian noise; XX = YY = V, XY = YX = noise;
* weights U(0.5, 1.5) f32 per polarisation; flags Bernoulli(p) per (row, chan)
  on all polarisations plus a few single-polarisation flags.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
from numpy.typing import NDArray

from .measurement_set import InMemoryMeasurementSet

SPEED_OF_LIGHT = 299792458.0
DEFAULT_SEED = 20241008


@dataclass
class PointSource:
    """A point source at direction cosines (l, m) with flux in Jy."""

    l: float  # noqa: E741
    m: float
    flux: float


def antenna_positions(n_ant: int, radius_m: float, rng) -> NDArray:
    """ENU antenna positions uniform in a disc, shape (n_ant, 3)."""
    r = radius_m * np.sqrt(rng.uniform(0.0, 1.0, n_ant))
    phi = rng.uniform(0.0, 2 * np.pi, n_ant)
    up = rng.normal(0.0, 2.0, n_ant)
    return np.stack([r * np.cos(phi), r * np.sin(phi), up], axis=1)


def uvw_tracks(
    n_rows: int,
    n_ant: int = 64,
    *,
    array_radius_m: float = 4000.0,
    latitude_deg: float = -30.7,
    dec_deg: float = -30.0,
    dump_s: float = 8.0,
    seed: int = DEFAULT_SEED,
) -> NDArray:
    """
    Earth-rotation uvw tracks in metres, shape (n_rows, 3) float64, rows in
    (time, baseline) order; the last time step is truncated to give exactly
    `n_rows` rows.
    """
    rng = np.random.default_rng(seed)
    enu = antenna_positions(n_ant, array_radius_m, rng)
    a1, a2 = np.triu_indices(n_ant, k=1)
    bl = enu[a2] - enu[a1]  # (nbl, 3) ENU
    lat = np.radians(latitude_deg)
    dec = np.radians(dec_deg)
    # ENU -> local equatorial XYZ
    x = -np.sin(lat) * bl[:, 1] + np.cos(lat) * bl[:, 2]
    y = bl[:, 0]
    z = np.cos(lat) * bl[:, 1] + np.sin(lat) * bl[:, 2]
    nbl = len(bl)
    n_times = -(-n_rows // nbl)
    omega = 7.292115e-5  # rad/s
    ha = (np.arange(n_times) - (n_times - 1) / 2.0) * dump_s * omega
    sh, ch = np.sin(ha)[:, None], np.cos(ha)[:, None]
    u = sh * x + ch * y
    v = -np.sin(dec) * ch * x + np.sin(dec) * sh * y + np.cos(dec) * z
    w = np.cos(dec) * ch * x - np.cos(dec) * sh * y + np.sin(dec) * z
    uvw = np.stack([u, v, w], axis=-1).reshape(-1, 3)[:n_rows]
    return np.ascontiguousarray(uvw, dtype=np.float64)


def channel_frequencies(
    nchan: int, f0: float = 856.0e6, bandwidth: Optional[float] = None
) -> NDArray:
    """f_k = f0 + k * bandwidth / nchan; bandwidth defaults to f0 (856 MHz)."""
    bw = f0 if bandwidth is None else bandwidth
    return f0 + np.arange(nchan, dtype=np.float64) * (bw / nchan)


def random_sources(
    n: int, fov_l: float, rng, flux_range=(0.1, 1.0)
) -> list[PointSource]:
    """`n` sources uniform in |l|, |m| < fov_l/2 with uniform fluxes."""
    lm = rng.uniform(-fov_l / 2, fov_l / 2, size=(n, 2))
    flux = rng.uniform(*flux_range, size=n)
    return [PointSource(float(a), float(b), float(f)) for (a, b), f in zip(lm, flux)]


def predict_visibilities(
    uvw_m: NDArray, freqs: NDArray, sources: list[PointSource]
) -> NDArray:
    """
    fp64 direct prediction, shape (nrow, nchan) complex128:
    V = sum_s F_s exp(-2 pi i f/c (u l + v m - w (n - 1))).
    """
    scale = freqs / SPEED_OF_LIGHT  # (nchan,)
    out = np.zeros((uvw_m.shape[0], freqs.size), dtype=np.complex128)
    for src in sources:
        n = np.sqrt(1.0 - src.l**2 - src.m**2)
        path = uvw_m[:, 0] * src.l + uvw_m[:, 1] * src.m - uvw_m[:, 2] * (n - 1.0)
        out += src.flux * np.exp(-2j * np.pi * path[:, None] * scale[None, :])
    return out


def make_measurement_set(
    n_rows: int,
    nchan: int,
    *,
    n_ant: int = 64,
    array_radius_m: float = 4000.0,
    f0: float = 856.0e6,
    bandwidth: Optional[float] = None,
    n_sources: int = 8,
    fov_l: float = 0.01,
    sources: Optional[list[PointSource]] = None,
    noise: float = 0.01,
    flag_fraction: float = 0.05,
    weight_spectrum: bool = True,
    cheap_visibilities: bool = False,
    seed: int = DEFAULT_SEED,
) -> InMemoryMeasurementSet:
    """
    Build a seeded synthetic `InMemoryMeasurementSet`.

    `cheap_visibilities=True` replaces the point-source prediction with
    random values (throughput runs: values do not affect gridding cost, uvw
    tracks - which drive tile populations - stay real).
    """
    rng = np.random.default_rng(seed)
    uvw = uvw_tracks(
        n_rows, n_ant, array_radius_m=array_radius_m, seed=seed
    )
    freqs = channel_frequencies(nchan, f0, bandwidth)
    if cheap_visibilities:
        stokes = (
            rng.standard_normal((n_rows, nchan), dtype=np.float32)
            + 1j * rng.standard_normal((n_rows, nchan), dtype=np.float32)
        ).astype(np.complex64)
    else:
        if sources is None:
            sources = random_sources(n_sources, fov_l, rng)
        stokes = predict_visibilities(uvw, freqs, sources)
    vis = np.empty((n_rows, nchan, 4), dtype=np.complex64)
    shape = (n_rows, nchan)

    def _noise():
        if noise == 0.0:
            return np.zeros(shape, dtype=np.complex64)
        return (
            noise
            * (rng.standard_normal(shape) + 1j * rng.standard_normal(shape))
            / np.sqrt(2)
        ).astype(np.complex64)

    vis[..., 0] = stokes + _noise()
    vis[..., 3] = stokes + _noise()
    vis[..., 1] = _noise()
    vis[..., 2] = _noise()
    if weight_spectrum:
        weights = rng.uniform(0.5, 1.5, size=(n_rows, nchan, 4)).astype(np.float32)
    else:
        weights = rng.uniform(0.5, 1.5, size=(n_rows, 4)).astype(np.float32)
    flags = np.zeros((n_rows, nchan, 4), dtype=bool)
    if flag_fraction > 0:
        flags |= (rng.uniform(size=shape) < flag_fraction)[..., None]
        # a few single-polarisation flags exercise the XX|YY fold
        flags[..., 0] |= rng.uniform(size=shape) < flag_fraction / 5
        flags[..., 3] |= rng.uniform(size=shape) < flag_fraction / 5
    return InMemoryMeasurementSet(uvw, vis, flags, weights, freqs)


def pixel_size_for_grid(
    uvw_m: NDArray, freqs: NDArray, num_pixels: int, sigma: float = 2.0,
    support: int = 8, fill: float = 0.9,
) -> float:
    """
    Pixel size (radians, sin-projected) such that the longest |u| or |v| lands
    at `fill` of the usable half-width of a (sigma * num_pixels)^2 grid.
    """
    uv_max = np.abs(uvw_m[:, :2]).max() * freqs.max() / SPEED_OF_LIGHT
    nu = int(round(sigma * num_pixels))
    usable = 0.5 - (support / 2 + 2) / nu
    return fill * usable / uv_max


def pixel_size_asec(pixsize_lm: float) -> float:
    """Inverse of the reference's asec -> lm conversion (`invert.py:163`)."""
    return float(np.degrees(np.arcsin(pixsize_lm)) * 3600.0)


# --- counter-based columns (strong-scaling runs: the same data at every N) ---

_M32 = 0xFFFFFFFF


def _hash32(x):
    """A 32-bit integer finaliser on int64 tensors holding values in
    [0, 2^32): two xorshift-multiply rounds (every product < 2^59, so the
    int64 arithmetic never wraps; shifts act on non-negative values only)."""
    x = (((x >> 16) ^ x) * 0x45D9F3B) & _M32
    x = (((x >> 16) ^ x) * 0x45D9F3B) & _M32
    return (x >> 16) ^ x


def _uniform(idx, stream: int, seed: int):
    """U(0, 1) float64 from the global visibility index `idx` (int64 tensor,
    < 2^32), a stream number and a seed: a pure function of (idx, stream,
    seed), so any rank - or any split of the rows - draws the same value."""
    import torch  # pylint: disable=import-outside-toplevel

    key = int(_hash32(torch.tensor(((seed * 0x9E3779B1) ^ (stream * 0x85EBCA6B)) & _M32, dtype=torch.int64)))
    h = _hash32((idx ^ key) & _M32)
    h = _hash32((h + stream * 0x27D4EB2F + 1) & _M32)
    return (h.to(torch.float64) + 0.5) * (1.0 / 4294967296.0)


def counter_columns(idx, seed: int = DEFAULT_SEED, flag_fraction: float = 0.05):
    """Visibilities and weights of global visibility indices `idx` = row *
    nchan + channel (int64 tensor, any shape, values < 2^32): complex64
    visibilities with standard-normal real and imaginary parts (Box-Muller),
    float32 weights U(0.5, 1.5) with `flag_fraction` of them zero (flagged).
    The strong-scaling benchmark draws every rank's strip this way, so the
    1G-visibility C4 image is the same image at every rank count."""
    import torch  # pylint: disable=import-outside-toplevel

    if idx.numel() and int(idx.max()) >= (1 << 32):
        raise ValueError("counter_columns: global indices must be < 2^32")
    u1 = _uniform(idx, 1, seed)
    u2 = _uniform(idx, 2, seed)
    r = torch.sqrt(-2.0 * torch.log(u1))
    ph = (2.0 * np.pi) * u2
    vis = torch.complex((r * torch.cos(ph)).to(torch.float32), (r * torch.sin(ph)).to(torch.float32))
    wgt = (_uniform(idx, 3, seed) + 0.5).to(torch.float32)
    wgt = torch.where(_uniform(idx, 4, seed) < flag_fraction, torch.zeros_like(wgt), wgt)
    return vis.contiguous(), wgt.contiguous()


def counter_columns_slices(rows, c0, c1, nchan: int, seed: int = DEFAULT_SEED, chunk: int = 1 << 25):
    """`counter_columns` of Tile-layout row slices (slice s: channels
    [c0[s], c1[s]) of MS row rows[s], visibilities concatenated in slice
    order), drawn in chunks of `chunk` visibilities -> (vis (nvis,) complex64,
    wgt (nvis,) float32) on the slices' device."""
    import torch  # pylint: disable=import-outside-toplevel

    rows, c0, c1 = rows.to(torch.int64), c0.to(torch.int64), c1.to(torch.int64)
    lengths = c1 - c0
    ends = torch.cumsum(lengths, 0)
    total = int(ends[-1]) if ends.numel() else 0
    vis = torch.empty(total, dtype=torch.complex64, device=rows.device)
    wgt = torch.empty(total, dtype=torch.float32, device=rows.device)
    for a in range(0, total, chunk):
        b = min(total, a + chunk)
        k = torch.arange(a, b, device=rows.device)
        sl = torch.searchsorted(ends, k, right=True)
        idx = rows[sl] * nchan + c0[sl] + (k - (ends[sl] - lengths[sl]))
        vis[a:b], wgt[a:b] = counter_columns(idx, seed)
    return vis, wgt
