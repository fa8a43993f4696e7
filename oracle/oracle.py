"""
TEST INFRASTRUCTURE ONLY - CPU oracle for the invert hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module; the product (`ska_sdp_cip_amd`) never does.

Contents (each restates a reference function; file:line under
/root/reference/src/ska_sdp_cip):

* `choose_params`   - grid / kernel / w-plane parameters (the choice ducc0 makes
                      inside ms2dirty), restated from
                      the spec in DESIGN.md, independently of the HIP library.
* `ms2dirty`        - dirty image: fp64 gridding (libcip_oracle.so, C/OpenMP)
                      + numpy FFT + grid correction + w-stacking screen + 1/n;
                      restates ducc0.wgridder.ms2dirty as called at
                      invert.py:170-183 (third-party ducc0 0.34.0,
                      poetry.lock:421-422, absent here: parity of the ducc
                      boundary is UNPINNED, see DESIGN.md "Oracle").
* `dft_dirty`       - the fp64 direct-DFT definition of ms2dirty (ducc0's test
                      suite definition); small cases only.
* `stokes_i`        - StokesIGridderInput.from_measurement_set_reader +
                      effective_weights (invert.py:72-116).
* `tile_mapping_sequential` - create_uvw_tile_mapping_sequential
                      (uvw_tiling/tiling_plan.py:29-61) with runs found by a
                      linear scan (same set as the bisection of :150-181).
* `balanced_chunk_bounds`, `split_tile_bounds` - measurement_set.py:361-391,
                      uvw_tiling/tile.py:155-211.

Pinned against the reference's own outputs: tests/golden/*.npz were produced by
importing the reference modules standalone (tests/golden/make_golden.py).
"""

from __future__ import annotations

import ctypes
import math
import subprocess
from pathlib import Path
from typing import Optional

import numpy as np

SPEED_OF_LIGHT = 299792458.0
HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libcip_oracle.so"
BASELINE_PATH = HERE / "_build" / "libcip_cpu_baseline.so"
_LIB = None
_BASE = None


def build() -> Path:
    """Compile libcip_oracle.so (gcc, OpenMP)."""
    subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
    return LIB_PATH


def _lib():
    global _LIB  # pylint: disable=global-statement
    if _LIB is None:
        if not LIB_PATH.exists():
            build()
        so = ctypes.CDLL(str(LIB_PATH))
        vp, i64, f64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int
        so.oracle_grid_plane.argtypes = [vp, i64, vp, i64, vp, vp, i64, i64, f64, f64, i32, i32, f64, f64,
                                         i64, i64, i32, vp]
        so.oracle_grid_plane.restype = i64
        so.oracle_kernel_ft.argtypes = [i32, vp, i64, vp]
        so.oracle_kernel_value.argtypes = [i32, i32, f64, ctypes.POINTER(ctypes.c_double)]
        so.oracle_dft.argtypes = [vp, i64, vp, i64, vp, vp, i64, i64, f64, f64, i32, i32, vp]
        _LIB = so
    return _LIB


def _baseline_lib():
    global _BASE  # pylint: disable=global-statement
    if _BASE is None:
        if not BASELINE_PATH.exists():
            build()
        so = ctypes.CDLL(str(BASELINE_PATH))
        vp, i64, f64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int
        so.cpu_grid_tiled.argtypes = [vp, i64, vp, i64, vp, vp, i64, i64, f64, f64, i32, i32, vp]
        so.cpu_grid_tiled.restype = i64
        _BASE = so
    return _BASE


# ------------------------------------------------------------- params ----
def _good_size(n: int) -> int:
    n = max(n, 16)
    m = n + (n & 1)
    while True:
        r = m
        for p in (2, 3, 5, 7):
            while r % p == 0:
                r //= p
        if r == 1:
            return m
        m += 2


def support_for_epsilon(eps: float) -> int:
    """Kernel support for a requested accuracy (DESIGN.md 'Accuracy')."""
    for w, bound in ((4, 2e-3), (6, 2e-5), (8, 3e-7), (10, 4e-9), (12, 5e-11), (14, 6e-13)):
        if eps >= bound:
            return w
    return 16


# The kernel shape rule (tools/gen_es_kernels.py beta_for_support, restated):
# beta = 2.3 W (Barnett et al.'s sigma = 2 choice) while the ES kernel's edge
# ratio F(1/4)/F(0) stays >= 0.03; larger supports take the beta at which it
# equals 0.03 (their grid / w corrections then amplify rounding no more than a
# W = 24 kernel's, and the aliasing stays at the fp64 floor).
LARGE_EDGE_RATIO = 0.03


def es_edge_ratio(W: int, beta: float, nu: float = 0.25) -> float:
    """F(nu) / F(0) of the exact ES kernel exp(beta (sqrt(1 - (2d/W)^2) - 1)),
    |d| < W/2 cells (40-point Gauss-Legendre per cell)."""
    x, wq = np.polynomial.legendre.leggauss(40)
    d = (np.arange(W)[:, None] - W / 2.0) + 0.5 * (x[None, :] + 1.0)
    t = 2.0 * d / W
    ph = np.where(np.abs(t) < 1.0, np.exp(beta * (np.sqrt(np.clip(1.0 - t * t, 0.0, None)) - 1.0)), 0.0)
    return float((wq * ph * np.cos(2.0 * math.pi * d * nu)).sum() / (wq * ph).sum())


def es_beta(W: int) -> float:
    """Kernel shape parameter of support W (the rule above; bisection)."""
    if W <= 16 or es_edge_ratio(W, 2.3 * W) >= LARGE_EDGE_RATIO:
        return 2.3 * W
    lo, hi = 2.3 * W, 40.0 * W
    for _ in range(100):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if es_edge_ratio(W, mid) < LARGE_EDGE_RATIO else (lo, mid)
    return 0.5 * (lo + hi)


def choose_params(npix_x, npix_y, px, py, epsilon=1e-4, support=None, do_wstacking=False,
                  wmin=0.0, wmax=0.0) -> dict:
    """Grid / kernel / plane parameters (spec: DESIGN.md 'Parameters')."""
    if npix_x % 2 or npix_y % 2:
        raise ValueError("npix must be even")
    W = int(support) if support else support_for_epsilon(epsilon)
    sigma = 2.0
    nu = _good_size(int(math.ceil(sigma * npix_x)))
    nv = _good_size(int(math.ceil(sigma * npix_y)))
    x0, y0 = -0.5 * npix_x * px, -0.5 * npix_y * py
    e = x0 * x0 + y0 * y0
    nmin = -e / (math.sqrt(1.0 - e) + 1.0)
    if do_wstacking:
        dw = 0.5 / sigma / abs(nmin)
        nplanes = int(math.ceil((wmax - wmin) / dw)) + W
        w0 = 0.5 * (wmin + wmax) - 0.5 * (nplanes - 1) * dw
    else:
        dw, nplanes, w0 = 1.0, 1, 0.0
    return dict(nu=nu, nv=nv, support=W, sigma=sigma, nplanes=nplanes, w0=w0, dw=dw, nmin=nmin,
                do_wstacking=bool(do_wstacking), beta=es_beta(W))


def kernel_ft(W: int, nus) -> np.ndarray:
    """F(nu) of the piecewise-polynomial kernel (cycles per cell)."""
    nus = np.ascontiguousarray(nus, dtype=np.float64)
    out = np.empty_like(nus)
    _lib().oracle_kernel_ft(int(W), nus.ctypes.data, nus.size, out.ctypes.data)
    return out


def kernel_value(W: int, piece: int, y: float) -> float:
    out = ctypes.c_double()
    _lib().oracle_kernel_value(int(W), int(piece), float(y), ctypes.byref(out))
    return out.value


def _as_inputs(uvw, freq, vis, wgt):
    uvw = np.ascontiguousarray(uvw, dtype=np.float64)
    freq = np.ascontiguousarray(freq, dtype=np.float64)
    vis = np.ascontiguousarray(vis, dtype=np.complex128)
    wgt = None if wgt is None else np.ascontiguousarray(wgt, dtype=np.float64)
    return uvw, freq, vis, wgt


def w_range(uvw, freq) -> tuple[float, float]:
    """min / max of w in wavelengths over all rows and channels."""
    fx = np.asarray(freq, dtype=np.float64) / SPEED_OF_LIGHT
    w = np.asarray(uvw, dtype=np.float64)[:, 2]
    cand = np.concatenate([w * fx.min(), w * fx.max()])
    return float(cand.min()), float(cand.max())


def grid_plane(uvw, freq, vis, wgt, params: dict, px: float, py: float, plane: int = 0,
               nthreads: int = 0) -> np.ndarray:
    """fp64 grid (nu, nv) complex128 of w-plane `plane` (0 in 2-D mode)."""
    uvw, freq, vis, wgt = _as_inputs(uvw, freq, vis, wgt)
    nu, nv = params["nu"], params["nv"]
    grid = np.zeros((nu, nv), dtype=np.complex128)
    bad = _lib().oracle_grid_plane(
        uvw.ctypes.data, uvw.shape[0], freq.ctypes.data, freq.size, vis.ctypes.data,
        None if wgt is None else wgt.ctypes.data, nu, nv, px, py, params["support"],
        int(params["do_wstacking"]), params["w0"], params["dw"], params["nplanes"], plane,
        int(nthreads), grid.ctypes.data)
    if bad < 0:
        raise ValueError("unsupported kernel support")
    if bad > 0:
        raise ValueError(f"{bad} visibilities fall outside the grid")
    return grid


def grid_plane_tiled(uvw, freq, vis, wgt, params: dict, px: float, py: float, nthreads: int = 0) -> np.ndarray:
    """CPU BASELINE (oracle/cpu_baseline.c, bench.py's cpu_baseline leg): the
    2-D grid by the tiled restatement of ducc0's CPU design; complex64 vis and
    float32 weights (or None) are read as given."""
    uvw = np.ascontiguousarray(uvw, dtype=np.float64)
    freq = np.ascontiguousarray(freq, dtype=np.float64)
    vis = np.ascontiguousarray(vis, dtype=np.complex64)
    wgt = None if wgt is None else np.ascontiguousarray(wgt, dtype=np.float32)
    nu, nv = params["nu"], params["nv"]
    grid = np.zeros((nu, nv), dtype=np.complex128)
    bad = _baseline_lib().cpu_grid_tiled(
        uvw.ctypes.data, uvw.shape[0], freq.ctypes.data, freq.size, vis.ctypes.data,
        None if wgt is None else wgt.ctypes.data, nu, nv, px, py, params["support"], int(nthreads),
        grid.ctypes.data)
    if bad < 0:
        raise ValueError("unsupported kernel support")
    return grid


def fft_backward(grid: np.ndarray, workers: int = 0) -> np.ndarray:
    """Unnormalised backward 2-D FFT (exp(+2 pi i)): scipy.fft with `workers`
    threads when scipy is present (numpy otherwise; the same fp64 transform)."""
    nu, nv = grid.shape
    try:
        import scipy.fft  # pylint: disable=import-outside-toplevel

        return scipy.fft.ifft2(grid, workers=workers or None) * (nu * nv)
    except ImportError:  # pragma: no cover - scipy is in the image
        return np.fft.ifft2(grid) * (nu * nv)


def baseline_ms2dirty(uvw, freq, vis, wgt, npix_x, npix_y, px, py, support=8, nthreads=0):
    """CPU BASELINE dirty image (2-D): tiled gridding + threaded FFT + crop +
    correction - the work one invert does, timed by bench.py's cpu_baseline."""
    prm = choose_params(npix_x, npix_y, px, py, support=support)
    nu, nv, W = prm["nu"], prm["nv"], prm["support"]
    g = grid_plane_tiled(uvw, freq, vis, wgt, prm, px, py, nthreads)
    ghat = fft_backward(g, nthreads)
    del g
    cx = 1.0 / kernel_ft(W, (np.arange(npix_x) - npix_x // 2) / nu)
    cy = 1.0 / kernel_ft(W, (np.arange(npix_y) - npix_y // 2) / nv)
    return _crop(ghat, npix_x, npix_y).real * cx[:, None] * cy[None, :]


def _crop(grid_hat: np.ndarray, npix_x: int, npix_y: int) -> np.ndarray:
    """(-1)^(p+q) G^[p mod nu, q mod nv] for p, q in [-npix/2, npix/2)."""
    nu, nv = grid_hat.shape
    p = np.arange(npix_x) - npix_x // 2
    q = np.arange(npix_y) - npix_y // 2
    sub = grid_hat[np.ix_(p % nu, q % nv)]
    sgn = np.where((p[:, None] + q[None, :]) % 2 == 0, 1.0, -1.0)
    return sgn * sub


def _nm1(npix_x, npix_y, px, py):
    l = (np.arange(npix_x) - npix_x // 2) * px  # noqa: E741
    m = (np.arange(npix_y) - npix_y // 2) * py
    e = l[:, None] ** 2 + m[None, :] ** 2
    return -e / (np.sqrt(1.0 - e) + 1.0)


def ms2dirty(uvw, freq, vis, wgt, npix_x, npix_y, px, py, epsilon=1e-4, support=None,
             do_wstacking=False, nthreads=0, return_params=False, planes=None):
    """fp64 dirty image of the oracle pipeline (same definition as the GPU).
    planes=(begin, end) (w-stacking): the share of w planes [begin, end) of
    the stack (cip_ms2dirty_wplanes); the shares of a partition of the stack
    sum to the image."""
    uvw, freq, vis, wgt = _as_inputs(uvw, freq, vis, wgt)
    wmin, wmax = w_range(uvw, freq) if do_wstacking else (0.0, 0.0)
    prm = choose_params(npix_x, npix_y, px, py, epsilon, support, do_wstacking, wmin, wmax)
    nu, nv, W = prm["nu"], prm["nv"], prm["support"]
    cx = 1.0 / kernel_ft(W, (np.arange(npix_x) - npix_x // 2) / nu)
    cy = 1.0 / kernel_ft(W, (np.arange(npix_y) - npix_y // 2) / nv)
    if not do_wstacking:
        g = grid_plane(uvw, freq, vis, wgt, prm, px, py, 0, nthreads)
        ghat = fft_backward(g, nthreads)  # backward, unnormalised: exp(+2 pi i)
        dirty = _crop(ghat, npix_x, npix_y).real * cx[:, None] * cy[None, :]
    else:
        nm1 = _nm1(npix_x, npix_y, px, py)
        acc = np.zeros((npix_x, npix_y))
        pb, pe = (0, prm["nplanes"]) if planes is None else (int(planes[0]), min(int(planes[1]), prm["nplanes"]))
        for p in range(pb, pe):
            g = grid_plane(uvw, freq, vis, wgt, prm, px, py, p, nthreads)
            ghat = fft_backward(g, nthreads)
            wp = prm["w0"] + p * prm["dw"]
            acc += (_crop(ghat, npix_x, npix_y) * np.exp(-2j * np.pi * wp * nm1)).real
        fw = kernel_ft(W, np.abs(prm["dw"] * nm1).ravel()).reshape(nm1.shape)
        dirty = acc * cx[:, None] * cy[None, :] / (fw * (nm1 + 1.0))
    if return_params:
        return dirty, prm
    return dirty


def dft_dirty(uvw, freq, vis, wgt, npix_x, npix_y, px, py, apply_w=False, nthreads=0):
    """Direct fp64 DFT dirty image (the definition)."""
    uvw, freq, vis, wgt = _as_inputs(uvw, freq, vis, wgt)
    out = np.empty((npix_x, npix_y))
    _lib().oracle_dft(uvw.ctypes.data, uvw.shape[0], freq.ctypes.data, freq.size, vis.ctypes.data,
                      None if wgt is None else wgt.ctypes.data, npix_x, npix_y, px, py,
                      int(bool(apply_w)), int(nthreads), out.ctypes.data)
    return out


def dft_directions(uvw, freq, vis, wgt, l, m):
    """Direct fp64 dirty image values at arbitrary directions (l, m) of the
    original tangent plane (same definition as dft_dirty, w term included):
    sum w Re{V exp(2 pi i f/c (u l + v m - w (n - 1)))}. Small cases only."""
    uvw = np.asarray(uvw, dtype=np.float64)
    fx = np.asarray(freq, dtype=np.float64) / SPEED_OF_LIGHT
    vis = np.asarray(vis).astype(np.complex128)
    wgt = np.ones(vis.shape) if wgt is None else np.asarray(wgt, dtype=np.float64)
    l = np.asarray(l, dtype=np.float64).ravel()
    m = np.asarray(m, dtype=np.float64).ravel()
    nm1 = -(l * l + m * m) / (np.sqrt(1.0 - l * l - m * m) + 1.0)
    out = np.zeros(l.size)
    wv = (wgt * vis)
    for c in range(fx.size):
        ph = 2.0 * np.pi * fx[c] * (np.outer(uvw[:, 0], l) + np.outer(uvw[:, 1], m) - np.outer(uvw[:, 2], nm1))
        out += (wv[:, c, None] * np.exp(1j * ph)).real.sum(axis=0)
    return out


def facet_rotation(l0, m0):
    """Q (3x3): the minimal rotation taking the phase centre (0, 0, 1) to the
    facet centre (l0, m0, n0) (restated for the facet tests: a facet pixel at
    (l', m') of the facet's tangent plane is the direction Q (l', m', n'))."""
    n0 = np.sqrt(1.0 - l0 * l0 - m0 * m0)
    axis = np.cross([0.0, 0.0, 1.0], [l0, m0, n0])
    s = np.linalg.norm(axis)
    if s == 0.0:
        return np.eye(3)
    k = axis / s
    kx = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return np.eye(3) + s * kx + (1.0 - n0) * (kx @ kx)


def facet_rephase(uvw, freq, vis, l0, m0):
    """The facet data (restated from the convention): with
    b = (u, v, -w), a source at s has delay d(s) = b.s - b.z; the facet frame
    holds V' = V exp(+2 pi i f/c d(s0)), s0 = (l0, m0, n0), and b' = Q^T b
    (Q = facet_rotation), stored as (u', v', w') = (b'_0, b'_1, -b'_2).
    numpy fp64; vis may be None (uvw only). Returns (uvw', vis' complex128)."""
    uvw = np.asarray(uvw, dtype=np.float64)
    b = uvw * np.array([1.0, 1.0, -1.0])
    n0m1 = -(l0 * l0 + m0 * m0) / (math.sqrt(1.0 - l0 * l0 - m0 * m0) + 1.0)
    delay = b[:, 0] * l0 + b[:, 1] * m0 + b[:, 2] * n0m1
    bp = b @ facet_rotation(l0, m0)  # rows: (Q^T b)^T = b^T Q
    uvw_out = np.ascontiguousarray(bp * np.array([1.0, 1.0, -1.0]))
    if vis is None:
        return uvw_out, None
    turns = delay[:, None] * (np.asarray(freq, dtype=np.float64)[None, :] / SPEED_OF_LIGHT)
    turns -= np.rint(turns)
    return uvw_out, np.asarray(vis).astype(np.complex128) * np.exp(2j * np.pi * turns)


def stokes(vis4, flags4, wgt4, which):
    """Stokes `which` from linear feeds (XX, XY, YX, YY) in numpy float32 /
    complex64 arithmetic (I as stokes_i) -> (vis c64, eff_w f32)."""
    vis4 = np.asarray(vis4)
    a, b = (0, 3) if which in "IQ" else (1, 2)
    half = np.float32(0.5)
    if which == "I":
        v = half * (vis4[..., 0] + vis4[..., 3])
    elif which == "Q":
        v = half * (vis4[..., 0] - vis4[..., 3])
    elif which == "U":
        v = half * (vis4[..., 1] + vis4[..., 2])
    else:
        d = vis4[..., 1] - vis4[..., 2]
        v = (half * d.imag + 1j * (-half * d.real)).astype(np.complex64)
    fl = np.logical_or(flags4[..., a], flags4[..., b])
    with np.errstate(divide="ignore", invalid="ignore"):
        w = (np.float32(4.0) / (np.float32(1.0) / wgt4[..., a] + np.float32(1.0) / wgt4[..., b])).astype(np.float32)
    return v.astype(np.complex64), (np.logical_not(fl) * w).astype(np.float32)


# ---------------------------------------------------- reference restated ----
def stokes_i(vis4, flags4, wgt4):
    """invert.py:86-116 and :72-76 -> (vis_i c64, flags_i bool, wgt_i f32, eff_w f32)."""
    vis4 = np.asarray(vis4)
    vis_i = (0.5 * (vis4[..., 0] + vis4[..., 3])).astype(np.complex64)
    flags_i = np.logical_or(flags4[..., 0], flags4[..., 3])
    with np.errstate(divide="ignore", invalid="ignore"):
        w = (np.float32(4.0) / (np.float32(1.0) / wgt4[..., 0] + np.float32(1.0) / wgt4[..., 3])).astype(
            np.float32)
    eff = (np.logical_not(flags_i) * w).astype(np.float32)
    return vis_i, flags_i, w, eff


def tile_mapping_sequential(uvw, tile_size, channel_freqs, row_offset=0) -> dict:
    """tiling_plan.py:29-61: {(iu, iv, iw): [(irow, c0, c1), ...]} in insertion order."""
    winv = np.asarray(channel_freqs, dtype=np.float64).reshape(-1, 1) / SPEED_OF_LIGHT
    ts = np.asarray(tile_size, dtype=np.float64)
    mapping: dict = {}
    for irow, row in enumerate(np.asarray(uvw, dtype=np.float64), start=row_offset):
        idx = np.floor(winv * (row / ts) + 0.5).astype(np.int64)
        change = np.ones(len(idx), dtype=bool)
        change[1:] = np.any(idx[1:] != idx[:-1], axis=1)
        starts = np.flatnonzero(change)
        stops = np.append(starts[1:], len(idx))
        for s, e in zip(starts, stops):
            key = tuple(int(v) for v in idx[s])
            mapping.setdefault(key, []).append((irow, int(s), int(e)))
    return mapping


def balanced_chunk_bounds(start: int, end: int, k: int):
    """measurement_set.py:379-391 (sizes :361-376)."""
    n = end - start
    q, r = divmod(n, k)
    out, lo = [], start
    for i in range(k):
        size = q + 1 if i < r else q
        out.append((lo, lo + size))
        lo += size
    return out


def split_tile_bounds(sizes, max_vis_per_chunk):
    """tile.py:155-211: row-slice index ranges of each chunk (never splits a slice)."""
    chunks, row, nrows, nvis = [], 0, 0, 0
    for size in sizes:
        if nvis + size > max_vis_per_chunk and nrows > 0:
            chunks.append((row, row + nrows))
            row += nrows
            nrows, nvis = 0, 0
        nrows += 1
        nvis += size
    if nrows:
        chunks.append((row, row + nrows))
    return chunks


def optional_int(x: Optional[int]) -> Optional[int]:
    return None if x is None else int(x)
