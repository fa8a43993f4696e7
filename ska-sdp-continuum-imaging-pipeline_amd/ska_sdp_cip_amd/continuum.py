"""
Full continuum invert (config C5: PSF + dirty images, 4 Stokes, facets) -
SURVEY.md 8(f) item 4. This goes beyond the reference, whose pipeline makes a
Stokes-I dirty image only (invert.py:119-149); every image here is made by
the same device invert (cip_ms2dirty), on inputs prepared on the device:

* Stokes I, Q, U, V + effective weights from the raw (rows, chans, 4)
  columns (cip_stokes; I is the reference's arithmetic, bit-exact);
* facets: the data rephased to each facet centre and the baselines rotated
  into the facet's frame (cip_facet_rephase), so each facet image is the
  dirty image on its own tangent plane - exact, also with w-stacking;
* PSF: unit visibilities with the Stokes-I weights (CIP_PSF), per facet frame.

Facets are independent images: with several GPUs (torch.distributed, one
process per GPU) rank r makes the facets k with k % world == r; there is no
exchange between ranks.
"""

from __future__ import annotations

from typing import Iterable, Optional, Sequence

import numpy as np

from .gridder import _require_gpu, device_facet_rephase, device_ms2dirty, device_stokes
from .invert import EPSILON, pixel_size_lm

try:
    import torch
except ModuleNotFoundError:  # pragma: no cover - torch is in the image
    torch = None


def facet_centres(n_facets_x: int, n_facets_y: int, facet_pixels: int, pixel_size: float) -> list:
    """Centres (l0, m0) of an n_facets_x x n_facets_y mosaic of facets of
    facet_pixels^2 pixels of `pixel_size` (sin-projected radians) around the
    phase centre, row-major in (x, y)."""
    step = facet_pixels * pixel_size
    return [((ix - (n_facets_x - 1) / 2.0) * step, (iy - (n_facets_y - 1) / 2.0) * step)
            for ix in range(n_facets_x) for iy in range(n_facets_y)]


def continuum_invert(
    vis4, flags4, wgt4, uvw, freq,
    facet_pixels: int,
    pixel_size_asec: float,
    *,
    facets: Optional[Sequence[tuple[float, float]]] = None,
    stokes: Iterable[str] = "IQUV",
    psf: bool = True,
    epsilon: float = EPSILON,
    support: Optional[int] = None,
    do_wstacking: bool = True,
    rank: int = 0,
    world: int = 1,
    reuse_plans: bool = True,
    single_precision_accumulation: bool = False,
) -> dict:
    """
    Dirty images (normalised by each Stokes parameter's weight sum) and PSFs
    (normalised: peak 1) of device-resident raw columns: vis4 (nrow, nchan, 4)
    complex64, flags4 bool/uint8, wgt4 float32, uvw (nrow, 3) f64, freq
    (nchan,) f64. `facets`: centres (l0, m0) (default: one facet at the phase
    centre). Returns {(name, k): fp64 device tensor (facet_pixels,
    facet_pixels)} with name in `stokes` or "PSF", for this rank's facets k.
    `reuse_plans`: a facet's later products reuse its first product's tile
    plan (the same rephased uvw; identical images, one planner per facet).
    `single_precision_accumulation`: the packed single-precision class (ducc0's
    float class of the reference's complex64 call) instead of fp64.
    """
    _require_gpu()
    pix = pixel_size_lm(pixel_size_asec)
    facets = [(0.0, 0.0)] if facets is None else list(facets)
    stokes = list(stokes)
    kw = dict(epsilon=epsilon, support=support, do_wstacking=do_wstacking,
              single_precision_accumulation=single_precision_accumulation)
    per_stokes = {s: device_stokes(vis4, flags4, wgt4, s) for s in stokes}
    wts = {s: eff for s, (_, eff) in per_stokes.items()}
    if psf and "I" not in wts:
        wts["I"] = device_stokes(vis4, flags4, wgt4, "I")[1]
    sums = {s: w.sum(dtype=torch.float64) for s, w in wts.items()}
    out = {}
    for k, (l0, m0) in enumerate(facets):
        if k % world != rank:
            continue
        # the facet's products share its rephased uvw: the first one plans,
        # the others reuse that tile plan (CIP_REUSE_PLAN)
        planned = False
        for s, (vis_s, eff) in per_stokes.items():
            uvw_f, vis_f = device_facet_rephase(uvw, freq, vis_s, l0, m0)
            img, _ = device_ms2dirty(uvw_f, freq, vis_f, eff, facet_pixels, facet_pixels, pix, pix,
                                     reuse_plan=planned and reuse_plans, **kw)
            planned = True
            out[(s, k)] = img.div_(sums[s])
        if psf:
            uvw_f, _ = device_facet_rephase(uvw, freq, None, l0, m0)
            img, _ = device_ms2dirty(uvw_f, freq, None, wts["I"], facet_pixels, facet_pixels, pix, pix, psf=True,
                                     reuse_plan=planned and reuse_plans, **kw)
            out[("PSF", k)] = img.div_(sums["I"])
    return out


def continuum_invert_measurement_set(ms_reader, facet_pixels: int, pixel_size_asec: float, **kwargs) -> dict:
    """`continuum_invert` of a measurement set reader's columns (moved to the
    current device once); images returned as float32 numpy arrays."""
    _require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())

    def t(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)

    res = continuum_invert(t(ms_reader.visibilities(), np.complex64), t(ms_reader.flags(), np.uint8),
                           t(ms_reader.weights(), np.float32), t(ms_reader.uvw(), np.float64),
                           t(ms_reader.channel_frequencies(), np.float64), facet_pixels, pixel_size_asec, **kwargs)
    return {k: v.to(torch.float32).cpu().numpy() for k, v in res.items()}


__all__ = ["continuum_invert", "continuum_invert_measurement_set", "facet_centres"]
