"""
`ms2dirty`: MI355X drop-in for `ducc0.wgridder.ms2dirty` as the reference
calls it (`/root/reference/src/ska_sdp_cip/invert.py:170-183`).

Host side only: moves arrays to HBM (torch tensors are used purely as device
buffers), calls `cip_ms2dirty` of libcip_hip.so on the current HIP stream and
returns the dirty image. Accepts numpy arrays (returns numpy) or CUDA/HIP
torch tensors (returns a torch tensor on the same device, no host round trip).

Definition computed (ducc0's documented ms2dirty):
    dirty[i, j] = (1/n) sum_{r,c} wgt[r,c] Re{ ms[r,c]
                  exp(2 pi i f_c/c (u_r l + v_r m - w_r (n - 1))) }
with l = (i - npix_x/2) pixsize_x, m = (j - npix_y/2) pixsize_y,
n = sqrt(1 - l^2 - m^2); in 2-D mode (do_wstacking=False) n := 1.
"""

from __future__ import annotations

from typing import Optional

import numpy as np

from . import _lib

try:  # torch is plumbing (device memory, streams); import lazily-safe
    import torch
except ModuleNotFoundError:  # pragma: no cover - torch is in the image
    torch = None


def _require_gpu():
    if torch is None or not torch.cuda.is_available():
        raise RuntimeError(
            "ska_sdp_cip_amd.ms2dirty needs a ROCm GPU (MI355X); no CPU fallback"
        )


def _to_device(x, dtype, device):
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x))
        return t.to(device=device, dtype=dtype, non_blocking=False)
    return x.to(device=device, dtype=dtype).contiguous()


_VIS_CODES = {}
_WGT_CODES = {}


def _codes():
    if not _VIS_CODES:
        _VIS_CODES.update({torch.complex64: _lib.CIP_C64, torch.complex128: _lib.CIP_C128})
        _WGT_CODES.update({torch.float32: _lib.CIP_F32, torch.float64: _lib.CIP_F64})
    return _VIS_CODES, _WGT_CODES


def device_ms2dirty(
    uvw: "torch.Tensor",
    freq: "torch.Tensor",
    vis: "torch.Tensor",
    wgt: Optional["torch.Tensor"],
    npix_x: int,
    npix_y: int,
    pixsize_x: float,
    pixsize_y: float,
    *,
    epsilon: float = 1e-4,
    support: Optional[int] = None,
    do_wstacking: bool = False,
    out: Optional["torch.Tensor"] = None,
    sum_weights: Optional["torch.Tensor"] = None,
    single_precision_accumulation: bool = False,
    psf: bool = False,
    normalise: bool = False,
    synchronize: bool = True,
    resident_inputs: bool = False,
    reuse_plan: bool = False,
    planes: Optional[tuple] = None,
) -> tuple["torch.Tensor", _lib.GridderParams]:
    """
    Device-resident ms2dirty: all tensors already in HBM on the current device.
    Returns (dirty fp64 tensor (npix_x, npix_y), params). `sum_weights`
    (fp64, 1 element) receives the sum of `wgt` when given.
    `single_precision_accumulation` (complex64 `vis` only) selects the packed
    single-precision class (CIP_ACC_SINGLE, include/cip.h): quantisation
    2^-19 of max|w V| per contribution, like ducc0's float gridding; the
    default accumulates every input in 64-bit fixed point (fp64 class).
    `psf=True` grids unit visibilities instead of `vis` (the point-spread
    function with the same weights; `vis` may then be None).
    `normalise=True` (CIP_NORMALISE) returns the image divided by the weight
    sum of this call (the reference's (1 / total_weight) * image,
    invert.py:119-149), fused into the FFT epilogue; not for partial images
    that are summed across ranks afterwards.
    `synchronize=False` (CIP_ASYNC) returns once the work is queued on the
    current stream: `out` / `sum_weights` are valid in stream order (the next
    kernel or copy on that stream sees them; the host must synchronise before
    reading them). The planner's two mid-call readbacks still wait.
    `resident_inputs=True` (CIP_PIPELINE, with `synchronize=False` only)
    promises that uvw / freq / vis / wgt were complete before the previous
    asynchronous call returned and stay unchanged (resident data, as in the
    benchmark): the planner of this call then runs beside the previous call's
    scatter and FFT instead of after all work queued on the stream.
    `reuse_plan=True` (CIP_REUSE_PLAN, not with `resident_inputs`) promises
    that uvw, freq and the row layout equal those of this thread's previous
    planned call (e.g. the Stokes parameters and PSF of one facet): if that
    call's geometry matches, its tile plan is used again and only the weight
    sum and max |w V| are computed (images identical to a planned call's).
    `planes=(begin, end)` (w-stacking only, cip_ms2dirty_wplanes): the partial
    image of w planes [begin, end) of the stack - the share of one GPU when the
    plane groups of ONE image are split over GPUs (SURVEY.md 8(e) option 2,
    `wplanes.py`); the partial images of a partition of [0, nplanes) sum to
    the whole image (the final w correction and `normalise` are linear and
    applied to each part; `sum_weights` is the whole call's weight sum).
    """
    if planes is not None and not do_wstacking:
        raise ValueError("planes=(begin, end) needs do_wstacking=True")
    if resident_inputs and synchronize:
        raise ValueError("resident_inputs=True needs synchronize=False")
    if reuse_plan and resident_inputs:
        raise ValueError("reuse_plan=True cannot be combined with resident_inputs=True")
    vis_codes, wgt_codes = _codes()
    if psf:
        vis = None  # never read
    elif vis is None or vis.dtype not in vis_codes:
        raise ValueError(f"vis dtype must be complex64/complex128, got {getattr(vis, 'dtype', None)}")
    if wgt is not None and wgt.dtype not in wgt_codes:
        raise ValueError(f"wgt dtype must be float32/float64, got {wgt.dtype}")
    nrow = uvw.shape[0]
    nchan = freq.shape[0]
    if tuple(uvw.shape) != (nrow, 3):
        raise ValueError("uvw must have shape (nrow, 3)")
    if vis is not None and tuple(vis.shape) != (nrow, nchan):
        raise ValueError(f"ms must have shape ({nrow}, {nchan}), got {tuple(vis.shape)}")
    if wgt is not None and tuple(wgt.shape) != (nrow, nchan):
        raise ValueError("wgt must have the shape of ms")
    if uvw.dtype != torch.float64 or freq.dtype != torch.float64:
        raise ValueError("uvw and freq must be float64")
    for t in (uvw, freq) + ((vis,) if vis is not None else ()) + ((wgt,) if wgt is not None else ()):
        _check_device_tensor(t, uvw.device, "device_ms2dirty inputs")
    if out is None:
        out = torch.empty((npix_x, npix_y), dtype=torch.float64, device=uvw.device)
    else:
        # the library writes npix_x * npix_y doubles through the raw pointer
        if out.dtype != torch.float64 or tuple(out.shape) != (int(npix_x), int(npix_y)):
            raise ValueError(f"out must be float64 of shape ({npix_x}, {npix_y}), "
                             f"got {out.dtype} {tuple(out.shape)}")
        _check_device_tensor(out, uvw.device, "out")
    if sum_weights is not None:
        if sum_weights.dtype != torch.float64 or sum_weights.numel() != 1:
            raise ValueError("sum_weights must be a float64 tensor of one element")
        _check_device_tensor(sum_weights, uvw.device, "sum_weights")
    params = _lib.GridderParams()
    with torch.cuda.device(uvw.device):
        stream = torch.cuda.current_stream(uvw.device).cuda_stream
        rc = _ms2dirty_call(uvw, freq, vis, wgt, vis_codes, wgt_codes, npix_x, npix_y, pixsize_x, pixsize_y,
                            epsilon, support, do_wstacking, single_precision_accumulation, psf, normalise,
                            stream, out, sum_weights, params, synchronize, resident_inputs, reuse_plan, planes)
    _lib.check(rc)
    return out, params


def _check_device_tensor(t, device, what):
    """Contiguous, on a GPU, and on `device` (the library works on the current
    device, which the callers set to `device`)."""
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{what}: need contiguous device tensors")
    if t.device != device:
        raise ValueError(f"{what}: tensor on {t.device}, expected {device}")


def _ms2dirty_call(uvw, freq, vis, wgt, vis_codes, wgt_codes, npix_x, npix_y, pixsize_x, pixsize_y, epsilon,
                   support, do_wstacking, single_precision_accumulation, psf, normalise, stream, out,
                   sum_weights, params, synchronize=True, resident_inputs=False, reuse_plan=False, planes=None):
    nrow = uvw.shape[0]
    nchan = freq.shape[0]
    head = (uvw.data_ptr(), nrow, freq.data_ptr(), nchan, None if vis is None else vis.data_ptr(),
            _lib.CIP_C64 if vis is None else vis_codes[vis.dtype],
            wgt.data_ptr() if wgt is not None else None,
            wgt_codes[wgt.dtype] if wgt is not None else _lib.CIP_NONE,
            int(npix_x), int(npix_y), float(pixsize_x), float(pixsize_y), float(epsilon),
            int(support or 0),
            (_lib.CIP_WSTACKING if do_wstacking else 0)
            | (_lib.CIP_ACC_SINGLE if single_precision_accumulation else 0)
            | (_lib.CIP_PSF if psf else 0)
            | (_lib.CIP_NORMALISE if normalise else 0)
            | (0 if synchronize else _lib.CIP_ASYNC)
            | (_lib.CIP_PIPELINE if resident_inputs else 0)
            | (_lib.CIP_REUSE_PLAN if reuse_plan else 0))
    tail = (stream, out.data_ptr(), sum_weights.data_ptr() if sum_weights is not None else None, params)
    if planes is not None:
        return _lib.lib().cip_ms2dirty_wplanes(*head, int(planes[0]), int(planes[1]), *tail)
    return _lib.lib().cip_ms2dirty(*head, *tail)


def device_ms2dirty_stokes_i(
    uvw: "torch.Tensor",
    freq: "torch.Tensor",
    vis4: Optional["torch.Tensor"],
    flags4: Optional["torch.Tensor"],
    wgt4: "torch.Tensor",
    npix_x: int,
    npix_y: int,
    pixsize_x: float,
    pixsize_y: float,
    *,
    epsilon: float = 1e-4,
    support: Optional[int] = None,
    do_wstacking: bool = False,
    out: Optional["torch.Tensor"] = None,
    sum_weights: Optional["torch.Tensor"] = None,
    single_precision_accumulation: bool = False,
    psf: bool = False,
    normalise: bool = False,
    synchronize: bool = True,
    resident_inputs: bool = False,
    reuse_plan: bool = False,
) -> tuple["torch.Tensor", _lib.GridderParams]:
    """
    device_ms2dirty on the raw linear-feed columns (cip_ms2dirty_stokes_i):
    vis4 (nrow, nchan, 4) complex64 XX, XY, YX, YY, flags4 (nrow, nchan, 4)
    bool/uint8 or None, wgt4 (nrow, nchan, 4) float32. Stokes I and the
    effective weights (reference invert.py:78-116) are formed inside the
    planner and scatter as each visibility is loaded - no intermediate
    columns; the image is bit-identical to device_stokes_i + device_ms2dirty.
    Keyword arguments as device_ms2dirty.
    """
    if resident_inputs and synchronize:
        raise ValueError("resident_inputs=True needs synchronize=False")
    if reuse_plan and resident_inputs:
        raise ValueError("reuse_plan=True cannot be combined with resident_inputs=True")
    nrow, nchan = uvw.shape[0], freq.shape[0]
    shape = (nrow, nchan, 4)
    if psf:
        vis4 = None
    elif vis4 is None or vis4.dtype != torch.complex64 or tuple(vis4.shape) != shape:
        raise ValueError(f"vis4 must be complex64 of shape {shape}")
    if wgt4 is None or wgt4.dtype != torch.float32 or tuple(wgt4.shape) != shape:
        raise ValueError(f"wgt4 must be float32 of shape {shape}")
    if flags4 is not None:
        if tuple(flags4.shape) != shape:
            raise ValueError(f"flags4 must have shape {shape}")
        if flags4.dtype == torch.bool:
            flags4 = flags4.view(torch.uint8)
        elif flags4.dtype != torch.uint8:
            raise ValueError("flags4 must be bool or uint8")
    if tuple(uvw.shape) != (nrow, 3) or uvw.dtype != torch.float64 or freq.dtype != torch.float64:
        raise ValueError("uvw must be float64 (nrow, 3) and freq float64")
    for t in (uvw, freq, wgt4) + tuple(x for x in (vis4, flags4) if x is not None):
        _check_device_tensor(t, uvw.device, "device_ms2dirty_stokes_i inputs")
    if out is None:
        out = torch.empty((npix_x, npix_y), dtype=torch.float64, device=uvw.device)
    elif out.dtype != torch.float64 or tuple(out.shape) != (int(npix_x), int(npix_y)):
        raise ValueError(f"out must be float64 of shape ({npix_x}, {npix_y})")
    else:
        _check_device_tensor(out, uvw.device, "out")
    if sum_weights is not None:
        if sum_weights.dtype != torch.float64 or sum_weights.numel() != 1:
            raise ValueError("sum_weights must be a float64 tensor of one element")
        _check_device_tensor(sum_weights, uvw.device, "sum_weights")
    params = _lib.GridderParams()
    with torch.cuda.device(uvw.device):
        stream = torch.cuda.current_stream(uvw.device).cuda_stream
        rc = _lib.lib().cip_ms2dirty_stokes_i(
            uvw.data_ptr(), nrow, freq.data_ptr(), nchan, None if vis4 is None else vis4.data_ptr(),
            None if flags4 is None else flags4.data_ptr(), wgt4.data_ptr(), int(npix_x), int(npix_y),
            float(pixsize_x), float(pixsize_y), float(epsilon), int(support or 0),
            (_lib.CIP_WSTACKING if do_wstacking else 0)
            | (_lib.CIP_ACC_SINGLE if single_precision_accumulation else 0)
            | (_lib.CIP_PSF if psf else 0)
            | (_lib.CIP_NORMALISE if normalise else 0)
            | (0 if synchronize else _lib.CIP_ASYNC)
            | (_lib.CIP_PIPELINE if resident_inputs else 0)
            | (_lib.CIP_REUSE_PLAN if reuse_plan else 0),
            stream, out.data_ptr(), sum_weights.data_ptr() if sum_weights is not None else None, params)
    _lib.check(rc)
    return out, params


def device_stokes(vis4: "torch.Tensor", flags4: "torch.Tensor", wgt4: "torch.Tensor", stokes: str = "I"):
    """
    Stokes parameter `stokes` ("I", "Q", "U", "V") on the device (cip_stokes;
    linear feeds XX, XY, YX, YY; I is the reference's invert.py:72-116,
    bit-exact): -> (visibilities complex64 (nrow, nchan), effective weights
    float32 (nrow, nchan)).
    """
    _require_gpu()
    if stokes not in _lib.STOKES_CODES:
        raise ValueError(f"stokes must be one of I, Q, U, V, got {stokes!r}")
    if vis4.dtype != torch.complex64 or wgt4.dtype != torch.float32:
        raise ValueError("vis4 must be complex64 and wgt4 float32")
    if vis4.dim() != 3 or vis4.shape[-1] != 4 or tuple(flags4.shape) != tuple(vis4.shape) or \
            tuple(wgt4.shape) != tuple(vis4.shape):
        raise ValueError("vis4, flags4, wgt4 must all have shape (nrow, nchan, 4)")
    fl = flags4.to(torch.uint8) if flags4.dtype != torch.uint8 else flags4
    for t in (vis4, fl, wgt4):
        if not t.is_contiguous() or not t.is_cuda:
            raise ValueError("device_stokes needs contiguous device tensors")
    nrow, nchan = vis4.shape[0], vis4.shape[1]
    vis_s = torch.empty((nrow, nchan), dtype=torch.complex64, device=vis4.device)
    eff = torch.empty((nrow, nchan), dtype=torch.float32, device=vis4.device)
    with torch.cuda.device(vis4.device):
        stream = torch.cuda.current_stream(vis4.device).cuda_stream
        _lib.check(_lib.lib().cip_stokes(vis4.data_ptr(), fl.data_ptr(), wgt4.data_ptr(), nrow * nchan,
                                         _lib.STOKES_CODES[stokes], stream, vis_s.data_ptr(), None, None,
                                         eff.data_ptr()))
    return vis_s, eff


def device_facet_rephase(uvw: "torch.Tensor", freq: "torch.Tensor", vis: Optional["torch.Tensor"],
                         l0: float, m0: float):
    """
    Facet data (cip_facet_rephase): visibilities rephased to the facet centre
    (l0, m0) of the image plane and baselines rotated into the facet's frame,
    so that device_ms2dirty of the result is the dirty image on the facet's own
    tangent plane centred on (l0, m0). Returns (uvw_f, vis_f); vis may be None
    (uvw only, for a facet PSF).
    """
    _require_gpu()
    vis_codes, _ = _codes()
    nrow, nchan = uvw.shape[0], freq.shape[0]
    if vis is not None and (vis.dtype not in vis_codes or tuple(vis.shape) != (nrow, nchan)):
        raise ValueError("vis must be complex64/complex128 of shape (nrow, nchan)")
    for t in (uvw, freq) + ((vis,) if vis is not None else ()):
        if not t.is_contiguous() or not t.is_cuda:
            raise ValueError("device_facet_rephase needs contiguous device tensors")
    uvw_f = torch.empty_like(uvw)
    vis_f = torch.empty_like(vis) if vis is not None else None
    with torch.cuda.device(uvw.device):
        stream = torch.cuda.current_stream(uvw.device).cuda_stream
        _lib.check(_lib.lib().cip_facet_rephase(
            uvw.data_ptr(), nrow, freq.data_ptr(), nchan, vis.data_ptr() if vis is not None else None,
            vis_codes[vis.dtype] if vis is not None else _lib.CIP_C64, float(l0), float(m0), stream,
            uvw_f.data_ptr(), vis_f.data_ptr() if vis_f is not None else None))
    return uvw_f, vis_f


def device_stokes_i(vis4: "torch.Tensor", flags4: "torch.Tensor", wgt4: "torch.Tensor"):
    """
    Stokes I on the device (cip_stokes_i; reference invert.py:72-116, bit-exact
    with its numpy arithmetic): (nrow, nchan, 4) complex64 visibilities,
    bool/uint8 flags and float32 weights -> (vis_i complex64 (nrow, nchan),
    effective weights float32 (nrow, nchan)).
    """
    _require_gpu()
    if vis4.dtype != torch.complex64 or wgt4.dtype != torch.float32:
        raise ValueError("vis4 must be complex64 and wgt4 float32")
    if vis4.dim() != 3 or vis4.shape[-1] != 4 or tuple(flags4.shape) != tuple(vis4.shape) or \
            tuple(wgt4.shape) != tuple(vis4.shape):
        raise ValueError("vis4, flags4, wgt4 must all have shape (nrow, nchan, 4)")
    fl = flags4.to(torch.uint8) if flags4.dtype != torch.uint8 else flags4
    for t in (vis4, fl, wgt4):
        if not t.is_contiguous() or not t.is_cuda:
            raise ValueError("device_stokes_i needs contiguous device tensors")
    nrow, nchan = vis4.shape[0], vis4.shape[1]
    vis_i = torch.empty((nrow, nchan), dtype=torch.complex64, device=vis4.device)
    eff = torch.empty((nrow, nchan), dtype=torch.float32, device=vis4.device)
    with torch.cuda.device(vis4.device):
        stream = torch.cuda.current_stream(vis4.device).cuda_stream
        _lib.check(_lib.lib().cip_stokes_i(vis4.data_ptr(), fl.data_ptr(), wgt4.data_ptr(), nrow * nchan, stream,
                                           vis_i.data_ptr(), None, None, eff.data_ptr()))
    return vis_i, eff


def ms2dirty(  # pylint: disable=too-many-arguments,unused-argument
    uvw,
    freq,
    ms,
    wgt=None,
    npix_x: int = None,
    npix_y: int = None,
    pixsize_x: float = None,
    pixsize_y: float = None,
    nu: int = 0,
    nv: int = 0,
    epsilon: float = 1e-4,
    do_wstacking: bool = False,
    nthreads: int = 1,
    verbosity: int = 0,
    mask=None,
    double_precision_accumulation: Optional[bool] = None,
    *,
    support: Optional[int] = None,
    device=None,
    return_params: bool = False,
):
    """
    Drop-in for `ducc0.wgridder.ms2dirty` (same positional order as the call
    at reference invert.py:170-183). `nu`, `nv`, `nthreads` and `verbosity`
    are accepted for signature compatibility and ignored (the grid is chosen
    from epsilon / `support`). Accumulation is 64-bit fixed point unless
    `double_precision_accumulation=False` is passed explicitly with complex64
    `ms` (ducc0's float gridding class, CIP_ACC_SINGLE); left at None it is the
    fp64 class, at least as accurate as ducc0 in every mode. `mask` (uint8,
    shape of ms) zeroes the weights where 0. Output dtype follows ducc:
    float32 for complex64 `ms`, else float64.
    """
    _require_gpu()
    if npix_x is None or npix_y is None or pixsize_x is None or pixsize_y is None:
        raise TypeError("npix_x, npix_y, pixsize_x and pixsize_y are required")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    numpy_in = isinstance(ms, np.ndarray)
    ms_dtype = ms.dtype
    single = ms_dtype in (np.complex64, torch.complex64)
    with torch.cuda.device(dev):
        uvw_d = _to_device(uvw, torch.float64, dev)
        freq_d = _to_device(np.asarray(freq, dtype=np.float64) if not torch.is_tensor(freq) else freq,
                            torch.float64, dev)
        vis_d = _to_device(ms, torch.complex64 if single else torch.complex128, dev)
        wgt_d = None
        if wgt is not None:
            wdt = torch.float32 if (wgt.dtype in (np.float32, torch.float32)) else torch.float64
            wgt_d = _to_device(wgt, wdt, dev)
        if mask is not None:
            m = _to_device(np.asarray(mask) if not torch.is_tensor(mask) else mask, torch.bool, dev)
            if wgt_d is None:
                wgt_d = m.to(torch.float32)
            else:
                wgt_d = wgt_d * m.to(wgt_d.dtype)
        dirty, params = device_ms2dirty(
            uvw_d, freq_d, vis_d, wgt_d, int(npix_x), int(npix_y), float(pixsize_x),
            float(pixsize_y), epsilon=epsilon, support=support, do_wstacking=do_wstacking,
            single_precision_accumulation=single and double_precision_accumulation is False)
        dirty = dirty.to(torch.float32) if single else dirty
        result = dirty.cpu().numpy() if numpy_in else dirty
    if return_params:
        return result, params
    return result
