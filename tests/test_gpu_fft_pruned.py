"""
The pruned FFT fast path (csrc/cip_fft.hip row pass + hipFFT column pass on
the kept half) against the fp64 oracle, at every grid size it serves
(nv = 1024 .. 8192, i.e. npix = 512 .. 4096 at sigma = 2), in 2-D and
w-stacking mode. Other sizes take the full 2-D hipFFT path (covered by
test_gpu_invert_parity.py at npix <= 256).
"""

import numpy as np
import pytest

import oracle
from ska_sdp_cip_amd import gridder, synthetic as syn
from ska_sdp_cip_amd.invert import StokesIGridderInput

pytestmark = pytest.mark.gpu

TIGHT = 1e-10


def _case(n_rows, nchan, seed=11):
    ms = syn.make_measurement_set(n_rows, nchan, n_ant=32, array_radius_m=3000.0, fov_l=0.02, seed=seed)
    gi = StokesIGridderInput.from_measurement_set_reader(ms)
    return gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)


@pytest.mark.parametrize("npix,wstack", [(512, False), (1024, False), (2048, False), (4096, False),
                                         (512, True)])
def test_pruned_fft_matches_oracle(gpu_device, npix, wstack):
    uvw, f, vis, w = _case(3_000 if npix < 4096 else 1_000, 4)
    px = syn.pixel_size_for_grid(uvw, f, npix, fill=0.4)
    gpu, prm = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=wstack,
                                return_params=True, double_precision_accumulation=True)
    assert prm.nu == 2 * npix
    ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=8, do_wstacking=wstack)
    sumw = float(w.astype(np.float64).sum())
    # float32 output for complex64 input: compare at float32 resolution of the peak
    tol = max(TIGHT, 4e-7 * float(np.abs(ref).max()) / sumw)
    assert float(np.abs(gpu - ref).max()) / sumw < tol


def test_pruned_fft_rectangular_image(gpu_device):
    # npix_x != npix_y: the row pass keeps npix_y columns of an nv-point transform
    uvw, f, vis, w = _case(2_000, 2)
    px = syn.pixel_size_for_grid(uvw, f, 1024, fill=0.4)
    import torch

    args = [torch.from_numpy(a).cuda() for a in (uvw, f, vis.astype(np.complex128), w.astype(np.float64))]
    gpu, prm = gridder.device_ms2dirty(*args, 768, 1024, px, px, support=8)
    ref = oracle.ms2dirty(uvw, f, vis, w, 768, 1024, px, px, support=8)
    sumw = float(w.astype(np.float64).sum())
    assert prm.nv == 2048
    assert float(np.abs(gpu.cpu().numpy() - ref).max()) / sumw < TIGHT
