"""Diagnostic: GPU and oracle vs the DFT at a given image size / support."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"), str(ROOT / "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from ska_sdp_cip_amd import gridder, synthetic as syn  # noqa: E402
from ska_sdp_cip_amd.invert import StokesIGridderInput  # noqa: E402

npix, W, nrows, nchan = (int(a) for a in sys.argv[1:5])
ms = syn.make_measurement_set(nrows, nchan, n_ant=16, array_radius_m=1500.0, fov_l=0.01, seed=21)
gi = StokesIGridderInput.from_measurement_set_reader(ms)
uvw, f, vis, w = gi.uvw, gi.channel_frequencies, gi.visibilities, gi.effective_weights().astype(np.float32)
px = syn.pixel_size_for_grid(uvw, f, npix, support=W)
sw = float(w.astype(np.float64).sum())
ref = oracle.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=False)
gpu = gridder.ms2dirty(uvw, f, vis, w, npix, npix, px, px, support=W, do_wstacking=False)
dft = oracle.dft_dirty(uvw, f, vis, w, npix, npix, px, px, apply_w=False, nthreads=16)
e = lambda a, b: float(np.abs(a - b).max()) / sw  # noqa: E731
print(f"npix {npix} W {W}: gpu-oracle {e(gpu, ref):.3e}  gpu-dft {e(gpu, dft):.3e}  oracle-dft {e(ref, dft):.3e}")
d = np.abs(gpu - ref)
i, j = np.unravel_index(np.argmax(d), d.shape)
print("worst pixel", i, j, "gpu", gpu[i, j], "oracle", ref[i, j], "dft", dft[i, j])
print("err by row distance from centre:", [float(np.abs(gpu - ref)[k].max() / sw) for k in (0, npix // 4, npix // 2, 3 * npix // 4, npix - 1)])
