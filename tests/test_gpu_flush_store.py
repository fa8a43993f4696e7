"""
The scatter flush's private-cell stores (csrc/cip_scatter.h: a tile's only
work unit stores the cells no neighbour's sub-grid reaches instead of adding
them with fp64 atomics; on by default for planes of >= 16384^2 cells, where
bench.py --config c4 checks the image against the oracle). A child process
forces them on for every grid (CIP_FLUSH_STORE=1, read once per process) and
its images must equal this process's (stores off below 16384^2) to the last
bits - the flush atomics may sum a cell's contributions in another order, hence
1e-12 of the peak: cip_ms2dirty in 2-D (fp64 class), the reference's
w-stacking call (packed class, plane groups), repeated calls on the kept-clean
grid, the uv-strip path (cip_grid_tiles with CIP_GRID_ZEROED, 1 and 3 virtual
ranks) and chunked accumulation (cip_grid_ms without the flag: never stores).
"""

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _images():
    import torch

    import oracle
    from ska_sdp_cip_amd import gridder, strips, synthetic as syn
    from ska_sdp_cip_amd.accumulate import GridAccumulator, w_range_rows

    ms = syn.make_measurement_set(6_000, 16, n_ant=24, array_radius_m=1500.0, seed=31)
    vis, _, _, w = oracle.stokes_i(ms.visibilities(), ms.flags(), ms.weights())
    uvw, f = ms.uvw(), ms.channel_frequencies()
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    tu, tf, tv, tw = t(uvw), t(f), t(vis.astype(np.complex64)), t(w.astype(np.float32))
    out = {}
    npix = 512
    px = syn.pixel_size_for_grid(uvw, f, npix)
    for rep in range(2):
        img, prm = gridder.device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, support=8, normalise=True)
        out[f"2d_{rep}"] = img.cpu().numpy()
    img, _ = gridder.device_ms2dirty(tu, tf, tv, tw, npix, npix, px, px, epsilon=1e-4, do_wstacking=True,
                                     single_precision_accumulation=True, normalise=True)
    out["refcall"] = img.cpu().numpy()
    for world in (1, 3):
        layout = strips.plan_strips(tu, tf, prm, px, npix, npix, world)
        datas = []
        for r in range(world):
            datas.append(strips.split_strip(tu, tf, tv, tw, prm, px, *layout.rows(r)))
        be = strips.HipStripBackend(prm, px, px, npix, npix, device=dev)
        out[f"strips_{world}"] = strips.invert_strips_local(datas, tf, layout, be).cpu().numpy()
    acc = GridAccumulator(npix, npix, px, px, support=8, do_wstacking=False, w_range=w_range_rows(uvw, f))
    for a, b in [(0, 2_000), (2_000, 2_001), (2_001, 6_000)]:
        acc.add_ms(t(uvw[a:b]), tf, tv[a:b], tw[a:b])
    out["chunked"] = acc.dirty()[0].cpu().numpy()
    torch.cuda.synchronize()
    return out


CHILD = """
import sys
sys.path[:0] = [{root!r}, {pkg!r}, {orc!r}, {tests!r}]
import numpy as np
import test_gpu_flush_store as t
np.savez({out!r}, **t._images())
"""


def test_private_cell_stores_equal_atomics(gpu_device, tmp_path):
    mine = _images()
    out = tmp_path / "stores.npz"
    code = CHILD.format(root=str(ROOT), pkg=str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"),
                        orc=str(ROOT / "oracle"), tests=str(ROOT / "tests"), out=str(out))
    env = dict(os.environ, CIP_FLUSH_STORE="1")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    ref = np.load(out)
    assert sorted(ref.files) == sorted(mine)
    for k, img in mine.items():
        peak = float(np.abs(ref[k]).max())
        assert peak > 0, k
        assert float(np.abs(img - ref[k]).max()) <= 1e-12 * peak, k
