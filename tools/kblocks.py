#!/usr/bin/env python3
"""EXPERIMENT: executed plane blocks of the packed plane-group scatter on the
C3 reference call, from a counting build (-DCIP_COUNT_KBLOCKS, loaded with
CIP_HIP_LIB). Prints visits, lane-blocks with work and wave-blocks executed."""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "ska-sdp-continuum-imaging-pipeline_amd"), str(ROOT)]


def main():
    import numpy as np
    import torch

    import bench
    from ska_sdp_cip_amd import _lib
    from ska_sdp_cip_amd.gridder import device_ms2dirty

    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    uvw, freq, vis, wgt, px, _, _ = bench.make_inputs(cfg, 0, 1, dev)
    so = _lib.lib()
    so.cip_debug_kblocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(192, dtype=np.uint64)
    so.cip_debug_kblocks(buf.ctypes.data, 1)
    device_ms2dirty(uvw, freq, vis, wgt, cfg["npix"], cfg["npix"], px, px, epsilon=1e-4, do_wstacking=True,
                    single_precision_accumulation=True)
    torch.cuda.synchronize()
    so.cip_debug_kblocks(buf.ctypes.data, 0)
    visits = int(buf[:64].sum())
    lane_blocks = int(buf[64:128].sum())
    wave_blocks_lanes = int(buf[128:].sum())  # each lane of a wave counts its wave's executed blocks
    print(json.dumps({"lane_visits": visits, "useful_lane_blocks": lane_blocks,
                      "executed_lane_blocks": wave_blocks_lanes,
                      "useful_blocks_per_visit": lane_blocks / max(visits, 1),
                      "executed_blocks_per_visit": wave_blocks_lanes / max(visits, 1),
                      "block_efficiency": lane_blocks / max(wave_blocks_lanes, 1)}))


if __name__ == "__main__":
    main()
