"""
The streaming reader protocol: `read_into` fills
caller-owned (pinned) arrays with exactly what the reference-style column
getters return, for bounded readers, WEIGHT-only sets and disjoint row blocks
filled from several threads; readers without it go through the copying
adapter. CPU only.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from ska_sdp_cip_amd import synthetic as syn
from ska_sdp_cip_amd.measurement_set import InMemoryMeasurementSet


def _empty(n, nchan):
    return {"uvw": np.empty((n, 3)), "vis4": np.empty((n, nchan, 4), np.complex64),
            "flags4": np.empty((n, nchan, 4), np.uint8), "wgt4": np.empty((n, nchan, 4), np.float32)}


def _check(out, r):
    assert np.array_equal(out["uvw"], r.uvw())
    assert np.array_equal(out["vis4"], r.visibilities(), equal_nan=True)
    assert np.array_equal(out["flags4"].astype(bool), r.flags())
    assert np.array_equal(out["wgt4"], r.weights())


@pytest.mark.parametrize("weight_only", [False, True])
def test_read_into_matches_getters(weight_only):
    ms = syn.make_measurement_set(300, 6, n_ant=8, seed=2)
    if weight_only:
        ms = InMemoryMeasurementSet(ms.uvw(), ms.visibilities(), ms.flags(), ms.weights()[:, 0, :],
                                    ms.channel_frequencies())
    for r in [ms] + ms.partition(3, 2):
        out = _empty(r.num_data_rows, r.num_channels)
        # disjoint row blocks from several threads
        with cf.ThreadPoolExecutor(4) as pool:
            n = r.num_data_rows
            list(pool.map(lambda a: r.read_into({k: v[a:a + 37] for k, v in out.items()}, a, min(n, a + 37)),
                          range(0, n, 37)))
        _check(out, r)


def test_copying_adapter():
    from ska_sdp_cip_amd.streaming import _CopyingReader

    ms = syn.make_measurement_set(120, 5, n_ant=8, seed=3)
    r = ms.partition(2, 1)[1]
    out = _empty(r.num_data_rows, r.num_channels)
    _CopyingReader(r).read_into(out, 0, r.num_data_rows)
    _check(out, r)
    part = _empty(10, r.num_channels)
    _CopyingReader(r).read_into(part, 5, 15)
    sub = r.partition(1, 1)[0]
    sub.set_row_bounds(r.row_start + 5, r.row_start + 15)
    _check(part, sub)
