"""
Pin the CPU oracle (oracle/oracle.py) against golden vectors produced by the
reference's own code (tests/golden/make_golden.py): tiling plans incl. tile
boundaries +-1 ulp and descending frequencies, Stokes-I / effective weights,
balanced chunk bounds / partitions (incl. the known answers of
reference tests/test_measurement_set_partition_indices.py:33-62), split_tile.
"""
from pathlib import Path

import numpy as np
import pytest

import oracle

GOLD = Path(__file__).resolve().parent / "golden"
TILING = np.load(GOLD / "tiling_plan.npz")
CASES = sorted({k.split("__")[0] for k in TILING.files if k.endswith("__key")})


def golden_mapping(name):
    g = {f: TILING[f"{name}__{f}"] for f in ("key", "irow", "c0", "c1", "tile_order")}
    out = {}
    for k, r, a, b in zip(g["key"].tolist(), g["irow"].tolist(), g["c0"].tolist(), g["c1"].tolist()):
        out.setdefault(tuple(k), []).append((r, a, b))
    return out


@pytest.mark.parametrize("name", CASES)
def test_oracle_tiling_plan_matches_reference(name):
    mapping = oracle.tile_mapping_sequential(TILING[f"{name}__uvw"], TILING[f"{name}__tile_size"],
                                             TILING[f"{name}__freq"], row_offset=7)
    gold = golden_mapping(name)
    assert list(mapping.keys()) == list(gold.keys())  # insertion order too
    assert mapping == gold


def test_each_sample_in_exactly_one_tile():
    # reference tests/uvw_tiling/test_uvw_tiling_plan.py:25-32
    name = "meerkat_ts3000_256ch"
    uvw, freq = TILING[f"{name}__uvw"], TILING[f"{name}__freq"]
    hits = np.zeros((len(uvw), len(freq)), dtype=int)
    for slices in oracle.tile_mapping_sequential(uvw, TILING[f"{name}__tile_size"], freq).values():
        for r, a, b in slices:
            hits[r, a:b] += 1
    assert (hits == 1).all()


def test_oracle_stokes_i_matches_reference():
    g = np.load(GOLD / "stokes_i.npz")
    vis_i, flags_i, w_i, eff = oracle.stokes_i(g["vis4"], g["flags4"], g["weights4"])
    assert vis_i.dtype == g["vis_i"].dtype and np.array_equal(vis_i, g["vis_i"])
    assert np.array_equal(flags_i, g["flags_i"])
    assert w_i.dtype == g["weights_i"].dtype
    np.testing.assert_array_equal(w_i, g["weights_i"])
    assert eff.dtype == g["eff_w"].dtype and np.array_equal(eff, g["eff_w"])


def test_oracle_balanced_bounds_match_reference():
    g = np.load(GOLD / "partition.npz")
    for key in g.files:
        if key.startswith("bounds_"):
            _, s, e, k = key.split("_")
            assert oracle.balanced_chunk_bounds(int(s), int(e), int(k)) == [tuple(x) for x in g[key].tolist()]
    # reference known answer (tests/test_measurement_set_partition_indices.py:51-61)
    assert g["5x1"].tolist() == [[0, 14843, 0, 4], [14843, 29686, 0, 4], [29686, 44529, 0, 4],
                                 [44529, 59372, 0, 4], [59372, 74214, 0, 4]]


def test_oracle_split_tile_matches_reference():
    g = np.load(GOLD / "tile_split.npz")
    sizes = g["chan_stop"] - g["chan_start"]
    for mv in (1, 25, 64, 100, 1000, 10_000):
        chunks = oracle.split_tile_bounds(sizes.tolist(), mv)
        assert [b - a for a, b in chunks] == g[f"split_{mv}__nrows"].tolist()
        assert [int(sizes[a:b].sum()) for a, b in chunks] == g[f"split_{mv}__nvis"].tolist()


def test_reference_ms2dirty_call_contract():
    # dtypes / arguments the reference passes to ms2dirty (invert.py:170-183)
    g = np.load(GOLD / "reorder_invert.npz")
    assert g["call_dtypes"].tolist() == ["float64", "float64", "complex64", "float32"]
    assert float(g["call_epsilon"][0]) == 1e-4 and bool(g["call_wstacking"][0])
    assert float(g["pixsize"][0]) == float(np.sin(np.radians(5.0 / 3600.0)))
