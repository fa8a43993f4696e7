"""
Host simulation of the scatter's LDS bank conflicts on the C3 benchmark tracks
(round 6): every visibility's footprint origin and bank class ((ix0 % 32) P +
iy0 % 32) % 32, tiles in tile order (MS order within a tile, as the stable
radix sort leaves them), 1024-position ordering windows, and per aligned
32-lane group of the scatter's waves the LDS cycles of one tap instruction =
the largest number of lanes on one bank pair.

Orders compared:
  level   - the planner's level-major class order (one sub-grid copy)
  pair2   - two sub-grid copies 16 elements apart: a lane of class c may add
            into copy 0 (bank c) or copy 1 (bank c + 16), so the two classes
            c, c + 16 share two banks; the window ordered level-major over the
            16 pair classes with two slots per level
Usage: python tools/sim_bank_conflicts.py [rows] [max_windows] [window]
"""
import sys

import numpy as np

sys.path.insert(0, "ska-sdp-continuum-imaging-pipeline_amd")
from ska_sdp_cip_amd import synthetic as syn  # noqa: E402


def origins(uvw, fx, nu, px, W):
    hw = W // 2
    x = (uvw[:, None] * fx[None, :]) * (nu * px) + float(nu // 2)
    return (np.floor(x - hw).astype(np.int64) + 1) % nu


def level_layout(cls, ncls, cap):
    """Positions of a window's items: level-major over ncls classes with `cap`
    slots per class and level -> the class sequence in position order."""
    counts = np.bincount(cls, minlength=ncls)
    seq = []
    lev = 0
    while True:
        row = [c for c in range(ncls) for k in range(cap) if counts[c] > lev * cap + k]
        if not row:
            break
        seq.extend(row)
        lev += 1
    return np.array(seq, dtype=np.int64)


def group_cost_single(seq):
    cost = 0
    for g in range(0, len(seq), 32):
        cost += np.bincount(seq[g:g + 32], minlength=32).max()
    return cost


def group_cost_pair(seq32):
    """seq32: classes (0..31) in position order; a group's cost with two copies
    = max over pair classes k of ceil(n_k / 2)."""
    cost = 0
    for g in range(0, len(seq32), 32):
        n = np.bincount(seq32[g:g + 32] % 16, minlength=16)
        cost += int(np.ceil(n.max() / 2))
    return cost


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 390_625
    maxw = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    win = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    nchan, npix, W = 256, 4096, 8
    uvw = syn.uvw_tracks(rows, 64, array_radius_m=4000.0, seed=20241008)
    freq = syn.channel_frequencies(nchan)
    px = syn.pixel_size_for_grid(uvw, freq, npix, support=8)
    nu = 2 * npix
    fx = freq / 299792458.0
    P = 32 + W - 1
    keys, clss = [], []
    for a in range(0, rows, 20000):
        ix = origins(uvw[a:a + 20000, 0], fx, nu, px, W)
        iy = origins(uvw[a:a + 20000, 1], fx, nu, px, W)
        keys.append(((iy // 32) * (nu // 32) + ix // 32).astype(np.int32).ravel())
        clss.append((((ix % 32) * P + iy % 32) % 32).astype(np.uint8).ravel())
    key = np.concatenate(keys)
    cls = np.concatenate(clss)
    order = np.argsort(key, kind="stable")
    key, cls = key[order], cls[order]
    starts = np.flatnonzero(np.r_[True, key[1:] != key[:-1]])
    ends = np.r_[starts[1:], key.size]
    rng = np.random.default_rng(1)
    wins = []
    for s, e in zip(starts, ends):
        for w0 in range(s, e, win):
            wins.append((w0, min(e, w0 + win)))
    pick = rng.choice(len(wins), size=min(maxw, len(wins)), replace=False)
    items = tot_single = tot_pair = groups_min = 0
    for k in pick:
        a, b = wins[k]
        c = cls[a:b].astype(np.int64)
        items += c.size
        groups_min += -(-c.size // 32)
        tot_single += group_cost_single(level_layout(c, 32, 1))
        # pair classes: level-major over c % 16 with two slots per level; the
        # class sequence within a level keeps c (either copy serves it)
        pc = c % 16
        seq_p = level_layout(pc, 16, 2)
        tot_pair += group_cost_pair(seq_p)
    print(f"window {win}: {rows} rows, {len(wins)} windows ({len(pick)} sampled), {items} items, W = {W}")
    print(f"  groups (>= items / 32): {groups_min}")
    print(f"  level-major, one copy : LDS cycles per group {tot_single / groups_min:.3f} "
          f"(extra {tot_single / groups_min - 1:.3f})")
    print(f"  pair classes, 2 copies: LDS cycles per group {tot_pair / groups_min:.3f} "
          f"(extra {tot_pair / groups_min - 1:.3f})")


if __name__ == "__main__":
    main()
