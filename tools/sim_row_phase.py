import sys, numpy as np
sys.path.insert(0, "/root/repo/ska-sdp-continuum-imaging-pipeline_amd"); sys.path.insert(0, "/root/repo/tools")
from ska_sdp_cip_amd import synthetic as syn
from sim_bank_conflicts import origins
rows = int(sys.argv[1]); maxw = int(sys.argv[2])
nchan, npix, W = 256, 4096, 8
full = syn.uvw_tracks(390625, 64, array_radius_m=4000.0, seed=20241008)
uvw = full[:rows]; freq = syn.channel_frequencies(nchan)
px = syn.pixel_size_for_grid(full, freq, npix, support=8)
nu = 2 * npix; fx = freq / 299792458.0; P = 32 + W - 1
ix = origins(uvw[:, 0], fx, nu, px, W); iy = origins(uvw[:, 1], fx, nu, px, W)
key = ((iy // 32) * (nu // 32) + ix // 32).ravel(); cls = (((ix % 32) * P + iy % 32) % 32).ravel()
order = np.argsort(key, kind="stable"); ks = key[order]; cs = cls[order]
starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]]); ends = np.r_[starts[1:], ks.size]
wins = [(w0, min(e, w0 + 1024)) for s, e in zip(starts, ends) for w0 in range(s, e, 1024)]
pick = np.random.default_rng(1).choice(len(wins), size=min(maxw, len(wins)), replace=False)
PM = P % 32
def bank_rows(c, h):
    # bank pair of a lane at tap row i (j common): c + P ((i + h) mod W)
    i = np.arange(W)
    return (c[:, None] + PM * ((i[None, :] + h[:, None]) % W)) % 32
def group_cost(c, h):
    tot = 0
    for g in range(0, len(c), 32):
        b = bank_rows(c[g:g+32], h[g:g+32])
        tot += np.mean([np.bincount(b[:, i], minlength=32).max() for i in range(W)])
    return tot
def level(eff):
    cnt = np.bincount(eff, minlength=32); rk = np.zeros(len(eff), np.int64); seen = np.zeros(32, np.int64)
    for j, x in enumerate(eff): rk[j] = seen[x]; seen[x] += 1
    S = np.array([np.minimum(cnt, r).sum() for r in range(cnt.max() + 1)])
    return S[rk] + np.array([((cnt > rk[j]) & (np.arange(32) < eff[j])).sum() for j in range(len(eff))])
def assign_greedy(c):
    # each item: h in {0,1}; effective class c or c + PM; balance counts greedily (largest classes first)
    cnt = np.zeros(32, np.int64); h = np.zeros(len(c), np.int64)
    base = np.bincount(c, minlength=32)
    for j in np.argsort(-base[c], kind="stable"):
        a, b = c[j], (c[j] + PM) % 32
        if cnt[b] < cnt[a]: h[j] = 1; cnt[b] += 1
        else: cnt[a] += 1
    return h
res = {}; gmin = 0
for k in pick:
    a, b = wins[k]; c = cs[a:b].astype(np.int64); n = len(c); gmin += -(-n // 32)
    pos = level(c); seq = np.empty(n, np.int64); seq[pos] = c
    0 and group_cost(seq, np.zeros(n, np.int64))
    pass
for k, v in res.items(): print(k, v / gmin)
def assign_greedy_n(c, H):
    cnt = np.zeros(32, np.int64); h = np.zeros(len(c), np.int64)
    base = np.bincount(c, minlength=32)
    for j in np.argsort(-base[c], kind="stable"):
        opts = [(c[j] + PM * k) % 32 for k in range(H)]
        k = int(np.argmin([cnt[o] for o in opts])); h[j] = k; cnt[opts[k]] += 1
    return h
for H in ():
    tot = 0.0; gmin = 0
    for k in pick:
        a, b = wins[k]; c = cs[a:b].astype(np.int64); n = len(c); gmin += -(-n // 32)
        h = assign_greedy_n(c, H); eff = (c + PM * h) % 32
        pos = level(eff); sc = np.empty(n, np.int64); sh = np.empty(n, np.int64); sc[pos] = c; sh[pos] = h
        tot += group_cost(sc, sh)
    print("H", H, tot / gmin)
def assign_cycle(c):
    n = np.bincount(c, minlength=32); tot = n.sum(); m = -(-tot // 32)
    k = np.zeros(32, np.int64)
    start = int(np.argmax(n))
    for it in range(2):
        for s in range(32):
            cc = (start + 1 + s * PM) % 32  # walk the cycle c -> c + PM
            prev = (cc - PM) % 32
            e = n[cc] + k[prev]
            k[cc] = min(n[cc], max(0, e - m))
    # items: the last k[c] of class c move (rank order = input order)
    h = np.zeros(len(c), np.int64); seen = np.zeros(32, np.int64)
    for j, x in enumerate(c):
        h[j] = 1 if seen[x] >= n[x] - k[x] else 0; seen[x] += 1
    return h
tot = 0.0; gmin = 0
for kk in pick[:0]:
    a, b = wins[kk]; c = cs[a:b].astype(np.int64); n = len(c); gmin += -(-n // 32)
    h = assign_cycle(c); eff = (c + PM * h) % 32
    pos = level(eff); sc = np.empty(n, np.int64); sh = np.empty(n, np.int64); sc[pos] = c; sh[pos] = h
    tot += group_cost(sc, sh)

def assign_excess(c, slack=0):
    n = np.bincount(c, minlength=32); m = -(-n.sum() // 32) + slack
    k = np.maximum(0, n - m)
    h = np.zeros(len(c), np.int64); seen = np.zeros(32, np.int64)
    for j, x in enumerate(c):
        h[j] = 1 if seen[x] >= n[x] - k[x] else 0; seen[x] += 1
    return h
for sl in (0, 2, -2):
    tot = 0.0; gmin = 0
    for kk in pick:
        a, b = wins[kk]; c = cs[a:b].astype(np.int64); n = len(c); gmin += -(-n // 32)
        h = assign_excess(c, sl); eff = (c + PM * h) % 32
        pos = level(eff); sc = np.empty(n, np.int64); sh = np.empty(n, np.int64); sc[pos] = c; sh[pos] = h
        tot += group_cost(sc, sh)
    print("excess slack", sl, tot / gmin)
