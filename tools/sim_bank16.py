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
key = ((iy // 32) * (nu // 32) + ix // 32).ravel()
elem = ((ix % 32) * P + iy % 32).ravel()  # element index of the footprint origin in the sub-grid
order = np.argsort(key, kind="stable"); ks = key[order]; es = elem[order]
starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]]); ends = np.r_[starts[1:], ks.size]
wins = [(w0, min(e, w0 + 1024)) for s, e in zip(starts, ends) for w0 in range(s, e, 1024)]
pick = np.random.default_rng(1).choice(len(wins), size=min(maxw, len(wins)), replace=False)
def level(cl, ncls):
    cnt = np.bincount(cl, minlength=ncls); rk = np.zeros(len(cl), np.int64); seen = np.zeros(ncls, np.int64)
    for j, x in enumerate(cl): rk[j] = seen[x]; seen[x] += 1
    S = np.array([np.minimum(cnt, r).sum() for r in range(cnt.max() + 1)])
    return S[rk] + np.array([((cnt > rk[j]) & (np.arange(ncls) < cl[j])).sum() for j in range(len(cl))])
def cost(seq_e, h, G=16, MOD=16):
    # per tap row i: lane bank = (e + P*((i+h) mod W)) mod MOD; groups of G lanes; cycles = max multiplicity
    tot = 0.0
    i = np.arange(W)
    for g in range(0, len(seq_e), G):
        e = seq_e[g:g+G]; hh = h[g:g+G]
        b = (e[:, None] + P * ((i[None, :] + hh[:, None]) % W)) % MOD
        tot += np.mean([np.bincount(b[:, r], minlength=MOD).max() for r in range(W)])
    return tot
res = {}
for name in ():
    tot = 0.0; gmin = 0
    for k in pick:
        a, b = wins[k]; e = es[a:b].astype(np.int64); n = len(e); gmin += -(-n // 16)
        if name == "plain": seq = e
        else:
            ncls = 32 if "32" in name else 16
            pos = level(e % ncls, ncls); seq = np.empty(n, np.int64); seq[pos] = e
        tot += cost(seq, np.zeros(n, np.int64))
    print(name, tot / gmin)
def assign_cycle(c, ncls, dP):
    n = np.bincount(c, minlength=ncls); tot = n.sum(); m = -(-tot // ncls)
    k = np.zeros(ncls, np.int64); start = int(np.argmax(n)); cc = start; kc = 0
    for s in range(2 * ncls):
        cc = (cc + dP) % ncls
        e = n[cc] + kc
        kc = min(n[cc], max(0, e - m)); k[cc] = kc
    h = np.zeros(len(c), np.int64); seen = np.zeros(ncls, np.int64)
    for j, x in enumerate(c):
        h[j] = 1 if seen[x] >= n[x] - k[x] else 0; seen[x] += 1
    return h
for ncls in ():
    dP = P % ncls
    tot = 0.0; gmin = 0
    for k in pick:
        a, b = wins[k]; e = es[a:b].astype(np.int64); n = len(e); gmin += -(-n // 16)
        c = e % ncls
        h = assign_cycle(c, ncls, dP); eff = (c + dP * h) % ncls
        pos = level(eff, ncls); seq = np.empty(n, np.int64); hs = np.empty(n, np.int64); seq[pos] = e; hs[pos] = h
        tot += cost(seq, hs)
    print("phases order", ncls, tot / gmin)
def assign_cycle1(c, ncls, dP, laps):
    n = np.bincount(c, minlength=ncls); tot = n.sum(); m = -(-tot // ncls)
    k = np.zeros(ncls, np.int64); start = int(np.argmax(n)); cc = start; kc = 0
    for s in range(laps * ncls):
        cc = (cc + dP) % ncls
        e = n[cc] + kc
        kc = min(n[cc], max(0, e - m)); k[cc] = kc
    h = np.zeros(len(c), np.int64); seen = np.zeros(ncls, np.int64)
    for j, x in enumerate(c):
        h[j] = 1 if seen[x] >= n[x] - k[x] else 0; seen[x] += 1
    return h
for laps in (1, 3):
    ncls = 16; dP = P % ncls
    tot = 0.0; gmin = 0
    for k in pick:
        a, b = wins[k]; e = es[a:b].astype(np.int64); n = len(e); gmin += -(-n // 16)
        c = e % ncls
        h = assign_cycle1(c, ncls, dP, laps); eff = (c + dP * h) % ncls
        pos = level(eff, ncls); seq = np.empty(n, np.int64); hs = np.empty(n, np.int64); seq[pos] = e; hs[pos] = h
        tot += cost(seq, hs)
    print("phases16 laps", laps, tot / gmin)
