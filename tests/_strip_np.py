"""
CPU restatement of the strip stages (test infrastructure only): the numpy /
oracle stand-in for HipStripBackend that the world-size-2 gloo test of
ska_sdp_cip_amd.strips plugs in. grid_strip grids with the oracle
(oracle/oracle.py grid_plane, transposed to gT[y][x]); pass_rows is the 1-D
backward FFT along u with the kept frequencies k = i - npix_x/2 (mod nu) laid
out in blocks of 4 (cip.h cip_strip_rows); pass_cols the backward FFT along v,
the crop sign (-1)^(p+q) and the grid correction (oracle.ms2dirty's
definition). w-stacking parameters: one buffer plane per w plane (grid_plane
per plane), pass_cols_wplane adds the plane's w-screened rows and
finish_rows applies the final w correction (oracle.ms2dirty's w-stacking
branch, restricted to the rank's image rows).
"""
import numpy as np
import torch

import oracle
from ska_sdp_cip_amd import strips
from ska_sdp_cip_amd.strips import COL_BLOCK


class NumpyStripBackend:
    def __init__(self, prm: dict, px: float, py: float, npix_x: int, npix_y: int, rows=None):
        self.prm, self.px, self.py = prm, float(px), float(py)
        self.npix_x, self.npix_y = int(npix_x), int(npix_y)
        self.nu, self.nv = prm["nu"], prm["nv"]
        self.nplanes = int(prm["nplanes"]) if prm.get("do_wstacking") else 1
        self.rows = None
        self.dirty = False
        self._alloc((0, self.nv) if rows is None else rows)
        W = prm["support"]
        self.cx = 1.0 / oracle.kernel_ft(W, (np.arange(npix_x) - npix_x // 2) / self.nu)
        self.cy = 1.0 / oracle.kernel_ft(W, (np.arange(npix_y) - npix_y // 2) / self.nv)

    def _alloc(self, rows):
        if self.rows != tuple(rows):
            self.rows = tuple(int(x) for x in rows)
            shape = (self.rows[1], self.nu, 2) if self.nplanes == 1 else (self.nplanes, self.rows[1], self.nu, 2)
            self.grid = torch.zeros(shape, dtype=torch.float64)

    def spawn(self):
        return NumpyStripBackend(self.prm, self.px, self.py, self.npix_x, self.npix_y, rows=self.rows)

    def bind(self, layout, rank):
        self._alloc(strips.strip_buffer_rows(layout, rank))
        return self

    def mark_clean(self):
        self.dirty = False

    def grid_strip(self, data, freq):
        if self.dirty:
            self.grid.zero_()
        self.dirty = True
        ns = data.slice_uvw.shape[0]
        nchan = freq.shape[0]
        sumw = torch.zeros(1, dtype=torch.float64)
        if ns == 0:
            return self.grid, sumw
        c0 = data.chan_start.numpy().astype(np.int64)
        c1 = data.chan_stop.numpy().astype(np.int64)
        vis = np.zeros((ns, nchan), np.complex128)
        wgt = np.zeros((ns, nchan))
        k = 0
        v = data.vis.numpy()
        w = None if data.wgt is None else data.wgt.numpy()
        for s in range(ns):
            n = c1[s] - c0[s]
            vis[s, c0[s]:c1[s]] = v[k:k + n]
            wgt[s, c0[s]:c1[s]] = 1.0 if w is None else w[k:k + n]
            k += n
        # the strip buffer's rows (row0 + k) mod nv; every other grid row must be empty
        row0, nrows = self.rows
        sel = (row0 + np.arange(nrows)) % self.nv
        rest = np.ones(self.nv, bool)
        rest[sel] = False
        for p in range(self.nplanes):
            g = oracle.grid_plane(data.slice_uvw.numpy(), freq.numpy(), vis, wgt, self.prm, self.px, self.py,
                                  p).T
            assert not np.any(g[rest]), "footprint outside the strip's rows"
            part = torch.view_as_real(torch.from_numpy(np.ascontiguousarray(g[sel])))
            if self.nplanes == 1:
                self.grid += part
            else:
                self.grid[p] += part
        sumw += float(wgt.sum())
        return self.grid, sumw

    def pass_rows(self, grid, y0, y1, plane=0):
        rows = torch.view_as_complex(grid[y0:y1].contiguous()).numpy()
        F = np.fft.ifft(rows, axis=1) * self.nu
        k = (np.arange(self.npix_x) - self.npix_x // 2) % self.nu
        sel = F[:, k]  # (h, npix_x)
        h = y1 - y0
        H = sel.reshape(h, self.npix_x // COL_BLOCK, COL_BLOCK).transpose(1, 0, 2)
        grid[y0:y1].zero_()
        return torch.view_as_real(torch.from_numpy(np.ascontiguousarray(H))).contiguous()

    def pass_cols(self, H, i0, i1, norm=None):
        Hc = torch.view_as_complex(H.contiguous()).numpy()  # (nb, nv, 4)
        cols = Hc.transpose(0, 2, 1).reshape(i1 - i0, self.nv)  # image row i0 + 4b + c
        F = np.fft.ifft(cols, axis=1) * self.nv
        q = np.arange(self.npix_y) - self.npix_y // 2
        p = np.arange(i0, i1) - self.npix_x // 2
        sub = F[:, q % self.nv]
        sgn = np.where((p[:, None] + q[None, :]) % 2 == 0, 1.0, -1.0)
        out = (sgn * sub).real * self.cx[i0:i1, None] * self.cy[None, :]
        if norm is not None:
            out = out / float(norm.reshape(-1)[0])
        return torch.from_numpy(np.ascontiguousarray(out))

    def _nm1_rows(self, i0, i1):
        l = (np.arange(i0, i1) - self.npix_x // 2) * self.px  # noqa: E741
        m = (np.arange(self.npix_y) - self.npix_y // 2) * self.py
        e = l[:, None] ** 2 + m[None, :] ** 2
        return -e / (np.sqrt(1.0 - e) + 1.0)

    def pass_cols_wplane(self, H, i0, i1, plane, first, acc):
        Hc = torch.view_as_complex(H.contiguous()).numpy()  # (nb, nv, 4)
        cols = Hc.transpose(0, 2, 1).reshape(i1 - i0, self.nv)
        F = np.fft.ifft(cols, axis=1) * self.nv
        q = np.arange(self.npix_y) - self.npix_y // 2
        p = np.arange(i0, i1) - self.npix_x // 2
        sgn = np.where((p[:, None] + q[None, :]) % 2 == 0, 1.0, -1.0)
        wp = self.prm["w0"] + plane * self.prm["dw"]
        val = (sgn * F[:, q % self.nv] * np.exp(-2j * np.pi * wp * self._nm1_rows(i0, i1))).real
        a = acc.numpy()
        if first:
            a[...] = val
        else:
            a += val
        return acc

    def finish_rows(self, acc, i0, i1, norm=None):
        nm1 = self._nm1_rows(i0, i1)
        fw = oracle.kernel_ft(self.prm["support"], np.abs(self.prm["dw"] * nm1).ravel()).reshape(nm1.shape)
        a = acc.numpy()
        a *= self.cx[i0:i1, None] * self.cy[None, :] / (fw * (nm1 + 1.0))
        if norm is not None:
            a /= float(norm.reshape(-1)[0])
        return acc
