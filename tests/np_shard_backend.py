"""Test double for the sharded-ICE backend protocol of hichap_master_amd.dist:
the same calls as the HIP backend (IceState), computed with the oracle's
NumPy restatement, so the exchange logic runs under gloo on CPU."""
import numpy as np

from oracle import ice_ref


class NumpyShard:
    def __init__(self, b1, b2, c, n, off, rows, tol=1e-5, max_iters=200, mad_max=5, min_nnz=10):
        chrom_of = np.repeat(np.arange(len(off) - 1), np.diff(off))
        self.b1, self.b2, self.c = ice_ref._active_pixels(np.asarray(b1), np.asarray(b2), np.asarray(c),
                                                          chrom_of, 1, False)
        self.n, self.off = n, np.asarray(off)
        self.lo, self.hi = rows
        self.tol, self.max_iters, self.mad_max, self.min_nnz = tol, max_iters, mad_max, min_nnz
        self.bias = np.ones(n)
        self.marg = np.zeros(n)
        self.iters, self.active, self.var, self.scale = 0, True, np.nan, np.nan

    def marg_local(self, mode, out, stream):
        import torch
        if mode == 0:
            w = (self.c != 0).astype(float)
        elif mode == 1:
            w = self.c
        else:
            w = self.c * self.bias[self.b1] * self.bias[self.b2]
        full = ice_ref.marginalize(self.b1, self.b2, w, self.n)
        out[: self.hi - self.lo] = torch.from_numpy(full[self.lo:self.hi])

    def set_marg(self, gathered, world, maxlen, rank_rows, stream):
        g = gathered.numpy().reshape(world, maxlen)
        for k in range(world):
            a, b = rank_rows[k], rank_rows[k + 1]
            self.marg[a:b] = g[k, : b - a]

    def filter_nnz(self, stream):
        self.bias[self.marg < self.min_nnz] = 0

    def filter_count_mad(self, stream):
        m = self.marg.copy()
        for lo, hi in zip(self.off[:-1], self.off[1:]):
            cm = m[lo:hi]
            m[lo:hi] = cm / np.median(cm[cm > 0])
        lg = np.log(m[m > 0])
        cut = np.exp(np.median(lg) - self.mad_max * np.median(np.abs(lg - np.median(lg))))
        self.bias[m < cut] = 0

    def update(self, stream):
        if not self.active:
            return
        nz = self.marg[self.marg != 0]
        self.iters += 1
        m = self.marg / nz.mean()
        m[m == 0] = 1
        self.bias /= m
        self.var, self.scale = nz.var(), nz.mean()
        if self.var < self.tol or self.iters >= self.max_iters:
            self.active = False

    def active_groups(self, stream):
        return int(self.active)

    def finalize(self, stream):
        w = self.bias.copy()
        w[w == 0] = np.nan
        return w / np.sqrt(self.scale), dict(iters=self.iters, var=self.var, scale=self.scale)
