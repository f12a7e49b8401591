"""cooler-file drop-in for HiCHap's two cooler touch points (SURVEY.md
§8(b) routes (i) and (iv), §8(f) row 1), on the HDF5 subset of ``h5.py``:

* ``balance_cooler(uri, ...)`` -- ``cooler balance --ignore-diags 1
  [--cis-only] --force {file}::{res}`` as matrixBuilding.py:708 / :713 /
  :1537 / :1542 / :1761 / :1766 run it: read ``pixels/`` and ``indexes/``,
  balance on the GPU (ice.py, the same ICE path as every other entry point),
  write ``bins/weight`` plus cooler's attributes (tol, min_nnz, min_count,
  mad_max, cis_only, ignore_diags, converged, var, scale, divisive_weights)
  in place, replacing an existing weight column (--force).
* ``Cooler(uri)`` with the reads StructureFind makes: ``chromnames``,
  ``matrix(balance=...).fetch(chrom)`` (StructureFind.py:513, :853, :859,
  :2006-2008) and ``bins().fetch(chrom)['weight']`` (:2010).
* ``create_cooler(uri_or_path, bins, pixels, ...)`` -- a writer for the same
  schema (cooler format v3, symmetric-upper storage), one or several
  resolutions per file as NPZ2Cooler writes them (matrixBuilding.py:200-211).

URIs are ``path::group`` (``group`` = ``10000``, ``/10000`` or
``resolutions/10000``) or a bare path (the root group).

PARITY UNPINNED against cooler itself (absent here):
tests/test_coolio.py checks the schema round trip, the weights against
ice.balance on the same pixel table, and fetch against a dense build.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

from . import h5


def parse_uri(uri):
    path, _, group = str(uri).partition("::")
    return path, group.strip("/")


def _col(g, name):
    return g[name].read()


class _BinSelector:
    def __init__(self, c):
        self._c = c

    def fetch(self, chrom):
        import pandas as pd
        c = self._c
        lo, hi = c.extent(chrom)
        g = c._g("bins")
        cols = {"chrom": np.array([chrom] * (hi - lo), dtype=object),
                "start": g["start"].read(lo, hi), "end": g["end"].read(lo, hi)}
        if "weight" in g:
            cols["weight"] = g["weight"].read(lo, hi)
        return pd.DataFrame(cols)

    def __getitem__(self, key):
        return _BinColumn(self._c, key)

    def __call__(self):
        return self


class _BinColumn:
    def __init__(self, c, key):
        self._c, self._k = c, key

    def fetch(self, chrom):
        return self._c.bins().fetch(chrom)[self._k]


class _MatrixSelector:
    def __init__(self, c, balance):
        self._c, self._b = c, balance

    def fetch(self, chrom):
        """Dense symmetric intra-chromosome matrix (raw counts, or
        ``w_i w_j count`` with NaN at masked bins when balanced)."""
        c = self._c
        lo, hi = c.extent(chrom)
        b1, b2, v = c.pixel_rows(lo, hi)
        keep = b2 < hi
        b1, b2, v = b1[keep] - lo, b2[keep] - lo, v[keep]
        n = hi - lo
        if self._b:
            w = c.weights()[lo:hi]
            M = np.zeros((n, n), dtype=np.float64)
            val = v * w[b1] * w[b2]
        else:
            M = np.zeros((n, n), dtype=v.dtype)
            val = v
        M[b1, b2] = val
        M[b2, b1] = val
        if self._b:
            bad = ~np.isfinite(c.weights()[lo:hi])
            M[bad, :] = np.nan
            M[:, bad] = np.nan
        return M


class Cooler:
    """Read access to one cooler (``path::group``)."""

    def __init__(self, uri):
        self.uri = uri
        self.path, self.group = parse_uri(uri)
        self._f = h5.File(self.path)
        self._root = self._f[self.group] if self.group else self._f.root
        self.info = dict(self._root.attrs)
        ch = self._g("chroms")
        names = ch["name"].read()
        self.chromnames = [x.decode() if isinstance(x, bytes) else str(x) for x in names]
        self.chromsizes = dict(zip(self.chromnames, ch["length"].read().tolist()))
        self._chrom_offset = self._g("indexes")["chrom_offset"].read().astype(np.int64)
        self.binsize = self.info.get("bin-size")
        self._w = None

    def _g(self, name):
        return self._root[name]

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def n_bins(self):
        return int(self._chrom_offset[-1])

    def offset(self, chrom):
        return int(self._chrom_offset[self.chromnames.index(chrom)])

    def extent(self, chrom):
        k = self.chromnames.index(chrom)
        return int(self._chrom_offset[k]), int(self._chrom_offset[k + 1])

    def chrom_offsets(self):
        return self._chrom_offset.copy()

    def pixels_table(self):
        """The whole pixel table (bin1_id, bin2_id, count)."""
        g = self._g("pixels")
        return _col(g, "bin1_id"), _col(g, "bin2_id"), _col(g, "count")

    def pixel_rows(self, lo, hi):
        """Pixels whose bin1 is in [lo, hi) (indexes/bin1_offset)."""
        off = self._g("indexes")["bin1_offset"].read(lo, hi + 1)
        a, b = int(off[0]), int(off[-1])
        g = self._g("pixels")
        return g["bin1_id"].read(a, b), g["bin2_id"].read(a, b), g["count"].read(a, b)

    def weights(self, name="weight"):
        if self._w is None:
            self._w = self._g("bins")[name].read()
        return self._w

    def matrix(self, balance=True):
        return _MatrixSelector(self, balance)

    def bins(self):
        return _BinSelector(self)


def balance_cooler(uri, ignore_diags=1, cis_only=False, mad_max=5, min_nnz=10, min_count=0, tol=1e-5,
                   max_iters=200, rescale_marginals=True, store=True, store_name="weight", stream=None):
    """``cooler balance`` on the GPU: returns ``(weights, stats)`` and, with
    ``store``, writes ``bins/<store_name>`` + attributes in place (replacing
    an existing column, as ``--force`` does)."""
    from . import ice
    with Cooler(uri) as c:
        b1, b2, cnt = c.pixels_table()
        off = c.chrom_offsets()
        n = c.n_bins
    if cnt.dtype.kind == "f":
        if np.any(cnt != np.floor(cnt)):
            raise ValueError("ICE on the GPU takes integer counts (HiCHap writes int32 counts, matrixBuilding.py:196)")
        cnt = cnt.astype(np.int64)
    w, st = ice.balance(b1, b2, cnt, n, off, ignore_diags=ignore_diags, cis_only=cis_only, mad_max=mad_max,
                        min_nnz=min_nnz, min_count=min_count, tol=tol, max_iters=max_iters,
                        rescale_marginals=rescale_marginals, stream=stream)
    if store:
        path, group = parse_uri(uri)
        attrs = {k: st[k] for k in ("tol", "min_nnz", "min_count", "mad_max", "cis_only", "ignore_diags",
                                    "converged", "var", "scale", "divisive_weights") if k in st}
        h5.append_dataset(path, (group + "/bins") if group else "bins", store_name, np.asarray(w, np.float64),
                          attrs)
    return w, st


def _bins_arrays(chromsizes, binsize):
    names, starts, ends, cids = [], [], [], []
    for k, (nm, L) in enumerate(chromsizes):
        s = np.arange(0, L, binsize, dtype=np.int32)  # cooler COORD_DTYPE
        starts.append(s)
        ends.append(np.minimum(s + binsize, L))
        cids.append(np.full(s.size, k, dtype=np.int32))
        names.append(nm)
    return names, np.concatenate(cids), np.concatenate(starts), np.concatenate(ends)


def cooler_tree(chromsizes, binsize, bin1, bin2, count, metadata=None, assembly=None):
    """The cooler v3 group (dict tree for h5.write_file) of one resolution.
    ``chromsizes``: [(name, length)] in file order; pixels upper triangle."""
    names, cid, start, end = _bins_arrays(chromsizes, binsize)
    nb = int(cid.size)
    bin1 = np.asarray(bin1, dtype=np.int64)
    bin2 = np.asarray(bin2, dtype=np.int64)
    count = np.asarray(count)
    if np.any(bin1 > bin2):
        raise ValueError("pixels must be upper-triangle (bin1 <= bin2)")
    if bin1.size and np.any(np.diff(bin1 * nb + bin2) <= 0):
        o = np.lexsort((bin2, bin1))
        bin1, bin2, count = bin1[o], bin2[o], count[o]
    chrom_offset = np.concatenate([[0], np.cumsum(np.bincount(cid, minlength=len(names)))]).astype(np.int64)
    bin1_offset = np.searchsorted(bin1, np.arange(nb + 1), side="left").astype(np.int64)
    attrs = {"format": "HDF5::Cooler", "format-version": 3, "bin-type": "fixed", "bin-size": int(binsize),
             "storage-mode": "symmetric-upper", "nbins": nb, "nchroms": len(names), "nnz": int(bin1.size),
             "generated-by": "hichap_master_amd", "creation-date": time.strftime("%Y-%m-%dT%H:%M:%S"),
             "metadata": json.dumps(metadata or {})}
    if assembly:
        attrs["assembly"] = assembly
    return {
        "@attrs": attrs,
        "chroms": {"name": np.array([n.encode() for n in names]),
                   "length": np.array([L for _, L in chromsizes], dtype=np.int32)},
        "bins": {"chrom": {"@data": cid, "@enum": [(nm, k) for k, nm in enumerate(names)]},
                 "start": start, "end": end},
        "pixels": {"bin1_id": bin1, "bin2_id": bin2, "count": count},
        "indexes": {"chrom_offset": chrom_offset, "bin1_offset": bin1_offset},
    }


def create_cooler(path, resolutions, metadata=None, assembly=None, mode="w"):
    """Write a file holding one cooler per resolution, as NPZ2Cooler does
    (group ``/<res>``, URI ``path::<res>``).  ``resolutions`` maps res ->
    (chromsizes [(name, length)], bin1, bin2, count[, metadata]).  mode "a"
    keeps the resolution groups an existing file already holds (those not
    given here; NPZ2Cooler's mode='a', :193-196): the file is rewritten with
    their pixels, bins (weight columns and attributes included) and
    metadata."""
    tree = {}
    if mode == "a" and os.path.exists(path):
        for grp in cooler_groups(path):
            if grp not in {str(r) for r in resolutions}:
                tree[grp] = _regroup(path, grp)
    for res, spec in resolutions.items():
        cs, b1, b2, c = spec[:4]
        meta = spec[4] if len(spec) > 4 else metadata
        tree[str(res)] = cooler_tree(cs, int(res), b1, b2, c, meta, assembly)
    h5.write_file(path, tree)


def cooler_groups(path):
    """Top-level groups of a file that hold a cooler (a ``pixels`` group)."""
    with h5.File(path) as f:
        return [k for k in f.root.keys() if "pixels" in f.root[k]]


def _regroup(path, grp):
    """One existing cooler group as a write_file tree (rewriting a file)."""
    with Cooler(f"{path}::{grp}") as c:
        cs = [(n, int(c.chromsizes[n])) for n in c.chromnames]
        b1, b2, cnt = c.pixels_table()
        meta = c.info.get("metadata")
        try:
            meta = json.loads(meta) if isinstance(meta, str) else meta
        except ValueError:
            meta = {"metadata": meta}
        t = cooler_tree(cs, int(c.binsize), b1, b2, cnt, meta, c.info.get("assembly"))
        g = c._g("bins")
        for k in g.keys():
            if k not in ("chrom", "start", "end"):
                d = g[k]
                t["bins"][k] = {"@attrs": dict(d.attrs), "@data": d.read()}
    return t
