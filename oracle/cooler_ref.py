"""ORACLE (test infrastructure only) -- the cooler-writing half of HiCHap's
matrix construction restated: NPZ2Cooler's pixel-table assembly
(matrixBuilding.py:100-303), WholeMatrixToSparseDict / IntraMatrixToSparseDict
(:457-525) on dense matrices, and cooler.merge_coolers as
TraditionalMatrixConstruction uses it (:680-695: the replicates' pixels of one
resolution summed).

The reference writes through the third-party `cooler` package (absent here,
SURVEY.md §8(c)); what it puts into `pixels/` and `bins/` is restated from
the reference's own generator (`_generator`, :261-303) and cooler's
`binnify` (bins [k res, min((k+1) res, length)) for k < ceil(length / res)).
Inputs are the reference's sparse dicts (structured arrays bin1 / bin2 / IF
in chromosome-local bins); the block extraction follows :274-298 with
scipy.sparse as the reference does (csr sums duplicates, lil symmetrises,
triu keeps the upper triangle).  PARITY of the cooler layout itself is
unpinned (cooler absent); the sparse dicts are pinned by the reference's own
TraditionalMatrixBuilding outputs (tests/golden/pairs_*.npz)."""
from __future__ import annotations

import numpy as np
from scipy import sparse

from oracle.pairs_ref import sort_chromosomes

S_DTYPE = np.dtype({"names": ["bin1", "bin2", "IF"], "formats": [np.int64, np.int64, np.float64]})


def _check(c, chroms):
    # NPZ2Cooler's filter (:145, :150-151, :215): no chroms = all
    chroms = set(chroms)
    return (not chroms) or (c.isdigit() and "#" in chroms) or (c in chroms)


def read_chromsizes(genome_lines, chroms):
    """NPZ2Cooler.readChromSize (:212-223) + Sort_Chromosomes (:135-138):
    [(name, length)] in cooler file order."""
    sizes = {}
    for line in genome_lines:
        f = line.strip().split()
        if not f:
            continue
        c = f[0].lstrip("chr")
        if _check(c, chroms):
            sizes[c] = int(f[1])
    return [(c, sizes[c]) for c in sort_chromosomes(list(sizes))]


def whole_to_sparse_dict(Bins, M):
    """WholeMatrixToSparseDict (:457-505) on a dense matrix."""
    order = sort_chromosomes(list(Bins))
    lib = {}
    for i, c1 in enumerate(order):
        for j in range(i, len(order)):
            c2 = order[j]
            s1, e1 = Bins[c1][0], Bins[c1][1] + 1
            s2, e2 = Bins[c2][0], Bins[c2][1] + 1
            blk = M[s1:e1, s2:e2]
            if c1 == c2:
                blk = np.triu(blk)
                key = c1
            else:
                key = c1 + "_" + c2
            x, y = np.nonzero(blk)
            t = np.zeros(x.size, dtype=S_DTYPE)
            t["bin1"], t["bin2"], t["IF"] = x, y, blk[x, y]
            lib[key] = t
    return lib


def intra_to_sparse_dict(D):
    """IntraMatrixToSparseDict (:508-525)."""
    out = {}
    for c, M in D.items():
        T = np.triu(M)
        x, y = np.nonzero(T)
        t = np.zeros(x.size, dtype=S_DTYPE)
        t["bin1"], t["bin2"], t["IF"] = x, y, T[x, y]
        out[c] = t
    return out


def npz2cooler_tables(datasets, genome_lines, chroms, onlyIntra, dtype="int"):
    """{res: (chromsizes, bin1, bin2, count)} as NPZ2Cooler writes them."""
    full = read_chromsizes(genome_lines, chroms)
    names = [c for c, _ in full]
    out = {}
    for res, lib in datasets.items():
        Map = {}
        for key in lib:
            if "_" not in key and _check(key, chroms):
                Map[(key, key)] = key
            else:
                tmp = key.split("_")
                if len(tmp) != 2:
                    continue
                if _check(tmp[0], chroms) and _check(tmp[1], chroms):
                    Map[(tmp[0], tmp[1])] = key
        subset = {c for pair in Map for c in pair}
        cs = [(c, L) for c, L in full if c in subset]
        cum = np.cumsum([int(np.ceil(L / res)) for _, L in cs])
        xs, ys, vs = [], [], []
        for i in range(len(full)):
            for j in range(i, len(full)):
                c1, c2 = names[i], names[j]
                if onlyIntra and c1 != c2:
                    continue
                if (c1, c2) in Map:
                    ci, cj = i, j
                elif (c2, c1) in Map:
                    c1, c2 = c2, c1
                    ci, cj = j, i
                else:
                    continue
                data = lib[Map[(c1, c2)]]
                x, y, v = np.asarray(data["bin1"]), np.asarray(data["bin2"]), np.asarray(data["IF"], np.float64)
                if x.size == 0:
                    continue  # (the reference's x.max() raises on an empty block)
                if ci > cj:
                    x, y = y, x
                    ci, cj = cj, ci
                if ci != cj:
                    tmp = sparse.csr_matrix((v, (x, y)), shape=(x.max() + 1, y.max() + 1))
                    tmp = tmp.tocoo()
                else:
                    L = max(x.max() + 1, y.max() + 1)
                    tmp = sparse.lil_matrix(sparse.csr_matrix((v, (x, y)), shape=(L, L)))
                    tmp[y, x] = tmp[x, y]
                    tmp = sparse.triu(tmp).tocoo()
                keep = tmp.data != 0
                r, c = tmp.row[keep].astype(np.int64), tmp.col[keep].astype(np.int64)
                if ci > 0:
                    r = r + cum[ci - 1]
                if cj > 0:
                    c = c + cum[cj - 1]
                xs.append(r)
                ys.append(c)
                vs.append(tmp.data[keep])
        b1 = np.concatenate(xs) if xs else np.zeros(0, np.int64)
        b2 = np.concatenate(ys) if ys else np.zeros(0, np.int64)
        val = np.concatenate(vs) if vs else np.zeros(0)
        # create_from_unordered / create_cooler(ordered): sorted by (bin1, bin2), equal pixels summed
        key = b1 * (int(cum[-1]) + 1 if cs else 1) + b2
        uk, inv = np.unique(key, return_inverse=True)
        tot = np.bincount(inv, val, minlength=uk.size)
        b1 = np.zeros(uk.size, np.int64)
        b2 = np.zeros(uk.size, np.int64)
        b1[inv] = np.concatenate(xs) if xs else b1
        b2[inv] = np.concatenate(ys) if ys else b2
        cnt = tot.astype(np.int32) if dtype == "int" else tot.astype(np.float64)
        out[res] = (cs, b1, b2, cnt)
    return out


def merge_tables(tables):
    """cooler.merge_coolers (:689-695) of one resolution: pixels summed."""
    cs = tables[0][0]
    b1 = np.concatenate([t[1] for t in tables])
    b2 = np.concatenate([t[2] for t in tables])
    v = np.concatenate([np.asarray(t[3], np.float64) for t in tables])
    n = int(max(b2.max(initial=0), b1.max(initial=0))) + 1
    uk, inv = np.unique(b1 * n + b2, return_inverse=True)
    tot = np.bincount(inv, v, minlength=uk.size)
    return cs, uk // n, uk % n, tot.astype(tables[0][3].dtype)
