#!/usr/bin/env python3
"""Golden vectors for pair binning from the REFERENCE's own functions.

Run in the build container only (reads /root/reference, absent on the GPU box):

    python tests/golden/make_golden_pairs.py

As in make_golden.py, the Python-2 source TEXT of HiCHap/matrixBuilding.py is
converted with lib2to3 in memory and the needed definitions are executed:
``TraditionalMatrixBuilding`` (+ Load_Genome, Get_Chro_Bins, Sort_Chromosomes,
WholeMatrixToSparseDict, IntraMatrixToSparseDict), ``TraditionalMatrixInAllelic``
and — for the haplotype passes, which live inline in
``HaplotypeMatrixBuilding`` (:1108-1240) — the statements of that function from
``Hap_Bins_Pos = {}`` to the end of the P_M pass, wrapped into a function.
Their `cat` subprocess is replaced by a reader of the same files (text lines).

Saved per case (``pairs_*.npz``): the input texts as uint8 arrays, the genome
file text, the parameters, and every output matrix as COO arrays
(``<lib>/<res>/<key>/{bin1,bin2,IF}`` for sparse dicts; upper-triangle
nonzeros of dense matrices).  Nothing converted is written to disk.
"""
from __future__ import annotations

import ast
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/HiCHap"
sys.path.insert(0, HERE)

from make_golden import _py3_source  # noqa: E402

FUNCS = ["Merge_beds", "Load_Genome", "Load_HaplotypeGenome", "Sort_Chromosomes", "Get_Chro_Bins",
         "Get_Chro_Bins_Haplotypes", "WholeMatrixToSparseDict", "IntraMatrixToSparseDict",
         "TraditionalMatrixBuilding", "TraditionalMatrixInAllelic"]


class _Log:
    def log(self, *a, **k):
        pass


class _Proc:
    def __init__(self, cmd, **kw):
        assert cmd[0] == "cat"
        lines = []
        for fn in cmd[1:]:
            with open(fn) as f:
                lines.append(f.read())
        self.stdout = _Lines("".join(lines))


class _Lines(list):
    def __init__(self, text):
        super().__init__(text.splitlines(keepends=True))

    def close(self):
        pass


class _Subprocess:
    PIPE = -1
    Popen = _Proc


def load_reference():
    for name, val in (("int", int), ("float", float), ("bool", bool)):
        if not hasattr(np, name):
            setattr(np, name, val)
    import copy
    import math
    ns = {"np": np, "math": math, "log": _Log(), "subprocess": _Subprocess, "copy": copy, "os": os}
    tree = ast.parse(_py3_source(os.path.join(REF, "matrixBuilding.py")))
    fdefs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert {f.name for f in fdefs} == set(FUNCS)
    exec(compile(ast.Module(body=fdefs, type_ignores=[]), "<matrixBuilding>", "exec"), ns)
    # the unimputed haplotype passes, inline in HaplotypeMatrixBuilding
    hmb = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "HaplotypeMatrixBuilding"][0]
    src = [ast.unparse(s) for s in hmb.body]
    i0 = next(i for i, s in enumerate(src) if s.startswith("Hap_Bins_Pos = {}"))
    i1 = next(i for i, s in enumerate(src) if s.startswith("DataSets['UnImputated_Whole']"))
    body = hmb.body[i0:i1] + ast.parse("return (UnImputated_Whole_Lib, UnImputated_Local_Lib)").body
    args = ast.arguments(posonlyargs=[], args=[ast.arg(arg=a) for a in
                                                ("files", "genomeSize", "wholeRes", "localRes", "chroms")],
                         kwonlyargs=[], kw_defaults=[], defaults=[])
    fn = ast.FunctionDef(name="HapUnImputed", args=args, body=body, decorator_list=[], returns=None)
    exec(compile(ast.fix_missing_locations(ast.Module(body=[fn], type_ignores=[])), "<HaplotypeMatrixBuilding>",
                 "exec"), ns)
    return ns


# ------------------------------------------------------------ synthetic inputs
GENOME = [("chr1", 2_950_000), ("chr2", 2_100_000), ("chr10", 1_200_000), ("chrX", 1_650_000),
          ("chrY", 900_000), ("chrM", 16_571), ("chrUn_gl000220", 161_802)]


def genome_text():
    return "".join(f"{c}\t{l}\n" for c, l in GENOME)


def _pos(rng, L, near_end=0.02):
    if rng.random() < near_end:
        return int(L - 1 - rng.integers(0, 50))
    return int(rng.integers(0, L))


def _pair(rng, names, cis=0.75):
    L = dict(GENOME)
    c1 = names[rng.integers(len(names))]
    p1 = _pos(rng, L[c1])
    if rng.random() < cis:
        c2 = c1
        p2 = int(min(max(p1 + rng.integers(-400_000, 400_000), 0), L[c1] - 1))
    else:
        c2 = names[rng.integers(len(names))]
        p2 = _pos(rng, L[c2])
    return c1, p1, c2, p2


def valid_bed_text(rng, n, names, crlf_every=0):
    out = []
    for k in range(n):
        c1, p1, c2, p2 = _pair(rng, names)
        sep = "\t" if k % 7 else "  \t "  # runs of mixed whitespace
        f = [f"SRR.{k}", c1, "+", str(p1), str(p1 // 4096), str(p1 // 4096 * 4096), str(p1), "0",
             c2, "-", str(p2), str(p2 // 4096), str(p2 // 4096 * 4096), str(p2), "0"]
        line = sep.join(f)
        end = "\r\n" if crlf_every and k % crlf_every == 0 else "\n"
        out.append(line + end)
    text = "".join(out)
    return text[:-1]  # final line without a newline


def allelic_text(rng, n, names, marks=("Both",)):
    out = []
    for k in range(n):
        c1, p1, c2, p2 = _pair(rng, names)
        out.append(f"{c1}\t{p1}\t{c2}\t{p2}\t{marks[rng.integers(len(marks))]}\n")
    return "".join(out)


# ------------------------------------------------------------ flattening
def flat_sparse(prefix, lib, out):
    for res, d in lib.items():
        for key, arr in d.items():
            for f in ("bin1", "bin2", "IF"):
                out[f"{prefix}/{res}/{key}/{f}"] = np.asarray(arr[f])


def flat_dense(prefix, lib, out):
    for res, d in lib.items():
        if isinstance(d, dict) and "Matrix" in d:
            items = {"__whole__": d["Matrix"]}
        else:
            items = d
        for key, M in items.items():
            M = np.asarray(M)
            i, j = np.nonzero(np.triu(M))
            out[f"{prefix}/{res}/{key}/bin1"] = i.astype(np.int64)
            out[f"{prefix}/{res}/{key}/bin2"] = j.astype(np.int64)
            out[f"{prefix}/{res}/{key}/IF"] = M[i, j].astype(np.float64)
            assert (M == M.T).all()


def text_arr(t):
    return np.frombuffer(t.encode(), dtype=np.uint8).copy()


def main():
    ref = load_reference()
    rng = np.random.default_rng(20201016)
    tmp = tempfile.mkdtemp()
    gpath = os.path.join(tmp, "genome.txt")
    with open(gpath, "w") as f:
        f.write(genome_text())
    cases = {}

    # 1. traditional, default chroms ['#', 'X'] (chrY / chrM / chrUn pairs skipped)
    names = [c for c, _ in GENOME]
    t1 = valid_bed_text(rng, 3000, names, crlf_every=11)
    W, L = ref["TraditionalMatrixBuilding"](bed_IO=t1.splitlines(keepends=True), genomeSize=gpath,
                                            wholeRes=[200000, 100000], localRes=[50000], chroms=["#", "X"])
    d = {"text": text_arr(t1), "genome": text_arr(genome_text()),
         "params": np.array(json.dumps(dict(wholeRes=[200000, 100000], localRes=[50000], chroms=["#", "X"])))}
    flat_sparse("whole", W, d)
    flat_sparse("local", L, d)
    cases["pairs_traditional"] = d

    # 2. traditional, chroms = [] (every genome chromosome, incl. chrM and the scaffold)
    t2 = valid_bed_text(rng, 1500, names)
    W, L = ref["TraditionalMatrixBuilding"](bed_IO=t2.splitlines(keepends=True), genomeSize=gpath,
                                            wholeRes=[500000], localRes=[100000, 40000], chroms=[])
    d = {"text": text_arr(t2), "genome": text_arr(genome_text()),
         "params": np.array(json.dumps(dict(wholeRes=[500000], localRes=[100000, 40000], chroms=[])))}
    flat_sparse("whole", W, d)
    flat_sparse("local", L, d)
    cases["pairs_traditional_allchroms"] = d

    # 3. TraditionalMatrixInAllelic over the five allelic beds (dense outputs)
    files = {}
    for kind in ("Bi_Allelic", "M_M", "M_P", "P_M", "P_P"):
        files[kind] = allelic_text(rng, 700, names, marks=("Both", "Both", "Both", "R1", "R2"))
    cat = "".join(files[k] for k in ("Bi_Allelic", "M_M", "M_P", "P_M", "P_P"))
    W, L = ref["TraditionalMatrixInAllelic"](bed_IO=cat.splitlines(keepends=True), genomeSize=gpath,
                                             wholeRes=[250000], localRes=[100000], chroms=["#", "X"])
    d = {"text": text_arr(cat), "genome": text_arr(genome_text()),
         "params": np.array(json.dumps(dict(wholeRes=[250000], localRes=[100000], chroms=["#", "X"])))}
    flat_dense("whole", W, d)
    flat_dense("local", L, d)
    cases["pairs_allelic_traditional"] = d

    # 4. the unimputed haplotype passes (M_M / P_P with 'Both' filter, M_P, P_M)
    paths = []
    for kind, text in files.items():
        p = os.path.join(tmp, f"Sample_Valid_{kind}.bed")
        with open(p, "w") as f:
            f.write(text)
        paths.append(p)
    UW, UL = ref["HapUnImputed"](files=paths, genomeSize=gpath, wholeRes=[250000], localRes=[100000],
                                 chroms=["#", "X"])
    d = {f"text_{k}": text_arr(v) for k, v in files.items()}
    d["genome"] = text_arr(genome_text())
    d["params"] = np.array(json.dumps(dict(wholeRes=[250000], localRes=[100000], chroms=["#", "X"])))
    flat_dense("whole", UW, d)
    flat_dense("local", UL, d)
    cases["pairs_haplotype_unimputed"] = d

    for name, d in cases.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print("wrote", path, len(d), "arrays")


if __name__ == "__main__":
    main()
