#!/usr/bin/env python3
"""Golden vectors for the haplotype imputation of HaplotypeMatrixBuilding
(HiCHap/matrixBuilding.py:1108-1494) from the REFERENCE's own code.

Run in the build container only:  python tests/golden/make_golden_impute.py

The statements of ``HaplotypeMatrixBuilding`` from ``Hap_Bins_Pos = {}``
(:1108) to ``DataSets['Imputated_Local'] = ...`` (:1494) — the unimputed
M_M / P_P / M_P / P_M passes and both imputation passes — are wrapped into a
function (lib2to3-converted in memory, as make_golden_pairs.py does) and run
on synthetic allelic beds; `cat` is replaced by a reader of the same files.
Saved: the bed texts, the genome file, the parameters and every matrix as
nonzero COO (imputed matrices are asymmetric: full nonzeros, not triu).
"""
from __future__ import annotations

import ast
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import _py3_source  # noqa: E402
from make_golden_pairs import GENOME, REF, _Log, _Subprocess, allelic_text, genome_text, text_arr  # noqa: E402

FUNCS = ["Merge_beds", "Load_Genome", "Load_HaplotypeGenome", "Sort_Chromosomes", "Get_Chro_Bins_Haplotypes",
         "GetNeighborhoodIndex", "GetNeighborhoodContacts"]


def load_reference():
    import copy
    import math
    for name, val in (("int", int), ("float", float), ("bool", bool)):
        if not hasattr(np, name):
            setattr(np, name, val)
    ns = {"np": np, "math": math, "log": _Log(), "subprocess": _Subprocess, "copy": copy, "os": os}
    tree = ast.parse(_py3_source(os.path.join(REF, "matrixBuilding.py")))
    fdefs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert {f.name for f in fdefs} == set(FUNCS)
    exec(compile(ast.Module(body=fdefs, type_ignores=[]), "<matrixBuilding>", "exec"), ns)
    hmb = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "HaplotypeMatrixBuilding"][0]
    src = [ast.unparse(s) for s in hmb.body]
    i0 = next(i for i, s in enumerate(src) if s.startswith("Hap_Bins_Pos = {}"))
    i1 = next(i for i, s in enumerate(src) if s.startswith("DataSets['Imputated_Local']"))
    body = hmb.body[i0:i1 + 1] + ast.parse(
        "return (UnImputated_Whole_Lib, UnImputated_Local_Lib, Imputated_Whole_Lib, Imputated_Local_Lib)").body
    names = ("files", "genomeSize", "wholeRes", "localRes", "chroms", "Imputation_region", "Imputation_min",
             "Imputation_ratio")
    args = ast.arguments(posonlyargs=[], args=[ast.arg(arg=a) for a in names], kwonlyargs=[], kw_defaults=[],
                         defaults=[])
    pre = ast.parse("DataSets = {}").body
    fn = ast.FunctionDef(name="HapImpute", args=args, body=pre + body, decorator_list=[], returns=None)
    exec(compile(ast.fix_missing_locations(ast.Module(body=[fn], type_ignores=[])), "<HaplotypeMatrixBuilding>",
                 "exec"), ns)
    return ns


def clustered_allelic(rng, n, names, marks, hot):
    """Allelic lines; a share of the inter-chromosome pairs fall in a few hot
    regions so that neighbourhood sums pass Imputation_min / ratio."""
    L = dict(GENOME)
    out = []
    for k in range(n):
        u = rng.random()
        if u < 0.35 and hot:
            (c1, a), (c2, b) = hot[rng.integers(len(hot))]
            p1 = int(min(max(a + rng.integers(-600_000, 600_000), 0), L[c1] - 1))
            p2 = int(min(max(b + rng.integers(-600_000, 600_000), 0), L[c2] - 1))
        else:
            c1 = names[rng.integers(len(names))]
            p1 = int(rng.integers(0, L[c1]))
            if rng.random() < 0.6:
                c2 = c1
                p2 = int(min(max(p1 + rng.integers(-500_000, 500_000), 0), L[c1] - 1))
            else:
                c2 = names[rng.integers(len(names))]
                p2 = int(rng.integers(0, L[c2]))
        out.append(f"{c1}\t{p1}\t{c2}\t{p2}\t{marks[rng.integers(len(marks))]}\n")
    return "".join(out)


def flat_dense(prefix, lib, out):
    for res, d in lib.items():
        items = {"__whole__": d["Matrix"]} if isinstance(d, dict) and "Matrix" in d else d
        for key, M in items.items():
            M = np.asarray(M)
            i, j = np.nonzero(M)
            out[f"{prefix}/{res}/{key}/bin1"] = i.astype(np.int64)
            out[f"{prefix}/{res}/{key}/bin2"] = j.astype(np.int64)
            out[f"{prefix}/{res}/{key}/IF"] = M[i, j].astype(np.float64)


def main():
    ref = load_reference()
    rng = np.random.default_rng(20201019)
    tmp = tempfile.mkdtemp()
    gpath = os.path.join(tmp, "genome.txt")
    with open(gpath, "w") as f:
        f.write(genome_text())
    names = ["chr1", "chr2", "chr10", "chrX", "chrY"]
    hot = [(("chr1", 1_400_000), ("chr2", 900_000)), (("chr10", 600_000), ("chrX", 800_000)),
           (("chr2", 1_500_000), ("chr1", 2_300_000))]
    cases = {}
    for name, wholeRes, localRes, region in (("impute_1res", [250000], [100000], 2_000_000),
                                             ("impute_fine", [100000], [50000], 1_000_000)):
        texts = {
            "M_M": clustered_allelic(rng, 4000, names, ("Both", "Both", "R1", "R2"), hot),
            "P_P": clustered_allelic(rng, 3000, names, ("Both", "R1", "R2", "R2"), hot),
            "M_P": allelic_text(rng, 600, names),
            "P_M": allelic_text(rng, 600, names),
            "Bi_Allelic": allelic_text(rng, 200, names),
        }
        paths = []
        for kind, t in texts.items():
            p = os.path.join(tmp, f"{name}_Valid_{kind}.bed")
            with open(p, "w") as f:
                f.write(t)
            paths.append(p)
        UW, UL, IW, IL = ref["HapImpute"](files=sorted(paths), genomeSize=gpath, wholeRes=wholeRes,
                                          localRes=localRes, chroms=["#", "X"], Imputation_region=region,
                                          Imputation_min=2, Imputation_ratio=0.9)
        d = {f"text_{k}": text_arr(v) for k, v in texts.items()}
        d["genome"] = text_arr(genome_text())
        d["params"] = np.array(json.dumps(dict(wholeRes=wholeRes, localRes=localRes, chroms=["#", "X"],
                                               region=region, min=2, ratio=0.9)))
        flat_dense("uwhole", UW, d)
        flat_dense("ulocal", UL, d)
        flat_dense("iwhole", IW, d)
        flat_dense("ilocal", IL, d)
        added = sum(np.asarray(IW[r]["Matrix"]).sum() - np.asarray(UW[r]["Matrix"]).sum() for r in wholeRes)
        print(name, "imputed whole-genome contacts added:", int(added))
        cases[name] = d
    for name, d in cases.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)


if __name__ == "__main__":
    main()
