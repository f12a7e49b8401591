#!/usr/bin/env python3
"""Golden vectors for the TAD boundary rules from the REFERENCE's own methods
(StructureFind.BoundaryMask :1126, BoundaryCall :1158, Candidate_domains
:1212, BoundaryFilter :1232, BoundaryToDomain :1271, init_parameter_state3/5/6
:918-1049).  Run in the build container only (reads /root/reference):

    python tests/golden/make_golden_tads.py

Same harness as make_golden.py (lib2to3 text conversion in memory, methods
extracted with ast, nothing converted written to disk).  One Py2 -> Py3
deviation, applied to the converted text: the structured arrays' byte-string
fields ('>S5', '>S1') become unicode ('<U5', '<U1'), because the reference
compares them with str literals, which Py2 treats as equal to bytes and Py3
does not.  The Viterbi paths fed to BoundaryCall are synthetic state runs (the
reference gets them from ghmm, absent here); the rules are what is pinned.
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

from make_golden import REF, _namespace, _py3_source  # noqa: E402

METHODS = ["BoundaryMask", "BoundaryCall", "Candidate_domains", "BoundaryFilter", "BoundaryToDomain",
           "init_parameter_state3", "init_parameter_state5", "init_parameter_state6"]


def load_reference():
    ns = _namespace()
    text = _py3_source(os.path.join(REF, "StructureFind.py"))
    text = text.replace("'>S5'", "'<U5'").replace("'>S1'", "'<U1'")
    tree = ast.parse(text)
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "StructureFind"][0]
    meths = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in METHODS]
    assert {m.name for m in meths} == set(METHODS)
    klass = ast.ClassDef(name="RefSF", bases=[], keywords=[], body=meths, decorator_list=[])
    exec(compile(ast.fix_missing_locations(ast.Module(body=[klass], type_ignores=[])), "<StructureFind>",
                 "exec"), ns)
    return ns["RefSF"]


def synth_chrom(rng, N, S, A):
    """DI with zero runs, gap bins, segments between gaps, and Viterbi-like
    state runs per segment (patterns of the boundary rules occur)."""
    DI = rng.normal(0, 8, N)
    gap = np.sort(rng.choice(np.arange(1, N - 1), size=N // 40, replace=False))
    runs = rng.integers(1, N - 6, 6)
    for r in runs:  # runs of consecutive gap bins
        gap = np.union1d(gap, np.arange(r, min(r + rng.integers(2, 9), N - 1)))
    for r in rng.integers(1, N - 8, N // 150):  # sparse clusters (every other bin): filter hits
        gap = np.union1d(gap, np.arange(r, r + 6, 2))
    gap = np.union1d(gap, [0, N - 1])
    DI[gap] = 0.0
    for r in rng.integers(0, N - 4, 5):  # isolated zero-DI runs
        DI[r:r + rng.integers(2, 5)] = 0.0
    segs = {}
    for a, b in zip(gap[:-1], gap[1:]):
        if b - a > 7:
            segs[(int(a) + 1, int(b))] = None
    paths = {}
    for (a, b) in segs:
        L = b - a
        path, s = [], int(rng.integers(0, S))
        while len(path) < L:
            path.extend([s] * int(rng.integers(1, 7)))
            p = np.asarray(A[s], float) + 0.05  # the prior's transitions, every state reachable
            s = int(rng.choice(S, p=p / p.sum()))
        paths[(a, b)] = (path[:L], float(rng.normal(-50, 10)))
    return DI, gap, segs, paths


def run_case(RefSF, rng, state_num, chroms, res=40000, min_tad=200000, max_tad=4000000):
    sf = RefSF()
    sf.Res, sf.state_num, sf.minTAD, sf.maxTAD = res, state_num, min_tad, max_tad
    sf.DI_all_train, sf.DI_dict, sf.Gap_all, sf.boundary_index = {}, {}, {}, {}
    out = {}
    A = getattr(sf, f"init_parameter_state{state_num}")()[0]
    for name, N in chroms:
        DI, gap, segs, paths = synth_chrom(rng, N, state_num, A)
        sf.DI_dict[name] = DI
        sf.Gap_all[name] = gap
        sf.DI_all_train[name] = {k: DI[k[0]:k[1]] for k in segs}
        bi = sf.BoundaryCall(paths_sub=paths, Gap_sub=gap, DI_len_sub=N)
        sf.boundary_index[name] = bi
        keys = sorted(paths)
        out[f"{name}_DI"] = DI
        out[f"{name}_gap"] = gap.astype(np.int64)
        out[f"{name}_seg"] = np.array(keys, dtype=np.int64)
        out[f"{name}_path"] = np.concatenate([np.array(paths[k][0], np.int64) for k in keys])
        out[f"{name}_rely"] = np.array([paths[k][1] for k in keys])
        out[f"{name}_call_boundary"] = bi["boundary"].astype(np.int64)
        out[f"{name}_call_state"] = bi["state"].astype("<U5")
        out[f"{name}_call_rely"] = bi["rely"].astype(np.float64)
        out[f"{name}_call_raw"] = bi["raw_state"].astype("<U1")
    sf.BoundaryFilter()
    sf.BoundaryToDomain()
    for name, _ in chroms:
        out[f"{name}_filt_state"] = sf.boundary_index[name]["state"].astype("<U5")
        out[f"{name}_filtered"] = np.asarray(sf.boundary_filtered[name], dtype=np.int64)
        out[f"{name}_dom_start"] = np.asarray(sf.Domain_dict[name]["start"], dtype=np.int64)
        out[f"{name}_dom_end"] = np.asarray(sf.Domain_dict[name]["end"], dtype=np.int64)
        out[f"{name}_cand_start"] = np.asarray(sf.candidate_domain[name]["start"], dtype=np.int64)
        out[f"{name}_cand_end"] = np.asarray(sf.candidate_domain[name]["end"], dtype=np.int64)
    out["chroms"] = np.array([c for c, _ in chroms])
    out["sizes"] = np.array([n for _, n in chroms], dtype=np.int64)
    out["res"], out["min_tad"], out["max_tad"], out["state_num"] = (np.int64(res), np.int64(min_tad),
                                                                    np.int64(max_tad), np.int64(state_num))
    return out


def main():
    RefSF = load_reference()
    rng = np.random.default_rng(20201016)
    sf = RefSF()
    priors = {}
    for k in (3, 5, 6):
        A, B, pi = getattr(sf, f"init_parameter_state{k}")()
        priors[f"A{k}"] = np.array(A, dtype=np.float64)
        priors[f"B{k}"] = np.array(B, dtype=np.float64)
        priors[f"pi{k}"] = np.array(pi, dtype=np.float64)
    cases = {
        "tads_state3": run_case(RefSF, rng, 3, [("1", 900), ("2", 640), ("X", 420)]),
        "tads_state5": run_case(RefSF, rng, 5, [("1", 800), ("7", 500)]),
        "tads_state3_res10k": run_case(RefSF, rng, 3, [("3", 1500)], res=10000, min_tad=50000, max_tad=1000000),
        "tads_priors": priors,
    }
    for name, d in cases.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print("wrote", path, len(d), "arrays")


if __name__ == "__main__":
    main()
