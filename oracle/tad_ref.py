"""ORACLE (test infrastructure only) — the TAD HMM decoding restated in NumPy.

ghmm's ``model.viterbi`` (called at HiCHap/StructureFind.py:1121) for a
continuous HMM with Gaussian-mixture emissions, B[i] = [means, variances,
weights].  ghmm is a third-party C library absent from /root/reference and
from this image (version unpinned), so this is the published log-space Viterbi
recursion (impossible transitions -inf, ties to the lowest state index),
pinned by exhaustive path enumeration on short sequences
(tests/test_tads.py) -- parity with ghmm itself is unpinned.
"""
from __future__ import annotations

import itertools

import numpy as np


def log_emission(x, mean, var, weight):
    """log sum_m w_m N(x; mu_m, v_m) for every state: (n, S)."""
    x = np.asarray(x, float)[:, None, None]
    with np.errstate(divide="ignore"):
        t = np.log(weight)[None] - 0.5 * np.log(2 * np.pi * var)[None] - 0.5 * (x - mean[None]) ** 2 / var[None]
    mx = np.max(t, axis=2, keepdims=True)
    return (mx + np.log(np.sum(np.exp(t - mx), axis=2, keepdims=True)))[..., 0]


def viterbi(x, A, pi, mean, var, weight):
    """(path, log_p) of the most probable state path."""
    with np.errstate(divide="ignore"):
        la, lpi = np.log(np.asarray(A, float)), np.log(np.asarray(pi, float))
    E = log_emission(x, np.asarray(mean, float), np.asarray(var, float), np.asarray(weight, float))
    n, S = E.shape
    delta = lpi + E[0]
    back = np.zeros((n, S), np.int64)
    for t in range(1, n):
        cand = delta[:, None] + la          # [from, to]
        back[t] = np.argmax(cand, axis=0)   # first maximum = lowest state
        delta = cand[back[t], np.arange(S)] + E[t]
    path = np.empty(n, np.int64)
    path[-1] = int(np.argmax(delta))
    for t in range(n - 1, 0, -1):
        path[t - 1] = back[t, path[t]]
    return path, float(np.max(delta))


def brute_force(x, A, pi, mean, var, weight):
    """max over all S^n paths of the joint log-probability (tiny n only)."""
    with np.errstate(divide="ignore"):
        la, lpi = np.log(np.asarray(A, float)), np.log(np.asarray(pi, float))
    E = log_emission(x, np.asarray(mean, float), np.asarray(var, float), np.asarray(weight, float))
    n, S = E.shape
    best, arg = -np.inf, None
    for p in itertools.product(range(S), repeat=n):
        v = lpi[p[0]] + E[0, p[0]] + sum(la[p[t - 1], p[t]] + E[t, p[t]] for t in range(1, n))
        if v > best:
            best, arg = v, p
    return np.array(arg), best
