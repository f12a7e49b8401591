"""TAD calling after the DI scan (hichap_master_amd/tads.py, StructureFind.py
:842-1342): the HMM priors and the boundary rules against golden vectors from
the reference's own methods (tests/golden/make_golden_tads.py); the Viterbi
decoder (host C++ behind hh_viterbi_gmm) against exhaustive path enumeration
and the NumPy oracle (ghmm itself is absent: parity with ghmm unpinned); the
whole chain on the GPU against the oracle's gap / DI scans."""
import os

import numpy as np
import pytest

from oracle import structure_ref, tad_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _sf(res=40000, min_tad=200000, max_tad=4000000, state_num=3, window=600000):
    from hichap_master_amd.StructureFind import StructureFind
    sf = StructureFind(Res=res)
    sf.TAD_parameter_init(minTAD=min_tad, maxTAD=max_tad, state_num=state_num, window=window, test_type="ttest")
    return sf


def test_priors_match_reference():
    d = np.load(os.path.join(GOLD, "tads_priors.npz"))
    sf = _sf()
    for k in (3, 5, 6):
        A, B, pi = getattr(sf, f"init_parameter_state{k}")()
        np.testing.assert_array_equal(np.array(A, float), d[f"A{k}"])
        np.testing.assert_array_equal(np.array(B, float), d[f"B{k}"])
        np.testing.assert_array_equal(np.array(pi, float), d[f"pi{k}"])


def _random_model(rng, S, M, zero_frac=0.25):
    A = rng.random((S, S)) * (rng.random((S, S)) > zero_frac)
    A[np.arange(S), rng.integers(0, S, S)] += 0.1  # every row has an exit
    A /= A.sum(axis=1, keepdims=True)
    pi = rng.random(S) + 0.05
    pi /= pi.sum()
    mean = rng.normal(0, 5, (S, M))
    var = rng.uniform(0.5, 9.0, (S, M))
    w = rng.random((S, M)) + 0.1
    w /= w.sum(axis=1, keepdims=True)
    return A, pi, mean, var, w


@pytest.mark.parametrize("seed", range(6))
def test_viterbi_exhaustive(seed):
    from hichap_master_amd.tads import GaussianMixtureHMM
    rng = np.random.default_rng(100 + seed)
    S = 3 if seed % 2 == 0 else 4
    A, pi, mean, var, w = _random_model(rng, S, 3)
    m = GaussianMixtureHMM(A, [[mean[i], var[i], w[i]] for i in range(S)], pi)
    for n in (1, 2, 5, 7 if S == 3 else 6):
        x = rng.normal(0, 6, n)
        path, logp = m.viterbi(x)
        bp, bl = tad_ref.brute_force(x, A, pi, mean, var, w)
        np.testing.assert_allclose(logp, bl, rtol=1e-12)
        np.testing.assert_array_equal(path, bp)


@pytest.mark.parametrize("k", [3, 5, 6])
def test_viterbi_matches_oracle_on_priors(k):
    """Long DI-like sequences under the reference's priors (the 5- and
    6-state models have forbidden transitions)."""
    from hichap_master_amd.tads import GaussianMixtureHMM
    sf = _sf()
    A, B, pi = getattr(sf, f"init_parameter_state{k}")()
    m = GaussianMixtureHMM(A, B, pi)
    rng = np.random.default_rng(k)
    x = np.cumsum(rng.normal(0, 1.5, 3000)) % 25 - 12
    x[rng.integers(0, x.size, 200)] = 0.0
    path, logp = m.viterbi(x)
    Bm = np.array(B, float)
    op, ol = tad_ref.viterbi(x, A, pi, Bm[:, 0], Bm[:, 1], Bm[:, 2])
    np.testing.assert_array_equal(path, op)
    np.testing.assert_allclose(logp, ol, rtol=1e-12)


def test_viterbi_rejects_bad_models():
    from hichap_master_amd._lib import HipLibraryError
    from hichap_master_amd.tads import GaussianMixtureHMM
    with pytest.raises(HipLibraryError):
        GaussianMixtureHMM([[1.0]], [[[0.0], [0.0], [1.0]]], [1.0]).viterbi([1.0])  # variance 0
    with pytest.raises(ValueError):
        GaussianMixtureHMM([[1.0, 0.0]], [[[0.0], [1.0], [1.0]]], [1.0])


@pytest.mark.parametrize("case", ["tads_state3", "tads_state5", "tads_state3_res10k"])
def test_boundary_rules_match_reference(case):
    d = np.load(os.path.join(GOLD, case + ".npz"))
    sf = _sf(res=int(d["res"]), min_tad=int(d["min_tad"]), max_tad=int(d["max_tad"]),
             state_num=int(d["state_num"]))
    sf.DI_dict, sf.Gap_all, sf.DI_all_train, sf.boundary_index = {}, {}, {}, {}
    chroms = [str(c) for c in d["chroms"]]
    for c in chroms:
        DI, gap, seg = d[f"{c}_DI"], d[f"{c}_gap"], d[f"{c}_seg"]
        sf.DI_dict[c], sf.Gap_all[c] = DI, gap
        sf.DI_all_train[c] = {(int(a), int(b)): DI[a:b] for a, b in seg}
        paths, pos = {}, 0
        for (a, b), r in zip(seg, d[f"{c}_rely"]):
            paths[(int(a), int(b))] = (list(d[f"{c}_path"][pos:pos + b - a]), float(r))
            pos += b - a
        bi = sf.BoundaryCall(paths_sub=paths, Gap_sub=gap, DI_len_sub=DI.size)
        np.testing.assert_array_equal(bi["boundary"], d[f"{c}_call_boundary"])
        np.testing.assert_array_equal(bi["state"], d[f"{c}_call_state"])
        np.testing.assert_array_equal(bi["rely"], d[f"{c}_call_rely"])
        np.testing.assert_array_equal(bi["raw_state"], d[f"{c}_call_raw"])
        sf.boundary_index[c] = bi
    sf.BoundaryFilter()
    sf.BoundaryToDomain()
    for c in chroms:
        np.testing.assert_array_equal(sf.boundary_index[c]["state"], d[f"{c}_filt_state"])
        np.testing.assert_array_equal(sf.boundary_filtered[c], d[f"{c}_filtered"])
        np.testing.assert_array_equal(sf.candidate_domain[c]["start"], d[f"{c}_cand_start"])
        np.testing.assert_array_equal(sf.candidate_domain[c]["end"], d[f"{c}_cand_end"])
        np.testing.assert_array_equal(sf.Domain_dict[c]["start"], d[f"{c}_dom_start"])
        np.testing.assert_array_equal(sf.Domain_dict[c]["end"], d[f"{c}_dom_end"])


def test_six_state_model_has_no_boundary_rule():
    sf = _sf(state_num=6)
    with pytest.raises(ValueError):
        sf.BoundaryCall({(1, 9): ([0] * 8, -1.0)}, np.array([0, 9]), 10)


@pytest.mark.gpu
def test_tad_chain_on_gpu_matches_oracle_scans():
    """run_TADs' numeric chain (GPU gap / DI scans, host Viterbi with the
    3-state model, boundary rules) == the same chain fed by the oracle's
    gap / DI scans."""
    from hichap_master_amd import _lib, synth
    from hichap_master_amd.tads import GaussianMixtureHMM
    _lib.require_gpu()
    rng = np.random.default_rng(5)
    mats = {}
    for c, n in (("1", 420), ("2", 300)):
        M = synth.dense_chrom(n, rng, A=30.0, gap_frac=0.04).astype(np.float64)
        tad = np.repeat(np.arange(n), rng.integers(6, 20, n))[:n]  # TAD blocks: contacts x 4 inside
        M = M * np.where(tad[:, None] == tad[None, :], 4.0, 1.0)
        w = 1.0 / np.sqrt(np.maximum(M.sum(axis=1), 1.0))
        mats[c] = M * w[:, None] * w[None, :]
    sf = _sf()
    A, B, pi = sf.init_parameter_state3()
    # a "trained" model at this data's DI scale: the priors' means x 0.25
    B = [[[m * 0.25 for m in b[0]], [v * 0.0625 for v in b[1]], b[2]] for b in B]
    model = GaussianMixtureHMM(A, B, pi)
    dom = sf.tad_domains(mats, model=model)
    ref = _sf()
    ref.model = model
    ref.DI_dict, ref.Gap_all, ref.DI_all_train = {}, {}, {}
    for c, M in mats.items():
        gap = structure_ref.get_gap(M, ref.minTAD, ref.Res)
        DI = structure_ref.get_di(M, gap, int(ref.window / ref.Res))
        np.testing.assert_array_equal(sf.Gap_all[c], gap)
        np.testing.assert_allclose(sf.DI_dict[c], DI, rtol=1e-12, atol=1e-12)
        ref.DI_dict[c], ref.Gap_all[c] = DI, gap
        filt = ref.Gap_Filter(gap, M)
        ref.DI_all_train[c] = ref.train_segments(gap, filt, DI, 7, float(gap.size) / M.shape[0] / 2.0)
    ref.modelPredict()
    ref.BoundaryFilter()
    ref.BoundaryToDomain()
    for c in mats:
        assert len(sf.boundary_index[c]) > 0 and len(dom[c]) > 0
        np.testing.assert_array_equal(dom[c]["start"], ref.Domain_dict[c]["start"])
        np.testing.assert_array_equal(dom[c]["end"], ref.Domain_dict[c]["end"])
