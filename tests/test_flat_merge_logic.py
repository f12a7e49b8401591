"""CPU restatement of the flat (merge-path) sweep's row bookkeeping
(hichap_master_amd/csrc/ice.hip: flat_step / flat_seg, plan split in
matrix.hip plan_tiles): lane-major runs of U uint4, row of a run's first
uint4 by bounded search over the compacted row starts, rows closed at their
starts, heads carried left by the segmented suffix scan.  Checked against
plain per-row sums on random ragged tiles (empty rows, one-uint4 rows,
rows spanning lanes, steps and the 64-lane wave), so the kernel's
bookkeeping is pinned independently of the GPU."""
import numpy as np
import pytest

NW = 8  # waves per block (kFlatWaves)


def plan_split(fst, nfr, Q):
    """tile_fw: per wave (first uint4, first compact row), wave 8 = (Q, nfr)."""
    out = []
    for w in range(NW + 1):
        tq = Q * w // NW
        i = int(np.searchsorted(fst[:nfr], tq, "left"))
        out.append((int(fst[i]) if i < nfr else Q, i))
    return out


def flat_seg(pay, fst, fr, nfr, acc, qa, qb, i0, i1, U, compact=None):
    """compact: None (row-id accumulation, flat_step) or a dict of compact
    row -> sum (flat_step_c: every row's first write must be a plain store
    by the lane holding its start, later ones adds by lane 0)."""
    if i0 >= i1:
        return
    ic, q0 = i0, qa
    while q0 < qb:
        L = []
        for lane in range(64):
            s = q0 + lane * U
            act = s < qb
            d = [pay[s + k] if s + k < qb else 0.0 for k in range(U)]
            lo, hi = ic, min(i1 - 1, ic + lane * U + 1)
            while lo < hi:
                mid = (lo + hi + 1) >> 1
                if fst[mid] <= s:
                    lo = mid
                else:
                    hi = mid - 1
            head = fst[lo] < s
            nb = [fst[min(lo + 1 + k, nfr)] for k in range(U)]
            rid = [fr[min(lo + k, nfr - 1)] for k in range(U)]
            x = h = 0.0
            inhead, j, done = head, 0, []
            for k in range(U):
                if k > 0 and s + k == nb[j] and s + k < qb:
                    if inhead:
                        h, inhead = x, False
                    else:
                        done.append((lo + j if compact is not None else rid[j], x))
                    x, j = 0.0, j + 1
                x += d[k]
            if inhead:
                h = x
            c = compact is not None
            L.append(dict(act=act, h=h if act else 0.0, F=(not act) or inhead, x=x,
                          tail=act and not inhead, orow=(lo + j) if c else rid[j], done=done, head=head,
                          rid0=lo if c else rid[0], last=lo + j))
        def store(r, v):
            if compact is None:
                acc[r] += v
            else:
                assert r not in compact, "a compact row's first write must be its only store"
                compact[r] = v

        for ln in L:
            for r, v in ln["done"]:
                store(r, v)
        H = [ln["h"] for ln in L]
        F = [ln["F"] for ln in L]
        o = 1
        while o < 64:
            Hn, Fn = list(H), list(F)
            for lane in range(64 - o):
                if F[lane]:
                    H[lane] += Hn[lane + o]
                    F[lane] = Fn[lane + o]
            o <<= 1
        for lane, ln in enumerate(L):
            if ln["tail"]:
                store(ln["orow"], ln["x"] + (H[lane + 1] if lane < 63 else 0.0))
        if L[0]["head"]:
            if compact is None:
                acc[L[0]["rid0"]] += H[0]
            else:
                assert L[0]["rid0"] in compact, "a continued row was stored before"
                compact[L[0]["rid0"]] += H[0]
        ic = L[63]["last"]
        q0 += 64 * U


@pytest.mark.parametrize("U,compact", [(2, False), (4, False), (2, True), (8, True)])
def test_flat_rows_bookkeeping(U, compact):
    rng = np.random.default_rng(7 + U)
    for _ in range(25):
        nrows = 512
        maxlen = int(rng.integers(1, 40))
        lens = rng.integers(0, maxlen + 1, nrows) * (rng.random(nrows) < rng.random())
        if rng.random() < 0.3:
            lens[rng.integers(0, nrows, 40)] = 1  # many one-uint4 rows
        rp = np.concatenate([[0], np.cumsum(lens)])
        Q = int(rp[-1])
        pay = rng.random(Q)
        nz = np.nonzero(lens)[0]
        nfr = len(nz)
        if nfr == 0:
            continue
        fr = np.zeros(nrows, int)
        fr[:nfr] = nz
        fst = np.full(nrows + 1, Q)
        fst[:nfr] = rp[nz]
        split = plan_split(fst, nfr, Q)
        acc = np.zeros(nrows)
        cmp = {} if compact else None
        for w in range(NW):
            (qa, i0), (qb, i1) = split[w], split[w + 1]
            flat_seg(pay, fst, fr, nfr, acc, qa, qb, i0, i1, U, cmp)
        if compact:
            assert sorted(cmp) == list(range(nfr))  # every nonempty row written
            for i, v in cmp.items():
                acc[fr[i]] += v
        ref = np.array([pay[rp[r]:rp[r + 1]].sum() for r in range(nrows)])
        np.testing.assert_allclose(acc, ref, rtol=1e-12, atol=1e-12)
