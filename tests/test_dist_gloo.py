"""world_size-2 gloo runs of the sharded ICE driver (hichap_master_amd.dist)
with a NumPy backend: the all-gather exchange, row partitioning and loop
control give the single-process oracle's weights on every rank."""
import os
import socket
import tempfile

import numpy as np
import pytest

from hichap_master_amd import dist, synth


def test_partition_rows_aligned_and_balanced():
    w = np.random.default_rng(0).integers(0, 100, size=5000)
    rr = dist.partition_rows(w, 4)
    assert rr[0] == 0 and rr[-1] == 5000
    assert all(x % dist.ROW_BLOCK == 0 for x in rr[1:-1])
    assert np.all(np.diff(rr) >= 0)
    loads = [w[a:b].sum() for a, b in zip(rr[:-1], rr[1:])]
    assert max(loads) < 1.35 * (w.sum() / 4)
    assert list(dist.partition_rows(w, 1)) == [0, 5000]
    # more ranks than blocks: empty shards allowed, ranges still cover [0, n)
    rr = dist.partition_rows(np.ones(300), 8)
    assert rr[0] == 0 and rr[-1] == 300 and np.all(np.diff(rr) >= 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, outdir):
    import torch
    import torch.distributed as tdist
    from tests.np_shard_backend import NumpyShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    b1, b2, c, off = case
    n = int(off[-1])
    rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), world)
    be = NumpyShard(b1, b2, c, n, off, (rr[rank], rr[rank + 1]), max_iters=400)
    ex = dist.Exchange(rr, torch.device("cpu"))
    w, st = dist.balance_sharded(be, ex, max_iters=400, check_every=8)
    np.save(os.path.join(outdir, f"w{rank}.npy"), w)
    np.save(os.path.join(outdir, f"it{rank}.npy"), np.array([st["iters"]]))
    tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_balance_gloo_matches_oracle(world):
    import torch.multiprocessing as mp
    from oracle import ice_ref
    rng = np.random.default_rng(11)
    case = synth.coo_genome([400, 300], rng, A=25.0, trans_density=0.01)
    b1, b2, c, off = case
    n = int(off[-1])
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), case, d), nprocs=world, start_method="spawn")
        ws = [np.load(os.path.join(d, f"w{r}.npy")) for r in range(world)]
        its = [int(np.load(os.path.join(d, f"it{r}.npy"))[0]) for r in range(world)]
    wr, sr = ice_ref.balance(b1, b2, c, n, off, max_iters=400)
    for w in ws:
        np.testing.assert_array_equal(w, ws[0])
        np.testing.assert_allclose(w, wr, rtol=1e-12, equal_nan=True)
    # the driver polls every 8 sweeps; converged groups stop updating
    assert its[0] == sr["iters"]


def test_lpt_assign_greedy():
    owner = dist.lpt_assign([10, 9, 8, 1, 1, 1], 2)
    loads = [sum(c for c, o in zip([10, 9, 8, 1, 1, 1], owner) if o == r) for r in range(2)]
    assert loads == [13, 17]  # 10 | 9, 8 | then the 1s to the lighter rank
    assert list(dist.lpt_assign([5, 5, 5], 1)) == [0, 0, 0]
    # hg19 autosomes at 25 kb, cost N^3 over 8 ranks: max load vs ideal (1.98e12 vs 1.27e12)
    Ns = np.array(synth.chrom_bins([synth.HG19[str(c)] for c in range(1, 23)], 25000), dtype=float)
    own = dist.lpt_assign(Ns ** 3, 8)
    worst = max(float(np.sum(Ns[own == r] ** 3)) for r in range(8))
    assert worst == float(Ns.max() ** 3) or worst < 1.6 * float(np.sum(Ns ** 3)) / 8


def _chrom_worker(rank, world, port, outdir):
    import torch.distributed as tdist
    from oracle import hichap_ref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    mats = {f"c{i}": synth.dense_chrom(n, rng, A=20.0) for i, n in enumerate([60, 90, 40, 75])}

    def body(key):
        TM = mats[key]
        return hichap_ref.sort_chromosomes([key]), int(TM.sum())

    res = dist.run_chromosomes(body, list(mats), [m.shape[0] ** 2 for m in mats.values()], rank, world,
                               gather=True)
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.array([res[k][1] for k in mats]))
    tdist.destroy_process_group()


def test_run_chromosomes_gloo():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_chrom_worker, args=(2, _free_port(), d), nprocs=2, start_method="spawn")
        a, b = np.load(os.path.join(d, "r0.npy")), np.load(os.path.join(d, "r1.npy"))
    rng = np.random.default_rng(5)
    want = [int(synth.dense_chrom(n, rng, A=20.0).sum()) for n in [60, 90, 40, 75]]
    assert list(a) == want and list(b) == want


def test_refine_weights_levels_measured_cost():
    """A shard measured slower per unit weight gets fewer rows next time."""
    w = np.ones(8192)
    rr = dist.partition_rows(w, 2)
    assert list(rr) == [0, 4096, 8192]
    # rows of the second half sweep 3x slower per weight unit
    w2 = dist.refine_weights(w, rr, [1.0, 3.0])
    np.testing.assert_allclose(w2[:4096].sum(), 1.0)
    np.testing.assert_allclose(w2[4096:].sum(), 3.0)
    rr2 = dist.partition_rows(w2, 2)
    assert rr2[1] > 4096 and rr2[1] % dist.ROW_BLOCK == 0
    cost = [w2[a:b].sum() for a, b in zip(rr2[:-1], rr2[1:])]
    assert max(cost) < 1.15 * (sum(cost) / 2)
    # zero-weight shard untouched, equal costs keep the partition
    np.testing.assert_array_equal(dist.refine_weights(np.zeros(10), [0, 5, 10], [1.0, 1.0]), np.zeros(10))
    np.testing.assert_array_equal(dist.partition_rows(dist.refine_weights(w, rr, [2.0, 2.0]), 2), rr)


def test_cis_plan_local_genome_reassembles():
    """--cis-only by chromosome (dist.cis_plan / local_genome): LPT owners,
    compact renumbering; the oracle's per-rank balances of the local genomes
    (MAD off: its cutoff is the one genome-wide step, exchanged on the GPU
    path) reassemble the whole-genome --cis-only result exactly."""
    from hichap_master_amd import dist, synth
    from oracle import ice_ref
    rng = np.random.default_rng(4)
    b1, b2, c, off = synth.coo_genome([300, 250, 200, 150, 100], rng, A=20.0, trans_density=0.02)
    n = int(off[-1])
    w_full, st_full = ice_ref.balance(b1, b2, c, n, off, cis_only=True, mad_max=0, max_iters=300)
    for world in (1, 2, 3):
        owner, cost = dist.cis_plan(b1, b2, off, world)
        assert sorted(set(owner.tolist())) == list(range(min(world, len(cost))))
        w = np.full(n, np.nan)
        for r in range(world):
            mine = np.flatnonzero(owner == r)
            lb1, lb2, lc, loff = dist.local_genome(b1, b2, c, off, mine)
            assert (lb1 <= lb2).all() and lb2.max() < loff[-1]
            wl, _ = ice_ref.balance(lb1, lb2, lc, int(loff[-1]), loff, cis_only=True, mad_max=0, max_iters=300)
            p = 0
            for ch in mine:
                k = int(off[ch + 1] - off[ch])
                w[off[ch]:off[ch + 1]] = wl[p:p + k]
                p += k
        np.testing.assert_array_equal(np.isnan(w), np.isnan(w_full))
        np.testing.assert_allclose(w, w_full, rtol=1e-13, equal_nan=True)
