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
    assert all(x % 256 == 0 for x in rr[1:-1])
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


@pytest.mark.parametrize("world", [2])
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
