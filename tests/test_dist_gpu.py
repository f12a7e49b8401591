"""Multi-process sharded ICE on the GPU.  World-size-2 runs of
hichap_master_amd.dist.balance_sharded / balance_capi (row shards) and
balance_cis_sharded (--cis-only, whole chromosomes per rank, no collective in
the iterations) with both ranks on cuda:0 and the gloo exchange (RCCL refuses
two ranks on one device), the sweep's side streams forced on: every rank's
weights equal the one-process HIP run (bitwise for row shards; 1e-12 for the
compact per-rank chromosome numbering) and the oracle within the ICE
tolerance.  test_rccl_every_gpu spawns one rank per GPU over the library's own
RCCL communicator on any box with >= 2 GPUs (skipped on a 1-GPU box); RCCL at
world 1 is covered by test_library_rccl_communicator_world1."""
import os
import socket
import tempfile

import numpy as np
import pytest

from hichap_master_amd import synth

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, cis_only, outdir, impl="python", rr_force=None):
    import torch
    import torch.distributed as tdist
    from hichap_master_amd import _lib, dist, ice
    torch.cuda.set_device(0)
    _lib.load()
    _lib.call("hh_set_device", 0)
    _lib.call("hh_tune", b"conc_min_bytes", 0)  # three sweep streams even on this small shard
    _lib.call("hh_tune", b"sweep_single", 0)    # (the single launch is checked first: off)
    if impl.endswith("_upper"):  # upper-triangle tiles: the column side crosses the ranks
        impl = impl[:-len("_upper")]
        _lib.call("hh_tune", b"upper_tiles", 1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b1, b2, c, off = case
        n = int(off[-1])
        rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), world)
        if rr_force is not None:
            rr = np.asarray(rr_force, dtype=np.int64)
        opts = ice.IceOptions(max_iters=400, cis_only=cis_only)
        if impl != "cis":
            m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, cis_only=cis_only,
                                              row_range=(rr[rank], rr[rank + 1]))
        if impl == "cis":
            # chromosomes by LPT, no collective in the iterations (gloo callback
            # for the one MAD exchange)
            cx = dist.CapiExchange([0, n], world, rank, backend="gloo")
            w, s_ = dist.balance_cis_sharded(b1, b2, c, n, off, rank, world,
                                             ice.IceOptions(max_iters=400, cis_only=True), cx)
            cx.close()
        elif impl == "capi":
            # the loop in C++ (hh_ice_balance_sharded), exchange = a gloo callback
            cx = dist.CapiExchange(rr, world, rank, backend="gloo")
            w, s_ = dist.balance_capi(m, opts, cx, torch.cuda.current_stream().cuda_stream)
            cx.close()
        else:
            st = ice.IceState(m, opts)
            ex = dist.Exchange(rr, torch.device("cuda", 0))
            assert not ex.fused
            w, s_ = dist.balance_sharded(st, ex, max_iters=400)
            st.close()
        torch.cuda.synchronize()
        if impl != "cis":
            m.close()
        np.save(os.path.join(outdir, f"w{rank}.npy"), w)
        np.save(os.path.join(outdir, f"it{rank}.npy"), np.atleast_1d(s_["iters"]))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("cis_only,impl", [(False, "python"), (True, "python"), (False, "capi"), (True, "capi"),
                                            (True, "cis")])
def test_balance_sharded_two_processes(cis_only, impl):
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib, ice
    from oracle import ice_ref
    _lib.require_gpu()
    rng = np.random.default_rng(21)
    case = synth.coo_genome([900, 700, 400], rng, A=25.0, trans_density=0.01)
    b1, b2, c, off = case
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=400)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), case, cis_only, d, impl), nprocs=2, start_method="spawn")
        ws = [np.load(os.path.join(d, f"w{r}.npy")) for r in range(2)]
        its = [np.load(os.path.join(d, f"it{r}.npy")) for r in range(2)]
    wr, sr = ice_ref.balance(b1, b2, c, n, off, cis_only=cis_only, max_iters=400)
    for w, it in zip(ws, its):
        if impl == "cis":  # compact per-rank numbering: same sums up to the row-block grouping
            np.testing.assert_array_equal(np.isnan(w), np.isnan(w_full))
            np.testing.assert_allclose(w, w_full, rtol=1e-12, equal_nan=True)
        else:
            np.testing.assert_array_equal(w, w_full)
        np.testing.assert_allclose(w, wr, rtol=1e-9, equal_nan=True)
        np.testing.assert_array_equal(it, np.atleast_1d(st_full["iters"]))
    np.testing.assert_array_equal(ws[0], ws[1])


@pytest.mark.parametrize("impl", ["python", "capi"])
def test_uptiles_two_processes(impl):
    """Upper-triangle tiles over two processes: the column side of each
    rank's strictly upper tiles reaches the other rank's rows through the
    int64 exchange (a torch.distributed reduce callback for the Python
    driver, the all-gather fallback summed in rank order for the C++ loop):
    every rank's weights equal the one-process upper-tile run bitwise."""
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib, ice
    from oracle import ice_ref
    from tests.shard_exchange import require_uptiles
    _lib.require_gpu()
    require_uptiles()
    rng = np.random.default_rng(23)
    case = synth.coo_genome([5000, 4000, 700], rng, A=8.0, trans_density=0.002)
    b1, b2, c, off = case
    n = int(off[-1])
    _lib.call("hh_tune", b"upper_tiles", 1)
    try:
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
        assert m.info()["upper"] == 1
        w_full, st_full = ice.balance_matrix(m, ice.IceOptions(max_iters=400))
        m.close()
    finally:
        _lib.call("hh_tune", b"upper_tiles", -1)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), case, False, d, impl + "_upper"), nprocs=2,
                           start_method="spawn")
        ws = [np.load(os.path.join(d, f"w{r}.npy")) for r in range(2)]
        its = [np.load(os.path.join(d, f"it{r}.npy")) for r in range(2)]
    wr, _ = ice_ref.balance(b1, b2, c, n, off, max_iters=400)
    for w, it in zip(ws, its):
        np.testing.assert_array_equal(w, w_full)
        np.testing.assert_array_equal(it, np.atleast_1d(st_full["iters"]))
    np.testing.assert_allclose(w_full, wr, rtol=1e-9, equal_nan=True)


def _fail_worker(rank, world, port, case, outdir):
    """rank 1 hands hh_ice_balance_sharded a shard that does not match
    rank_rows: both ranks must raise (agreed status), neither may hang in the
    exchange."""
    import torch
    import torch.distributed as tdist
    from hichap_master_amd import _lib, dist, ice
    torch.cuda.set_device(0)
    _lib.load()
    _lib.call("hh_set_device", 0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b1, b2, c, off = case
        n = int(off[-1])
        rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), world)
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(int(rr[rank]), int(rr[rank + 1])))
        rr_seen = np.array(rr, dtype=np.int64)
        if rank == 1:  # this rank's rank_rows disagree with the shard it holds
            rr_seen[1] = rr[1] - 512 if rr[1] >= 512 else rr[1] + 512
        cx = dist.CapiExchange(rr_seen, world, rank, backend="gloo")
        msg = "no error"
        try:
            dist.balance_capi(m, ice.IceOptions(max_iters=50), cx, torch.cuda.current_stream().cuda_stream)
        except Exception as e:  # noqa: BLE001
            msg = str(e)
        cx.close()
        m.close()
        with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
            f.write(msg)
    finally:
        tdist.destroy_process_group()


def test_sharded_failure_on_one_rank_raises_everywhere():
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib
    _lib.require_gpu()
    rng = np.random.default_rng(5)
    case = synth.coo_genome([900, 700], rng, A=20.0, trans_density=0.01)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_fail_worker, args=(2, _free_port(), case, d), nprocs=2, start_method="spawn")
        e0 = open(os.path.join(d, "err0.txt")).read()
        e1 = open(os.path.join(d, "err1.txt")).read()
    assert "rank 1 of 2 failed" in e0, e0
    assert "does not hold rank_rows" in e1, e1


def test_library_rccl_communicator_world1():
    """hh_comm_* (the library-owned RCCL communicator) at world 1 on the box's
    one GPU, and the C++ sharded balance at world 1 equal to hh_ice_balance."""
    import ctypes as C
    import torch
    from hichap_master_amd import _lib, dist, ice
    _lib.require_gpu()
    uid = C.create_string_buffer(128)
    _lib.call("hh_comm_unique_id", uid)
    h = C.c_void_p()
    _lib.call("hh_comm_init", uid, 1, 0, C.byref(h))
    x = torch.arange(1000, dtype=torch.float64, device="cuda")
    y = torch.zeros_like(x)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("hh_comm_allgather", C.c_void_p(x.data_ptr()), 1000, C.c_void_p(y.data_ptr()), h, C.c_void_p(s))
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    _lib.call("hh_comm_free", h)
    rng = np.random.default_rng(5)
    b1, b2, c, off = synth.coo_genome([800, 600], rng, A=25.0, trans_density=0.01)
    n = int(off[-1])
    m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off)
    opts = ice.IceOptions(max_iters=300)
    w1, s1 = ice.balance_matrix(m, opts)
    cx = dist.CapiExchange([0, n], 1, 0)
    w2, s2 = dist.balance_capi(m, opts, cx)
    np.testing.assert_array_equal(w1, w2)
    assert s1["iters"] == s2["iters"]


def _rccl_worker(rank, world, port, case, case1, outdir):
    """One rank per GPU over the library's own RCCL communicator (xGMI):
    genome-wide row shards (hh_ice_balance_sharded, one ncclAllGather of the
    marginals per iteration) and --cis-only by chromosome
    (hh_ice_balance_cis_local, no collective in the iterations)."""
    import torch
    import torch.distributed as tdist
    from hichap_master_amd import _lib, dist, ice
    torch.cuda.set_device(rank)
    _lib.load()
    _lib.call("hh_set_device", rank)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)  # bootstrap for the ncclUniqueId only
    try:
        b1, b2, c, off = case
        n = int(off[-1])
        rr = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), world)
        cx = dist.CapiExchange(rr, world, rank, backend="nccl")
        m = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(rr[rank], rr[rank + 1]))
        w, s_ = dist.balance_capi(m, ice.IceOptions(max_iters=400), cx, torch.cuda.current_stream().cuda_stream)
        m.close()
        wc, sc = dist.balance_cis_sharded(b1, b2, c, n, off, rank, world,
                                          ice.IceOptions(max_iters=400, cis_only=True), cx)
        cx.close()
        # the empty-rank cases an 8-GPU node meets on small matrices: one
        # genome-wide shard without rows (world - 1 real shards, an empty one
        # in the middle), and --cis-only with one chromosome (world - 1
        # chromosome-less ranks)
        w1 = dist.partition_rows(np.bincount(b1, minlength=n) + np.bincount(b2, minlength=n), world - 1)
        rre = np.insert(w1, world // 2, w1[world // 2])
        cxe = dist.CapiExchange(rre, world, rank, backend="nccl")
        me = ice.ContactMatrix.from_pixels(b1, b2, c, n, off, row_range=(rre[rank], rre[rank + 1]))
        we, se = dist.balance_capi(me, ice.IceOptions(max_iters=400), cxe, torch.cuda.current_stream().cuda_stream)
        me.close()
        e1, e2, ec, eoff = case1
        w1c, s1c = dist.balance_cis_sharded(e1, e2, ec, int(eoff[-1]), eoff, rank, world,
                                            ice.IceOptions(max_iters=400, cis_only=True), cxe)
        torch.cuda.synchronize()
        cxe.close()
        np.save(os.path.join(outdir, f"we{rank}.npy"), we)
        np.save(os.path.join(outdir, f"w1c{rank}.npy"), w1c)
        np.save(os.path.join(outdir, f"ite{rank}.npy"), np.array([se["iters"]]))
        np.save(os.path.join(outdir, f"w{rank}.npy"), w)
        np.save(os.path.join(outdir, f"wc{rank}.npy"), wc)
        np.save(os.path.join(outdir, f"it{rank}.npy"), np.array([s_["iters"]]))
        np.save(os.path.join(outdir, f"itc{rank}.npy"), np.atleast_1d(sc["iters"]))
    finally:
        tdist.destroy_process_group()


def test_rccl_every_gpu():
    """RCCL at world = every GPU of the box (skipped below 2: RCCL refuses
    two ranks on one device): the genome-wide sharded balance is bitwise the
    one-GPU run (small matrix: the unit plan sits at its floor, so shards
    sum every row in the same order) and the chromosome-dealt --cis-only run
    equals the one-GPU --cis-only run to 1e-12 with the same iterations."""
    import torch
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib, ice
    _lib.require_gpu()
    world = min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("one GPU on this box: RCCL at world > 1 needs >= 2 devices")
    rng = np.random.default_rng(33)
    case = synth.coo_genome([1100, 900, 700, 500, 300], rng, A=25.0, trans_density=0.01)
    b1, b2, c, off = case
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, max_iters=400)
    wc_full, stc_full = ice.balance(b1, b2, c, n, off, cis_only=True, max_iters=400)
    case1 = synth.coo_genome([1500], rng, A=25.0)
    w1_full, _ = ice.balance(*case1[:3], int(case1[3][-1]), case1[3], cis_only=True, max_iters=400)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rccl_worker, args=(world, _free_port(), case, case1, d), nprocs=world,
                           start_method="spawn")
        for r in range(world):
            np.testing.assert_array_equal(np.load(os.path.join(d, f"w{r}.npy")), w_full)
            assert int(np.load(os.path.join(d, f"it{r}.npy"))[0]) == st_full["iters"]
            wc = np.load(os.path.join(d, f"wc{r}.npy"))
            np.testing.assert_array_equal(np.isnan(wc), np.isnan(wc_full))
            np.testing.assert_allclose(wc, wc_full, rtol=1e-12, equal_nan=True)
            np.testing.assert_array_equal(np.load(os.path.join(d, f"itc{r}.npy")), stc_full["iters"])
            np.testing.assert_array_equal(np.load(os.path.join(d, f"we{r}.npy")), w_full)
            assert int(np.load(os.path.join(d, f"ite{r}.npy"))[0]) == st_full["iters"]
            np.testing.assert_allclose(np.load(os.path.join(d, f"w1c{r}.npy")), w1_full, rtol=1e-12, equal_nan=True)


@pytest.mark.parametrize("impl", ["capi", "python"])
def test_empty_genomewide_shard_world3(impl):
    """World 3 on a 2-row-block matrix: one rank holds no rows (what
    partition_rows gives whenever ranks outnumber row blocks, e.g. the RCCL
    test's 3 500 bins at world 8).  The empty rank still joins every
    all-gather; every rank's weights equal the one-process run bitwise."""
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib, ice
    _lib.require_gpu()
    rng = np.random.default_rng(44)
    case = synth.coo_genome([600, 400], rng, A=25.0, trans_density=0.01)
    b1, b2, c, off = case
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, max_iters=400)
    for rr in ([0, 512, 512, n], [0, 0, 512, n], [0, 512, n, n]):
        with tempfile.TemporaryDirectory() as d:
            mp.start_processes(_worker, args=(3, _free_port(), case, False, d, impl, rr), nprocs=3,
                               start_method="spawn")
            for r in range(3):
                np.testing.assert_array_equal(np.load(os.path.join(d, f"w{r}.npy")), w_full)
                assert int(np.load(os.path.join(d, f"it{r}.npy"))[0]) == st_full["iters"]


def test_chromosomeless_cis_ranks_world4():
    """--cis-only over 4 ranks with 2 chromosomes: ranks 2 and 3 get no
    chromosome and only join the MAD exchange and the final gather; every
    rank's weights equal the one-process --cis-only run to 1e-12 with the
    same per-chromosome iterations."""
    import torch.multiprocessing as mp
    from hichap_master_amd import _lib, ice
    _lib.require_gpu()
    rng = np.random.default_rng(45)
    case = synth.coo_genome([900, 700], rng, A=25.0, trans_density=0.01)
    b1, b2, c, off = case
    n = int(off[-1])
    w_full, st_full = ice.balance(b1, b2, c, n, off, cis_only=True, max_iters=400)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(4, _free_port(), case, True, d, "cis"), nprocs=4, start_method="spawn")
        for r in range(4):
            w = np.load(os.path.join(d, f"w{r}.npy"))
            np.testing.assert_array_equal(np.isnan(w), np.isnan(w_full))
            np.testing.assert_allclose(w, w_full, rtol=1e-12, equal_nan=True)
            np.testing.assert_array_equal(np.load(os.path.join(d, f"it{r}.npy")), st_full["iters"])
