"""Multi-GPU drivers: one process per GPU.

Genome-wide ICE: rows sharded, one all-gather of the per-bin marginal per
iteration over RCCL (xGMI).  Per-chromosome work (two-step correction,
compartment PCA, DI scans): whole chromosomes dealt to ranks by LPT on their
cost, no collective on the data path (``lpt_assign`` / ``run_chromosomes``).

Each rank holds complete symmetric rows ``[rank_rows[r], rank_rows[r+1])`` of
the pixel-chunk matrix, so the marginal of its own rows is exact locally; the
only exchange per iteration is an all-gather of those marginals (n_bins x 8 B
in total: 4.9 MB for the diploid 10 kb genome).  Every rank then runs the
identical variance / bias update on the full vector.  Every
reduction is a fixed tree, so the weights are bitwise reproducible for a fixed
unit plan; the work-unit size adapts to each shard's payload, which regroups a
row's partial sums, so runs with different world sizes agree to ~1e-15
relative rather than bitwise (bitwise whenever the unit plan is the same, e.g.
small matrices at the unit-size floor, or a pinned hh_tune("unit_entries")).

The driver is written against a small backend protocol (``marg_local``,
``set_marg``, ``filter_nnz``, ``filter_count_mad``, ``update``,
``active_groups``, ``finalize``) so that the exchange logic is exercised by
world-size-2 ``gloo`` tests on CPU as well as by the HIP backend
(``hichap_master_amd.ice.IceState``) on GPUs.
"""
from __future__ import annotations

import numpy as np


ROW_BLOCK = 512  # shards are whole 512-row blocks of the tiled layout


def partition_rows(row_weight, world: int, align: int = ROW_BLOCK) -> np.ndarray:
    """Contiguous row ranges with ~equal total weight (e.g. stored slots per
    row), cut at multiples of ``align``.  Returns ``rank_rows[world + 1]``."""
    w = np.asarray(row_weight, dtype=np.float64)
    n = w.size
    if world <= 1 or n == 0:
        return np.array([0, n], dtype=np.int64)
    nb = (n + align - 1) // align
    wb = np.zeros(nb * align)
    wb[:n] = w
    cum = np.concatenate([[0.0], np.cumsum(wb.reshape(nb, align).sum(axis=1))])
    tot = cum[-1]
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, tot * r / world, side="left"))
        cuts.append(min(max(c, cuts[-1]), nb))
    cuts.append(nb)
    return np.minimum(np.asarray(cuts, dtype=np.int64) * align, n)


def refine_weights(row_weight, rank_rows, shard_cost) -> np.ndarray:
    """Per-row weights rescaled so each shard's rows carry its measured cost
    (e.g. sweep ms): w'_i = w_i * cost_r / W_r for the rows of shard r (W_r =
    the shard's total weight).  Stored payload alone mis-prices rows whose
    bytes sweep at different rates (4-bit band slots are VALU-bound, sparse
    flat tiles latency-bound); one measured refinement of ``partition_rows``
    levels the slowest rank.  A shard with zero weight keeps its weights."""
    w = np.asarray(row_weight, dtype=np.float64)
    rr = np.asarray(rank_rows, dtype=np.int64)
    cost = np.asarray(shard_cost, dtype=np.float64)
    out = w.copy()
    for r in range(rr.size - 1):
        W = w[rr[r]:rr[r + 1]].sum()
        if W > 0 and cost[r] > 0:
            out[rr[r]:rr[r + 1]] *= cost[r] / W
    return out


def lpt_assign(costs, world: int) -> np.ndarray:
    """Longest-processing-time-first: items in decreasing cost (ties by
    index) each go to the least-loaded rank (ties by lowest rank).  Returns
    ``owner[i]``; deterministic, so every rank computes the same plan."""
    c = np.asarray(costs, dtype=np.float64)
    owner = np.zeros(c.size, dtype=np.int64)
    load = np.zeros(max(int(world), 1))
    for i in sorted(range(c.size), key=lambda k: (-c[k], k)):
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += c[i]
    return owner


def run_chromosomes(fn, keys, costs, rank: int, world: int, gather: bool = False, group=None):
    """Run ``fn(key)`` for this rank's share of ``keys`` (LPT on ``costs``).
    Returns {key: result} for the local keys, or for every key on every rank
    with ``gather=True`` (``all_gather_object``; meant for small results such
    as PC vectors, not N x N matrices)."""
    owner = lpt_assign(costs, world)
    local = {k: fn(k) for k, o in zip(keys, owner) if o == rank}
    if not gather or world == 1:
        return local
    import torch.distributed as tdist
    parts = [None] * world
    tdist.all_gather_object(parts, local, group=group)
    out = {}
    for p in parts:
        out.update(p)
    return {k: out[k] for k in keys}


class Exchange:
    """All-gather of per-rank padded marginals through torch.distributed
    (backend "nccl" = RCCL on ROCm; "gloo" on CPU)."""

    def __init__(self, rank_rows, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.group = group
        self.rank_rows = np.asarray(rank_rows, dtype=np.int64)
        self.world = self.rank_rows.size - 1
        self.maxlen = int(np.max(np.diff(self.rank_rows))) if self.world else 0
        self.maxlen = max(self.maxlen, 1)
        self.local = torch.zeros(self.maxlen, dtype=torch.float64, device=device)
        self.gathered = torch.zeros(self.world * self.maxlen, dtype=torch.float64, device=device)
        self._views = list(self.gathered.view(self.world, self.maxlen).unbind(0))
        be = dist.get_backend(group) if dist.is_initialized() else "none"
        self.fused = be == "nccl"

    def reduce_callback(self):
        """An hh_reduce_fn over this group: the column side of the
        upper-triangle tiles (per-rank padded int64 blocks summed, this
        rank's block returned; integer sums, so any reduction order is
        exact)."""
        return _python_reduce_scatter(self.world, self.dist.get_rank(self.group), self.group,
                                      on_device=self.fused)

    def all_gather(self):
        if self.world == 1:
            self.gathered.copy_(self.local)
        elif self.fused:
            self.dist.all_gather_into_tensor(self.gathered, self.local, group=self.group)
        else:
            self.dist.all_gather(self._views, self.local, group=self.group)


def _stream():
    import torch
    if torch.cuda.is_available():
        return torch.cuda.current_stream().cuda_stream
    return None


def run_filters(backend, ex: Exchange):
    s = _stream()
    bind = getattr(backend, "bind_exchange", None)
    if bind is not None:  # the column side of upper-triangle tiles crosses ranks
        bind(ex)
    backend.marg_local(0, ex.local, s)
    ex.all_gather()
    backend.set_marg(ex.gathered, ex.world, ex.maxlen, ex.rank_rows, s)
    backend.filter_nnz(s)
    backend.marg_local(1, ex.local, s)
    ex.all_gather()
    backend.set_marg(ex.gathered, ex.world, ex.maxlen, ex.rank_rows, s)
    backend.filter_count_mad(s)


def iterate(backend, ex: Exchange, n: int):
    """``n`` ICE iterations (no host synchronisation)."""
    s = _stream()
    for _ in range(n):
        backend.marg_local(2, ex.local, s)
        ex.all_gather()
        backend.set_marg(ex.gathered, ex.world, ex.maxlen, ex.rank_rows, s)
        backend.update(s)


def balance_sharded(backend, ex: Exchange, max_iters: int, check_every: int = 8):
    """Filters + ICE iterations until every group converged or max_iters.
    Returns ``backend.finalize()`` (identical on every rank)."""
    s = _stream()
    run_filters(backend, ex)
    done = 0
    while done < max_iters:
        k = min(check_every, max_iters - done)
        iterate(backend, ex, k)
        done += k
        if backend.active_groups(s) == 0:
            break
    return backend.finalize(s)


# ----------------------------------------------------------- C-ABI driver
# The same sharded ICE with the iteration loop in C++ (hh_ice_*_sharded):
# the exchange is a C function pointer, the library's RCCL all-gather
# (hh_comm_allgather over a communicator it owns) or, for CPU-side path checks
# (gloo), a Python callback.

def _cb_type():
    import ctypes as C
    return C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p)


class CapiExchange:
    """(function pointer, user) pair for hh_ice_*_sharded.

    ``backend="nccl"``: the library owns an RCCL communicator; rank 0 makes
    the ncclUniqueId and ``torch.distributed`` broadcasts it (any other means
    would do for a non-Python caller).  ``"gloo"``: a Python callback
    all-gathering through host memory (path checks with every rank on one
    GPU, where RCCL refuses duplicate devices)."""

    def __init__(self, rank_rows, world, rank, backend="nccl", group=None):
        import ctypes as C
        from . import _lib
        self.rank_rows = np.ascontiguousarray(rank_rows, dtype=np.int64)
        self.world, self.rank = int(world), int(rank)
        self._comm = None
        self._cb = None
        lib = _lib.load()
        if self.world == 1:
            self.fn, self.user = None, None
        elif backend == "nccl":
            import torch
            import torch.distributed as tdist
            # every rank reaches every collective below whatever fails, and
            # all ranks raise together (a caller can then fall back as one)
            uid = C.create_string_buffer(128)
            err = None
            if self.rank == 0:
                try:
                    _lib.call("hh_comm_unique_id", uid)
                except Exception as e:  # noqa: BLE001
                    err = e
            obj = [bytes(uid.raw) if self.rank == 0 and err is None else None]
            tdist.broadcast_object_list(obj, src=0, group=group)
            if obj[0] is None:
                raise RuntimeError(f"ncclGetUniqueId failed on rank 0: {err}")
            uid = C.create_string_buffer(obj[0], 128)
            h = C.c_void_p()
            try:
                _lib.call("hh_comm_init", uid, self.world, self.rank, C.byref(h))
                ok = 1
            except Exception as e:  # noqa: BLE001
                err, ok = e, 0
            flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
            tdist.all_reduce(flag, op=tdist.ReduceOp.MIN, group=group)
            if int(flag.item()) == 0:
                if ok:
                    _lib.call("hh_comm_free", h)
                raise RuntimeError(f"RCCL communicator init failed on a rank ({err})")
            self._comm = h
            self.fn = C.cast(lib.hh_comm_allgather, C.c_void_p)
            self.user = h
        else:
            self._cb = _python_allgather(self.world, group)
            self.fn = C.cast(self._cb, C.c_void_p)
            self.user = None

    def close(self):
        if self._comm is not None:
            from ._lib import call
            call("hh_comm_free", self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _python_allgather(world, group=None):
    """An hh_allgather_fn over torch.distributed's CPU path (gloo)."""
    import ctypes as C
    import torch
    import torch.distributed as tdist
    from ._lib import call

    def cb(send, count, recv, user, stream):
        try:
            st = C.c_void_p(stream) if stream else None
            buf = torch.empty(int(count), dtype=torch.float64, device="cuda")
            call("hh_device_copy", C.c_void_p(buf.data_ptr()), C.c_void_p(send), 8 * int(count), st)
            call("hh_synchronize", st)
            cpu = buf.cpu()
            parts = [torch.empty_like(cpu) for _ in range(world)]
            tdist.all_gather(parts, cpu, group=group)
            g = torch.cat(parts).cuda()
            torch.cuda.synchronize()
            call("hh_device_copy", C.c_void_p(recv), C.c_void_p(g.data_ptr()), 8 * int(count) * world, st)
            call("hh_synchronize", st)
            return 0
        except Exception:  # never raise through C
            return -2
    return _cb_type()(cb)


def _python_reduce_scatter(world, rank, group=None, on_device=False):
    """An hh_reduce_fn over torch.distributed: ``send`` holds ``world``
    blocks of ``count`` int64, ``recv`` gets the element-wise sum of every
    rank's block ``rank``.  ``on_device``: reduce_scatter_tensor on the
    device (nccl); otherwise an all_reduce through host memory (gloo)."""
    import ctypes as C
    import torch
    import torch.distributed as tdist
    from ._lib import call

    def cb(send, count, recv, user, stream):
        try:
            st = C.c_void_p(stream) if stream else None
            n = int(count)
            buf = torch.empty(world * n, dtype=torch.int64, device="cuda")
            call("hh_device_copy", C.c_void_p(buf.data_ptr()), C.c_void_p(send), 8 * world * n, st)
            call("hh_synchronize", st)
            if on_device:
                out = torch.empty(n, dtype=torch.int64, device="cuda")
                tdist.reduce_scatter_tensor(out, buf, group=group)
            else:
                cpu = buf.cpu()
                tdist.all_reduce(cpu, group=group)
                out = cpu[rank * n:(rank + 1) * n].cuda()
            torch.cuda.synchronize()
            call("hh_device_copy", C.c_void_p(recv), C.c_void_p(out.data_ptr()), 8 * n, st)
            call("hh_synchronize", st)
            return 0
        except Exception:  # never raise through C
            return -2
    return _cb_type()(cb)


def balance_capi(m, opts, ex: CapiExchange, stream=None):
    """Filters + ICE to convergence on this rank's shard, loop in C++
    (hh_ice_balance_sharded).  Returns (weights, stats), identical on every
    rank."""
    import ctypes as C
    from .ice import _stats
    from ._lib import call, ptr
    inf = m.info()
    G = inf["n_chroms"] if inf["cis_only"] else 1
    w = np.empty(inf["n_bins"], np.float64)
    scale, var = np.empty(G), np.empty(G)
    iters, conv = np.empty(G, np.int32), np.empty(G, np.int32)
    secs = C.c_double(0)
    call("hh_ice_balance_sharded", m.handle, C.byref(opts.c_opts()), ex.world, ex.rank, ptr(ex.rank_rows),
         ex.fn, ex.user, ptr(w), ptr(scale), ptr(var), ptr(iters), ptr(conv), C.byref(secs), stream)
    st = _stats(opts, scale, var, iters, conv, inf["cis_only"])
    st["sweep_seconds"] = secs.value
    return w, st


def filters_capi(st, ex: CapiExchange, stream=None):
    from ._lib import call, ptr
    call("hh_ice_filters_sharded", st._h, ex.world, ptr(ex.rank_rows), ex.fn, ex.user, stream)


def iterate_capi(st, ex: CapiExchange, n: int, stream=None):
    """``n`` ICE iterations enqueued from C++ (one call, no host polling)."""
    from ._lib import call, ptr
    call("hh_ice_run_sharded", st._h, ex.world, ptr(ex.rank_rows), ex.fn, ex.user, int(n), stream)


# ------------------------------------------- --cis-only, chromosomes by LPT
# `cooler balance --cis-only` (matrixBuilding.py:713,
# :1542, :1766) needs no collective in its iterations: every chromosome is
# its own ICE group, so whole chromosomes are dealt to ranks (LPT on their
# cis pixels) and each rank balances a compact matrix of its own
# chromosomes.  The one exchange is cooler's genome-wide MAD cutoff over the
# per-chromosome-normalised raw marginals (hh_ice_balance_cis_local); the
# weights are gathered once at the end.

def cis_plan(bin1, bin2, chrom_offsets, world: int):
    """``(owner[chrom], cis pixels per chrom)``: LPT on cis pixels."""
    off = np.asarray(chrom_offsets, dtype=np.int64)
    nc = off.size - 1
    c1 = np.searchsorted(off, np.asarray(bin1), side="right") - 1
    c2 = np.searchsorted(off, np.asarray(bin2), side="right") - 1
    cost = np.bincount(c1[c1 == c2], minlength=nc).astype(np.float64)
    return lpt_assign(cost, world), cost


def local_genome(bin1, bin2, count, chrom_offsets, chroms):
    """The cis pixels of ``chroms`` (ascending chromosome indices) renumbered
    into a compact genome: ``(b1, b2, count, local_offsets)``."""
    off = np.asarray(chrom_offsets, dtype=np.int64)
    chroms = np.asarray(sorted(chroms), dtype=np.int64)
    sizes = np.diff(off)[chroms]
    loff = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    shift = np.zeros(off.size - 1, dtype=np.int64)
    shift[chroms] = loff[:-1] - off[chroms]
    keep = np.zeros(off.size - 1, dtype=bool)
    keep[chroms] = True
    b1 = np.asarray(bin1, dtype=np.int64)
    b2 = np.asarray(bin2, dtype=np.int64)
    c1 = np.searchsorted(off, b1, side="right") - 1
    c2 = np.searchsorted(off, b2, side="right") - 1
    sel = (c1 == c2) & keep[np.clip(c1, 0, off.size - 2)]
    sh = shift[c1[sel]]
    return b1[sel] + sh, b2[sel] + sh, np.asarray(count)[sel], loff


def balance_cis_capi(m_local, opts, ex: CapiExchange, max_local_bins: int, stream=None):
    """hh_ice_balance_cis_local on this rank's compact matrix: ``(weights of
    the local bins, per-local-chromosome scale, var, iters, converged,
    sweep seconds)``."""
    import ctypes as C
    from ._lib import call, ptr
    inf = m_local.info()
    G = inf["n_chroms"]
    w = np.empty(inf["n_bins"], np.float64)
    scale, var = np.empty(G), np.empty(G)
    iters, conv = np.empty(G, np.int32), np.empty(G, np.int32)
    secs = C.c_double(0)
    call("hh_ice_balance_cis_local", m_local.handle, C.byref(opts.c_opts()), ex.world, int(max_local_bins),
         ex.fn, ex.user, ptr(w), ptr(scale), ptr(var), ptr(iters), ptr(conv), C.byref(secs), stream)
    return w, scale, var, iters, conv, secs.value


def balance_cis_sharded(bin1, bin2, count, n_bins, chrom_offsets, rank: int, world: int, opts, ex: CapiExchange,
                        group=None, stream=None):
    """`cooler balance --cis-only` over ``world`` ranks, chromosomes by LPT,
    no collective in the iterations.  Returns ``(weights, stats)`` for the
    whole genome on every rank (as ``ice.balance`` with ``cis_only=True``)."""
    from .ice import ContactMatrix, _stats
    off = np.asarray(chrom_offsets, dtype=np.int64)
    owner, _ = cis_plan(bin1, bin2, off, world)
    sizes = np.diff(off)
    max_local = max(int(sizes[owner == r].sum()) for r in range(world))
    mine = np.flatnonzero(owner == rank)
    loc = None
    if mine.size:
        b1, b2, c, loff = local_genome(bin1, bin2, count, off, mine)
        m = ContactMatrix.from_pixels(b1, b2, c, int(loff[-1]), loff, opts.ignore_diags, True, stream=stream)
        try:
            loc = balance_cis_capi(m, opts, ex, max_local, stream)
        finally:
            m.close()
    elif world > 1:  # a rank without chromosomes still joins the MAD exchange
        b1, b2, c, loff = np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0), np.array([0, 1])
        m = ContactMatrix.from_pixels(b1, b2, c, 1, loff, opts.ignore_diags, True, stream=stream)
        try:
            balance_cis_capi(m, opts, ex, max_local, stream)
        finally:
            m.close()
    parts = [(mine, loc)]
    if world > 1:
        import torch.distributed as tdist
        parts = [None] * world
        tdist.all_gather_object(parts, (mine, loc), group=group)
    nc = off.size - 1
    w = np.full(int(n_bins), np.nan)
    scale, var = np.full(nc, np.nan), np.full(nc, np.nan)
    iters, conv = np.zeros(nc, np.int32), np.zeros(nc, np.int32)
    secs = 0.0
    for chroms, res in parts:
        if res is None:
            continue
        wl, sc, vr, it, cv, t = res
        p = 0
        for k, ch in enumerate(chroms):
            n = int(sizes[ch])
            w[off[ch]:off[ch] + n] = wl[p:p + n]
            p += n
            scale[ch], var[ch], iters[ch], conv[ch] = sc[k], vr[k], it[k], cv[k]
        secs = max(secs, t)
    st = _stats(opts, scale, var, iters, conv, True)
    st["sweep_seconds"] = secs
    return w, st
