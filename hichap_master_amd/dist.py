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
