"""Row shards of one matrix balanced in one process on one GPU (the sharded
driver's exchanges without a process group): the marginal all-gather by hand,
and the column side of upper-triangle tiles through an
hh_reduce_fn served by one thread per shard (test infrastructure)."""
import ctypes as C
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np


class ThreadReduce:
    """hh_reduce_fn between the shard states of this process: every caller
    (user = its rank) deposits its ``world`` padded int64 blocks, then sums
    block ``rank`` over the ranks (integers: exact in any order)."""

    def __init__(self, world):
        from hichap_master_amd import dist
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.cb = dist._cb_type()(self._cb)
        self.fn = C.cast(self.cb, C.c_void_p)

    def _cb(self, send, count, recv, user, stream):
        import torch
        from hichap_master_amd._lib import call
        try:
            rank, n, st = int(user or 0), int(count), C.c_void_p(stream) if stream else None
            buf = torch.empty(self.world * n, dtype=torch.int64, device="cuda")
            call("hh_device_copy", C.c_void_p(buf.data_ptr()), C.c_void_p(send), 8 * self.world * n, st)
            call("hh_synchronize", st)
            self.slots[rank] = buf
            self.bar.wait()
            out = sum(self.slots[k][rank * n:(rank + 1) * n] for k in range(self.world))
            torch.cuda.synchronize()
            call("hh_device_copy", C.c_void_p(recv), C.c_void_p(out.data_ptr()), 8 * n, st)
            call("hh_synchronize", st)
            self.bar.wait()
            return 0
        except Exception:  # noqa: BLE001  (never raise through C)
            self.bar.abort()
            return -2


def balance_states(states, rr, max_iters):
    """Filters + ICE over the shard states (``states[k]`` holds rows
    ``rr[k] .. rr[k + 1]``); returns every state's ``finalize()``."""
    import torch
    from hichap_master_amd._lib import call, ptr
    W = len(rr) - 1
    maxlen = int(np.max(np.diff(rr)))
    loc = [torch.zeros(maxlen, dtype=torch.float64, device="cuda") for _ in range(W)]
    gat = torch.zeros(W * maxlen, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    red = ThreadReduce(W)
    rr64 = np.ascontiguousarray(rr, dtype=np.int64)
    for k in range(W):
        call("hh_ice_set_column_exchange", states[k]._h, W, k, ptr(rr64), red.fn, C.c_void_p(k), None, None)
    with ThreadPoolExecutor(W) as pool:
        def exchange(mode):
            if mode == 2 and W > 1:  # the column exchange blocks until every shard's sweep is in
                for f in [pool.submit(states[k].marg_local, mode, loc[k], s) for k in range(W)]:
                    f.result()
            else:
                for k in range(W):
                    states[k].marg_local(mode, loc[k], s)
            for k in range(W):
                gat[k * maxlen:(k + 1) * maxlen].copy_(loc[k])
            for k in range(W):
                states[k].set_marg(gat, W, maxlen, rr, s)
        exchange(0)
        for st_ in states:
            st_.filter_nnz(s)
        exchange(1)
        for st_ in states:
            st_.filter_count_mad(s)
        for it in range(max_iters):
            exchange(2)
            for st_ in states:
                st_.update(s)
            if it % 8 == 7 and states[0].active_groups(s) == 0:
                break
        return [st_.finalize(s) for st_ in states]


def require_uptiles():
    """Skip unless the loaded library has upper-triangle tiles (the 4096-column
    build, libhichap_hip_up.so; tests/test_uptiles_variant_gpu.py runs these
    cases against it in a child process)."""
    import pytest
    from hichap_master_amd._lib import HipLibraryError, call
    try:
        call("hh_tune", b"upper_tiles", 1)
    except HipLibraryError:
        pytest.skip("upper-triangle tiles: 4096-column build only (run by test_uptiles_variant_gpu.py)")
    finally:
        call("hh_tune", b"upper_tiles", -1)
