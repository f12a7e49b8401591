// Sharded genome-wide ICE driven from C++: one process
// per GPU, each holding whole 512-row blocks of the matrix; per iteration one
// all-gather of the local marginals (n_bins x 8 B in total), then the
// identical variance / bias update on every rank.  The exchange is a
// function pointer, so any transport fits; the library provides RCCL's
// (hh_comm_*: a communicator it owns, ncclUniqueId passed in by the caller,
// ncclAllGather on the library's stream over xGMI).  No Python in the loop:
// the iteration is enqueued back to back and the host polls convergence every
// check_every iterations, as hh_ice_balance does on one GPU.
//
// Replaces the per-process `cooler balance` subprocess of matrixBuilding.py:708
// for whole-genome matrices sharded across the GPUs of a node.
#include <chrono>
#include <cstring>

#include <rccl/rccl.h>

#include "ice_internal.hpp"

using namespace hh;

struct hh_comm {
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0, device = 0;
};

namespace {
void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) HH_THROW(HH_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
}  // namespace

extern "C" {

int hh_comm_unique_id(uint8_t* id) {
    return guard([&] {
        HH_REQUIRE(id, "null");
        ncclUniqueId u;
        nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof(u));
    });
}

int hh_comm_init(const uint8_t* id, int32_t world, int32_t rank, hh_comm** out) {
    return guard([&] {
        HH_REQUIRE(id && out && world >= 1 && 0 <= rank && rank < world, "bad arguments");
        auto c = std::make_unique<hh_comm>();
        HIP_CHECK(hipGetDevice(&c->device));
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        nccl_check(ncclCommInitRank(&c->comm, world, u, rank), "ncclCommInitRank");
        c->world = world;
        c->rank = rank;
        *out = c.release();
    });
}

int hh_comm_free(hh_comm* c) {
    return guard([&] {
        if (c && c->comm) (void)ncclCommDestroy(c->comm);
        delete c;
    });
}

int hh_comm_allgather(const double* send, int64_t count, double* recv, void* comm, void* stream) {
    return guard([&] {
        auto* c = static_cast<hh_comm*>(comm);
        HH_REQUIRE(c && c->comm && count >= 0, "bad arguments");
        nccl_check(ncclAllGather(send, recv, (size_t)count, ncclFloat64, c->comm, as_stream(stream)), "ncclAllGather");
    });
}

int hh_comm_reduce_scatter(const int64_t* send, int64_t count, int64_t* recv, void* comm, void* stream) {
    return guard([&] {
        auto* c = static_cast<hh_comm*>(comm);
        HH_REQUIRE(c && c->comm && count >= 0, "bad arguments");
        nccl_check(ncclReduceScatter(send, recv, (size_t)count, ncclInt64, ncclSum, c->comm, as_stream(stream)),
                   "ncclReduceScatter");
    });
}

}  // extern "C"

namespace {

// A sharded run keeps every rank in step even when one rank fails: a rank
// whose local step throws remembers the error, skips its remaining local
// work, but keeps calling the all-gather the others are waiting in; at each
// agreement point (after setup, after the filters, every check_every
// iterations, at the end) one double per rank says whether it is still good,
// and every rank then raises together -- the failing one with its own error,
// the others naming it -- instead of the peers hanging in the exchange (ADVICE
// r2).  A failure of the all-gather itself is not recoverable here.
struct Sharded {
    hh_ice* S = nullptr;
    int world = 1;
    std::vector<int64_t> rr;
    int64_t maxlen = 1;
    hh_allgather_fn ag = nullptr;
    void* user = nullptr;
    hh::DBuf<double> local, gathered, sb, gb;
    void* stream = nullptr;
    int err_rc = 0;
    std::string err;
    bool failed() const { return err_rc != 0; }
    template <class F>
    void attempt(F&& f) {  // a local step: an exception marks this rank failed
        if (failed()) return;
        try {
            f();
        } catch (const hh::Error& e) {
            err_rc = e.code;
            err = e.what();
        } catch (const std::bad_alloc&) {
            err_rc = HH_ERR_OOM;
            err = "out of host memory";
        } catch (const std::exception& e) {
            err_rc = HH_ERR_STATE;
            err = e.what();
        }
    }
    void gather(const double* send, int64_t count, double* recv) {
        const int rc = ag(const_cast<double*>(send), count, recv, user, stream);
        if (rc) HH_THROW(rc < 0 ? rc : HH_ERR_HIP, std::string("all-gather callback failed: ") + hh_last_error());
    }
    static void ok(int r) {
        if (r) throw hh::Error(r, hh_last_error());
    }
    void exchange(int mode) {
        attempt([&] { ok(hh_ice_marg_local(S, mode, local.p, stream)); });
        if (world == 1) {
            attempt([&] {
                HIP_CHECK(hipMemcpyAsync(gathered.p, local.p, sizeof(double) * maxlen, hipMemcpyDeviceToDevice,
                                         hh::as_stream(stream)));
            });
        } else {
            gather(local.p, maxlen, gathered.p);  // always: the peers are in it
        }
        attempt([&] { ok(hh_ice_set_marg(S, gathered.p, world, maxlen, rr.data(), stream)); });
    }
    // every rank: raise if any rank has failed
    void agree() {
        int bad = failed() ? 0 : -1;
        if (world > 1) {
            const double v = failed() ? 0.0 : 1.0;
            std::vector<double> h(world, 0.0);
            HIP_CHECK(hipMemcpyAsync(sb.p, &v, sizeof(double), hipMemcpyHostToDevice, hh::as_stream(stream)));
            gather(sb.p, 1, gb.p);
            HIP_CHECK(hipMemcpyAsync(h.data(), gb.p, sizeof(double) * world, hipMemcpyDeviceToHost,
                                     hh::as_stream(stream)));
            HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream)));
            for (int r = world - 1; r >= 0; --r)
                if (h[r] != 1.0) bad = r;
        }
        if (bad < 0) return;
        if (failed()) throw hh::Error(err_rc, err);
        HH_THROW(HH_ERR_STATE, "rank " + std::to_string(bad) + " of " + std::to_string(world) +
                                   " failed; the sharded run stopped on every rank");
    }
    // the exchange buffers (a failure here is agreed on like any other)
    void setup(hh_ice* S_, const int64_t* rank_rows) {
        S = S_;
        attempt([&] {
            HH_REQUIRE(S && rank_rows, "bad arguments");
            rr.assign(rank_rows, rank_rows + world + 1);
            for (int r = 0; r < world; ++r) {
                HH_REQUIRE(rr[r] <= rr[r + 1], "rank_rows not monotone");
                maxlen = std::max<int64_t>(maxlen, rr[r + 1] - rr[r]);
            }
            local.alloc(maxlen);
            local.zero(hh::as_stream(stream));
            gathered.alloc((size_t)world * maxlen);
            // the column side of upper-triangle tiles: RCCL's reduce-scatter
            // when the exchange is the library's own, else through `ag`
            const bool rccl = ag == hh_comm_allgather;
            ok(hh_ice_set_column_exchange(S, world, -1, rr.data(), rccl ? hh_comm_reduce_scatter : nullptr,
                                          rccl ? user : nullptr, ag, user));
        });
    }
    void filters() {
        exchange(0);
        attempt([&] { ok(hh_ice_filter_nnz(S, stream)); });
        exchange(1);
        attempt([&] { ok(hh_ice_filter_count_mad(S, stream)); });
        attempt([&] { HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream))); });
    }
    void iterate(int n) {
        for (int k = 0; k < n; ++k) {
            exchange(2);
            attempt([&] { ok(hh_ice_update(S, stream)); });
        }
    }
};

// world, the exchange and the two status buffers; an error here is
// identical on every rank (the arguments of the call), so it is not agreed
Sharded make_sharded(int32_t world, hh_allgather_fn ag, void* user, void* stream) {
    HH_REQUIRE(world >= 1, "bad arguments");
    HH_REQUIRE(world == 1 || ag, "an all-gather function is required for world > 1");
    Sharded X;
    X.world = world;
    X.ag = ag;
    X.user = user;
    X.stream = stream;
    X.sb.alloc(1);
    X.gb.alloc((size_t)world);
    return X;
}

}  // namespace

extern "C" {

int hh_ice_filters_sharded(hh_ice* S, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                           void* stream) {
    return guard([&] {
        Sharded X = make_sharded(world, allgather, user, stream);
        X.setup(S, rank_rows);
        X.agree();
        X.filters();
        X.agree();
    });
}

int hh_ice_run_sharded(hh_ice* S, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                       int32_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(n >= 0, "bad arguments");
        Sharded X = make_sharded(world, allgather, user, stream);
        X.setup(S, rank_rows);
        X.agree();
        X.iterate(n);
        X.attempt([&] { HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream))); });  // buffers return to the pool
        X.agree();
    });
}

int hh_ice_balance_sharded(hh_matrix* m, const hh_ice_opts* o, int32_t world, int32_t rank, const int64_t* rank_rows,
                           hh_allgather_fn allgather, void* user, double* weights, double* scale, double* var,
                           int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream) {
    hh_ice* S = nullptr;
    const int rc = guard([&] {
        HH_REQUIRE(o && 0 <= rank && rank < world, "bad arguments");
        Sharded X = make_sharded(world, allgather, user, stream);
        X.attempt([&] {
            Sharded::ok(hh_ice_create(m, o, &S));
            hh_matrix_info inf{};
            Sharded::ok(hh_matrix_get_info(m, &inf));
            HH_REQUIRE(rank_rows && inf.row_lo == rank_rows[rank] && inf.row_hi == rank_rows[rank + 1],
                       "the matrix shard does not hold rank_rows[rank] .. rank_rows[rank + 1]");
        });
        if (!X.failed()) X.setup(S, rank_rows);
        X.agree();
        X.filters();
        X.agree();
        const auto t0 = std::chrono::steady_clock::now();
        int32_t done = 0;
        while (done < o->max_iters) {
            const int k = std::min(o->check_every > 0 ? o->check_every : 8, o->max_iters - done);
            X.iterate(k);
            done += k;
            int32_t na = 0;
            X.attempt([&] { Sharded::ok(hh_ice_active_groups(S, &na, stream)); });
            X.agree();  // na is then the same on every rank (from gathered data)
            if (na == 0) break;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (sweep_seconds) *sweep_seconds = std::chrono::duration<double>(t1 - t0).count();
        Sharded::ok(hh_ice_finalize(S, weights, scale, var, iters, converged, stream));  // local: no peer waits
    });
    if (S) hh_ice_free(S);
    return rc;
}

}  // extern "C"
