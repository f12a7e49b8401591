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

}  // extern "C"

namespace {

struct Sharded {
    hh_ice* S;
    int world;
    std::vector<int64_t> rr;
    int64_t maxlen;
    hh_allgather_fn ag;
    void* user;
    hh::DBuf<double> local, gathered;
    void* stream;
    void exchange(int mode) {
        auto ok = [](int r) { if (r) throw hh::Error(r, hh_last_error()); };
        ok(hh_ice_marg_local(S, mode, local.p, stream));
        if (world == 1) {
            HIP_CHECK(hipMemcpyAsync(gathered.p, local.p, sizeof(double) * maxlen, hipMemcpyDeviceToDevice,
                                     hh::as_stream(stream)));
        } else {
            const int rc = ag(local.p, maxlen, gathered.p, user, stream);
            if (rc) HH_THROW(rc < 0 ? rc : HH_ERR_HIP, std::string("all-gather callback failed: ") + hh_last_error());
        }
        ok(hh_ice_set_marg(S, gathered.p, world, maxlen, rr.data(), stream));
    }
};

Sharded make_sharded(hh_ice* S, int32_t world, const int64_t* rank_rows, hh_allgather_fn ag, void* user, void* stream) {
    HH_REQUIRE(S && world >= 1 && rank_rows, "bad arguments");
    HH_REQUIRE(world == 1 || ag, "an all-gather function is required for world > 1");
    Sharded X{S, world, std::vector<int64_t>(rank_rows, rank_rows + world + 1), 1, ag, user, {}, {}, stream};
    for (int r = 0; r < world; ++r) {
        HH_REQUIRE(X.rr[r] <= X.rr[r + 1], "rank_rows not monotone");
        X.maxlen = std::max<int64_t>(X.maxlen, X.rr[r + 1] - X.rr[r]);
    }
    X.local.alloc(X.maxlen);
    X.local.zero(hh::as_stream(stream));
    X.gathered.alloc((size_t)world * X.maxlen);
    return X;
}

}  // namespace

extern "C" {

int hh_ice_filters_sharded(hh_ice* S, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                           void* stream) {
    return guard([&] {
        Sharded X = make_sharded(S, world, rank_rows, allgather, user, stream);
        auto ok = [](int r) { if (r) throw hh::Error(r, hh_last_error()); };
        X.exchange(0);
        ok(hh_ice_filter_nnz(S, stream));
        X.exchange(1);
        ok(hh_ice_filter_count_mad(S, stream));
        HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream)));
    });
}

int hh_ice_run_sharded(hh_ice* S, int32_t world, const int64_t* rank_rows, hh_allgather_fn allgather, void* user,
                       int32_t n, void* stream) {
    return guard([&] {
        HH_REQUIRE(n >= 0, "bad arguments");
        Sharded X = make_sharded(S, world, rank_rows, allgather, user, stream);
        auto ok = [](int r) { if (r) throw hh::Error(r, hh_last_error()); };
        for (int k = 0; k < n; ++k) {
            X.exchange(2);
            ok(hh_ice_update(S, stream));
        }
        HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream)));  // buffers return to the pool
    });
}

int hh_ice_balance_sharded(hh_matrix* m, const hh_ice_opts* o, int32_t world, int32_t rank, const int64_t* rank_rows,
                           hh_allgather_fn allgather, void* user, double* weights, double* scale, double* var,
                           int32_t* iters, int32_t* converged, double* sweep_seconds, void* stream) {
    hh_ice* S = nullptr;
    int rc = hh_ice_create(m, o, &S);
    if (rc) return rc;
    rc = guard([&] {
        HH_REQUIRE(rank_rows && 0 <= rank && rank < world, "bad arguments");
        hh_matrix_info inf{};
        auto ok = [](int r) { if (r) throw hh::Error(r, hh_last_error()); };
        ok(hh_matrix_get_info(m, &inf));
        HH_REQUIRE(inf.row_lo == rank_rows[rank] && inf.row_hi == rank_rows[rank + 1],
                   "the matrix shard does not hold rank_rows[rank] .. rank_rows[rank + 1]");
        Sharded X = make_sharded(S, world, rank_rows, allgather, user, stream);
        X.exchange(0);
        ok(hh_ice_filter_nnz(S, stream));
        X.exchange(1);
        ok(hh_ice_filter_count_mad(S, stream));
        HIP_CHECK(hipStreamSynchronize(hh::as_stream(stream)));
        const auto t0 = std::chrono::steady_clock::now();
        int32_t done = 0;
        while (done < o->max_iters) {
            const int k = std::min(o->check_every > 0 ? o->check_every : 8, o->max_iters - done);
            for (int j = 0; j < k; ++j) {
                X.exchange(2);
                ok(hh_ice_update(S, stream));
            }
            done += k;
            int32_t na = 0;
            ok(hh_ice_active_groups(S, &na, stream));
            if (na == 0) break;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (sweep_seconds) *sweep_seconds = std::chrono::duration<double>(t1 - t0).count();
        ok(hh_ice_finalize(S, weights, scale, var, iters, converged, stream));
    });
    hh_ice_free(S);
    return rc;
}

}  // extern "C"
