// comm_abi.hip — gnsship_comm_*: the multi-GPU fan-out of the C ABI (include/gnsship.h) on RCCL.
//
// GNSS-SDR feeds every channel from the same signal-conditioner output (gnss_flowgraph.cc:
// 1127-1136, one connect() per channel).  With channels sharded over GPUs — one process per GPU —
// that connection becomes one RCCL broadcast of the raw IF block over xGMI from the rank that reads
// the front end; afterwards each rank tracks its channel shard (or searches its PRN shard) on its
// own, and only the small per-PRN acquisition results travel back (all-gather).  Collectives run on
// the context's stream, so they are ordered against the engine's own launches without a host wait.
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <new>

#include "engine.h"

struct gnsship_comm {
    gnsship_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, n_ranks = 1;
};

namespace {

int rccl_fail(gnsship_ctx* ctx, ncclResult_t r, const char* where)
{
    if (ctx) {
        char buf[256];
        std::snprintf(buf, sizeof(buf), "%s: %s", where, ncclGetErrorString(r));
        ctx->last_error = buf;
    }
    return GNSSHIP_E_RCCL;
}

int select_device(gnsship_ctx* ctx)
{
    const hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) {
        ctx->last_error = std::string("hipSetDevice: ") + hipGetErrorString(e);
        return GNSSHIP_E_DEVICE;
    }
    return GNSSHIP_OK;
}

}  // namespace

#define RCCL_TRY(ctx, expr)                                        \
    do {                                                           \
        ncclResult_t _r = (expr);                                  \
        if (_r != ncclSuccess) return rccl_fail((ctx), _r, #expr); \
    } while (0)

extern "C" int gnsship_comm_unique_id(void* id)
{
    if (!id) return GNSSHIP_E_INVAL;
    static_assert(sizeof(ncclUniqueId) == GNSSHIP_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GNSSHIP_E_RCCL;
    std::memcpy(id, &u, sizeof(u));
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_create(gnsship_ctx* ctx, int n_ranks, int rank, const void* id, gnsship_comm** out)
{
    if (!ctx || !id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return GNSSHIP_E_INVAL;
    *out = nullptr;
    if (const int rc = select_device(ctx)) return rc;
    auto* c = new (std::nothrow) gnsship_comm;
    if (!c) return GNSSHIP_E_NOMEM;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return rccl_fail(ctx, r, "ncclCommInitRank");
    }
    c->ctx = ctx;
    c->rank = rank;
    c->n_ranks = n_ranks;
    *out = c;
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_rank(gnsship_comm* c, int* rank, int* n_ranks)
{
    if (!c) return GNSSHIP_E_INVAL;
    if (rank) *rank = c->rank;
    if (n_ranks) *n_ranks = c->n_ranks;
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_broadcast(gnsship_comm* c, void* dev_buf, size_t bytes, int root)
{
    if (!c || (!dev_buf && bytes) || root < 0 || root >= c->n_ranks) return GNSSHIP_E_INVAL;
    if (!bytes) return GNSSHIP_OK;
    if (const int rc = select_device(c->ctx)) return rc;
    RCCL_TRY(c->ctx, ncclBroadcast(dev_buf, dev_buf, bytes, ncclUint8, root, c->comm, c->ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_allgather(gnsship_comm* c, const void* dev_send, void* dev_recv, size_t bytes_per_rank)
{
    if (!c || ((!dev_send || !dev_recv) && bytes_per_rank)) return GNSSHIP_E_INVAL;
    if (!bytes_per_rank) return GNSSHIP_OK;
    if (const int rc = select_device(c->ctx)) return rc;
    RCCL_TRY(c->ctx, ncclAllGather(dev_send, dev_recv, bytes_per_rank, ncclUint8, c->comm, c->ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_allreduce_max_f64(gnsship_comm* c, double* dev_buf, size_t count)
{
    if (!c || (!dev_buf && count)) return GNSSHIP_E_INVAL;
    if (!count) return GNSSHIP_OK;
    if (const int rc = select_device(c->ctx)) return rc;
    RCCL_TRY(c->ctx, ncclAllReduce(dev_buf, dev_buf, count, ncclFloat64, ncclMax, c->comm, c->ctx->stream));
    return GNSSHIP_OK;
}

extern "C" int gnsship_comm_destroy(gnsship_comm* c)
{
    if (!c) return GNSSHIP_E_INVAL;
    int rc = GNSSHIP_OK;
    if (c->comm) {
        select_device(c->ctx);
        (void)hipStreamSynchronize(c->ctx->stream);
        if (ncclCommDestroy(c->comm) != ncclSuccess) rc = GNSSHIP_E_RCCL;
    }
    delete c;
    return rc;
}
