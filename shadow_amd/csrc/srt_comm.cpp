// srt_comm.cpp -- communicator for the row-sharded multi-GPU routing build.
//
// The reference has no collective at all: compute_shortest_paths fans sources
// out over a rayon pool inside one process (src/main/network/graph/mod.rs:190-208).
// Here source rows are sharded over the GPUs of one node (one process per GPU)
// and the two real exchange steps of the blocked closure go over xGMI:
//   - per round: broadcast of the pivot block-row from its owner;
//   - at the end: in-place all-gather of the path-key rows.
// Transport: RCCL (native, on the plan's stream) or host callbacks.
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <new>

#include "srt_internal.h"

namespace {
void set_err(srt_err *err, int code, const char *msg) {
    if (!err) return;
    std::memset(err, 0, sizeof *err);
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}
}  // namespace

namespace srt {

srt_status comm_bcast(srt_comm *c, void *buf, size_t bytes, int root, hipStream_t s, srt_err *err) {
    if (c->nccl) {
        ncclResult_t r = ncclBroadcast(buf, buf, bytes, ncclUint8, root, (ncclComm_t)c->nccl, s);
        if (r != ncclSuccess) {
            char m[200];
            std::snprintf(m, sizeof m, "ncclBroadcast: %s", ncclGetErrorString(r));
            set_err(err, SRT_ERR_COMM, m);
            return SRT_ERR_COMM;
        }
        return SRT_OK;
    }
    if (hipStreamSynchronize(s) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "hipStreamSynchronize before bcast callback");
        return SRT_ERR_HIP;
    }
    if (c->bcast(c->user, buf, bytes, root) != 0) {
        set_err(err, SRT_ERR_COMM, "bcast callback failed");
        return SRT_ERR_COMM;
    }
    return SRT_OK;
}

srt_status comm_allgather_inplace(srt_comm *c, void *buf, size_t bytes_per_rank, hipStream_t s,
                                  srt_err *err) {
    if (c->nccl) {
        char *base = (char *)buf;
        ncclResult_t r = ncclAllGather(base + (size_t)c->rank * bytes_per_rank, base, bytes_per_rank,
                                       ncclUint8, (ncclComm_t)c->nccl, s);
        if (r != ncclSuccess) {
            char m[200];
            std::snprintf(m, sizeof m, "ncclAllGather: %s", ncclGetErrorString(r));
            set_err(err, SRT_ERR_COMM, m);
            return SRT_ERR_COMM;
        }
        return SRT_OK;
    }
    if (hipStreamSynchronize(s) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "hipStreamSynchronize before allgather callback");
        return SRT_ERR_HIP;
    }
    if (c->allgather(c->user, buf, bytes_per_rank) != 0) {
        set_err(err, SRT_ERR_COMM, "allgather callback failed");
        return SRT_ERR_COMM;
    }
    return SRT_OK;
}

}  // namespace srt

extern "C" {

srt_status srt_comm_unique_id(uint8_t out[128], srt_err *err) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    if (!out) {
        set_err(err, SRT_ERR_INVALID, "null out");
        return SRT_ERR_INVALID;
    }
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_err(err, SRT_ERR_COMM, ncclGetErrorString(r));
        return SRT_ERR_COMM;
    }
    std::memcpy(out, &id, sizeof id);
    if (err) std::memset(err, 0, sizeof *err);
    return SRT_OK;
}

srt_status srt_comm_init(const uint8_t id[128], int nranks, int rank, int device, srt_comm **comm,
                         srt_err *err) {
    if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(err, SRT_ERR_INVALID, "bad communicator arguments");
        return SRT_ERR_INVALID;
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "hipSetDevice failed");
        return SRT_ERR_HIP;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRank(&c, nranks, uid, rank);
    if (r != ncclSuccess) {
        char m[200];
        std::snprintf(m, sizeof m, "ncclCommInitRank: %s", ncclGetErrorString(r));
        set_err(err, SRT_ERR_COMM, m);
        return SRT_ERR_COMM;
    }
    srt_comm *sc = new (std::nothrow) srt_comm();
    if (!sc) {
        ncclCommDestroy(c);
        set_err(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    sc->nranks = nranks;
    sc->rank = rank;
    sc->nccl = c;
    *comm = sc;
    if (err) std::memset(err, 0, sizeof *err);
    return SRT_OK;
}

srt_status srt_comm_init_callbacks(int nranks, int rank, srt_bcast_fn bcast,
                                   srt_allgather_fn allgather, void *user, srt_comm **comm,
                                   srt_err *err) {
    if (!comm || !bcast || !allgather || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(err, SRT_ERR_INVALID, "bad communicator arguments");
        return SRT_ERR_INVALID;
    }
    srt_comm *sc = new (std::nothrow) srt_comm();
    if (!sc) {
        set_err(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    sc->nranks = nranks;
    sc->rank = rank;
    sc->bcast = bcast;
    sc->allgather = allgather;
    sc->user = user;
    *comm = sc;
    if (err) std::memset(err, 0, sizeof *err);
    return SRT_OK;
}

void srt_comm_destroy(srt_comm *comm) {
    if (!comm) return;
    if (comm->nccl) ncclCommDestroy((ncclComm_t)comm->nccl);
    delete comm;
}

}  // extern "C"
