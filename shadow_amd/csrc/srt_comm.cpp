// srt_comm.cpp -- communicator for the row-sharded multi-GPU routing build.
//
// The reference has no collective at all: compute_shortest_paths fans sources
// out over a rayon pool inside one process (src/main/network/graph/mod.rs:190-208).
// Here source rows are sharded over the GPUs of one node and the exchange
// steps of the blocked closure go over xGMI (pivot-row broadcasts, row / tile
// all-gathers).  Transports: RCCL (one process per GPU, on the plan's stream),
// in-process (one host thread per GPU of one process: the way Shadow's single
// process reaches every GPU, srt_opts.n_gpus), or host callbacks (any
// host-side collective, e.g. torch.distributed/gloo in tests).
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

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

// In-process transport (srt_comm_init_local): the N ranks are N host threads
// of one process, one per device (or several on one device, for tests).  A
// collective is stream-ordered like RCCL's, with no host synchronisation of
// the device:
//   1. every rank records `ready` on its stream and publishes its buffer;
//   2. host barrier (every rank has enqueued its record and published);
//   3. each rank's stream waits for the other ranks' `ready` events and one
//      kernel (srt_peer.hip) reads their slots straight out of their buffers
//      (xGMI peer reads; peer access enabled at init);
//   4. every rank records `done`; host barrier; each stream waits for every
//      `done`, so no rank overwrites its slot while another still reads it.
// A failed rank aborts the group: the others' barriers return an error
// instead of waiting for it.
struct LocalGroup {
    int n = 0;
    std::vector<int> dev;
    std::vector<hipEvent_t> ready, done;
    // integrity: every collective's contributions are checksummed by their
    // senders (sums[r], on rank r's device) before `ready`, and every receiver
    // checksums what it received (tmp[r][q]) and compares with the sender's
    // word over xGMI; a mismatch sets bad[r] (on rank r's device), which
    // srt_plan_sync / the in-process builds report as SRT_ERR_COMM
    std::vector<unsigned long long *> sums, tmp;
    std::vector<uint32_t *> bad;
    int corrupt_rank = -1;  // test knob SRT_TEST_CORRUPT_PEER = rank: flips a received byte
    std::vector<const uint8_t *> ptr;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0, refs = 0;
    uint64_t gen = 0;
    bool aborted = false;

    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != g || aborted; });
        return !aborted;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

namespace {
// one in-process collective: rank c->rank contributes `own` (published as the
// base of its buffer) and gathers into dst; root >= 0: a broadcast from root
srt_status local_collective(srt_comm *c, uint8_t *buf, uint64_t bytes, int root, hipStream_t s, srt_err *err) {
    LocalGroup *G = c->local;
    const int r = c->rank, N = G->n;
    if (root < 0 || root == r) checksum(root < 0 ? buf + (uint64_t)r * bytes : buf, bytes, G->sums[r], s);
    hipError_t e = hipEventRecord(G->ready[r], s);
    if (e != hipSuccess) {
        G->abort();
        set_err(err, SRT_ERR_HIP, "local collective: hipEventRecord");
        return SRT_ERR_HIP;
    }
    G->ptr[r] = buf;
    if (!G->barrier()) {
        set_err(err, SRT_ERR_COMM, "local collective: another rank failed");
        return SRT_ERR_COMM;
    }
    const bool receive = root < 0 || root != r;
    if (receive) {
        PeerSrcs src{};
        for (int q = 0; q < N; ++q) {
            src.p[q] = G->ptr[q];
            if (q != r && (root < 0 || q == root)) (void)hipStreamWaitEvent(s, G->ready[q], 0);
        }
        peer_gather(buf, src, bytes, N, r, root, s);
        for (int q = 0; q < N; ++q) {
            if (q == r || (root >= 0 && q != root)) continue;
            uint8_t *slot = root < 0 ? buf + (uint64_t)q * bytes : buf;
            if (r == G->corrupt_rank) corrupt_byte(slot, bytes, s);
            checksum(slot, bytes, G->tmp[r] + q, s);
            checksum_cmp(G->tmp[r] + q, G->sums[q], G->bad[r], s);
        }
    }
    e = hipEventRecord(G->done[r], s);
    if (e != hipSuccess) {
        G->abort();
        set_err(err, SRT_ERR_HIP, "local collective: hipEventRecord");
        return SRT_ERR_HIP;
    }
    if (!G->barrier()) {
        set_err(err, SRT_ERR_COMM, "local collective: another rank failed");
        return SRT_ERR_COMM;
    }
    // every reader of this rank's slot is done before its stream moves on (a
    // broadcast's root waits for all; a receiver only for itself)
    if (root < 0 || root == r)
        for (int q = 0; q < N; ++q)
            if (q != r) (void)hipStreamWaitEvent(s, G->done[q], 0);
    if (hipGetLastError() != hipSuccess) {
        G->abort();
        set_err(err, SRT_ERR_HIP, "local collective: copy launch failed");
        return SRT_ERR_HIP;
    }
    return SRT_OK;
}
}  // namespace

bool local_corrupt(srt_comm *c) {
    if (!c || !c->local) return false;
    uint32_t b = 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(c->local->dev[c->rank]);
    const bool bad = hipMemcpy(&b, c->local->bad[c->rank], 4, hipMemcpyDeviceToHost) != hipSuccess || b != 0;
    (void)hipSetDevice(cur);
    return bad;
}

srt_status comm_bcast(srt_comm *c, void *buf, size_t bytes, int root, hipStream_t s, srt_err *err) {
    if (c->local) return local_collective(c, (uint8_t *)buf, bytes, root, s, err);
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
    if (c->local) return local_collective(c, (uint8_t *)buf, bytes_per_rank, -1, s, err);
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

srt_status srt_comm_init_local(int nranks, const int32_t *devices, srt_comm **comms, srt_err *err) {
    if (!comms || nranks < 1 || nranks > srt::MAX_LOCAL_RANKS) {
        set_err(err, SRT_ERR_INVALID, "bad communicator arguments (1 to 16 local ranks)");
        return SRT_ERR_INVALID;
    }
    srt::LocalGroup *G = new (std::nothrow) srt::LocalGroup();
    if (!G) {
        set_err(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    G->n = nranks;
    G->ptr.assign(nranks, nullptr);
    G->ready.assign(nranks, nullptr);
    G->done.assign(nranks, nullptr);
    int cur = 0;
    (void)hipGetDevice(&cur);
    hipError_t e = hipSuccess;
    for (int r = 0; r < nranks && e == hipSuccess; ++r) {
        const int d = devices ? devices[r] : r;
        G->dev.push_back(d);
        e = hipSetDevice(d);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&G->ready[r], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&G->done[r], hipEventDisableTiming);
        void *sm = nullptr, *tm = nullptr, *bd = nullptr;
        if (e == hipSuccess) e = hipMalloc(&sm, 8);
        if (e == hipSuccess) e = hipMalloc(&tm, 8ull * nranks);
        if (e == hipSuccess) e = hipMalloc(&bd, 4);
        if (e == hipSuccess) e = hipMemset(bd, 0, 4);
        G->sums.push_back((unsigned long long *)sm);
        G->tmp.push_back((unsigned long long *)tm);
        G->bad.push_back((uint32_t *)bd);
    }
    if (const char *k = std::getenv("SRT_TEST_CORRUPT_PEER")) G->corrupt_rank = std::atoi(k);
    // peer access between every pair of distinct devices (xGMI reads)
    for (int a = 0; a < nranks && e == hipSuccess; ++a)
        for (int b = 0; b < nranks && e == hipSuccess; ++b) {
            if (G->dev[a] == G->dev[b]) continue;
            int ok = 0;
            if (hipDeviceCanAccessPeer(&ok, G->dev[a], G->dev[b]) != hipSuccess || !ok) {
                e = hipErrorPeerAccessUnsupported;
                break;
            }
            if ((e = hipSetDevice(G->dev[a])) != hipSuccess) break;
            e = hipDeviceEnablePeerAccess(G->dev[b], 0);
            if (e == hipErrorPeerAccessAlreadyEnabled) {
                (void)hipGetLastError();
                e = hipSuccess;
            }
        }
    (void)hipSetDevice(cur);
    if (e != hipSuccess) {
        for (hipEvent_t ev : G->ready)
            if (ev) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : G->done)
            if (ev) (void)hipEventDestroy(ev);
        for (auto *q : G->sums) (void)hipFree(q);
        for (auto *q : G->tmp) (void)hipFree(q);
        for (auto *q : G->bad) (void)hipFree(q);
        char m[200];
        std::snprintf(m, sizeof m, "srt_comm_init_local: %s", hipGetErrorString(e));
        set_err(err, SRT_ERR_HIP, m);
        delete G;
        return SRT_ERR_HIP;
    }
    // every comm made holds one reference; on a failed allocation the
    // references of the comms not made are dropped first, so destroying the
    // made ones frees G (and its events) with the last of them
    G->refs = nranks;
    for (int r = 0; r < nranks; ++r) {
        srt_comm *c = new (std::nothrow) srt_comm();
        if (!c) {
            if (r == 0) {
                for (hipEvent_t ev : G->ready)
                    if (ev) (void)hipEventDestroy(ev);
                for (hipEvent_t ev : G->done)
                    if (ev) (void)hipEventDestroy(ev);
                delete G;
            } else {
                G->refs = r;
                for (int q = 0; q < r; ++q) srt_comm_destroy(comms[q]);
            }
            set_err(err, SRT_ERR_OOM, "out of host memory");
            return SRT_ERR_OOM;
        }
        c->nranks = nranks;
        c->rank = r;
        c->local = G;
        comms[r] = c;
    }
    if (err) std::memset(err, 0, sizeof *err);
    return SRT_OK;
}

void srt_comm_abort(srt_comm *comm) {
    if (comm && comm->local) comm->local->abort();
}

void srt_comm_destroy(srt_comm *comm) {
    if (!comm) return;
    if (comm->nccl) ncclCommDestroy((ncclComm_t)comm->nccl);
    if (srt::LocalGroup *G = comm->local) {
        bool last;
        {
            std::lock_guard<std::mutex> lk(G->m);
            last = --G->refs == 0;
        }
        if (last) {
            for (hipEvent_t ev : G->ready)
                if (ev) (void)hipEventDestroy(ev);
            for (hipEvent_t ev : G->done)
                if (ev) (void)hipEventDestroy(ev);
            for (auto *q : G->sums) (void)hipFree(q);
            for (auto *q : G->tmp) (void)hipFree(q);
            for (auto *q : G->bad) (void)hipFree(q);
            delete G;
        }
    }
    delete comm;
}

}  // extern "C"
