// srt_api.cpp -- host side of the MI355X routing-table build: the C ABI of
// include/srt.h, plan lifetime, validation and the key-representation choice.
//
// Mirrors the reference call sequence of NetworkGraph::compute_shortest_paths
// (src/main/network/graph/mod.rs:183-228):
//   1. shortest paths between in-use nodes (here: device kernels);
//   2. diagonal := the unique self-loop edge, else "No edge connecting node X
//      to X" / "More than one edge connecting node X to X" (mod.rs:210-217,
//      256-293) -- validated on the host before any device work, in node order;
//   3. every ordered pair must be reachable (the assert at mod.rs:219) ->
//      SRT_ERR_DISCONNECTED.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <numeric>
#include <string>
#include <vector>

#include "srt_internal.h"

using srt::KeyParams;

namespace {

void set_err(srt_err *err, int code, const char *msg, uint32_t a = 0, uint32_t b = 0) {
    if (!err) return;
    err->code = code;
    err->a_id = a;
    err->b_id = b;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

void clear_err(srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
}

srt_status hip_fail(srt_err *err, hipError_t e, const char *what) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    set_err(err, SRT_ERR_HIP, buf);
    return e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
}

#define HIP_TRY(expr, what)                                \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return hip_fail(err, e_, what); \
    } while (0)

uint32_t node_id(const srt_csr *g, uint32_t idx) { return g->node_ids ? g->node_ids[idx] : idx; }

// Edge lookup with petgraph's edges_connecting semantics (mod.rs:256-293):
// count adjacency entries of row a whose far endpoint is b.
int count_edges(const srt_csr *g, uint32_t a, uint32_t b, uint64_t *lat, float *loss) {
    int c = 0;
    for (uint64_t k = g->row_ptr[a]; k < g->row_ptr[a + 1]; ++k)
        if (g->col[k] == b) {
            if (c == 0) {
                *lat = g->lat_ns[k];
                *loss = g->loss[k];
            }
            ++c;
        }
    return c;
}

srt_status edge_error(srt_err *err, int c, uint32_t a_id, uint32_t b_id) {
    char buf[160];
    if (c == 0) {
        std::snprintf(buf, sizeof buf, "No edge connecting node %u to %u", a_id, b_id);
        set_err(err, SRT_ERR_NO_EDGE, buf, a_id, b_id);
        return SRT_ERR_NO_EDGE;
    }
    std::snprintf(buf, sizeof buf, "More than one edge connecting node %u to %u", a_id, b_id);
    set_err(err, SRT_ERR_MULTI_EDGE, buf, a_id, b_id);
    return SRT_ERR_MULTI_EDGE;
}

int bits_for(unsigned __int128 x) {  // number of bits to represent x
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

// Choose the packed-key representation (see KeyParams) and prove it exact.
//
// Every value the closure stores is the key of a simple path whose latency is
// at most Lmax (units of g), and every candidate is the sum of two stored
// values.  Lmax = max edge latency when every ordered pair of graph nodes has
// an edge (the initial matrix is finite and values only decrease), else
// (V-1) * max edge latency.  A stored path has at most H = min(V-1,
// Lmax / min_edge_latency) hops.  So with W usable bits (53 for f64 keys, 62
// for u64 keys):
//   latency field: 2*Lmax (+1) must fit in W - qb bits;
//   loss field:    2*H*max_q must stay < 2^qb (no carry into the latency);
// then key sums are exact integers and lexicographic (latency, loss) order is
// plain numeric order.  s (the loss resolution) must be >= 24, i.e. loss
// quantisation <= 2^-25 per hop; otherwise the next wider key is tried.
bool fit_width(int W, unsigned __int128 lat_field, unsigned __int128 hops2, double max_nl, KeyParams *kp) {
    const int lbits = bits_for(lat_field);
    if (lbits > W) return false;
    if (max_nl == 0.0) {  // loss-free graph: key = latency units, loss field empty
        kp->qb = 0;
        kp->s = 0;
        kp->scale = 1.0;
        kp->inv_scale = 1.0;
        kp->q_cap = 0;
        return true;
    }
    const int qb = W - lbits;
    const double room = std::ldexp(1.0, qb) / ((double)hops2 * max_nl);
    int s = (int)std::floor(std::log2(room)) - 1;  // one bit of margin for rounding
    s = std::min(s, 52);
    if (s < 24) return false;
    kp->qb = (uint32_t)qb;
    kp->s = s;
    kp->scale = std::ldexp(1.0, s);
    kp->inv_scale = std::ldexp(1.0, -s);
    kp->q_cap = (uint64_t)std::llrint(kp->nlr_cap * kp->scale);
    return true;
}

bool choose_key_params(const srt_csr *g, KeyParams *kp, bool *f64, std::string *why) {
    uint64_t gcd = 0, maxlat = 0, minlat = ~0ull;
    double max_nl = 0.0;
    const double NLR_CAP = 40.0;  // reliability < e^-40 ~ 4e-18: loss == 1.0f in f32
    for (uint64_t k = 0; k < g->n_adj; ++k) {
        const uint64_t l = g->lat_ns[k];
        gcd = std::gcd(gcd, l);
        maxlat = std::max(maxlat, l);
        minlat = std::min(minlat, l);
        const double nl = -std::log1p(-(double)g->loss[k]);
        max_nl = std::max(max_nl, std::min(nl, NLR_CAP));
    }
    if (gcd == 0) gcd = 1;
    kp->g = gcd;
    kp->nlr_cap = NLR_CAP;
    const uint64_t V = g->n_nodes;
    // complete: every node has an edge to every other node
    bool complete = V > 0;
    {
        std::vector<uint32_t> stamp(V, 0);
        for (uint64_t u = 0; u < V && complete; ++u) {
            uint64_t distinct = 0;
            for (uint64_t k = g->row_ptr[u]; k < g->row_ptr[u + 1]; ++k) {
                const uint32_t v = g->col[k];
                if (v != u && stamp[v] != u + 1) {
                    stamp[v] = (uint32_t)(u + 1);
                    ++distinct;
                }
            }
            complete = distinct == V - 1;
        }
    }
    const uint64_t maxu = maxlat / gcd, minu = std::max<uint64_t>(minlat / gcd, 1);
    const unsigned __int128 Lmax = complete ? (unsigned __int128)maxu : (unsigned __int128)(V ? V - 1 : 0) * maxu;
    unsigned __int128 H = V ? V - 1 : 0;
    if (minlat != ~0ull && Lmax / minu < H) H = Lmax / minu;
    const unsigned __int128 lat_field = 2 * Lmax + 1;
    const unsigned __int128 hops2 = 2 * H + 1;
    if (fit_width(53, lat_field, hops2, max_nl, kp)) {
        *f64 = true;
        return true;
    }
    if (fit_width(62, lat_field, hops2, max_nl, kp)) {
        *f64 = false;
        return true;
    }
    *why = "latency range and loss resolution do not fit a 62-bit exact key";
    return false;
}

template <typename T>
srt_status dmalloc(T **p, size_t count, srt_err *err) {
    void *ptr = nullptr;
    hipError_t e = hipMalloc(&ptr, std::max<size_t>(count, 1) * sizeof(T));
    if (e != hipSuccess) return hip_fail(err, e, "hipMalloc");
    *p = (T *)ptr;
    return SRT_OK;
}

void free_plan_buffers(srt_plan *p) {
    hipFree(p->d_row_ptr);
    hipFree(p->d_col);
    hipFree(p->d_lat);
    hipFree(p->d_loss);
    hipFree(p->d_nodes);
    hipFree(p->d_D);
    hipFree(p->d_out_lat);
    hipFree(p->d_out_loss);
    hipFree(p->d_sl_lat);
    hipFree(p->d_sl_loss);
    hipFree(p->d_stats);
    hipFree(p->d_pack);
    hipFree(p->d_draws);
}

}  // namespace

extern "C" {

int srt_abi_version(void) { return SRT_ABI_VERSION; }

int srt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

srt_status srt_plan_create(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                           const srt_opts *opts, srt_plan **plan_out, srt_err *err) {
    clear_err(err);
    if (!g || !plan_out || (n && !nodes) || !g->row_ptr || (g->n_adj && (!g->col || !g->lat_ns || !g->loss))) {
        set_err(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *plan_out = nullptr;
    // in-use nodes must be valid and unique (they come from a HashSet)
    std::vector<uint8_t> seen(g->n_nodes, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (nodes[i] >= g->n_nodes || seen[nodes[i]]) {
            set_err(err, SRT_ERR_INVALID, "in-use node list has an out-of-range or duplicate NodeIndex");
            return SRT_ERR_INVALID;
        }
        seen[nodes[i]] = 1;
    }
    if (g->row_ptr[g->n_nodes] != g->n_adj) {
        set_err(err, SRT_ERR_INVALID, "row_ptr[n_nodes] != n_adj");
        return SRT_ERR_INVALID;
    }
    // self-loop of every in-use node, in node order (mod.rs:210-217)
    std::vector<uint64_t> sl_lat(n);
    std::vector<float> sl_loss(n);
    for (uint32_t i = 0; i < n; ++i) {
        const int c = count_edges(g, nodes[i], nodes[i], &sl_lat[i], &sl_loss[i]);
        if (c != 1) return edge_error(err, c, node_id(g, nodes[i]), node_id(g, nodes[i]));
    }

    srt_plan *p = new (std::nothrow) srt_plan();
    if (!p) {
        set_err(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    p->V = g->n_nodes;
    p->Vp = ((g->n_nodes + srt::FW_B - 1) / srt::FW_B) * srt::FW_B;
    if (p->Vp == 0) p->Vp = srt::FW_B;
    p->rb0 = 0;
    p->rb1 = p->Vp / srt::FW_B;
    p->n = n;
    p->n_adj = g->n_adj;
    p->nodes.assign(nodes, nodes + n);
    p->identity_nodes = (n == g->n_nodes);
    for (uint32_t i = 0; i < n && p->identity_nodes; ++i) p->identity_nodes = nodes[i] == i;
    if (g->node_ids) p->node_ids.assign(g->node_ids, g->node_ids + g->n_nodes);

    std::string why;
    if (!choose_key_params(g, &p->kp, &p->key_f64, &why)) {
        delete p;
        set_err(err, SRT_ERR_UNSUPPORTED, ("packed key unavailable: " + why).c_str());
        return SRT_ERR_UNSUPPORTED;
    }
    p->algo = SRT_ALGO_FW;
    char d[160];
    std::snprintf(d, sizeof d, "fw:%s B=%d g=%llu qb=%u s=%d V=%u n=%u", p->key_f64 ? "f64key" : "u64key",
                  srt::FW_B, (unsigned long long)p->kp.g, p->kp.qb, p->kp.s, p->V, n);
    p->desc = d;

    int dev = opts && opts->device >= 0 ? opts->device : -1;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    p->device = dev;
    srt_status st;
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess) {
        delete p;
        return hip_fail(err, e, "hipSetDevice");
    }
    e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete p;
        return hip_fail(err, e, "hipStreamCreate");
    }
    p->own_stream = true;
    {
        int lo = 0, hi = 0;
        hipDeviceGetStreamPriorityRange(&lo, &hi);
        e = hipStreamCreateWithPriority(&p->side_stream, hipStreamNonBlocking, hi);
        if (e != hipSuccess) {
            hipStreamDestroy(p->stream);
            delete p;
            return hip_fail(err, e, "hipStreamCreateWithPriority");
        }
    }
    hipEventCreate(&p->ev_begin);
    hipEventCreate(&p->ev_end);
    hipEventCreateWithFlags(&p->ev_cross, hipEventDisableTiming);
    hipEventCreateWithFlags(&p->ev_pivot, hipEventDisableTiming);

#define PLAN_TRY(x)                \
    do {                           \
        st = (x);                  \
        if (st != SRT_OK) {        \
            srt_plan_destroy(p);   \
            return st;             \
        }                          \
    } while (0)
    PLAN_TRY(dmalloc(&p->d_row_ptr, (size_t)g->n_nodes + 1, err));
    PLAN_TRY(dmalloc(&p->d_col, g->n_adj, err));
    PLAN_TRY(dmalloc(&p->d_lat, g->n_adj, err));
    PLAN_TRY(dmalloc(&p->d_loss, g->n_adj, err));
    PLAN_TRY(dmalloc(&p->d_nodes, n, err));
    PLAN_TRY(dmalloc(&p->d_D, (size_t)p->Vp * p->Vp, err));
    PLAN_TRY(dmalloc(&p->d_out_lat, (size_t)n * n, err));
    PLAN_TRY(dmalloc(&p->d_out_loss, (size_t)n * n, err));
    PLAN_TRY(dmalloc(&p->d_sl_lat, n, err));
    PLAN_TRY(dmalloc(&p->d_sl_loss, n, err));
    PLAN_TRY(dmalloc(&p->d_stats, 2, err));
#undef PLAN_TRY
    auto up = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, p->stream);
    };
    if ((e = up(p->d_row_ptr, g->row_ptr, ((size_t)g->n_nodes + 1) * 8)) != hipSuccess ||
        (e = up(p->d_col, g->col, g->n_adj * 4)) != hipSuccess ||
        (e = up(p->d_lat, g->lat_ns, g->n_adj * 8)) != hipSuccess ||
        (e = up(p->d_loss, g->loss, g->n_adj * 4)) != hipSuccess ||
        (e = up(p->d_nodes, nodes, (size_t)n * 4)) != hipSuccess ||
        (e = up(p->d_sl_lat, sl_lat.data(), (size_t)n * 8)) != hipSuccess ||
        (e = up(p->d_sl_loss, sl_loss.data(), (size_t)n * 4)) != hipSuccess ||
        (e = hipStreamSynchronize(p->stream)) != hipSuccess) {
        srt_plan_destroy(p);
        return hip_fail(err, e, "upload");
    }
    *plan_out = p;
    return SRT_OK;
}

srt_status srt_plan_run_async(srt_plan *p, srt_err *err) {
    clear_err(err);
    if (!p) {
        set_err(err, SRT_ERR_INVALID, "null plan");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    hipEventRecord(p->ev_begin, p->stream);
    srt::fw_init(p);
    srt_status st = srt::fw_rounds(p, err);
    if (st != SRT_OK) return st;
    srt::fw_extract(p);
    hipEventRecord(p->ev_end, p->stream);
    HIP_TRY(hipGetLastError(), "kernel launch");
    p->ran = true;
    return SRT_OK;
}

srt_status srt_plan_sync(srt_plan *p, srt_err *err) {
    clear_err(err);
    if (!p) {
        set_err(err, SRT_ERR_INVALID, "null plan");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
    // collect timings
    float ms = 0.f;
    p->total_ms = 0.0;
    if (hipEventElapsedTime(&ms, p->ev_begin, p->ev_end) == hipSuccess) p->total_ms = ms;
    p->p3_ms = 0.0;
    for (uint64_t i = 0; i < p->p3_launches; ++i) {
        if (hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]) == hipSuccess) p->p3_ms += ms;
    }
    return SRT_OK;
}

srt_status srt_plan_run(srt_plan *p, srt_err *err) {
    srt_status s = srt_plan_run_async(p, err);
    if (s != SRT_OK) return s;
    return srt_plan_sync(p, err);
}

srt_status srt_plan_fetch(srt_plan *p, srt_path *out, uint64_t *min_latency_ns, srt_err *err) {
    clear_err(err);
    if (!p || !p->ran) {
        set_err(err, SRT_ERR_INVALID, "plan has not been run");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    unsigned long long stats[2];
    HIP_TRY(hipMemcpyAsync(stats, p->d_stats, sizeof stats, hipMemcpyDeviceToHost, p->stream), "stats");
    HIP_TRY(hipStreamSynchronize(p->stream), "sync");
    if (stats[1] != 0) {
        char buf[200];
        const unsigned long long nn = (unsigned long long)p->n * p->n;
        std::snprintf(buf, sizeof buf,
                      "assertion `left == right` failed: %llu != %llu (graph not connected)",
                      nn - stats[1], nn);
        set_err(err, SRT_ERR_DISCONNECTED, buf);
        return SRT_ERR_DISCONNECTED;
    }
    if (min_latency_ns) *min_latency_ns = stats[0];
    if (out && p->n) {
        const size_t total = (size_t)p->n * p->n;
        if (!p->d_pack) {
            void *ptr = nullptr;
            hipError_t e = hipMalloc(&ptr, total * sizeof(srt_path));
            if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(pack)");
            p->d_pack = (srt_path *)ptr;
        }
        srt::pack_paths(p);
        HIP_TRY(hipMemcpyAsync(out, p->d_pack, total * sizeof(srt_path), hipMemcpyDeviceToHost,
                               p->stream),
                "download");
        HIP_TRY(hipStreamSynchronize(p->stream), "sync");
    }
    return SRT_OK;
}

srt_status srt_plan_table(srt_plan *p, uint64_t **d_lat, float **d_loss, uint32_t *n) {
    if (!p) return SRT_ERR_INVALID;
    if (d_lat) *d_lat = p->d_out_lat;
    if (d_loss) *d_loss = p->d_out_loss;
    if (n) *n = p->n;
    return SRT_OK;
}

const char *srt_plan_describe(const srt_plan *p) { return p ? p->desc.c_str() : ""; }

void *srt_plan_stream(srt_plan *p) { return p ? (void *)p->stream : nullptr; }

srt_status srt_plan_kernel_stats(const srt_plan *p, double *dominant_ms, uint64_t *launches,
                                 double *dominant_work, double *total_ms) {
    if (!p) return SRT_ERR_INVALID;
    if (dominant_ms) *dominant_ms = p->p3_ms;
    if (launches) *launches = p->p3_launches;
    if (dominant_work) *dominant_work = p->p3_work;
    if (total_ms) *total_ms = p->total_ms;
    return SRT_OK;
}

void srt_plan_destroy(srt_plan *p) {
    if (!p) return;
    hipSetDevice(p->device);
    if (p->stream) hipStreamSynchronize(p->stream);
    free_plan_buffers(p);
    for (hipEvent_t e : p->ev) hipEventDestroy(e);
    if (p->ev_begin) hipEventDestroy(p->ev_begin);
    if (p->ev_end) hipEventDestroy(p->ev_end);
    if (p->ev_cross) hipEventDestroy(p->ev_cross);
    if (p->ev_pivot) hipEventDestroy(p->ev_pivot);
    if (p->side_stream) {
        hipStreamSynchronize(p->side_stream);
        hipStreamDestroy(p->side_stream);
    }
    if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
    delete p;
}

srt_status srt_plan_bind_comm(srt_plan *p, srt_comm *comm, srt_err *err) {
    clear_err(err);
    if (!p || !comm) {
        set_err(err, SRT_ERR_INVALID, "null plan or communicator");
        return SRT_ERR_INVALID;
    }
    HIP_TRY(hipSetDevice(p->device), "hipSetDevice");
    // pad the node range so every rank owns the same number of block-rows
    // (equal all-gather chunks); padded nodes are isolated and never in use
    const uint32_t unit = (uint32_t)srt::FW_B * (uint32_t)comm->nranks;
    const uint32_t Vp = std::max<uint32_t>(((p->V + unit - 1) / unit) * unit, unit);
    if (Vp != p->Vp) {
        void *ptr = nullptr;
        hipError_t e = hipMalloc(&ptr, (size_t)Vp * Vp * sizeof(uint64_t));
        if (e != hipSuccess) return hip_fail(err, e, "hipMalloc(D)");
        HIP_TRY(hipFree(p->d_D), "hipFree");
        p->d_D = (uint64_t *)ptr;
        p->Vp = Vp;
    }
    const uint32_t nblk = p->Vp / srt::FW_B, per = nblk / (uint32_t)comm->nranks;
    p->comm = comm;
    p->rb0 = per * (uint32_t)comm->rank;
    p->rb1 = p->rb0 + per;
    char d[64];
    std::snprintf(d, sizeof d, " ranks=%d rows=[%u,%u)", comm->nranks, p->rb0 * srt::FW_B, p->rb1 * srt::FW_B);
    p->desc += d;
    return SRT_OK;
}

srt_status srt_compute_shortest_paths(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                                      srt_path *out, uint64_t *min_latency_ns,
                                      const srt_opts *opts, srt_err *err) {
    srt_plan *p = nullptr;
    srt_status s = srt_plan_create(g, nodes, n, opts, &p, err);
    if (s != SRT_OK) return s;
    s = srt_plan_run(p, err);
    if (s == SRT_OK) s = srt_plan_fetch(p, out, min_latency_ns, err);
    srt_plan_destroy(p);
    return s;
}

}  // extern "C"
