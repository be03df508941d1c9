// srt_routing.cpp -- dense RoutingInfo behind the C ABI (include/srt.h).
//
// The reference builds routing info in three sequential N^2 passes after the
// shortest paths (sim_config.rs:424-461, graph/mod.rs:428-477): rayon's
// HashMap<(NodeIndex, NodeIndex), PathProperties> is re-keyed pair by pair into
// a new HashMap<(u32, u32), _> of GML ids (to_ids), and RoutingInfo then
// answers path() by hashing and counts packets in a RwLock<HashMap>.  Here the
// table the GPU built stays dense (row-major over the in-use nodes, the
// srt_path mirror of PathProperties), one GML id -> row map replaces the N^2
// re-keying (a direct array when the ids are dense, else a sorted array with
// binary search), and the packet counters are a dense array of atomics with
// the reference's saturating add -- no lock on the send path.  The shortest-
// path table is kept in the record form the build downloaded it in (6 or 8
// bytes a pair, srt::CompactTable) and decoded per path() call: no n^2
// expansion into srt_path (4.3 GB at 16k nodes) on the host.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "srt_internal.h"

struct srt_routing_info {
    uint32_t n = 0;
    srt::CompactTable t;                     // n * n paths (compact records or srt_path)
    std::atomic<uint64_t> *counters = nullptr;  // n * n, calloc'd: untouched pairs cost no memory
    std::vector<int32_t> dense;              // id -> row when ids are dense (-1: not in use)
    std::vector<std::pair<uint32_t, uint32_t>> sorted;  // (id, row) otherwise
    bool has_min = false;
    uint64_t min_latency = 0;

    int64_t row(uint32_t id) const {
        if (!dense.empty() || sorted.empty()) return id < dense.size() ? dense[id] : -1;
        auto it = std::lower_bound(sorted.begin(), sorted.end(), std::make_pair(id, 0u));
        return it != sorted.end() && it->first == id ? (int64_t)it->second : -1;
    }
};

namespace {

void rerr(srt_err *err, int code, const char *msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

// allocate the table and counters and the id -> row map; ids[i] = GML id of row i
srt_status make_info(uint32_t n, const uint32_t *ids, srt_routing_info **out, srt_err *err) {
    srt_routing_info *ri = new (std::nothrow) srt_routing_info();
    if (!ri) {
        rerr(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    ri->n = n;
    const size_t nn = (size_t)n * n;
    ri->counters = static_cast<std::atomic<uint64_t> *>(std::calloc(std::max<size_t>(nn, 1), sizeof(uint64_t)));
    if (!ri->counters) {
        srt_routing_info_destroy(ri);
        rerr(err, SRT_ERR_OOM, "out of host memory (routing table)");
        return SRT_ERR_OOM;
    }
    uint32_t max_id = 0;
    for (uint32_t i = 0; i < n; ++i) max_id = std::max(max_id, ids[i]);
    if (n && (uint64_t)max_id < 4ull * n + 1024) {
        ri->dense.assign((size_t)max_id + 1, -1);
        for (uint32_t i = 0; i < n; ++i) ri->dense[ids[i]] = (int32_t)i;
    } else {
        ri->sorted.resize(n);
        for (uint32_t i = 0; i < n; ++i) ri->sorted[i] = {ids[i], i};
        std::sort(ri->sorted.begin(), ri->sorted.end());
    }
    *out = ri;
    return SRT_OK;
}

// an srt_path table of n * n entries for ri->t (direct paths, plans)
srt_status full_table(srt_routing_info *ri, srt_err *err) {
    ri->t.release();
    ri->t.n = ri->n;
    ri->t.bytes = SRT_RI_PATH16;
    ri->t.full = static_cast<srt_path *>(std::malloc(std::max<size_t>((size_t)ri->n * ri->n, 1) * sizeof(srt_path)));
    if (!ri->t.full) {
        rerr(err, SRT_ERR_OOM, "out of host memory (routing table)");
        return SRT_ERR_OOM;
    }
    return SRT_OK;
}

void diag_from_full(srt_routing_info *ri) {
    ri->t.diag.resize(ri->n);
    for (uint32_t i = 0; i < ri->n; ++i) ri->t.diag[i] = ri->t.full[(size_t)i * ri->n + i];
}

std::vector<uint32_t> gml_ids(const srt_csr *g, const uint32_t *nodes, uint32_t n) {
    std::vector<uint32_t> ids(n);
    for (uint32_t i = 0; i < n; ++i) ids[i] = g->node_ids ? g->node_ids[nodes[i]] : nodes[i];
    return ids;
}

}  // namespace

extern "C" {

srt_status srt_routing_info_build(const srt_csr *g, const uint32_t *nodes, uint32_t n, int use_shortest_paths,
                                  const srt_opts *opts, srt_routing_info **out, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!g || !out || (n && !nodes)) {
        rerr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *out = nullptr;
    std::vector<uint8_t> seen(g->n_nodes, 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (nodes[i] >= g->n_nodes || seen[nodes[i]]) {
            rerr(err, SRT_ERR_INVALID, "in-use node list has an out-of-range or duplicate NodeIndex");
            return SRT_ERR_INVALID;
        }
        seen[nodes[i]] = 1;
    }
    const std::vector<uint32_t> ids = gml_ids(g, nodes, n);
    srt_routing_info *ri = nullptr;
    srt_status st = make_info(n, ids.data(), &ri, err);
    if (st != SRT_OK) return st;
    uint64_t mn = ~0ull;
    if (use_shortest_paths) {
        st = srt::routing_build(g, nodes, n, opts, &ri->t, &mn, err);
    } else {
        st = full_table(ri, err);
        if (st == SRT_OK) st = srt_get_direct_paths(g, nodes, n, ri->t.full, &mn, opts, err);
        if (st == SRT_OK) diag_from_full(ri);
    }
    if (st != SRT_OK) {
        srt_routing_info_destroy(ri);
        return st;
    }
    ri->has_min = n > 0;
    ri->min_latency = mn;
    *out = ri;
    return SRT_OK;
}

srt_status srt_routing_info_from_plan(srt_plan *plan, srt_routing_info **out, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan || !out) {
        rerr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *out = nullptr;
    std::vector<uint32_t> ids(plan->n);
    for (uint32_t i = 0; i < plan->n; ++i)
        ids[i] = plan->node_ids.empty() ? plan->nodes[i] : plan->node_ids[plan->nodes[i]];
    srt_routing_info *ri = nullptr;
    srt_status st = make_info(plan->n, ids.data(), &ri, err);
    if (st != SRT_OK) return st;
    uint64_t mn = ~0ull;
    st = full_table(ri, err);
    if (st == SRT_OK) st = srt_plan_fetch(plan, ri->t.full, &mn, err);
    if (st == SRT_OK) diag_from_full(ri);
    if (st != SRT_OK) {
        srt_routing_info_destroy(ri);
        return st;
    }
    ri->has_min = plan->n > 0;
    ri->min_latency = mn;
    *out = ri;
    return SRT_OK;
}

srt_status srt_routing_info_path(const srt_routing_info *ri, uint32_t src_id, uint32_t dst_id, srt_path *out) {
    if (!ri || !out) return SRT_ERR_INVALID;
    const int64_t i = ri->row(src_id), j = ri->row(dst_id);
    if (i < 0 || j < 0) return SRT_ERR_INVALID;
    *out = ri->t.at((uint64_t)i, (uint64_t)j);
    return SRT_OK;
}

void srt_routing_info_increment_packet_count(srt_routing_info *ri, uint32_t src_id, uint32_t dst_id) {
    if (!ri) return;
    const int64_t i = ri->row(src_id), j = ri->row(dst_id);
    if (i < 0 || j < 0) return;
    std::atomic<uint64_t> &c = ri->counters[(size_t)i * ri->n + (size_t)j];
    uint64_t v = c.load(std::memory_order_relaxed);
    // x.saturating_add(1) (mod.rs:453)
    while (v != ~0ull && !c.compare_exchange_weak(v, v + 1, std::memory_order_relaxed)) {
    }
}

void srt_routing_info_add_packet_counts(srt_routing_info *ri, const uint64_t *counts) {
    if (!ri || !counts) return;
    const size_t nn = (size_t)ri->n * ri->n;
    for (size_t k = 0; k < nn; ++k) {
        const uint64_t a = counts[k];
        if (!a) continue;
        std::atomic<uint64_t> &c = ri->counters[k];
        uint64_t v = c.load(std::memory_order_relaxed), w;
        do {
            w = v > ~0ull - a ? ~0ull : v + a;
        } while (v != w && !c.compare_exchange_weak(v, w, std::memory_order_relaxed));
    }
}

uint64_t srt_routing_info_packet_count(const srt_routing_info *ri, uint32_t src_id, uint32_t dst_id) {
    if (!ri) return 0;
    const int64_t i = ri->row(src_id), j = ri->row(dst_id);
    if (i < 0 || j < 0) return 0;
    return ri->counters[(size_t)i * ri->n + (size_t)j].load(std::memory_order_relaxed);
}

int srt_routing_info_smallest_latency_ns(const srt_routing_info *ri, uint64_t *out) {
    if (!ri || !ri->has_min) return 0;
    if (out) *out = ri->min_latency;
    return 1;
}

int64_t srt_routing_info_row(const srt_routing_info *ri, uint32_t gml_id) { return ri ? ri->row(gml_id) : -1; }

uint32_t srt_routing_info_size(const srt_routing_info *ri) { return ri ? ri->n : 0; }

int srt_routing_info_record_bytes(const srt_routing_info *ri) { return ri ? ri->t.bytes : 0; }

const srt_path *srt_routing_info_table(const srt_routing_info *ri) {
    return ri && ri->t.bytes == SRT_RI_PATH16 ? ri->t.full : nullptr;
}

void srt_routing_info_copy_table(const srt_routing_info *ri, srt_path *out) {
    if (!ri || !out) return;
    for (uint64_t i = 0; i < ri->n; ++i)
        for (uint64_t j = 0; j < ri->n; ++j) out[i * ri->n + j] = ri->t.at(i, j);
}

void srt_routing_info_destroy(srt_routing_info *ri) {
    if (!ri) return;
    ri->t.release();
    std::free(ri->counters);
    delete ri;
}

}  // extern "C"
