// srt_ip.cpp -- IpAssignment and the batched IP -> table-row resolution of the
// packet stage, behind the C ABI (include/srt.h).
//
// Reference: IpAssignment (src/main/network/graph/mod.rs:352-420): a
// HashMap<IpAddr, node id>; assign_ip refuses an address twice
// (IpPreviouslyAssignedError, :343-350, :383-394); assign hands out the next
// free address after the last one it gave, from 11.0.0.1 upward, skipping the
// ".0" and ".255" addresses (:371-381, :406-420); get_nodes is the set of
// assigned node ids (:402-404), the in-use nodes of generate_routing_info
// (sim_config.rs:136-140).  assign_ips (sim_config.rs:399-420) registers the
// hosts with a configured address first, then assigns the rest in host order.
//
// The send path resolves each packet's source and destination address to a
// node and the node to its path twice per packet (WorkerShared::latency and
// ::reliability, worker.rs:539-553) through two HashMap lookups each.  Here
// the assignment is frozen once per simulation into an IP -> table-row map
// (srt::IpTable): a direct array over the address span when the addresses are
// compact (auto-assigned ones are consecutive), else an open-addressing table;
// the same lookup runs on host threads (srt_ip_resolve_rows) and inside the
// device packet round (srt_packet_batch_ip, srt_packet.hip).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>

#include "srt_internal.h"

struct srt_ip_assignment {
    std::unordered_map<uint32_t, uint32_t> map;  // IPv4 (host order) -> node id
    uint32_t last = 11u << 24;                    // 11.0.0.0 (mod.rs:366)
};

struct srt_ip_resolver {
    srt::IpTable t{};                 // host view
    std::vector<int32_t> direct;      // span entries (mode 1)
    std::vector<uint64_t> hash;       // 1 << bits slots (mode 2)
    std::mutex mu;                    // device copies are made on first use
    void *dev_buf[srt::MAX_DEVICES] = {};
    srt::IpTable dev_t[srt::MAX_DEVICES] = {};
    ~srt_ip_resolver() {
        for (int d = 0; d < srt::MAX_DEVICES; ++d)
            if (dev_buf[d]) {
                (void)hipSetDevice(d);
                (void)hipFree(dev_buf[d]);
            }
    }
};

namespace {

void ierr(srt_err *err, int code, const char *msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

inline uint32_t be_to_host(uint32_t x) { return __builtin_bswap32(x); }

// IpAssignment::increment_address (mod.rs:406-420): the next address whose
// last octet is neither 0 nor 255
uint32_t increment_address(uint32_t x) {
    for (;;) {
        x += 1;
        const uint32_t o = x & 0xffu;
        if (o != 0 && o != 255) return x;
    }
}

}  // namespace

namespace srt {
srt_status ip_table_device(srt_ip_resolver *r, int device, IpTable *out, srt_err *err) {
    if (device < 0 || device >= MAX_DEVICES) {
        ierr(err, SRT_ERR_INVALID, "device ordinal out of range");
        return SRT_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(r->mu);
    if (!r->dev_buf[device]) {
        const size_t bytes = r->t.mode == 1 ? r->direct.size() * 4 : r->hash.size() * 8;
        void *d = nullptr;
        if (hipSetDevice(device) != hipSuccess || hipMalloc(&d, std::max<size_t>(bytes, 8)) != hipSuccess) {
            ierr(err, SRT_ERR_OOM, "hipMalloc(ip table) failed");
            return SRT_ERR_OOM;
        }
        const void *src = r->t.mode == 1 ? (const void *)r->direct.data() : (const void *)r->hash.data();
        if (bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            ierr(err, SRT_ERR_HIP, "upload of the ip table failed");
            return SRT_ERR_HIP;
        }
        r->dev_buf[device] = d;
        r->dev_t[device] = r->t;
        r->dev_t[device].direct = r->t.mode == 1 ? static_cast<const int32_t *>(d) : nullptr;
        r->dev_t[device].hash = r->t.mode == 2 ? static_cast<const uint64_t *>(d) : nullptr;
    }
    *out = r->dev_t[device];
    return SRT_OK;
}
}  // namespace srt

extern "C" {

srt_status srt_ip_assignment_create(srt_ip_assignment **out) {
    if (!out) return SRT_ERR_INVALID;
    *out = new (std::nothrow) srt_ip_assignment();
    return *out ? SRT_OK : SRT_ERR_OOM;
}

void srt_ip_assignment_destroy(srt_ip_assignment *ia) { delete ia; }

srt_status srt_ip_assignment_assign_ip(srt_ip_assignment *ia, uint32_t node_id, uint32_t ipv4_be, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!ia) {
        ierr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    // Entry::Occupied -> IpPreviouslyAssignedError (mod.rs:388-391)
    if (!ia->map.emplace(be_to_host(ipv4_be), node_id).second) {
        ierr(err, SRT_ERR_INVALID, "IP address has already been assigned");
        return SRT_ERR_INVALID;
    }
    return SRT_OK;
}

uint32_t srt_ip_assignment_assign(srt_ip_assignment *ia, uint32_t node_id) {
    if (!ia) return 0;
    // loop until an unused address (mod.rs:371-381); last_assigned_addr
    // advances past addresses assign_ip took
    for (;;) {
        ia->last = increment_address(ia->last);
        if (ia->map.emplace(ia->last, node_id).second) return be_to_host(ia->last);
    }
}

int srt_ip_assignment_get_node(const srt_ip_assignment *ia, uint32_t ipv4_be, uint32_t *node_id) {
    if (!ia) return 0;
    auto it = ia->map.find(be_to_host(ipv4_be));
    if (it == ia->map.end()) return 0;
    if (node_id) *node_id = it->second;
    return 1;
}

uint32_t srt_ip_assignment_get_nodes(const srt_ip_assignment *ia, uint32_t *out, uint32_t cap) {
    if (!ia) return 0;
    std::vector<uint32_t> v;
    v.reserve(ia->map.size());
    for (const auto &kv : ia->map) v.push_back(kv.second);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if (out)
        for (uint32_t i = 0; i < cap && i < v.size(); ++i) out[i] = v[i];
    return (uint32_t)v.size();
}

uint32_t srt_ip_assignment_size(const srt_ip_assignment *ia) { return ia ? (uint32_t)ia->map.size() : 0; }

srt_status srt_ip_resolver_create(const srt_ip_assignment *ia, const uint32_t *row_ids, uint32_t n_rows,
                                  srt_ip_resolver **out, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!ia || !out || (n_rows && !row_ids)) {
        ierr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    *out = nullptr;
    // GML node id -> table row (RoutingInfo's rows: the in-use nodes in table order)
    std::unordered_map<uint32_t, int32_t> id_row;
    id_row.reserve(n_rows * 2 + 1);
    for (uint32_t i = 0; i < n_rows; ++i)
        if (!id_row.emplace(row_ids[i], (int32_t)i).second) {
            ierr(err, SRT_ERR_INVALID, "duplicate node id in the table's rows");
            return SRT_ERR_INVALID;
        }
    srt_ip_resolver *r = new (std::nothrow) srt_ip_resolver();
    if (!r) {
        ierr(err, SRT_ERR_OOM, "out of host memory");
        return SRT_ERR_OOM;
    }
    // (ip, row) of the addresses whose node has a row; an address of a node
    // that is not in the table resolves like an unassigned one (the
    // reference's path() is None for it)
    std::vector<std::pair<uint32_t, int32_t>> e;
    e.reserve(ia->map.size());
    uint32_t lo = ~0u, hi = 0;
    for (const auto &kv : ia->map) {
        auto it = id_row.find(kv.second);
        if (it == id_row.end()) continue;
        e.emplace_back(kv.first, it->second);
        lo = std::min(lo, kv.first);
        hi = std::max(hi, kv.first);
    }
    const uint64_t span = e.empty() ? 0 : (uint64_t)hi - lo + 1;
    if (e.empty() || span <= std::max<uint64_t>(4 * e.size(), 1u << 16)) {
        r->t.mode = 1;
        r->t.base = e.empty() ? 0 : lo;
        r->t.span = (uint32_t)span;
        r->direct.assign(std::max<uint64_t>(span, 1), -1);
        for (const auto &x : e) r->direct[x.first - lo] = x.second;
        r->t.direct = r->direct.data();
    } else {
        uint32_t bits = 4;
        while ((1ull << bits) < 2 * e.size()) ++bits;
        r->t.mode = 2;
        r->t.bits = bits;
        r->hash.assign(1ull << bits, 0);
        const uint64_t mask = (1ull << bits) - 1;
        for (const auto &x : e) {
            uint64_t s = srt::ip_hash(x.first, bits);
            while (r->hash[s]) s = (s + 1) & mask;
            r->hash[s] = (uint64_t)x.first << 32 | (uint32_t)(x.second + 1);
        }
        r->t.hash = r->hash.data();
    }
    *out = r;
    return SRT_OK;
}

void srt_ip_resolver_destroy(srt_ip_resolver *r) { delete r; }

srt_status srt_ip_resolve_rows(const srt_ip_resolver *r, const uint32_t *ips_be, uint64_t n, int32_t *rows) {
    if (!r || (n && (!ips_be || !rows))) return SRT_ERR_INVALID;
    const srt::IpTable t = r->t;
    auto body = [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; ++i) rows[i] = srt::ip_lookup(t, be_to_host(ips_be[i]));
    };
    // large batches on host threads (a round's packets: two lookups each)
    const unsigned T = n >= (1u << 18) ? std::min(16u, std::max(1u, std::thread::hardware_concurrency())) : 1u;
    if (T == 1) {
        body(0, n);
        return SRT_OK;
    }
    std::vector<std::thread> th;
    for (unsigned k = 0; k < T; ++k) th.emplace_back(body, n * k / T, n * (k + 1) / T);
    for (auto &x : th) x.join();
    return SRT_OK;
}

}  // extern "C"
