// host_check.cpp -- the GPU-free host code of libsrt and the oracle under
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitize.py builds
// it with tests/asan/Makefile and runs it on the CPU).  It drives:
//   * srt_gml.cpp   GML ingest: generated graphs, truncations and byte flips
//   * srt_scan.cpp  the CSR scan: random CSRs with planted errors, on threads
//   * srt_xz.cpp    the .xz decoder: the blobs named on the command line
//                   (made by Python's liblzma) intact, truncated and flipped
//   * srt_ip.cpp    IpAssignment and the resolver's host lookups, threaded
//   * srt_routing.cpp RoutingInfo: path / counters from 8 threads over
//                   a compact table (the device build is replaced by
//                   routing_build below, which fills a host table)
//   * the oracle    GML parse + Dijkstra + direct paths
// Any sanitizer report aborts the process (halt_on_error); exit 0 = clean.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srt.h"
#include "../../oracle/srt_oracle.h"
#include "../../shadow_amd/csrc/srt_internal.h"
#include "../../shadow_amd/csrc/srt_scan.h"

#define CHECK(c, ...)                                         \
    do {                                                      \
        if (!(c)) {                                           \
            std::fprintf(stderr, "CHECK failed: " __VA_ARGS__); \
            std::fprintf(stderr, "\n");                       \
            std::exit(1);                                     \
        }                                                     \
    } while (0)

// ---- stand-ins for the device build the RoutingInfo code links against ----
// (the harness has no GPU: these fill the table on the host)
namespace srt {
void init_wait() {}
srt_status routing_build(const srt_csr *, const uint32_t *, uint32_t n, const srt_opts *, CompactTable *t,
                         uint64_t *min_latency, srt_err *) {
    t->bytes = SRT_RI_REC6;
    t->n = n;
    t->g = 1000;
    t->lat16 = static_cast<uint16_t *>(std::malloc(std::max<size_t>((size_t)n * n, 1) * 2));
    t->loss = static_cast<float *>(std::malloc(std::max<size_t>((size_t)n * n, 1) * 4));
    for (size_t k = 0; k < (size_t)n * n; ++k) {
        t->lat16[k] = (uint16_t)(1 + k % 300);
        t->loss[k] = (float)(k % 97) / 1000.0f;
    }
    t->diag.assign(n, srt_path{7, 0.5f, 0});
    *min_latency = 1000;
    return SRT_OK;
}
}  // namespace srt
extern "C" srt_status srt_get_direct_paths(const srt_csr *, const uint32_t *, uint32_t, srt_path *, uint64_t *,
                                           const srt_opts *, srt_err *) {
    return SRT_ERR_UNSUPPORTED;
}
extern "C" srt_status srt_plan_fetch(srt_plan *, srt_path *, uint64_t *, srt_err *) { return SRT_ERR_UNSUPPORTED; }

namespace {

std::string gml(uint32_t n, std::mt19937_64 &rng, bool directed) {
    std::string s = std::string("graph [\n  directed ") + (directed ? "1" : "0") + "\n";
    for (uint32_t i = 0; i < n; ++i) s += "  node [\n    id " + std::to_string(i * 3 + 1) + "\n    host_bandwidth_up \"1 Gbit\"\n  ]\n";
    const char *units[] = {"ms", "us", "ns", "s", "m", "h", "μs", ""};
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = directed ? 0 : i; j < n; ++j) {
            if (i != j && rng() % 3 == 0) continue;
            s += "  edge [\n    source " + std::to_string(i * 3 + 1) + "\n    target " + std::to_string(j * 3 + 1) +
                 "\n    latency \"" + std::to_string(1 + rng() % 300) + " " + units[rng() % 8] + "\"\n";
            if (rng() % 2) s += "    packet_loss 0." + std::to_string(rng() % 1000) + "\n";
            s += "  ]\n";
        }
    return s + "]\n";
}

void check_gml(std::mt19937_64 &rng) {
    int ok = 0, bad = 0;
    for (int it = 0; it < 60; ++it) {
        std::string t = gml(2 + rng() % 24, rng, rng() % 2);
        if (it % 3 == 1) t.resize(rng() % t.size());                     // truncated
        if (it % 3 == 2) t[rng() % t.size()] = (char)(rng() % 256);     // a flipped byte
        srt_gml *g = nullptr;
        srt_err e{};
        if (srt_gml_parse(t.data(), t.size(), &g, &e) == SRT_OK) {
            srt_csr c{};
            CHECK(srt_gml_csr(g, &c) == SRT_OK, "csr");
            uint64_t sum = 0;
            for (uint64_t k = 0; k < c.n_adj; ++k) sum += c.col[k] + c.lat_ns[k];
            (void)sum;
            srt_gml_free(g);
            ++ok;
        } else {
            ++bad;
        }
        char err[256];
        or_graph *og = or_gml_parse(t.data(), t.size(), err, sizeof err);
        if (og) or_graph_free(og);
    }
    std::printf("gml: %d parsed, %d rejected\n", ok, bad);
}

void check_scan(std::mt19937_64 &rng) {
    for (int it = 0; it < 20; ++it) {
        const uint32_t V = 50 + rng() % 300;
        std::vector<uint64_t> rp(V + 1, 0), lat;
        std::vector<uint32_t> col;
        std::vector<float> loss;
        for (uint32_t u = 0; u < V; ++u) {
            const uint32_t d = rng() % 40;
            for (uint32_t k = 0; k < d; ++k) {
                col.push_back(rng() % (V + (it % 5 == 0 ? 3 : 0)));  // sometimes out of range
                lat.push_back((rng() % 300) * 1000000ull + (it % 7 == 0 ? rng() % 2 : 0));
                loss.push_back(it % 4 == 0 && rng() % 50 == 0 ? 1.5f : (float)(rng() % 100) / 1000.f);
            }
            rp[u + 1] = col.size();
        }
        srt_csr c{V, 0, col.size(), rp.data(), col.data(), lat.data(), loss.data(), nullptr};
        srt::CsrStats cs;
        srt::csr_scan(&c, &cs, true);
        (void)srt::first_bad_loss(&c);
    }
    std::printf("scan: ok\n");
}

std::vector<uint8_t> slurp(const char *path) {
    std::vector<uint8_t> b;
    FILE *f = std::fopen(path, "rb");
    if (!f) return b;
    int c;
    while ((c = std::fgetc(f)) != EOF) b.push_back((uint8_t)c);
    std::fclose(f);
    return b;
}

void check_xz(int argc, char **argv, std::mt19937_64 &rng) {
    int good = 0, rejected = 0;
    for (int a = 1; a < argc; ++a) {
        const std::vector<uint8_t> blob = slurp(argv[a]);
        CHECK(!blob.empty(), "read %s", argv[a]);
        for (int v = 0; v < 12; ++v) {
            std::vector<uint8_t> b = blob;
            if (v >= 1 && v <= 4) b.resize(rng() % b.size());
            if (v >= 5) b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8));
            uint8_t *out = nullptr;
            size_t n = 0;
            srt_err e{};
            if (srt_xz_decompress(b.data(), b.size(), &out, &n, &e) == SRT_OK) {
                ++good;
                srt_free(out);
            } else {
                ++rejected;
            }
        }
    }
    std::printf("xz: %d decoded, %d rejected\n", good, rejected);
}

void check_ip(std::mt19937_64 &rng) {
    srt_ip_assignment *ia = nullptr;
    CHECK(srt_ip_assignment_create(&ia) == SRT_OK, "ia");
    for (int k = 0; k < 3000; ++k) {
        if (rng() % 4 == 0) {
            srt_err e{};
            (void)srt_ip_assignment_assign_ip(ia, (uint32_t)(rng() % 500), (uint32_t)rng(), &e);
        } else {
            (void)srt_ip_assignment_assign(ia, (uint32_t)(rng() % 500));
        }
    }
    std::vector<uint32_t> nodes(srt_ip_assignment_get_nodes(ia, nullptr, 0));
    srt_ip_assignment_get_nodes(ia, nodes.data(), (uint32_t)nodes.size());
    srt_ip_resolver *r = nullptr;
    srt_err e{};
    CHECK(srt_ip_resolver_create(ia, nodes.data(), (uint32_t)nodes.size(), &r, &e) == SRT_OK, "resolver");
    std::vector<uint32_t> ips(400000);
    for (auto &x : ips) x = (uint32_t)rng();
    std::vector<int32_t> rows(ips.size());
    CHECK(srt_ip_resolve_rows(r, ips.data(), ips.size(), rows.data()) == SRT_OK, "resolve");
    srt_ip_resolver_destroy(r);
    srt_ip_assignment_destroy(ia);
    std::printf("ip: ok\n");
}

void check_routing_info() {
    const uint32_t n = 300;
    std::vector<uint32_t> ids(n), nodes(n);
    std::vector<uint64_t> rp(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) ids[i] = 5 * i + 2, nodes[i] = i;
    srt_csr c{n, 0, 0, rp.data(), nullptr, nullptr, nullptr, ids.data()};
    srt_routing_info *ri = nullptr;
    srt_err e{};
    CHECK(srt_routing_info_build(&c, nodes.data(), n, 1, nullptr, &ri, &e) == SRT_OK, "build: %s", e.msg);
    std::vector<std::thread> th;
    std::atomic<uint64_t> hits{0};
    for (int t = 0; t < 8; ++t)
        th.emplace_back([&, t] {
            std::mt19937 r(t);
            for (int k = 0; k < 200000; ++k) {
                const uint32_t a = 5 * (r() % (n + 3)) + 2, b = 5 * (r() % n) + 2;
                srt_path p;
                if (srt_routing_info_path(ri, a, b, &p) == SRT_OK) hits++;
                srt_routing_info_increment_packet_count(ri, a, b);
            }
        });
    for (auto &x : th) x.join();
    std::vector<uint64_t> counts((size_t)n * n, 3);
    srt_routing_info_add_packet_counts(ri, counts.data());
    std::vector<srt_path> full((size_t)n * n);
    srt_routing_info_copy_table(ri, full.data());
    uint64_t mn = 0;
    CHECK(srt_routing_info_smallest_latency_ns(ri, &mn) == 1, "min");
    srt_routing_info_destroy(ri);
    std::printf("routing info: %llu paths\n", (unsigned long long)hits.load());
}

void check_oracle(std::mt19937_64 &rng) {
    const std::string t = gml(40, rng, false);
    char err[256];
    or_graph *og = or_gml_parse(t.data(), t.size(), err, sizeof err);
    CHECK(og, "oracle parse: %s", err);
    const uint32_t n = or_graph_num_nodes(og), m = or_graph_num_edges(og);
    std::vector<uint32_t> ids(n), src(m), dst(m), nodes(n);
    std::vector<uint64_t> lat(m);
    std::vector<float> loss(m);
    or_graph_node_ids(og, ids.data());
    or_graph_edges(og, src.data(), dst.data(), lat.data(), loss.data());
    for (uint32_t i = 0; i < n; ++i) nodes[i] = i;
    or_edge_list el{n, m, src.data(), dst.data(), lat.data(), loss.data(), or_graph_directed(og)};
    std::vector<uint64_t> ol((size_t)n * n);
    std::vector<float> op((size_t)n * n);
    or_err e{};
    for (int mode = 0; mode < 2; ++mode)
        (void)or_compute_shortest_paths(&el, ids.data(), nodes.data(), n, n, ol.data(), op.data(), 4, mode, &e);
    (void)or_get_direct_paths(&el, ids.data(), nodes.data(), n, ol.data(), op.data(), &e);
    or_graph_free(og);
    std::printf("oracle: ok\n");
}

}  // namespace

int main(int argc, char **argv) {
    std::mt19937_64 rng(2026);
    check_gml(rng);
    check_scan(rng);
    check_xz(argc, argv, rng);
    check_ip(rng);
    check_routing_info();
    check_oracle(rng);
    std::printf("host_check: clean\n");
    return 0;
}
