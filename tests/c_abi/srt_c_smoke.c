/* Calls the drop-in boundary (include/srt.h) from plain C, as Shadow's Rust
 * FFI would: builds the reference's own 3-node test graph
 * (src/main/network/graph/mod.rs:559-647) as petgraph adjacency CSR, runs
 * srt_compute_shortest_paths with both kernel families and srt_get_direct_paths
 * on a complete graph, and checks the reference's golden latencies and error
 * texts, then builds the dense RoutingInfo (srt_routing_info_*) by GML id.  Exit 0 = pass.  Built by tests/c_abi/Makefile (gcc, links
 * shadow_amd/libsrt.so); run by tests/test_gpu_c_abi.py on the GPU box. */
#include <stdio.h>
#include <string.h>

#include "../../include/srt.h"

static int fails = 0;
#define CHECK(c, ...)                      \
    do {                                   \
        if (!(c)) {                        \
            fprintf(stderr, __VA_ARGS__);  \
            fputc('\n', stderr);           \
            ++fails;                       \
        }                                  \
    } while (0)

/* graph.edges(u) of the reference's 3-node test graph, GML edge order
 * (mod.rs:576-610): self-loops 3333/5555/7777 ns, 0->1 3, 1->0 5, 0->2 7,
 * 2->1 11; undirected = the same edges traversable both ways. */
static void three_node(int directed, srt_csr *g, uint64_t *row_ptr, uint32_t *col, uint64_t *lat, float *loss) {
    static const uint32_t S[] = {0, 1, 2, 0, 1, 0, 2};
    static const uint32_t Dd[] = {0, 1, 2, 1, 0, 2, 1};
    static const uint64_t L[] = {3333, 5555, 7777, 3, 5, 7, 11};
    const int m = 7;
    uint64_t cnt[4] = {0, 0, 0, 0};
    for (int i = 0; i < m; ++i) {
        cnt[S[i] + 1]++;
        if (!directed && S[i] != Dd[i]) cnt[Dd[i] + 1]++;
    }
    for (int v = 0; v < 3; ++v) cnt[v + 1] += cnt[v];
    memcpy(row_ptr, cnt, sizeof cnt);
    uint64_t fill[3] = {cnt[0], cnt[1], cnt[2]};
    for (int i = 0; i < m; ++i) {
        uint64_t k = fill[S[i]]++;
        col[k] = Dd[i], lat[k] = L[i], loss[k] = 0.0f;
        if (!directed && S[i] != Dd[i]) {
            k = fill[Dd[i]]++;
            col[k] = S[i], lat[k] = L[i], loss[k] = 0.0f;
        }
    }
    g->n_nodes = 3;
    g->directed = (uint32_t)directed;
    g->n_adj = cnt[3];
    g->row_ptr = row_ptr;
    g->col = col;
    g->lat_ns = lat;
    g->loss = loss;
    g->node_ids = NULL;
}

int main(void) {
    if (srt_abi_version() != SRT_ABI_VERSION) return 2;
    if (srt_device_count() <= 0) {
        fprintf(stderr, "no HIP device\n");
        return 3;
    }
    /* mod.rs:626-644 golden latencies */
    static const uint64_t gold_dir[9] = {3333, 3, 7, 5, 5555, 12, 16, 11, 7777};
    static const uint64_t gold_und[9] = {3333, 3, 7, 3, 5555, 10, 7, 10, 7777};
    for (int directed = 0; directed < 2; ++directed)
        for (uint32_t algo = SRT_ALGO_FW; algo <= SRT_ALGO_SSSP; ++algo) {
            srt_csr g;
            uint64_t row_ptr[4], lat[16];
            uint32_t col[16];
            float loss[16];
            three_node(directed, &g, row_ptr, col, lat, loss);
            const uint32_t nodes[3] = {0, 1, 2};
            srt_path out[9];
            uint64_t mn = 0;
            srt_opts o = {algo, -1, 0, 0};
            srt_err err;
            srt_status st = srt_compute_shortest_paths(&g, nodes, 3, out, &mn, &o, &err);
            CHECK(st == SRT_OK, "directed=%d algo=%u: status %d %s", directed, algo, (int)st, err.msg);
            for (int i = 0; i < 9 && st == SRT_OK; ++i)
                CHECK(out[i].latency_ns == (directed ? gold_dir : gold_und)[i], "directed=%d algo=%u entry %d: %llu",
                      directed, algo, i, (unsigned long long)out[i].latency_ns);
            CHECK(mn == 3, "min latency %llu", (unsigned long long)mn);
        }
    /* a missing self-loop: the reference's error text (mod.rs:267-268) */
    {
        srt_csr g;
        uint64_t row_ptr[4] = {0, 1, 1, 1};
        uint32_t col[1] = {0};
        uint64_t lat[1] = {5};
        float loss[1] = {0.f};
        uint32_t ids[3] = {10, 20, 30};
        g.n_nodes = 3, g.directed = 1, g.n_adj = 1, g.row_ptr = row_ptr, g.col = col, g.lat_ns = lat;
        g.loss = loss, g.node_ids = ids;
        const uint32_t nodes[2] = {0, 1};
        srt_path out[4];
        srt_err err;
        srt_status st = srt_compute_shortest_paths(&g, nodes, 2, out, NULL, NULL, &err);
        CHECK(st == SRT_ERR_NO_EDGE && strcmp(err.msg, "No edge connecting node 20 to 20") == 0, "error text: %d %s",
              (int)st, err.msg);
    }
    /* generate_routing_info + RoutingInfo (sim_config.rs:424-461, mod.rs:428-477)
     * on the directed 3-node graph with GML ids 10/20/30, in-use nodes in
     * HashSet-like order: path() by GML id, None for an unknown id, the
     * smallest latency, saturating counters */
    {
        srt_csr g;
        uint64_t row_ptr[4], lat[16];
        uint32_t col[16];
        float loss[16];
        three_node(1, &g, row_ptr, col, lat, loss);
        const uint32_t ids[3] = {10, 20, 30};
        g.node_ids = ids;
        const uint32_t nodes[3] = {2, 0, 1};
        srt_routing_info *ri = NULL;
        srt_err err;
        srt_status st = srt_routing_info_build(&g, nodes, 3, 1, NULL, &ri, &err);
        CHECK(st == SRT_OK && ri, "routing info: %d %s", (int)st, err.msg);
        if (ri) {
            for (uint32_t a = 0; a < 3; ++a)
                for (uint32_t b = 0; b < 3; ++b) {
                    srt_path p;
                    st = srt_routing_info_path(ri, ids[a], ids[b], &p);
                    CHECK(st == SRT_OK && p.latency_ns == gold_dir[a * 3 + b], "path(%u,%u) = %llu", ids[a],
                          ids[b], (unsigned long long)p.latency_ns);
                }
            srt_path p;
            CHECK(srt_routing_info_path(ri, 10, 99, &p) == SRT_ERR_INVALID, "unknown id must be None");
            uint64_t mn = 0;
            CHECK(srt_routing_info_smallest_latency_ns(ri, &mn) == 1 && mn == 3, "smallest latency %llu",
                  (unsigned long long)mn);
            CHECK(srt_routing_info_row(ri, 30) == 0 && srt_routing_info_row(ri, 10) == 1, "rows");
            srt_routing_info_increment_packet_count(ri, 20, 30);
            srt_routing_info_increment_packet_count(ri, 20, 30);
            CHECK(srt_routing_info_packet_count(ri, 20, 30) == 2, "packet count");
            srt_routing_info_destroy(ri);
        }
    }
    /* the packet stage's host side from plain C (ABI 4): IpAssignment
     * (mod.rs:352-420) and its resolver, the host RNG helpers */
    {
        srt_ip_assignment *ia = NULL;
        CHECK(srt_ip_assignment_create(&ia) == SRT_OK && ia, "ip assignment");
        const uint32_t a0 = srt_ip_assignment_assign(ia, 30), a1 = srt_ip_assignment_assign(ia, 10);
        /* 11.0.0.1 and 11.0.0.2 in network byte order */
        CHECK(a0 == 0x0100000Bu && a1 == 0x0200000Bu, "assign %08x %08x", a0, a1);
        srt_err e;
        CHECK(srt_ip_assignment_assign_ip(ia, 20, 0x0300000Bu, &e) == SRT_OK, "assign_ip");
        CHECK(srt_ip_assignment_assign_ip(ia, 20, 0x0300000Bu, &e) == SRT_ERR_INVALID &&
                  strcmp(e.msg, "IP address has already been assigned") == 0,
              "assign_ip twice: %s", e.msg);
        uint32_t node = 0;
        CHECK(srt_ip_assignment_get_node(ia, a1, &node) == 1 && node == 10, "get_node");
        const uint32_t row_ids[3] = {30, 10, 20};
        srt_ip_resolver *res = NULL;
        CHECK(srt_ip_resolver_create(ia, row_ids, 3, &res, &e) == SRT_OK, "resolver");
        const uint32_t q[4] = {a0, a1, 0x0300000Bu, 0x0400000Bu};
        int32_t rows[4];
        CHECK(srt_ip_resolve_rows(res, q, 4, rows) == SRT_OK && rows[0] == 0 && rows[1] == 1 && rows[2] == 2 &&
                  rows[3] == -1,
              "resolve rows %d %d %d %d", rows[0], rows[1], rows[2], rows[3]);
        srt_ip_resolver_destroy(res);
        srt_ip_assignment_destroy(ia);
        uint64_t st4[4] = {1, 2, 3, 4}, d[2];
        srt_xoshiro_next_u64(st4, 2, d);
        CHECK(d[0] == 41943041ull && d[1] == 58720359ull, "xoshiro256++ vector");
        srt_xoshiro_seed_from_u64(0, st4);
        CHECK(st4[0] == 0xe220a8397b1dcdafull, "SplitMix64(0)");
    }
    if (fails) {
        fprintf(stderr, "%d check(s) failed\n", fails);
        return 1;
    }
    printf("c abi ok\n");
    return 0;
}
