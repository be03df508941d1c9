/*
 * srt_oracle.h -- CPU restatement of Shadow's routing-table build and packet
 * drop decision.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only as the checker / the timed CPU baseline.  The product
 * (shadow_amd, libsrt) never links or calls anything in this directory.
 *
 * Every function restates a named piece of the reference (paths are relative
 * to the Shadow v3.1.0 tree):
 *   - GML grammar:           src/lib/gml-parser/src/parser.rs:45-273
 *   - node/edge validation:  src/main/network/graph/mod.rs:28-111
 *   - graph build:           src/main/network/graph/mod.rs:134-181
 *   - Time units:            src/main/utility/units.rs:218-280, 377-439
 *   - PathProperties:        src/main/network/graph/mod.rs:296-340
 *   - shortest paths:        src/main/network/graph/mod.rs:183-228 (+ petgraph
 *                            0.6.4 algo::dijkstra, restated in srt_oracle.c)
 *   - direct paths:          src/main/network/graph/mod.rs:230-293
 *   - send_packet decision:  src/main/core/worker.rs:326-410, 539-553
 *   - host RNG seeding:      src/main/core/sim_config.rs:46-53, 222-244,
 *                            src/main/host/host.rs:233 (rand_xoshiro 0.6.0,
 *                            rand 0.8.5, std DefaultHasher = SipHash-1-3)
 *
 * Parity pinning: see oracle/README.md and DESIGN.md section "Oracle".
 */
#ifndef SRT_ORACLE_H
#define SRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OR_OK = 0,
    OR_ERR_NO_EDGE = 1,      /* "No edge connecting node {a} to {b}"            */
    OR_ERR_MULTI_EDGE = 2,   /* "More than one edge connecting node {a} to {b}" */
    OR_ERR_DISCONNECTED = 3, /* assert_eq!(paths.len(), nodes.len().pow(2))    */
    OR_ERR_PARSE = 4,        /* GML / unit / validation error                   */
    OR_ERR_ARG = 5,
};

/* ---------------- RNG (rand_xoshiro 0.6.0 / rand 0.8.5 / std SipHash13) ---- */
uint64_t or_splitmix64_next(uint64_t *state);
void or_xoshiro_seed_from_u64(uint64_t seed, uint64_t s[4]);
uint64_t or_xoshiro_next(uint64_t s[4]);
double or_gen_f64(uint64_t s[4]);
uint64_t or_siphash13_str(const uint8_t *bytes, size_t len);
/* generic SipHash-c-d (for checking against the published SipHash-2-4 vector) */
uint64_t or_siphash_cd(const uint8_t *m, size_t len, uint64_t k0, uint64_t k1, int c, int d);
/* node_seed of a host: first u64 of seed_from_u64(general_seed) XOR hash(hostname) */
uint64_t or_host_seed(uint32_t general_seed, const char *hostname);

/* ---------------- units (units.rs:405-439, 377-388) ------------------------ */
/* parse a Time<TimePrefix> string and convert to nanoseconds.
 * *value_out = the parsed value in its own unit (for the `latency != 0` check). */
int or_parse_time_ns(const char *s, size_t len, uint64_t *ns_out, uint64_t *value_out,
                     char *err, size_t errlen);

/* ---------------- GML -> graph ---------------------------------------------- */
typedef struct or_graph or_graph;
or_graph *or_gml_parse(const char *text, size_t len, char *err, size_t errlen);
void or_graph_free(or_graph *g);
int or_graph_directed(const or_graph *g);
uint32_t or_graph_num_nodes(const or_graph *g);
uint32_t or_graph_num_edges(const or_graph *g); /* GML edges (not adjacency entries) */
/* node index (GML order) -> gml id */
void or_graph_node_ids(const or_graph *g, uint32_t *ids_out);
/* gml id -> node index, -1 if absent (last node with that id wins, like HashMap insert) */
int64_t or_graph_index_of(const or_graph *g, uint32_t id);
/* edges in GML order, endpoints as node indices */
void or_graph_edges(const or_graph *g, uint32_t *src, uint32_t *dst, uint64_t *lat_ns,
                    float *loss);

/* ---------------- routing build --------------------------------------------- */
/* A graph given as a GML-order edge list (endpoints are node indices). Undirected
 * graphs traverse every edge both ways; self-loops appear once (petgraph). */
typedef struct {
    uint32_t n_nodes;
    uint32_t n_edges;
    const uint32_t *src;
    const uint32_t *dst;
    const uint64_t *lat_ns;
    const float *loss;
    int directed;
} or_edge_list;

typedef struct {
    int code;
    uint32_t a_id, b_id; /* gml ids for NO_EDGE / MULTI_EDGE */
    char msg[256];
} or_err;

/* compute_shortest_paths (mod.rs:183-228).  nodes = in-use node indices (any
 * order, unique), ids = gml id of every node index (for error text).
 * out[i*n+j] = path nodes[i] -> nodes[j].
 * mode 0: faithful restatement (hash-map scores, `nodes.contains` filter, per
 *         source map, sequential merge) -- the "ref-cpu" baseline;
 * mode 1: array-based Dijkstra with identical arithmetic ("opt-cpu").
 * threads <= 0 means all logical CPUs (rayon's default pool).
 * src_count < n limits the run to the first src_count sources (timing samples):
 * rows >= src_count are left untouched and no diag/connectivity checks are done
 * on them. */
int or_compute_shortest_paths(const or_edge_list *g, const uint32_t *ids, const uint32_t *nodes,
                              uint32_t n, uint32_t src_count, uint64_t *lat_out,
                              float *loss_out, int threads, int mode, or_err *err);

/* get_direct_paths (mod.rs:230-252) */
int or_get_direct_paths(const or_edge_list *g, const uint32_t *ids, const uint32_t *nodes,
                        uint32_t n, uint64_t *lat_out, float *loss_out, or_err *err);

/* PathProperties + PathProperties (mod.rs:322-331) */
void or_path_add(uint64_t lat_a, float loss_a, uint64_t lat_b, float loss_b, uint64_t *lat_o,
                 float *loss_o);

/* ---------------- packet decision (worker.rs:326-410) ----------------------- */
typedef struct {
    uint32_t src_host; /* index into host RNG states */
    uint32_t src_row;  /* table row of the source host's node        */
    uint32_t dst_row;  /* table column of the destination host's node */
    uint32_t payload_size;
    uint64_t t_ns; /* current emulated time when sent               */
} or_pkt;

enum { OR_PDS_NONE = 0, OR_PDS_INET_SENT = 1u << 8, OR_PDS_INET_DROPPED = 1u << 9 };

/* Sequential restatement: packets are processed in array order; each uses the
 * next draw of its source host's stream.  rng: 4*u64 per host, in/out.
 * counters (optional, n*n) incremented per sent packet.
 * min_latency_out: min delay over sent packets (UINT64_MAX if none).
 * next_event_out: min deliver time over sent packets (UINT64_MAX if none). */
void or_packet_batch(const uint64_t *lat_tab, const float *loss_tab, uint32_t n,
                     const or_pkt *pkts, uint64_t n_pkts, uint64_t *rng, uint64_t round_end_ns,
                     uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint32_t *flags_out,
                     uint64_t *deliver_out, uint64_t *counters, uint64_t *min_latency_out,
                     uint64_t *next_event_out);

#ifdef __cplusplus
}
#endif
#endif
