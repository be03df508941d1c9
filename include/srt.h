/*
 * srt.h -- C ABI of the MI355X-native Shadow routing-table build ("srt").
 *
 * This is the drop-in boundary behind Shadow's Rust network-graph API.  Each
 * entry point names the reference interface it replaces (paths relative to the
 * Shadow v3.1.0 tree, see INTEGRATION.md for the Rust-side binding):
 *
 *   srt_compute_shortest_paths  <- NetworkGraph::compute_shortest_paths
 *                                  src/main/network/graph/mod.rs:183-228
 *   srt_get_direct_paths        <- NetworkGraph::get_direct_paths
 *                                  src/main/network/graph/mod.rs:230-252
 *   min_latency_ns out-params   <- RoutingInfo::get_smallest_latency_ns
 *                                  src/main/network/graph/mod.rs:474-476
 *   srt_packet_batch            <- Worker::send_packet decision
 *                                  src/main/core/worker.rs:326-410 (+ :539-553)
 *   srt_gml_parse               <- NetworkGraph::parse / gml_parser::parse
 *                                  src/main/network/graph/mod.rs:134-181
 *   srt_gml_parse_file          <- load_network_graph + read_xz
 *                                  src/main/network/graph/mod.rs:479-509
 *   srt_ip_assignment_* / srt_ip_resolver_* / srt_packet_batch_ip
 *                               <- IpAssignment (mod.rs:352-420) and the
 *                                  send path's lookups (worker.rs:539-553)
 *   srt_xoshiro_* / srt_host_node_seed
 *                               <- Host::random (host.rs:122, 233) seeding
 *                                  (sim_config.rs:47-53, 222-244)
 *   srt_routing_info_*          <- generate_routing_info + RoutingInfo
 *                                  src/main/core/sim_config.rs:424-461,
 *                                  src/main/network/graph/mod.rs:428-477
 *
 * Conventions (mirroring the reference's FFI: plain C types, no exceptions
 * across the boundary, caller-owned outputs):
 *   - All pointers in srt_csr / outputs are HOST pointers unless a function
 *     says "device".  Inputs are borrowed for the duration of the call.
 *   - Node references are petgraph NodeIndex values (0..n_nodes-1, GML order).
 *   - out[i*n + j] is the path nodes[i] -> nodes[j] (row-major over the
 *     caller's in-use node list, which may be in any order).
 *   - Every function returns an srt_status and fills *err (may be NULL) with
 *     the reference's error text for NO_EDGE / MULTI_EDGE.
 *   - Library functions are thread-compatible: concurrent calls on different
 *     srt_plan objects are fine; one plan is used by one thread at a time.
 */
#ifndef SRT_H
#define SRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRT_ABI_VERSION 4

typedef enum {
    SRT_OK = 0,
    SRT_ERR_NO_EDGE = 1,      /* "No edge connecting node {a} to {b}"   (mod.rs:267-268) */
    SRT_ERR_MULTI_EDGE = 2,   /* "More than one edge connecting node {a} to {b}" (:270-274) */
    SRT_ERR_DISCONNECTED = 3, /* reference panics: assert_eq!(paths.len(), n^2) (:219) */
    SRT_ERR_INVALID = 4,      /* bad arguments / parse error */
    SRT_ERR_HIP = 5,          /* HIP runtime failure */
    SRT_ERR_OOM = 6,
    SRT_ERR_UNSUPPORTED = 7,
    SRT_ERR_COMM = 8, /* RCCL failure */
} srt_status;

typedef struct {
    int32_t code;
    uint32_t a_id; /* GML ids named in NO_EDGE / MULTI_EDGE messages */
    uint32_t b_id;
    char msg[256];
} srt_err;

/* The graph as petgraph holds it: for every NodeIndex u, the EdgeReferences of
 * graph.edges(u) (directed: outgoing; undirected: all incident edges, the far
 * endpoint as `col`, self-loops once).  Parallel edges are allowed. */
typedef struct {
    uint32_t n_nodes;
    uint32_t directed;        /* informational; adjacency already encodes it */
    uint64_t n_adj;           /* number of adjacency entries */
    const uint64_t *row_ptr;  /* n_nodes + 1 */
    const uint32_t *col;      /* n_adj */
    const uint64_t *lat_ns;   /* n_adj, latency already converted to ns (mod.rs:336) */
    const float *loss;        /* n_adj, packet_loss in [0,1] */
    const uint32_t *node_ids; /* n_nodes GML ids (error text); NULL = use NodeIndex */
} srt_csr;

/* #[repr(C)] mirror of PathProperties (mod.rs:296-303), 16 bytes */
typedef struct {
    uint64_t latency_ns;
    float packet_loss;
    uint32_t _pad;
} srt_path;

/* FW: blocked min-plus Floyd-Warshall on the latencies + the exact-loss fold
 * (dense graphs); SSSP: batched multi-source sweeps (sparse graphs); LEVEL:
 * per-source bucket (Dial) Dijkstra over the edges of at most B units, B a
 * proved bound on every shortest path (dense graphs of small diameter in units
 * of the latency gcd); AUTO: the cheapest that applies, priced from measured
 * rates (the plan description names the choice and the prices) */
typedef enum { SRT_ALGO_AUTO = 0, SRT_ALGO_FW = 1, SRT_ALGO_SSSP = 2, SRT_ALGO_LEVEL = 3 } srt_algo;

typedef struct {
    uint32_t algo;   /* srt_algo */
    int32_t device;  /* HIP device ordinal (the first one when n_gpus > 1), -1 = current */
    uint32_t flags;  /* SRT_OPT_* */
    uint32_t n_gpus; /* 0 or 1: one GPU; N > 1: the build (srt_compute_shortest_paths,
                        srt_routing_info_build) shards over devices device .. device+N-1
                        with one host thread each in the calling process (srt_comm_init_local) */
} srt_opts;
/* flags: every one of the n_gpus ranks on `device` (tests the multi-GPU schedules on one GPU) */
#define SRT_OPT_SAME_DEVICE 1u

/* ------------------------------------------------------------------ info */
int srt_abi_version(void);
/* number of visible HIP devices (0 when no GPU); never fails */
int srt_device_count(void);

/* ------------------------------------------------------ one-shot host API */
/* compute_shortest_paths over the in-use nodes.  out: n*n entries (caller
 * allocated).  *min_latency_ns (may be NULL) = get_smallest_latency_ns() of the
 * resulting table, diagonal included. */
srt_status srt_compute_shortest_paths(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                                      srt_path *out, uint64_t *min_latency_ns,
                                      const srt_opts *opts, srt_err *err);

/* get_direct_paths: table = the unique edge between every ordered pair. */
srt_status srt_get_direct_paths(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                                srt_path *out, uint64_t *min_latency_ns, const srt_opts *opts,
                                srt_err *err);

/* ---------------------------------------------- device-resident plan API */
/* A plan holds the graph and the routing table in HBM so a caller (bench,
 * multi-GPU driver, the packet stage) can time or chain the build without
 * PCIe copies.  Table layout in HBM: SoA, row-major n*n: u64 latency_ns and
 * f32 packet_loss. */
typedef struct srt_plan srt_plan;

/* Uploads the graph, validates self-loops of the in-use nodes (mod.rs:210-217)
 * and chooses the kernel family; no shortest-path work yet. */
srt_status srt_plan_create(const srt_csr *g, const uint32_t *nodes, uint32_t n,
                           const srt_opts *opts, srt_plan **plan, srt_err *err);
/* Full routing build on the plan's stream; blocks until done. */
srt_status srt_plan_run(srt_plan *plan, srt_err *err);
/* Same, enqueue only (caller synchronises with srt_plan_sync). */
srt_status srt_plan_run_async(srt_plan *plan, srt_err *err);
srt_status srt_plan_sync(srt_plan *plan, srt_err *err);
/* Post-run: connectivity check + min latency; copies the table out if out != NULL. */
srt_status srt_plan_fetch(srt_plan *plan, srt_path *out, uint64_t *min_latency_ns,
                          srt_err *err);
/* device pointers of the table (valid until srt_plan_destroy) */
srt_status srt_plan_table(srt_plan *plan, uint64_t **d_latency_ns, float **d_packet_loss,
                          uint32_t *n);
/* human-readable kernel/representation choice, e.g. "fw:packed64 g=1000000 qb=38 s=30" */
const char *srt_plan_describe(const srt_plan *plan);
/* hipStream_t of the plan (as void*) */
void *srt_plan_stream(srt_plan *plan);
/* Timing of the last run's dominant kernel (FW phase-3 "rest" launches or the
 * SSSP sweep): summed ms and number of launches, measured with HIP events on
 * the plan's stream; dominant_work = relaxations those launches performed;
 * total_ms = the whole build on the device. */
srt_status srt_plan_kernel_stats(const srt_plan *plan, double *dominant_ms,
                                 uint64_t *dominant_launches, double *dominant_work,
                                 double *total_ms);
/* Phase breakdown of the last run (HIP events on the plan's streams). */
typedef struct {
    double total_ms;            /* the whole build on the device */
    double dominant_ms;         /* FW phase-3 rest launches / SSSP sweeps, summed */
    uint64_t dominant_launches;
    double dominant_work;       /* relaxations (FW) / algorithmic bytes (SSSP) of those launches */
    double loss_ms;             /* dense: exact-loss pass (tight-edge CSR + fold), 0 for SSSP */
    uint64_t tight_edges;       /* dense: edges of the tight-edge CSR */
    uint32_t sharded_tail;      /* dense, comm bound: 1 = the loss pass ran on this rank's own
                                   closure rows (no key all-gather; tight-edge lists and
                                   u32 + f32 table rows exchanged), 0 = replicated */
    uint32_t sparse_split;      /* reserved, 0 (an earlier split latency/loss sweep, removed) */
    uint64_t sparse_sweeps;     /* sparse: sweep launches of the last run, summed over its source
                                   launches (each covers every group in flight) */
    uint32_t loss_fold;         /* dense: 1 = the level fold (tight edges walked by weight class
                                   from the smaller latency level), 0 = the single-direction scan */
    uint32_t reserved0;
    uint64_t edge_visits;       /* level solve: class-CSR entries the last run's rows walked (ABI 2) */
    double create_device_ms;    /* device work of srt_plan_create, once per graph: bound proofs, the
                                   level probes, the symmetry check (ABI 4) */
} srt_timing;
srt_status srt_plan_timing(const srt_plan *plan, srt_timing *out);
/* C tiles (128 x 128 keys) the last FW run's dominant launches loaded and
 * stored, summed over those launches (0 for the SSSP sweep): the algorithmic
 * C traffic is tiles x 128^2 x 2 x sizeof(key). */
srt_status srt_plan_kernel_tiles(const srt_plan *plan, uint64_t *dominant_tiles);
void srt_plan_destroy(srt_plan *plan);

/* -------------------------------------------------------- multi-GPU (RCCL) */
/* One process per GPU.  Rank 0 calls srt_comm_unique_id, ships the 128 bytes
 * to the other ranks (e.g. torch.distributed broadcast), then every rank calls
 * srt_comm_init on its device.  A plan bound to a communicator computes only
 * its own source rows and all-gathers the table over xGMI. */
typedef struct srt_comm srt_comm;
srt_status srt_comm_unique_id(uint8_t out[128], srt_err *err);
srt_status srt_comm_init(const uint8_t id[128], int nranks, int rank, int device,
                         srt_comm **comm, srt_err *err);
void srt_comm_destroy(srt_comm *comm);
/* Host-callback transport with the same semantics (used to run the sharded
 * build over any host-side collective, e.g. torch.distributed/gloo in tests).
 * Each callback is invoked with the plan's stream idle and must have completed
 * the collective on the DEVICE buffer before returning 0.
 *   bcast:     d_buf[0..bytes) from rank `root` to all ranks;
 *   allgather: in place, rank r contributes d_buf[r*bytes_per_rank ..). */
typedef int (*srt_bcast_fn)(void *user, void *d_buf, uint64_t bytes, int root);
typedef int (*srt_allgather_fn)(void *user, void *d_buf, uint64_t bytes_per_rank);
srt_status srt_comm_init_callbacks(int nranks, int rank, srt_bcast_fn bcast,
                                   srt_allgather_fn allgather, void *user, srt_comm **comm,
                                   srt_err *err);
/* In-process transport: nranks communicators (comms[0 .. nranks)) for nranks
 * host threads of THIS process, rank r on devices[r] (NULL: device r; a device
 * may repeat -- several ranks on one GPU, for testing the schedules).  Every
 * rank's plan is driven by its own thread; collectives stay stream-ordered
 * (events + one peer-read kernel, peer access enabled between the devices).
 * Up to 16 ranks.  srt_comm_abort releases the other ranks of a failed one. */
srt_status srt_comm_init_local(int nranks, const int32_t *devices, srt_comm **comms, srt_err *err);
void srt_comm_abort(srt_comm *comm);
/* Binds the plan to a communicator: from now on srt_plan_run computes only
 * this rank's block-rows of the closure, broadcasts each round's pivot
 * block-row from its owner and all-gathers the path keys at the end, so every
 * rank holds the full table.  The communicator must outlive the plan. */
srt_status srt_plan_bind_comm(srt_plan *plan, srt_comm *comm, srt_err *err);
/* Row sharding without an exchange, for plans whose source rows are
 * independent (LEVEL and SSSP: one Dijkstra per source, the rayon fan-out of
 * mod.rs:190-208): from now on srt_plan_run computes only table rows
 * [rank*n/nranks, (rank+1)*n/nranks) (other rows are not written) and the
 * connectivity check / min latency of srt_plan_fetch cover those rows;
 * srt_plan_fetch refuses `out` (read the rows through srt_plan_table).  The
 * multi-process form of srt_opts.n_gpus: each rank's rows stay in its HBM or go
 * to the host over its own link, no collective.  FW plans (the closure needs
 * every pivot row): SRT_ERR_UNSUPPORTED -- bind a communicator instead. */
srt_status srt_plan_shard_rows(srt_plan *plan, int nranks, int rank, srt_err *err);

/* ------------------------------------------------------- packet delivery */
/* One outgoing inter-host packet, in the source host's send order. */
typedef struct {
    uint32_t src_host; /* index of the source host's RNG state */
    uint32_t src_row;  /* table row of the source host's node */
    uint32_t dst_row;  /* table column of the destination host's node */
    uint32_t payload_size;
    uint64_t t_ns; /* emulated time at send */
} srt_pkt;

enum { SRT_PDS_NONE = 0, SRT_PDS_INET_SENT = 1u << 8, SRT_PDS_INET_DROPPED = 1u << 9 };

typedef struct {
    uint64_t round_end_ns;
    uint64_t bootstrap_end_ns;
    uint64_t sim_end_ns;
} srt_round;

/* Batched Worker::send_packet decision for one scheduling round, on the device.
 * All pointers are DEVICE pointers on the plan's device.  Packets must be
 * grouped by source host: host_pkt_ptr[h]..host_pkt_ptr[h+1] are host h's
 * packets in send order (n_hosts + 1 entries).  rng: 4 x u64 xoshiro256++ state
 * per host, advanced in place by one draw per non-completed packet.
 * flags/deliver: per packet.  counters (may be NULL): n*n u64 per-path packet
 * counts (RoutingInfo::increment_packet_count).  stats (device, 2 x u64):
 * [0] = min latency of sent packets (runahead), [1] = min deliver time
 * (next event time); both UINT64_MAX when nothing was sent, and they are
 * min-combined with their previous contents (initialise to UINT64_MAX). */
srt_status srt_packet_batch(srt_plan *plan, const srt_pkt *d_pkts, const uint32_t *d_host_pkt_ptr,
                            uint32_t n_hosts, uint64_t n_pkts, uint64_t *d_rng,
                            const srt_round *round, uint32_t *d_flags, uint64_t *d_deliver,
                            uint64_t *d_counters, uint64_t *d_stats, srt_err *err);

/* Batched Worker::push_packet_to_host (worker.rs:629-639) for the packets
 * srt_packet_batch marked SENT: each becomes Event::new_packet
 * (core/work/event.rs:20-31) whose src_host_event_id is its source host's
 * next event id (Host::get_new_event_id, host.rs:691-695) in send order, and
 * each destination host's events come out in its event queue's pop order:
 * deliver time, then source host id, then event id (event.rs:85-150).  Host
 * index order (the packet grouping of srt_packet_batch) is HostId order.
 * All pointers are DEVICE pointers.  dst_host: destination host of every
 * packet (< n_dst_hosts).  event_base: per source host, its next event id
 * (advanced in place by its number of sent packets).  Outputs: event_id per
 * packet (UINT64_MAX for packets not sent); order[0 .. n_sent): the sent
 * packets' indices grouped by destination host, each group in pop order;
 * dst_ptr[0 .. n_dst_hosts]: group offsets (dst_ptr[n_dst_hosts] = n_sent).
 * Asynchronous on the plan's stream (it never waits for the device): each
 * destination's group is sorted in on-chip memory; a group of more than 1024
 * events, or a sent packet whose destination is out of range, is flagged:
 * call srt_packet_events_status before reading the results (it redoes a batch
 * with a big group exactly).  The unsent tail of order[] is unspecified. */
srt_status srt_packet_events(srt_plan *plan, const uint32_t *d_host_pkt_ptr, uint32_t n_hosts, uint64_t n_pkts,
                             const uint32_t *d_flags, const uint64_t *d_deliver, const uint32_t *d_dst_host,
                             uint32_t n_dst_hosts, uint64_t *d_event_base, uint64_t *d_event_id,
                             uint32_t *d_order, uint32_t *d_dst_ptr, srt_err *err);
/* Synchronises the plan's stream: SRT_ERR_INVALID ("destination host index
 * out of range") if an srt_packet_events call since the last check met one;
 * if the last call had a destination group too big for the on-chip sort,
 * redoes that call's sort exactly (its arrays must still be valid) and
 * returns SRT_OK; else SRT_OK. */
srt_status srt_packet_events_status(srt_plan *plan, srt_err *err);

/* ---------------------------------------------------- IP assignment (a10) */
/* IpAssignment<u32> (src/main/network/graph/mod.rs:352-420): IPv4 address ->
 * GML node id.  Addresses cross the ABI in network byte order, as Shadow's C
 * exports pass them (in_addr_t, worker.rs:669-700).  Single-threaded use
 * (sim_config.rs:399-420 fills it once, on the main thread). */
typedef struct srt_ip_assignment srt_ip_assignment;
srt_status srt_ip_assignment_create(srt_ip_assignment **out);
void srt_ip_assignment_destroy(srt_ip_assignment *ia);
/* assign_ip (mod.rs:383-394): SRT_ERR_INVALID "IP address has already been
 * assigned" (IpPreviouslyAssignedError) when the address is taken */
srt_status srt_ip_assignment_assign_ip(srt_ip_assignment *ia, uint32_t node_id, uint32_t ipv4_be, srt_err *err);
/* assign (mod.rs:371-381): the next free address after the last one assign
 * handed out, from 11.0.0.1 upward, skipping *.0 and *.255 (:406-420);
 * returns it (network byte order) */
uint32_t srt_ip_assignment_assign(srt_ip_assignment *ia, uint32_t node_id);
/* get_node (mod.rs:397-399): 1 and *node_id, or 0 (None) */
int srt_ip_assignment_get_node(const srt_ip_assignment *ia, uint32_t ipv4_be, uint32_t *node_id);
/* get_nodes (mod.rs:402-404): the distinct assigned node ids, ascending, up to
 * cap of them into out (may be NULL); returns how many there are */
uint32_t srt_ip_assignment_get_nodes(const srt_ip_assignment *ia, uint32_t *out, uint32_t cap);
uint32_t srt_ip_assignment_size(const srt_ip_assignment *ia);

/* The assignment frozen against a routing table for the send path: IPv4 ->
 * table row (the row of the address's node; row_ids[i] = GML id of table row
 * i, e.g. the in-use nodes in srt_routing_info / srt_plan order).  Replaces the
 * two get_node lookups + the path() hash of every WorkerShared::latency /
 * reliability call (worker.rs:539-553).  Immutable: thread-safe. */
typedef struct srt_ip_resolver srt_ip_resolver;
srt_status srt_ip_resolver_create(const srt_ip_assignment *ia, const uint32_t *row_ids, uint32_t n_rows,
                                  srt_ip_resolver **out, srt_err *err);
void srt_ip_resolver_destroy(srt_ip_resolver *r);
/* host batch: rows[i] = table row of ips_be[i], -1 when the address is not
 * assigned or its node has no row (the reference's None) */
srt_status srt_ip_resolve_rows(const srt_ip_resolver *r, const uint32_t *ips_be, uint64_t n, int32_t *rows);

/* A packet by address: srt_pkt with the table row / column replaced by the
 * source / destination IPv4 (network byte order, packet_getSourceIP /
 * packet_getDestinationIP, worker.rs:341-345).  Same 24-byte layout. */
typedef struct {
    uint32_t src_host;
    uint32_t src_ip;
    uint32_t dst_ip;
    uint32_t payload_size;
    uint64_t t_ns;
} srt_pkt_ip;
/* srt_packet_batch with each packet's addresses resolved on the device
 * through `res` (its table is uploaded to the plan's device on first use).
 * Asynchronous like srt_packet_batch: a packet that is not completed and has
 * an address without a row (the reference's reliability(..).unwrap() panic,
 * worker.rs:359) is reported by the next srt_packet_status. */
srt_status srt_packet_batch_ip(srt_plan *plan, srt_ip_resolver *res, const srt_pkt_ip *d_pkts,
                               const uint32_t *d_host_pkt_ptr, uint32_t n_hosts, uint64_t n_pkts, uint64_t *d_rng,
                               const srt_round *round, uint32_t *d_flags, uint64_t *d_deliver, uint64_t *d_counters,
                               uint64_t *d_stats, srt_err *err);
/* Synchronises the plan's stream; SRT_ERR_INVALID if an srt_packet_batch_ip
 * since the last check met an unresolvable address, else SRT_OK. */
srt_status srt_packet_status(srt_plan *plan, srt_err *err);

/* ------------------------------------------------------ host RNG (a12) */
/* The host's Xoshiro256PlusPlus (host.rs:122, 233; rand_xoshiro 0.6.0) as the
 * 4 x u64 state srt_packet_batch advances.  Host-side helpers so the caller
 * can seed states, continue a stream on the host (the syscalls' draws,
 * host.rs:1373-1385) and check the hand-off; see INTEGRATION.md section 4. */
/* seed_from_u64 (SplitMix64 outputs as the four words) */
void srt_xoshiro_seed_from_u64(uint64_t seed, uint64_t state[4]);
/* count next_u64 draws (out may be NULL), state advanced in place */
void srt_xoshiro_next_u64(uint64_t state[4], uint64_t count, uint64_t *out);
/* a host's node_seed (sim_config.rs:47-53, 222-244): the first next_u64 of
 * seed_from_u64(general_seed) ^ DefaultHasher(hostname) (SipHash-1-3) */
uint64_t srt_host_node_seed(uint32_t general_seed, const char *hostname, size_t len);

/* ------------------------------------------------------------- RoutingInfo */
/* Dense RoutingInfo keyed by GML node ids: replaces the
 * HashMap<(u32,u32), PathProperties> and the RwLock<HashMap> packet counters of
 * RoutingInfo (mod.rs:428-477), and the NodeIndex -> GML id re-keying of every
 * pair in generate_routing_info (sim_config.rs:436-458): the table stays
 * row-major over the in-use nodes and a GML id -> row map resolves ids.
 * Thread-safe for concurrent path() / increment_packet_count() calls (worker
 * threads); build and destroy from one thread. */
typedef struct srt_routing_info srt_routing_info;

/* generate_routing_info (sim_config.rs:424-461) in one call: the in-use nodes
 * are NodeIndex values (node_id_to_index of the GML ids); use_shortest_paths
 * selects srt_compute_shortest_paths (mod.rs:183-228) or srt_get_direct_paths
 * (mod.rs:230-252); g->node_ids gives the GML ids (NULL: NodeIndex).  Errors
 * as those functions'. */
srt_status srt_routing_info_build(const srt_csr *g, const uint32_t *nodes, uint32_t n, int use_shortest_paths,
                                  const srt_opts *opts, srt_routing_info **out, srt_err *err);
/* The same over a plan that has run (srt_plan_run): fetches its table. */
srt_status srt_routing_info_from_plan(srt_plan *plan, srt_routing_info **out, srt_err *err);
/* RoutingInfo::path (mod.rs:444-446): SRT_OK and *out, or SRT_ERR_INVALID when
 * either GML id is not an in-use node (the reference's None). */
srt_status srt_routing_info_path(const srt_routing_info *ri, uint32_t src_id, uint32_t dst_id, srt_path *out);
/* RoutingInfo::increment_packet_count (mod.rs:449-456): saturating +1 (an id
 * that is not in use is ignored: the reference would panic on the missing
 * path when logging) */
void srt_routing_info_increment_packet_count(srt_routing_info *ri, uint32_t src_id, uint32_t dst_id);
/* adds a device round's per-pair counters (srt_packet_batch's n*n array,
 * copied to the host) into the counters, saturating */
void srt_routing_info_add_packet_counts(srt_routing_info *ri, const uint64_t *counts);
uint64_t srt_routing_info_packet_count(const srt_routing_info *ri, uint32_t src_id, uint32_t dst_id);
/* RoutingInfo::get_smallest_latency_ns (mod.rs:474-476): 0 = None (empty), 1 = *out set */
int srt_routing_info_smallest_latency_ns(const srt_routing_info *ri, uint64_t *out);
/* table row of a GML id (the srt_pkt src_row / dst_row of its host), -1 if not in use */
int64_t srt_routing_info_row(const srt_routing_info *ri, uint32_t gml_id);
uint32_t srt_routing_info_size(const srt_routing_info *ri);
/* Storage of the table.  srt_routing_info_build keeps the dense build's table
 * in the record form it was downloaded in and decodes in path(): 6 bytes a
 * pair (latency / g as u16 + f32 loss) for u16-key closures (C1-C3: 1.6 GB
 * at 16k nodes instead of 4.3 GB of srt_path), 8 bytes (u32 + f32) for other
 * closures whose latencies fit u32 units, else srt_path; the diagonal (the
 * raw self-loops) is kept apart. */
#define SRT_RI_PATH16 16  /* srt_path records */
#define SRT_RI_REC8 8     /* {latency / g u32, loss f32} */
#define SRT_RI_REC6 6     /* latency / g u16 array + loss f32 array */
int srt_routing_info_record_bytes(const srt_routing_info *ri);
/* the dense table as srt_path, row-major size x size, rows in in-use order
 * (read-only) -- only for SRT_RI_PATH16 storage, else NULL (use path() or
 * srt_routing_info_copy_table) */
const srt_path *srt_routing_info_table(const srt_routing_info *ri);
/* the whole table decoded into out[size * size] (any storage) */
void srt_routing_info_copy_table(const srt_routing_info *ri, srt_path *out);
void srt_routing_info_destroy(srt_routing_info *ri);

/* --------------------------------------------------------------- start-up */
/* Shadow builds the routing info once, at setup (sim_config.rs:136-140 ->
 * generate_routing_info, sim_config.rs:424-461), so that one call is a cold
 * one: it would pay the HIP runtime start, the load of this library's kernels
 * and the pinning of the transfer staging on top of the build.  srt_init does
 * those three on `device` (-1: the current device) and returns when done;
 * srt_init_async starts it on a library thread and returns at once, so the
 * simulator can call it first thing in main and parse its config and GML
 * graph meanwhile.  Every build (and srt_init) waits for a pending init.
 * Idempotent; errors of an async init surface in the next srt_init call.
 * Exit during an async init is safe without the caller's help: the calling
 * thread's exit (return from main, exit()) joins the init thread before any
 * atexit handler or static destructor runs.  srt_init_wait only waits for a
 * pending async init (no device work). */
srt_status srt_init(int device, srt_err *err);
void srt_init_async(int device);
void srt_init_wait(void);

/* --------------------------------------------------------------- GML ingest */
/* Parses Shadow GML text (gml-parser grammar + NetworkGraph validation) into a
 * library-owned graph; srt_gml_csr exposes its petgraph adjacency. */
typedef struct srt_gml srt_gml;
srt_status srt_gml_parse(const char *text, size_t len, srt_gml **out, srt_err *err);
srt_status srt_gml_csr(const srt_gml *g, srt_csr *csr);
void srt_gml_free(srt_gml *g);

/* load_network_graph's file sources (mod.rs:494-509) + NetworkGraph::parse:
 * reads `path`, decompresses it when xz != 0 (read_xz, mod.rs:479-492: the
 * .xz container with LZMA2 blocks and CRC32 / CRC64 / SHA-256 / no checks,
 * what lzma-rs 0.3.0 decodes), checks UTF-8 (String::from_utf8) and parses.
 * Errors carry the reference's contexts: "Failed to open file: \"{path}\""
 * / "Failed to read file: {path}" / "Failed to decompress file: ...". */
srt_status srt_gml_parse_file(const char *path, int xz, srt_gml **out, srt_err *err);
/* read_xz's decompression alone: *out (library-allocated, free with srt_free,
 * NUL-terminated for convenience) holds *out_len decompressed bytes */
srt_status srt_xz_decompress(const uint8_t *in, size_t len, uint8_t **out, size_t *out_len, srt_err *err);
void srt_free(void *p);

#ifdef __cplusplus
}
#endif
#endif /* SRT_H */
