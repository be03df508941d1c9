// srt_internal.h -- shared declarations of the gfx950 routing-table build.
// Not part of the ABI (include/srt.h is).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srt.h"

namespace srt {

// Path key for the dense min-plus closure: the path LATENCY in units of g
// (the gcd of all edge latencies), nothing else.
//
// The reference orders paths lexicographically by (latency_ns, packet_loss)
// (graph/mod.rs:305-313) and folds loss as 1-(1-a)(1-b) in f32
// (mod.rs:322-331), a non-associative fold that Floyd-Warshall's joins of
// path halves cannot reproduce.  So the closure computes only the exact
// latencies, and the loss of every pair is recomputed afterwards, bit for bit,
// by the left fold over the tight shortest-path DAG (srt_loss.hip, SURVEY.md
// S-R6).  Keys are exact integers: u16 when every candidate sum (two stored
// latencies, each <= lmax) stays below KEY16_INF (packed: v_pk_add_u16 +
// v_pk_min_u16 relax two keys per instruction pair -- the fastest), else u32
// below KEY32_INF (v_add_u32 + v_min3_u32), else f64 below 2^53, else u64
// below KEY_INF; the host proves it (choose_key_params in srt_api.cpp).
constexpr uint64_t KEY_INF = 1ull << 62;  // INF + INF < 2^64: no wrap in the closure
constexpr uint32_t KEY32_INF = 0x7fffffffu;  // u32 keys: INF + INF < 2^32
constexpr uint16_t KEY16_INF = 0x7fff;       // u16 keys: INF + INF < 2^16

// closure key representation (srt_plan::key_type); u32 < f64 < u64 in speed
enum KeyType { KEY_U32 = 0, KEY_F64 = 1, KEY_U64 = 2, KEY_U16 = 3 };
inline size_t key_bytes(int t) { return t == KEY_U16 ? 2 : t == KEY_U32 ? 4 : 8; }

struct KeyParams {
    uint64_t g;     // latency unit (gcd of all edge latencies, ns)
    uint64_t lmax;  // bound on any finite closure value, in units of g
    bool lat32;     // lmax < 2^32 - 1: the loss pass keeps latencies as u32
};

// FW tile geometry: B x B blocks, one block-row/column per round.
constexpr int FW_B = 128;
// level solve (SRT_ALGO_LEVEL): the row (u16 level, f32 loss, u16 member per
// vertex) in the 160 KB LDS beside the 8 KB level table
constexpr uint32_t LEVEL_V_MAX = 18400;

// In-edge of the sparse SSSP (srt_sssp.hip): the source vertex u of an
// adjacency entry u -> v, its latency in units of g and 1 - loss rounded to f32
// (the reference's `1f32 - other.packet_loss`, mod.rs:328).  16 B, one
// global_load_dwordx4 per lane.
struct InEdge {
    uint32_t u;
    uint32_t w;
    float eb;
    uint32_t pad;
};

// IPv4 (host order) -> table row of the packet stage (srt_ip.cpp): a direct
// array over [base, base + span) (mode 1) or open addressing over 1 << bits
// slots {ip << 32 | row + 1} (mode 2, 0 = empty); -1 = no row
constexpr int MAX_DEVICES = 64;
struct IpTable {
    uint32_t mode, base, span, bits;
    const int32_t *direct;
    const uint64_t *hash;
};
__host__ __device__ inline uint64_t ip_hash(uint32_t ip, uint32_t bits) {
    return (uint64_t)((ip * 0x9E3779B1u) >> (32 - bits));
}
__host__ __device__ inline int32_t ip_lookup(const IpTable &t, uint32_t ip) {
    if (t.mode == 1) {
        const uint32_t k = ip - t.base;
        return k < t.span ? t.direct[k] : -1;
    }
    const uint64_t mask = (1ull << t.bits) - 1;
    for (uint64_t s = ip_hash(ip, t.bits);; s = (s + 1) & mask) {
        const uint64_t v = t.hash[s];
        if (!v) return -1;
        if ((uint32_t)(v >> 32) == ip) return (int32_t)(uint32_t)v - 1;
    }
}

}  // namespace srt

struct srt_ip_resolver;
namespace srt {
// the resolver's table on `device` (uploaded on first use)
srt_status ip_table_device(srt_ip_resolver *r, int device, IpTable *out, srt_err *err);
struct LocalGroup;  // srt_comm.cpp: the ranks of one process (srt_comm_init_local)
constexpr int MAX_LOCAL_RANKS = 16;
// source buffers of one in-process collective, by rank (a kernel argument)
struct PeerSrcs {
    const uint8_t *p[MAX_LOCAL_RANKS];
};
// all-gather (only < 0): dst's slots [q * bytes, ...) <- src.p[q]'s, q != skip;
// broadcast (only = root): dst[0, bytes) <- src.p[root][0, bytes); on stream s
// (srt_peer.hip)
void peer_gather(uint8_t *dst, const PeerSrcs &src, uint64_t bytes, int nranks, int skip, int only, hipStream_t s);
// the in-process transports' integrity check (srt_peer.hip): *out = a
// position-weighted checksum of d[0, bytes) (out zeroed first); *bad |= 1 when
// *a != *b (b may live on a peer device); corrupt_byte flips a bit of the last
// byte of d[0, bytes) -- a value bit of the payloads' last record, never an
// index (test knob SRT_TEST_CORRUPT_PEER)
void checksum(const void *d, uint64_t bytes, unsigned long long *out, hipStream_t s);
void checksum_cmp(const unsigned long long *a, const unsigned long long *b, uint32_t *bad, hipStream_t s);
void corrupt_byte(void *d, uint64_t bytes, hipStream_t s);
// rank r of an in-process group: 1 when a collective it received did not match
// its senders' checksums (read after the rank's stream is synchronised)
bool local_corrupt(srt_comm *c);
}  // namespace srt

struct srt_comm {
    int nranks = 1;
    int rank = 0;
    srt::LocalGroup *local = nullptr;  // in-process transport (one host thread per rank)
    void *nccl = nullptr;  // ncclComm_t when the RCCL transport is used
    srt_bcast_fn bcast = nullptr;
    srt_allgather_fn allgather = nullptr;
    void *user = nullptr;
};

struct srt_plan {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t V = 0;   // graph nodes
    uint32_t Vp = 0;  // padded to FW_B
    uint32_t n = 0;   // in-use nodes
    uint64_t n_adj = 0;
    int algo = SRT_ALGO_FW;
    srt::KeyParams kp{};
    int key_type = srt::KEY_F64;  // closure keys: u32 / f64 (exact integers < 2^53) / u64
    bool fw_glds = true;   // FW tiles staged by LDS-DMA (false: register staging)
    bool fw_f16 = false;   // u16-stored keys relaxed as f16 integers (every finite distance < 1024 units)
    // u16/f16 phase 1 (the pivot block's closure): 1 = two FW steps per
    // barrier, 0 = one (knob SRT_FW_P1 for A/B).  (Min-plus squaring to the
    // fixpoint was tried: 1 CU does a whole 128^3 product per square, real
    // blocks need 2-4 squares, and its 66 KB of LDS waited behind the rest
    // launch for a CU -- median 44 us, tail 1.2 ms, against 33 us.)
    int fw_p1 = 1;
    bool fw_small_chain = false;  // quarter-tile kernels for the look-ahead chain (sharded)
    bool fw_unique_edges = false; // no parallel edges: FW init stores instead of atomic min
    bool d_f16 = false;           // D holds f16 keys now (the init wrote them; fw_rounds converts back)
    // rounds per row all-gather of the symmetric sharded schedule (knob
    // SRT_FW_SYM_GROUP; 1 = fw_rounds_sym_sharded's one-round chain).
    // Emulated C3, g = 1 / 2 / 4: 8 ranks 21.9 / 20.0 / 22.4 ms, 4 ranks 24.2 /
    // 22.6 / 26.0, 2 ranks 37.3 / 34.5 (stream-memory hand-offs instead of
    // events measured the same: 19.8 / 22.8 / 34.4)
    uint32_t fw_sym_group = 2;
    bool fw_sym = false;          // D symmetric (fw_sym_check): rest launches run the triangle
    bool fw_sym_known = false;
    uint32_t *d_flag32 = nullptr; // device scratch flag (symmetry check)
    // symmetric sharded schedule (fw_rounds_sym_sharded): tile (i, j), i <= j,
    // belongs to rank (i + j) mod N
    uint32_t *d_tl_all = nullptr;      // N x tl_max lists, entries (i << 16) | j
    uint32_t *d_tl_cnt = nullptr;      // N counts
    uint32_t *d_tl_cross = nullptr;    // own tiles with i == k or j == k, concatenated over k
    std::vector<uint32_t> tl_cross_off;
    uint32_t sym_g = 0;  // the group size the lists and slots above are laid out for
    uint32_t tl_max = 0, tl_own = 0;
    uint16_t *d_rowslots = nullptr;    // N x ceil(nblk / N) tiles: the per-round row exchange
    uint16_t *d_fbuf = nullptr;        // N x tl_max tiles: the final exchange
    bool fw_xcd = false;          // triangle rest: XCD remap of the order (measured no faster: off)
    // square rest order: plain row-major, dealt round-robin over the XCDs, by
    // default -- C3 forced square (SRT_FW_SYM=0), rest per build: remapped +
    // banded 119.3 ms, remapped 120.5, neither 117.9 (the remap concentrates
    // the group's short tiles on one XCD; see the triangle order in srt_fw.hip)
    uint32_t fw_band_h = 1;       // triangle rest: rows per band (power of 2; 1 measured best)
    bool fw_band = false;         // grouped launches: banded tile order (knob SRT_FW_BAND=1, read at create)
    uint32_t emulate_ranks = 0;   // measurement only, see fw_rounds_t
    bool emu_closed = false;
    // end-to-end build (srt_compute_shortest_paths): the loss array is uploaded
    // while the closure runs, and the fold runs in chunks of fold_chunk_rows
    // table rows (ev_fold after each) so their download overlaps the next
    const float *h_loss_defer = nullptr;
    // end-to-end builds: the losses are range-checked on the device as they
    // are uploaded; the first bad entry (~0 if none) lands in h_lossbad
    unsigned long long *d_lossbad = nullptr, *h_lossbad = nullptr;
    std::thread loss_checker;  // level plans: the range check of every loss on host threads (h_lossbad)
    void *d_lidx = nullptr;    // level plans' loss upload: needed entries' indices (u32), then their losses
    uint64_t lidx_cap = 0;
    uint32_t fold_chunk_rows = 0;
    std::vector<hipEvent_t> ev_fold;      // emulation: D holds the closure (first run done)
    uint64_t emu_tight = 0, emu_maxw = 0;  // emulation: tight edges / max latency of the closure
    std::string desc;
    bool identity_nodes = false;
    bool ident_rows = false;  // the adjacency is V identity rows (host scan, CsrStats::ident)
    bool ident_nodes = false;  // the in-use nodes are 0 .. V-1 in order (nodes[j] = j, n = V)
    double create_device_ms = 0.0;  // device work of srt_plan_create (probes, symmetry / bound checks)
    bool in_create = false;         // srt_plan_create is running: its kernels are timed (srt::cspan_*)
    std::vector<hipEvent_t> cspan;  // event pairs around those kernels

    // device buffers
    uint64_t *d_row_ptr = nullptr;
    uint32_t *d_col = nullptr;
    uint64_t *d_lat = nullptr;
    float *d_loss = nullptr;
    uint32_t *d_nodes = nullptr;
    uint64_t *d_D = nullptr;  // Vp*Vp path keys (key_bytes(key_type) each)
    uint64_t *d_out_lat = nullptr;
    float *d_out_loss = nullptr;
    uint64_t *d_sl_lat = nullptr;
    float *d_sl_loss = nullptr;
    std::vector<uint64_t> h_sl_lat;  // the self-loops on the host too (the compact downloads'
    std::vector<float> h_sl_loss;    // diagonal: a self-loop need not fit their latency field)
    unsigned long long *d_stats = nullptr;  // [0] min latency, [1] unreachable pairs
    srt_path *d_pack = nullptr;             // AoS staging for fetch
    void *d_pack8 = nullptr;                // 8-byte staging of the compact end-to-end download
    uint32_t *d_up32 = nullptr;             // u32 latency slots of the piece-pipelined upload
    uint64_t *d_draws = nullptr;            // packet stage: one RNG draw per packet (a host block's
    uint64_t draws_cap = 0;                 // draws overflowing its LDS) + per-block minima
    uint4 *d_pkt_tab = nullptr;             // packet stage: the table as 16-B {latency, loss} records
    uint64_t pkt_tab_run = 0;               // ... packed from the build numbered run_no (0: none)
    uint64_t run_no = 0;                    // builds of this plan (srt_plan_run_async)
    uint32_t *d_pkt_bad = nullptr;          // packet stage: bit 0 = a packet's address had no row
    void *d_ev_scratch = nullptr;           // packet events: per-destination counts + cursors
    uint32_t *d_ev_bad = nullptr;    // srt_packet_events: bit 0 a destination out of range, bit 2 a group over EV_CAP
    struct EvCall {                  // the last srt_packet_events call (exact fallback)
        const uint32_t *flags;
        const uint64_t *deliver;
        const uint32_t *dst;
        uint32_t n_dst;
        uint32_t *order, *dst_ptr;
        uint32_t n;
    } ev_last{};
    size_t ev_scratch_cap = 0;

    // host copies needed after create
    std::vector<uint32_t> nodes;
    std::vector<uint32_t> node_ids;

    // timing of the last run
    std::vector<hipEvent_t> ev;  // pairs around each phase-3 (rest) launch
    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    hipEvent_t ev_cross = nullptr, ev_pivot = nullptr;  // look-ahead hand-offs M <-> S
    hipStream_t side_stream = nullptr;                  // high-priority pivot stream
    hipStream_t comm_stream = nullptr;                  // pivot-row broadcasts (multi-GPU)
    hipEvent_t ev_row = nullptr, ev_bcast = nullptr;    // S -> C (row ready), C -> S/M (row received)
    hipEvent_t ev_upload = nullptr;                     // end-to-end: deferred loss upload done (C -> M)
    uint64_t p3_launches = 0;
    double p3_work = 0.0;  // relaxations done by the timed launches
    uint64_t p3_tiles = 0;  // C tiles those launches loaded and stored
    double p3_ms = 0.0, total_ms = 0.0;
    bool ran = false;

    // multi-GPU: this rank computes block-rows [rb0, rb1) of the closure
    srt_comm *comm = nullptr;
    uint32_t rb0 = 0, rb1 = 0;

    // sparse SSSP (algo == SRT_ALGO_SSSP, srt_sssp.hip)
    uint64_t *d_in_ptr = nullptr;        // V + 1
    std::vector<uint32_t> h_bfs_rank;    // BFS discovery rank per vertex (empty: table order)
    std::vector<uint32_t> h_spt_rank;    // shortest-latency-tree level rank (frontier: order within a launch)
    uint32_t *d_sperm = nullptr;         // n: sweep slot q -> table row (rows [sperm_r0, sperm_r1) permuted)
    uint32_t sperm_r0 = 0, sperm_r1 = 0;
    srt::InEdge *d_in_edge = nullptr;    // n_in_edges (self-loops dropped)
    uint64_t n_in_edges = 0;
    uint64_t *d_sD = nullptr;            // sssp_nb * V * 64 keys
    uint64_t *d_smask = nullptr;         // 2 * sssp_nb * V change masks
    uint32_t *d_sflag = nullptr;         // 12 * sssp_nb: convergence flags + delta ring (srt_sssp.hip)
    uint8_t *d_sact = nullptr;           // 3 * groups * V target-activation bytes (tail sweeps)
    bool sssp_act_on = true;             // knob SRT_SSSP_ACT=0 turns target activation off
    uint32_t sssp_act_from = 0;          // knob SRT_SSSP_ACT=k>1: from sweep k (0: from the last launch)
    uint32_t *h_sflag = nullptr;         // pinned host copy
    uint32_t sssp_nb = 0;                // 64-source words in flight (groups x sssp_r)
    uint32_t sssp_r = 1;                 // 64-source words per lane (group = 64 * sssp_r sources)
    uint64_t sssp_g = 1;                 // latency unit
    uint64_t sssp_sweeps = 0;            // sweeps of the last run (all groups)
    // delta-stepping bucket width in latency units (0: ungated sweeps, the
    // default); knob SRT_SSSP_DELTA = the factor of the mean in-edge latency
    uint32_t sssp_delta = 0;
    uint64_t sssp_tmax = 0;              // sweep count past which the sweep reports non-convergence
    uint64_t *d_spend = nullptr;         // sssp_nb * V pending-key masks (delta-stepping)
    // latency-first frontier sweeps (srt_frontier.hip), the sparse default when
    // every finite distance is < 0xFFFF units (eccentricity proof)
    bool sssp_frontier = false;
    uint32_t fr_nb = 0;                  // 512-source blocks per launch
    uint32_t fr_grid = 0;                // sweep workgroups (a few per CU; waves loop over the items)
    bool fr_sym = false;                 // latency-symmetric graph: launches seed from earlier rows
    uint32_t fr_lblocks = 0;             // blocks of d_fl (every block of the rows when fr_sym, else fr_nb)
    uint16_t *d_fl = nullptr;            // fr_lblocks * V * 512 u16 latencies (units of g)
    float *d_fp = nullptr;               // fr_nb * V * 512 f32 losses
    uint8_t *d_ftight = nullptr;         // fr_nb * n_in_edges * 64 tight-source bytes
    uint2 *d_fce = nullptr;              // fr_nb * n_in_edges compacted tight in-edges (u, 1 - e)
    uint32_t *d_fcnt = nullptr;          // fr_nb * V tight in-edge counts
    uint32_t fr_first = 0;               // blocks of a smaller first launch (0: equal launches)
    uint32_t *d_fctl = nullptr;          // 8 sweep-mode words (srt_frontier.hip sweep_mode)
    void *d_fchg = nullptr;              // fr_nb * V change records (srt_frontier.hip Chg, 16 B)
    uint32_t *d_fact = nullptr;          // fr_nb * V activation stamps
    uint8_t *d_ffin = nullptr;           // fr_nb * V: item exact from the start (symmetric seeding)
    // the frontier's vertex order (hubs spread over the 64-vertex chunks):
    // in-use nodes, out-CSR (self-loops dropped) renumbered; d_in_ptr /
    // d_in_edge of a frontier plan are in this order too
    uint32_t *d_fnodes = nullptr;
    uint64_t *d_frow_ptr = nullptr;
    uint32_t *d_fcol = nullptr;
    std::vector<uint32_t> h_fnodes;
    bool fr_symg = false;                // latency-symmetric adjacency: out-neighbours = in-edge sources
    uint8_t *d_fsb = nullptr;            // 2 x fr_nb * V * 64: per-source loss change bits (double-buffered)
    uint32_t *d_fdone = nullptr;         // V: block (of this rank's rows) in which the vertex is a source, ~0 none
    std::vector<uint32_t> h_fdone;
    uint32_t *d_fimp = nullptr;          // last sweep that improved anything
    uint32_t *h_fimp = nullptr;          // pinned copy
    uint32_t fr_t = 1;                   // sweep stamp counter (grows across launches and builds)
    uint64_t fr_lat_sweeps = 0, fr_loss_sweeps = 0;  // productive sweeps of the last run
    std::vector<uint32_t> h_sperm;       // host copy of d_sperm (kept alive for the async upload)
    // table rows this rank computes ([0, n) single-GPU); the table is allocated
    // with rows_alloc >= n rows so the row all-gather has equal chunks
    uint32_t row0 = 0, row1 = 0, rows_alloc = 0;
    unsigned long long *d_rstats = nullptr;  // 2 per rank: min latency, unreachable

    // exact-loss pass of the dense build (srt_loss.hip): the tight-edge pull
    // CSR (every edge u -> v whose latency equals the closure's D[u][v]) and
    // per-workgroup scratch
    uint8_t *d_tflag = nullptr;      // n_adj: adjacency entry is a tight edge
    uint32_t *d_tcnt = nullptr;      // V: in-degree count / fill cursor
    uint64_t *d_tptr = nullptr;      // V + 1
    uint32_t *d_tu = nullptr;        // t_cap: source vertex (unpacked form)
    void *d_tw = nullptr;            // t_cap: latency in units of g (u32 or u64; unpacked form)
    float *d_teb = nullptr;          // t_cap: 1 - loss, rounded once in f32 (unpacked form)
    uint64_t *d_tpk = nullptr;       // t_cap: packed form, (1-e) bits << 32 | (w << ubits) | u, rows sorted by w
    uint64_t *d_tpk2 = nullptr;      // t_cap: packed form before the sort
    void *d_tsort_tmp = nullptr;     // rocPRIM segmented sort scratch
    size_t tsort_tmp_cap = 0;
    uint64_t *d_tmaxw = nullptr;     // max latency (units) of a tight edge
    uint64_t t_cap = 0, t_edges = 0; // capacity / tight edges of the last run
    bool t_packed = false;           // the last run used the packed, w-sorted form
    bool t_push = false;             // the last run's CSR is the push form (rows by source)
    uint64_t *h_tcount = nullptr;    // pinned: [0] total tight edges, [1] max tight latency
    // level fold (srt_loss.hip level_loss_kernel): the tight edges grouped by
    // (vertex, exact weight class w = 1..15) twice -- out-rows in d_tpk, in-rows
    // in d_tpk2, entries (1-e) bits << 32 | other endpoint; class w of vertex x
    // is [tcls[x*16 + w-1], tcls[x*16 + w]) (in-rows: offset V*16 + 1)
    bool t_level = false;            // the last run built the class CSRs (and folds by levels)
    uint32_t t_q = 1;                // level width of the fold, units of g (1: exact levels; > 1: quantized)
    uint32_t t_cls = 16;             // class offsets per vertex of the level fold's CSRs (16 or 32)
    uint32_t *d_tcw = nullptr;       // quantized fold: each class entry's exact weight (out, then in), t_cap each
    uint64_t lvl_cap = 0;            // level solve: class entries d_tpk / d_tpk2 hold (the probe's count)
    bool lvl_sym_lat = false;        // level solve: identity rows, mirrored latencies (lvl_sym_tile_kernel)
    bool lvl_sym = false;            // ... and mirrored losses: the class in-rows are the out-rows
    uint16_t *d_lat16 = nullptr;     // symmetric level plans: the adjacency's latencies in units of g (< 0xffff), written by the symmetry check
    bool lvl_single = false;         // the last class-CSR build made out-rows only (in-rows = out-rows)
    uint64_t lvl_est = 0;            // the probe's entry-count estimate (sizes the arrays before its one pass)
    uint64_t lvl_maxu = 0;           // the longest edge, units of g (the estimate's scale)
    // sharded class CSR (symmetric level plans over W ranks): rank r builds the
    // out-rows of vertices [r * vr, (r + 1) * vr) into entry slot r (lvl_seg_cap
    // entries a slot, so the offsets are absolute) and the slots are
    // all-gathered (level_csr_sharded)
    uint64_t lvl_seg_cap = 0;
    uint32_t *d_lvl_offstage = nullptr;  // W * vr * cls class offsets, slot r = rank r's vertices
    uint64_t lvl_offstage_cap = 0;
    unsigned long long *d_lvl_counts = nullptr;  // W per-rank entry counts (sizing)
    uint32_t lvl_emu_ranks = 0;      // measurement (srt_plan_shard_rows + SRT_LVL_SHARD_EMU=1): rank row0's slice
    bool lvl_emu_built = false;      // ... every slice built once (the first run); later runs rebuild the own one
    unsigned long long *d_rowctr = nullptr;  // level solve: the rows dealt by a counter (LevelCtx::row_ctr)
    unsigned long long *d_lvisit = nullptr;  // level solve: class entries the last run walked
    uint32_t lvl_q = 0, lvl_rb = 0, lvl_vb = 0;  // quantized level solve: bucket width (units), entry field bits
    uint16_t *d_lmem = nullptr;              // its per-workgroup scratch (lmem_cap u16)
    uint64_t lmem_cap = 0;
    uint64_t lvl_visits = 0;                 // its host copy (srt_plan_sync)
    uint64_t tcw_cap = 0;            // d_tcw entries
    uint32_t *d_tcls = nullptr;      // 2 * (V*16 + 1) class offsets
    uint32_t *d_tccnt = nullptr;     // 2 * (V*16 + 1) class counts / fill cursors
    uint64_t tcls_cap = 0;           // entries of d_tcls and d_tccnt
    void *d_tscan_tmp = nullptr;     // rocPRIM scan scratch
    size_t tscan_tmp_cap = 0;
    void *d_lscratch = nullptr;      // per workgroup: order array (+ rows if not in LDS)
    size_t lscratch_cap = 0;
    hipEvent_t ev_loss0 = nullptr, ev_loss1 = nullptr;  // around the loss pass
    double loss_ms = 0.0;            // exact-loss pass of the last run (tight CSR + fold)

    // sharded dense tail (comm bound, srt_loss.hip fw_loss_sharded): the loss
    // pass of rank r covers the in-use sources inside its own closure
    // block-rows (their D rows are final locally, so no key all-gather); the
    // tight edges of its own adjacency rows are all-gathered as a list; its
    // table rows travel as u32 latency units + f32 loss and are expanded into
    // the table on every rank
    bool shard_tail = false;               // this run used the sharded tail
    bool row_shard = false;                // srt_plan_shard_rows: rows [row0, row1) only, no exchange
    bool tail_expanded = false;            // ... and expanded its chunks behind their all-gathers
    std::vector<uint32_t> lrow_cnt;        // per rank: loss-pass rows
    uint32_t lrow_max = 0;                 // staging rows per rank (tail_q chunks of tail_cr rows)
    uint32_t tail_q = 1, tail_cr = 0;      // the fold runs in tail_q chunks; chunk c's all-gather
                                           // overlaps the fold of chunk c + 1
    std::vector<hipEvent_t> ev_tail;       // per chunk: fold done (M -> C), then all-gather done
    uint32_t *d_lrows = nullptr;           // slot (c * nranks + r) * tail_cr + k: rank r's row
                                           // c * tail_cr + k (~0: padding)
    uint32_t *d_slat = nullptr;            // nranks * lrow_max * n: latency units (~0: unreachable),
                                           // u16 when stage16 (u16 keys), else u32
    bool stage16 = false;
    bool fw_full_d = false;                // the closure left the whole D on every rank (symmetric sharded)
    bool stage_loss_only = false;          // ... so the tail stages and exchanges only the loss; the
                                           // latencies come from D (expand_rows_kernel)
    float *d_sloss = nullptr;              // nranks * lrow_max * n
    uint4 *d_tlist = nullptr;              // tlist_cap allocated slots of tight edges {v, u, w, 1-e bits} (v = ~0: pad)
    uint64_t tlist_cap = 0;
    unsigned long long *d_tinfo = nullptr; // 2 per rank: local tight-edge count, max tight latency
    unsigned long long *d_tcursor = nullptr;  // list fill cursor
    unsigned long long *h_tinfo = nullptr; // pinned copy of d_tinfo
};

namespace srt {
// plan creation's kernels, timed by event pairs on the plan's stream while
// p->in_create (srt_timing.create_device_ms sums them; host work between the
// pairs -- allocation, count read-backs -- is not device time)
void cspan_begin(srt_plan *p);
void cspan_end(srt_plan *p);
// A host routing table in the record form of its download (srt_routing.cpp
// decodes it per path() call): SRT_RI_REC6 = lat16[n*n] (latency / g, 0xFFFF
// unreachable) + loss[n*n]; SRT_RI_REC8 = rec8[n*n] {latency / g (~0:
// unreachable), loss bits}; SRT_RI_PATH16 = full[n*n].  The diagonal (the raw
// self-loops, mod.rs:210-217) is diag[n] in every form.
struct CompactTable {
    int bytes = SRT_RI_PATH16;
    uint32_t n = 0;
    uint64_t g = 1;
    uint16_t *lat16 = nullptr;
    float *loss = nullptr;
    uint2 *rec8 = nullptr;
    srt_path *full = nullptr;
    std::vector<srt_path> diag;
    srt_path at(uint64_t i, uint64_t j) const {
        if (i == j) return diag[i];
        const uint64_t e = i * n + j;
        srt_path q{};
        if (bytes == SRT_RI_REC6) {
            q.latency_ns = lat16[e] == 0xffffu ? ~0ull : (uint64_t)lat16[e] * g;
            q.packet_loss = loss[e];
        } else if (bytes == SRT_RI_REC8) {
            const uint2 r = rec8[e];
            q.latency_ns = r.x == 0xffffffffu ? ~0ull : (uint64_t)r.x * g;
            q.packet_loss = __builtin_bit_cast(float, r.y);
        } else {
            q = full[e];
        }
        return q;
    }
    void release() {
        std::free(lat16);
        std::free(loss);
        std::free(rec8);
        std::free(full);
        lat16 = nullptr;
        loss = nullptr;
        rec8 = nullptr;
        full = nullptr;
    }
};
// generate_routing_info's shortest-path build straight into a CompactTable
// (srt_api.cpp): the end-to-end build of srt_compute_shortest_paths with the
// downloaded records kept as they are; *min_latency as that function's
srt_status routing_build(const srt_csr *g, const uint32_t *nodes, uint32_t n, const srt_opts *opts, CompactTable *t,
                         uint64_t *min_latency, srt_err *err);
// waits for a pending srt_init_async (srt_api.cpp)
void init_wait();
// loads the code object of every kernel translation unit (srt_init)
hipError_t preload_kernels();
// collectives (srt_comm.cpp)
srt_status comm_bcast(srt_comm *c, void *buf, size_t bytes, int root, hipStream_t s, srt_err *err);
srt_status comm_allgather_inplace(srt_comm *c, void *buf, size_t bytes_per_rank, hipStream_t s,
                                  srt_err *err);
// kernels (srt_fw.hip)
void fw_init(srt_plan *p);
srt_status fw_sym_check(srt_plan *p, srt_err *err);
// key-width proof: a bound on every finite distance (ns) from one source's
// in- and out-eccentricity, ~0 if none (srt_fw.hip)
srt_status fw_ecc_bound(srt_plan *p, uint32_t max_sweeps, uint64_t *bound_ns, uint32_t *sweeps, srt_err *err);
srt_status fw_rounds(srt_plan *p, srt_err *err);
// sharded closure: every rank's block-rows of D to every rank (the loss
// pass's fallback when the sharded tail does not apply)
srt_status fw_gather_keys(srt_plan *p, srt_err *err);
// exact-loss pass (srt_loss.hip): tight-edge CSR from the closure, then the
// f32 left fold over the tight DAG for table rows [row0, row1); writes the
// table rows, the raw self-loop diagonal and (min latency, unreachable) into
// d_stats
srt_status fw_loss(srt_plan *p, unsigned long long *d_stats, srt_err *err);
// level solve (srt_loss.hip, SRT_ALGO_LEVEL): the create-time bound on every
// in-use shortest path over the edges <= wmax units (~0: none; visits: edges a
// row walks), and the build of rows [row0, row1) into the table
srt_status level_probe(srt_plan *p, uint64_t wmax, uint32_t wc, uint64_t *bound, uint64_t *visits, srt_err *err);
srt_status level_run(srt_plan *p, unsigned long long *d_stats, srt_err *err);
// what a level solve launch reads and writes: a plan's buffers (level_ctx),
// or a peer device's copies of its class CSRs (the in-process multi-GPU build)
struct LevelCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t V = 0, n = 0, t_cls = 16;
    uint64_t g = 1;
    const uint32_t *tcls = nullptr;  // 2 * (V * t_cls + 1) class offsets (out, then in)
    const uint64_t *ce_out = nullptr, *ce_in = nullptr;
    const uint32_t *nodes = nullptr;
    const uint64_t *sl_lat = nullptr;
    const float *sl_loss = nullptr;
    uint64_t *out_lat = nullptr;
    float *out_loss = nullptr;
    unsigned long long *visits = nullptr;  // class entries walked (nullable)
    uint32_t q = 0, rb = 0, vb = 0;        // quantized solve: bucket width (units), remainder / vertex bits of an entry
    uint16_t *lmem = nullptr;              // quantized solve: level_scratch_bytes of per-workgroup scratch
    bool idn = false;                      // nodes[j] = j, n = V, n % 4 == 0: the vectorised row output
    unsigned long long *row_ctr = nullptr; // level solve: {next row, workgroups done}, 0 between launches (nullable: rows dealt statically)
};
LevelCtx level_ctx(srt_plan *p);
// the class CSRs of a level plan at its bound (the run's first step)
srt_status level_prepare(srt_plan *p, srt_err *err);
// rows [r0, r1) staged (row r0 + k at k * n) as u16 (stage_mode 1) or u32 (2)
// latency units + f32 loss, or as 8-byte records {u32 units, loss bits} (3,
// quantized plans only); (min latency, unreachable) min/added into d_stats, on
// c.stream
void level_solve_stage(const LevelCtx &c, uint32_t r0, uint32_t r1, uint32_t lmax, void *stage_lat,
                       float *stage_loss, uint32_t stage_mode, unsigned long long *d_stats);
// bytes of the quantized solve's scratch on `device` for V vertices (0 unless quant)
size_t level_scratch_bytes(int device, uint32_t V, bool quant);
// bits of a vertex index < V in a quantized class entry
uint32_t level_vbits(uint32_t V);
// the shortest non-self-loop edge latency of the plan's uploaded graph, ns
srt_status level_min_edge(srt_plan *p, uint64_t *min_ns, srt_err *err);
// *sym = the adjacency is V x V identity rows whose pairs of latency <= wmax
// units mirror each other exactly (and their losses when with_loss: d_loss
// uploaded) -- a level plan then builds no in-rows
srt_status level_sym_check(srt_plan *p, uint64_t wmax_units, bool with_loss, bool *sym, srt_err *err);
// the adjacency indices (u32) of the entries a level plan's class CSRs read
// (latency <= kp.lmax units, not a self-loop) into d_idx (cap entries), their
// count into *d_cnt; and the scatter of gathered losses into d_loss
void level_loss_index(srt_plan *p, uint32_t *d_idx, uint64_t cap, unsigned long long *d_cnt, hipStream_t s);
void loss_scatter(const uint32_t *d_idx, const float *d_val, uint64_t count, float *d_loss, hipStream_t s);
// *d_ok cleared when an uploaded loss (identity rows) differs from its mirror's
void loss_mirror_check(const uint32_t *d_idx, uint64_t count, uint64_t V, const float *d_loss, uint32_t *d_ok,
                       hipStream_t s);
// d_stats = (~0, 0) on stream s
void level_stats_init(unsigned long long *d_stats, hipStream_t s);
// sharded tail: every rank's staged rows (d_slat / d_sloss, all-gathered) into the table
void expand_shard_rows(srt_plan *p, int nranks);
// table entries [first, first + count) -> d_pack[0, count) as srt_path
void pack_paths(srt_plan *p, uint64_t first, uint64_t count, srt_path *dst, hipStream_t s);
// the same entries as 8-byte (latency / g as u32, loss bits) records (kp.lat32 plans)
void pack_paths8(srt_plan *p, uint64_t first, uint64_t count, void *dst, hipStream_t s);
// piece-pipelined upload: dst[i] = src[i] (u32 -> u64); dst[k] = k % V (identity rows)
void widen_u32(uint64_t *dst, const uint32_t *src, uint64_t count, hipStream_t s);
void iota_rows(uint32_t *dst, uint64_t count, uint32_t V, hipStream_t s);
// first loss entry outside [0, 1] of [k0, k0 + count) atomic-min'ed into *d_first
void loss_check(const float *d_loss, uint64_t count, uint64_t k0, unsigned long long *d_first, hipStream_t s);
// u16-key plans: u16 latency units, then the f32 losses at byte offset loss_off
void pack_paths6(srt_plan *p, uint64_t first, uint64_t count, void *dst, uint64_t loss_off, hipStream_t s);
// 5-byte records (lmax <= 510): u8 units, then the loss bits with the 9th unit bit in the sign
void pack_paths5(srt_plan *p, uint64_t first, uint64_t count, void *dst, uint64_t loss_off, hipStream_t s);
// kernels (srt_sssp.hip)
srt_status sssp_run(srt_plan *p, unsigned long long *d_stats, srt_err *err);
// kernels (srt_frontier.hip): the latency-first frontier sweeps
srt_status frontier_run(srt_plan *p, unsigned long long *d_stats, srt_err *err);
uint64_t frontier_block_bytes(uint32_t V, uint64_t E);
size_t frontier_chg_bytes();
void reduce_rank_stats(srt_plan *p, int nranks);
}  // namespace srt
