// srt_frontier.hip -- latency-first batched sparse SSSP over a ballot-compacted
// frontier, gfx950.
//
// Replaces NetworkGraph::compute_shortest_paths (src/main/network/graph/mod.rs:183-228)
// for sparse graphs (config C4: 100k-node AS-like graph, average degree 8) when
// every finite shortest latency is below 0xFFFF units of g (the eccentricity
// proof, srt_fw.hip fw_ecc_bound; C4: ~750 units).  The reference runs one
// petgraph Dijkstra per in-use source (mod.rs:195-198); here 512 sources
// ("a block") move together through two label-correcting phases:
//
//  1. Latency.  L[b][v][512] u16: one 128-B line holds a 64-source word of one
//     vertex, so a gather along an in-edge costs one line per changed word (the
//     packed u64 (latency, loss) key of srt_sssp.hip cost four).  Relaxation
//     is v_pk_add_u16 (clamp) + v_pk_min_u16, 8 sources a lane.
//  2. Tightness.  One pass stores, per (in-edge, lane), the 8-bit mask of the
//     lane's sources for which the edge ends a shortest path: L(s,u) + w ==
//     L(s,v) (the loss of a pair is the left fold along tight
//     edges only).
//  3. Loss.  P[b][v][512] f32 from 2.0 ("not reached"), sources 0:
//     P(s,v) = min over tight in-edges of 1 - (1 - P(s,u)) * (1 - e), one
//     rounding per op (mod.rs:322-331, __fmul_rn, -ffp-contract=off), folded
//     only from reached parents (P <= 1).  The fold is monotone in P(s,u), so
//     the label-correcting fixpoint over the tight DAG is petgraph's
//     lexicographic (latency, loss) minimum bit for bit; and since a parent is
//     reached only with its final loss when it has one tight parent itself
//     (1.007 tight in-edges per pair at C4), most pairs are written once.
//
// Frontier.  Items are (block, vertex).  act[b][v] holds the sweep that must
// process the item; a wave that improves (b, v) in sweep t stores t + 1 into
// act[b][x] of every out-neighbour x.  Sweep t's waves scan act in 64-item
// chunks, ballot the entries >= t (a mark for t + 1 may have overwritten one
// for t during the sweep: the item is then processed in both) and process only
// those -- the grid is capped at a few workgroups per CU, so a sweep costs its
// active items plus one coalesced 256-B scan per chunk, not a dispatch per
// vertex.  chg[b][v] = (sweep << 8) | changed words: a reader in sweep t
// gathers word w of u only if u changed it in sweep t - 1 or t (Gauss-Seidel:
// values written earlier in the same sweep may be read; every write also marks
// the readers for the next sweep).  Sweep stamps only grow (across phases,
// launches and builds), so neither array is ever cleared.
//
// Order: items are block-major, so the waves of a sweep work through one or
// two blocks at a time and the rows they gather (100 MB a block at C4) stay
// in the Infinity Cache; sources enter blocks in BFS order (srt_api.cpp
// bfs_rank), so a word's sources change at the same vertices in the same
// sweeps.
#include <algorithm>
#include <cstdio>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr uint32_t FR_SRC = 512;     // sources per block (8 words of 64)
constexpr int FR_WAVES = 4;          // waves per sweep workgroup
constexpr int FR_EB = 8;              // edges gathered per batch (loads in flight per lane)
constexpr int FR_EBL = 2;            // loss sweep: edges gathered per batch (2 x 16 B a lane each)
constexpr int FR_MG = 8;             // loss sweep: in-edges whose masks load together (multiple of 4)
constexpr uint32_t L16_INF = 0xffffu;

// The sweeps are latency-bound chains of dependent gathers: 8 waves a SIMD
// (<= 64 VGPRs, a few bytes of spill) beat fewer, fatter waves -- C4 1.03 s
// at 5 waves/SIMD (92 VGPRs, 4 loss edges a batch) -> 0.79 s.
#define FR_OCC __attribute__((amdgpu_waves_per_eu(8, 8)))
#ifndef FR_COUNT
#define FR_COUNT 0
#endif

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_add_sat(uint32_t x, uint32_t w2) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, x),
                                                                      __builtin_bit_cast(u16x2, w2)));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, x),
                                                                  __builtin_bit_cast(u16x2, y)));
}
__device__ __forceinline__ uint4 relax8(uint4 best, uint4 x, uint32_t w2) {
    best.x = pk_min(best.x, pk_add_sat(x.x, w2));
    best.y = pk_min(best.y, pk_add_sat(x.y, w2));
    best.z = pk_min(best.z, pk_add_sat(x.z, w2));
    best.w = pk_min(best.w, pk_add_sat(x.w, w2));
    return best;
}
// bit i of the result: source i of the lane's 8 -- (x_i + w == own_i), both finite
__device__ __forceinline__ uint32_t tight8(uint4 x, uint4 own, uint32_t w) {
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, os[4] = {own.x, own.y, own.z, own.w};
    uint32_t m = 0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t a = (xs[h] >> (16 * k)) & 0xffffu, o = (os[h] >> (16 * k)) & 0xffffu;
            if (a != L16_INF && o != L16_INF && a + w == o) m |= 1u << (2 * h + k);
        }
    }
    return m;
}
// the fold of mod.rs:322-331 with eb = 1 - edge loss (rounded once, f32)
__device__ __forceinline__ float fold(float a, float eb) { return 1.0f - __fmul_rn(1.0f - a, eb); }


// Change record of (b, v): the sweep that last improved it and the lanes
// whose sources improved (a lane = 8 sources), one 16-B store so a reader
// sees a consistent pair.
struct Chg {
    uint32_t stamp, pad;
    uint64_t lanes;
};

// The marks of v's out-neighbours for sweep t + 1, plain stores (stamps only
// grow, and final items are flagged apart, so a mark never lowers anything and
// needs no read first).  Latency-symmetric graphs: the out-neighbours are the
// in-edge sources [e0, e1); else the CSR row.
__device__ __forceinline__ void mark_rows(uint32_t *act_b, uint32_t v, uint32_t t, bool sym, const InEdge *in_edge,
                                          uint64_t e0, uint64_t e1, const uint64_t *__restrict__ row_ptr,
                                          const uint32_t *__restrict__ col, int lane) {
    if (sym) {
        for (uint64_t k = e0 + lane; k < e1; k += 64) act_b[in_edge[k].u] = t + 1;
    } else {
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t x = col[k];
            if (x != v) act_b[x] = t + 1;
        }
    }
}
// the same with the in-edge sources already in the lanes' registers (eu_last:
// the last in-edge chunk, the only one at <= 64 in-edges)
__device__ __forceinline__ void mark(uint32_t *act_b, uint32_t v, uint32_t t, bool sym, const InEdge *in_edge,
                                     uint32_t eu_last, uint64_t e0, uint64_t e1, const uint64_t *__restrict__ row_ptr,
                                     const uint32_t *__restrict__ col, int lane) {
    if (sym && e1 - e0 <= 64) {
        if (e0 + lane < e1) act_b[eu_last] = t + 1;
    } else {
        mark_rows(act_b, v, t, sym, in_edge, e0, e1, row_ptr, col, lane);
    }
}

// Dense sweeps.  In the heavy sweeps of a phase nearly every item of the
// launch is marked and improves (C4: 4.7M of 4.9M items in each of ~10 loss
// sweeps), so the activity flags and the marks cost stores and scans for
// nothing.  ctl[t & 3] counts the items sweep t improved, ctl[4 + (t & 3)] says
// that sweep t stored no marks.  Sweep t runs dense (every item, no activity
// read) if sweep t - 1 improved more than dense_min items or stored no marks,
// and stores no marks if sweep t - 1 improved more than nomark_min
// (> dense_min): a sweep after one that stored none is dense, so no mark is
// ever missing.  The host zeroes ctl before a phase (sweep t0 -- the seeds --
// counts 0: sweep t0 + 1 runs on the seeds' marks).
struct SweepMode {
    bool dense, mark;
};
__device__ __forceinline__ SweepMode sweep_mode(uint32_t *ctl, uint32_t t, uint32_t dense_min, uint32_t nomark_min) {
    const uint32_t pc = ctl[(t - 1) & 3], pn = ctl[4 + ((t - 1) & 3)];
    SweepMode m;
    m.dense = pn != 0 || pc > dense_min;
    m.mark = pc <= nomark_min;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // sweep t + 1 counts from 0; this sweep's mark flag
        ctl[(t + 1) & 3] = 0;
        ctl[4 + (t & 3)] = m.mark ? 0u : 1u;
    }
    return m;
}
__device__ __forceinline__ void count_improved(uint32_t *ctl, uint32_t t, uint32_t n, int lane) {
    if (lane == 0 && n) atomicAdd(&ctl[t & 3], n);
}

// the phase's last-improvement stamp, once per wave at the end of a sweep
// (every improving wave stores the same value: read first, a hot word)
__device__ __forceinline__ void note_improved(uint32_t *last, uint32_t t, bool any, int lane) {
    if (__ballot(any) && lane == 0 && __builtin_nontemporal_load(last) != t) *last = t;
}

// the lanes of u that changed in sweep t - 1 or t (0 if none)
__device__ __forceinline__ uint64_t changed_lanes(const Chg *chg_b, uint32_t u, uint32_t t) {
    const Chg c = chg_b[u];
    return c.stamp + 1 >= t ? c.lanes : 0ull;
}

// -------------------------------------------------------------- seeds
// slot q of the launch (q < nsrc): block q / 512, source q % 512 of it; the
// table row is perm[q0 + q] (perm null: q0 + q), the source vertex nodes[row].
// Phase 1 (L given): L = 0 and the source's lane marked changed in sweep t0;
// phase 3: P = 0 and the source's change bit set.  Either way its
// out-neighbours are marked for sweep t0 + 1.
__global__ void fr_seed_kernel(uint16_t *__restrict__ L, float *__restrict__ P, uint8_t *__restrict__ sbits, Chg *chg,
                               uint32_t *act, const uint32_t *__restrict__ nodes, const uint32_t *__restrict__ perm,
                               uint32_t V, uint32_t q0, uint32_t nsrc, uint32_t t0,
                               const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nsrc) return;
    const uint32_t b = q / FR_SRC, i = q % FR_SRC;
    const uint32_t src = nodes[perm ? perm[q0 + q] : q0 + q];
    const uint64_t row = (uint64_t)b * V + src;
    uint32_t *act_b = act + (uint64_t)b * V;
    if (L) {
        L[row * FR_SRC + i] = 0;
        Chg c;
        c.stamp = t0;
        c.pad = 0;
        c.lanes = 1ull << (i / 8);  // sources of a launch are distinct vertices
        chg[row] = c;
    } else {
        P[row * FR_SRC + i] = 0.0f;
        sbits[row * 64 + i / 8] = (uint8_t)(1u << (i % 8));  // the source's own change bit
    }
    for (uint64_t k = row_ptr[src]; k < row_ptr[src + 1]; ++k) {
        const uint32_t x = col[k];
        if (x != src) act_b[x] = t0 + 1;
    }
}

// Symmetric seeding (undirected graphs: L(s, v) = L(v, s)).  The rows of
// earlier launches are exact, so for every source s_i of this launch and
// every source v of an earlier block b', L[b][v][i] = L[b'][s_i][i'] -- a
// 64 x 64 tile transpose through LDS per (block pair, chunk pair).
// blockIdx.x: (b - B0) * 8 + chunk of i; blockIdx.y: b' * 8 + chunk of i'.
__global__ __launch_bounds__(256) void fr_sym_copy_kernel(uint16_t *L, const uint32_t *__restrict__ nodes,
                                                          const uint32_t *__restrict__ perm, uint32_t V,
                                                          uint32_t row0, uint32_t row1, uint32_t B0) {
    __shared__ uint16_t tile[64][66];
    __shared__ uint32_t sv[64], dv[64];
    const uint32_t b = B0 + blockIdx.x / 8, i0 = (blockIdx.x % 8) * 64;
    const uint32_t bp = blockIdx.y / 8, j0 = (blockIdx.y % 8) * 64;
    const int tid = threadIdx.x;
    if (tid < 64) {
        const uint32_t qa = row0 + b * FR_SRC + i0 + tid, qb = row0 + bp * FR_SRC + j0 + tid;
        sv[tid] = qa < row1 ? nodes[perm ? perm[qa] : qa] : ~0u;  // this launch's sources s_i
        dv[tid] = qb < row1 ? nodes[perm ? perm[qb] : qb] : ~0u;  // earlier sources v_j
    }
    __syncthreads();
    // read: row s_i of block b', entries j0 .. j0+63 (128 B, 2 B a thread)
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int ii = idx / 64, jj = idx % 64;
        uint16_t x = L16_INF;
        if (sv[ii] != ~0u) x = L[((uint64_t)bp * V + sv[ii]) * FR_SRC + j0 + jj];
        tile[jj][ii] = x;
    }
    __syncthreads();
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int jj = idx / 64, ii = idx % 64;
        if (dv[jj] != ~0u) L[((uint64_t)b * V + dv[jj]) * FR_SRC + i0 + ii] = tile[jj][ii];
    }
}

// Symmetric seeding, activity: an item (b, v) whose v is a source of an
// earlier block (done[v] < B0) is final -- fin = 1, changed in every lane in
// sweep t0; every other item is active in sweep t0 + 1.
__global__ void fr_sym_act_kernel(uint32_t *act, uint8_t *fin, Chg *chg, const uint32_t *__restrict__ done, uint32_t V,
                                  uint32_t NB, uint32_t B0, uint32_t t0) {
    const uint64_t n = (uint64_t)NB * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = (uint32_t)(e % V);
        const bool f = done[v] < B0;
        fin[e] = f;
        act[e] = t0 + 1;
        if (f) {
            Chg c;
            c.stamp = t0;
            c.pad = 0;
            c.lanes = ~0ull;
            chg[e] = c;
        }
    }
}

// ------------------------------------------------------- latency sweep
// One wave per active item (b, v): the 8 sources of lane l are 8l .. 8l+7.
// Per 64 in-edges: one edge and its source's changed lanes per lane, a ballot
// of the edges whose source changed in sweep t-1 or t, then batches of FR_EB
// gathers (16 B a lane, only the lanes whose sources changed) and the packed
// relaxation.  The own row is loaded first (independent of the chain).
__global__ __launch_bounds__(FR_WAVES * 64) FR_OCC void fr_lat_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V, uint32_t NB,
    uint16_t *L, Chg *chg, uint32_t *act, const uint8_t *__restrict__ fin, uint32_t *last, uint32_t t, bool sym,
    const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col, uint32_t *ctl, uint32_t dense_min,
    uint32_t nomark_min) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * FR_WAVES + (threadIdx.x >> 6), nwaves = gridDim.x * FR_WAVES;
    const uint32_t cpb = (V + 63) / 64, nchunks = cpb * NB;
    bool any_imp = false;
    uint32_t n_imp = 0;
    const SweepMode md = sweep_mode(ctl, t, dense_min, nomark_min);
    for (uint32_t c = __builtin_amdgcn_readfirstlane(wave); c < nchunks; c += nwaves) {
        const uint32_t b = c / cpb, v0 = (c % cpb) * 64;
        uint32_t *act_b = act + (uint64_t)b * V;
        const bool in = v0 + lane < V;
        const uint32_t a = in && !md.dense ? act_b[v0 + lane] : 0u;
        const bool f = in && fin[(uint64_t)b * V + v0 + lane];
        uint64_t items = __ballot((md.dense ? in : a >= t) && !f);
        uint4 *Lb = reinterpret_cast<uint4 *>(L + (uint64_t)b * V * FR_SRC);
        Chg *chg_b = chg + (uint64_t)b * V;
        if (!items) continue;
        // software-pipelined like the loss sweep: the next item's head (row
        // bounds, first 64 in-edges and their sources' change records) is
        // loaded while the current item's gathers are in flight.  A record
        // read early may miss a change of this sweep; its writer marked v for
        // sweep t + 1 anyway.
        uint32_t v = v0 + __builtin_ctzll(items);
        items &= items - 1;
        uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
        uint32_t eu = 0, ew = 0;
        uint64_t m = 0;
        if (e0 + lane < e1) {
            const InEdge e = in_edge[e0 + lane];
            eu = e.u;
            ew = e.w < L16_INF ? e.w : L16_INF;
            m = changed_lanes(chg_b, eu, t);
        }
        for (;;) {
            const bool more = items != 0;
            const uint32_t vn = more ? v0 + __builtin_ctzll(items) : v;
            if (more) items &= items - 1;
            // candidates only; the own row is read at the end by the lanes
            // that gathered anything (most lanes of an active item gather
            // nothing: reading every row cost 1 KB an item a sweep)
            uint4 best = make_uint4(~0u, ~0u, ~0u, ~0u);
            bool gat = false;
            const Chg old = chg_b[v];  // own record, for the kept lanes
            uint64_t ne0 = 0, ne1 = 0, nm = 0;
            uint32_t neu = 0, new_ = 0;
            bool pre = !more;
            for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
                if (c0 != e0) {  // chunks past the head
                    const uint64_t k = c0 + lane;
                    eu = 0;
                    ew = 0;
                    m = 0;
                    if (k < e1) {
                        const InEdge e = in_edge[k];
                        eu = e.u;
                        ew = e.w < L16_INF ? e.w : L16_INF;
                        m = changed_lanes(chg_b, eu, t);
                    }
                }
                uint64_t am = __ballot(m != 0);
                while (am) {
                    uint4 x[FR_EB];
                    uint32_t w2[FR_EB];
#pragma unroll
                    for (int q = 0; q < FR_EB; ++q) {
                        x[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
                        w2[q] = 0;
                        if (am) {
                            const int j = __builtin_ctzll(am);
                            am &= am - 1;
                            const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                            const uint32_t w = __builtin_amdgcn_readlane(ew, j);
                            const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)m, j);
                            const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(m >> 32), j);
                            w2[q] = w | (w << 16);
                            if (((lane < 32 ? mlo : mhi) >> (lane & 31)) & 1u) {
                                x[q] = Lb[(uint64_t)u * 64 + lane];
                                gat = true;
                            }
                        }
                    }
                    if (!pre) {  // the next item's head, behind this batch's gathers
                        pre = true;
                        ne0 = in_ptr[vn];
                        ne1 = in_ptr[vn + 1];
                        if (ne0 + lane < ne1) {
                            const InEdge e = in_edge[ne0 + lane];
                            neu = e.u;
                            new_ = e.w < L16_INF ? e.w : L16_INF;
                            nm = changed_lanes(chg_b, neu, t);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < FR_EB; ++q) best = relax8(best, x[q], w2[q]);
                }
            }
            if (!pre) {  // nothing gathered for v
                ne0 = in_ptr[vn];
                ne1 = in_ptr[vn + 1];
                if (ne0 + lane < ne1) {
                    const InEdge e = in_edge[ne0 + lane];
                    neu = e.u;
                    new_ = e.w < L16_INF ? e.w : L16_INF;
                    nm = changed_lanes(chg_b, neu, t);
                }
            }
            uint4 own = make_uint4(0u, 0u, 0u, 0u);
            if (gat) {
                own = Lb[(uint64_t)v * 64 + lane];
                best.x = pk_min(best.x, own.x);
                best.y = pk_min(best.y, own.y);
                best.z = pk_min(best.z, own.z);
                best.w = pk_min(best.w, own.w);
            }
            const bool imp = gat && (best.x != own.x || best.y != own.y || best.z != own.z || best.w != own.w);
            const uint64_t im = __ballot(imp);
            if (im) {
                any_imp = true;
                ++n_imp;
                if (imp) Lb[(uint64_t)v * 64 + lane] = best;
                if (lane == 0) {  // this sweep's lanes, and those of sweep t - 1 that readers may still need
                    Chg cnew;
                    cnew.stamp = t;
                    cnew.pad = 0;
                    cnew.lanes = im | (old.stamp + 1 == t ? old.lanes : 0ull);
                    chg_b[v] = cnew;
                }
                if (md.mark) mark(act_b, v, t, sym, in_edge, eu, e0, e1, row_ptr, col, lane);
            }
            if (!more) break;
            v = vn;
            e0 = ne0;
            e1 = ne1;
            eu = neu;
            ew = new_;
            m = nm;
        }
    }
    note_improved(last, t, any_imp, lane);
    count_improved(ctl, t, n_imp, lane);
}

// ---------------------------------------------------------- tight pass
// Every item (b, v): the in-edges k = (u -> v) of v that end a shortest path
// for at least one of the block's 512 sources (C4: about a third of them),
// compacted in in-edge order to positions e0 = in_ptr[v], e0 + 1, ...:
// ce[b * E + e0 + j] = (u, 1 - e) and tight[(b * E + e0 + j) * 64 + lane] =
// the lane's 8-bit mask of sources s with L(s,u) + w == L(s,v);
// cnt[b * V + v] = how many.  The loss sweeps walk only these, so an item's
// scan costs its tight edges, not its degree.  A wave takes 64-vertex chunks,
// as the sweeps do: every chunk holds one hub (slot 0, srt_api.cpp's vertex
// order), so the waves stay balanced -- striding single items by the wave
// count (a multiple of 64) put every hub on the same few waves (C4: 33 -> 90
// ms).
__global__ __launch_bounds__(FR_WAVES * 64) void fr_tight_kernel(const uint64_t *__restrict__ in_ptr,
                                                                 const InEdge *__restrict__ in_edge, uint32_t V,
                                                                 uint32_t NB, uint64_t E,
                                                                 const uint16_t *__restrict__ L,
                                                                 uint8_t *__restrict__ tight, uint2 *__restrict__ ce,
                                                                 uint32_t *__restrict__ cnt, float *__restrict__ P) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * FR_WAVES + (threadIdx.x >> 6), nwaves = gridDim.x * FR_WAVES;
    const uint32_t cpb = (V + 63) / 64, nchunks = cpb * NB;
    for (uint32_t c = __builtin_amdgcn_readfirstlane(wave); c < nchunks; c += nwaves)
    for (uint32_t v = (c % cpb) * 64, vend = std::min(V, v + 64); v < vend; ++v) {
        const uint32_t b = c / cpb;
        const uint4 *Lb = reinterpret_cast<const uint4 *>(L + (uint64_t)b * V * FR_SRC);
        const uint4 own = Lb[(uint64_t)v * 64 + lane];
        uint8_t *tb = tight + (uint64_t)b * E * 64 + lane;
        uint2 *cb = ce + (uint64_t)b * E;
        {  // the loss phase starts from P = 2.0 ("not reached"), stored here beside the reads
            float4 *pv = reinterpret_cast<float4 *>(P + (uint64_t)b * V * FR_SRC) + (uint64_t)v * 128 + 2 * lane;
            const float4 two = make_float4(2.f, 2.f, 2.f, 2.f);
            pv[0] = two;
            pv[1] = two;
        }
        const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
        uint64_t j = e0;  // next compacted position (wave-uniform)
        for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
            const uint64_t k = c0 + lane;
            uint32_t eu = 0, ew = 0, eb = 0;
            if (k < e1) {
                const InEdge e = in_edge[k];
                eu = e.u;
                ew = e.w;
                eb = __float_as_uint(e.eb);
            }
            const uint32_t n = e1 - c0 < 64 ? (uint32_t)(e1 - c0) : 64u;
            const uint64_t jc = j;
            uint64_t keep = 0;  // the chunk's edges kept
            for (uint32_t j0 = 0; j0 < n; j0 += FR_EB) {
                uint4 x[FR_EB];
                uint32_t w[FR_EB];
#pragma unroll
                for (int q = 0; q < FR_EB; ++q) {
                    w[q] = 0;
                    x[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
                    if (j0 + q < n) {
                        const uint32_t u = __builtin_amdgcn_readlane(eu, j0 + q);
                        w[q] = __builtin_amdgcn_readlane(ew, j0 + q);
                        x[q] = Lb[(uint64_t)u * 64 + lane];
                    }
                }
#pragma unroll
                for (int q = 0; q < FR_EB; ++q)
                    if (j0 + q < n) {
                        const uint32_t m = tight8(x[q], own, w[q]);
                        if (__ballot(m != 0)) {
                            tb[j * 64] = (uint8_t)m;
                            keep |= 1ull << (j0 + q);
                            ++j;
                        }
                    }
            }
            if ((keep >> lane) & 1ull)
                cb[jc + __builtin_popcountll(keep & ((1ull << lane) - 1ull))] = make_uint2(eu, eb);
        }
        if (lane == 0) cnt[(uint64_t)b * V + v] = (uint32_t)(j - e0);
    }
}

// ---------------------------------------------------------- loss sweep
// Pull over the item's compacted tight in-edges (the tight pass) with
// per-source change bits, double-buffered:
// sb_cur[b][u][lane] = the lane's sources of u whose loss changed in sweep
// t - 1, sb_next = those of sweep t (cleared before it; read as well, so a
// change made earlier in the same sweep is picked up at once, Gauss-Seidel).
// Per in-edge the lane loads its tight byte (in-edge order: the item's edges
// are contiguous) and u's two change bytes; only where they meet does it
// gather u's 8 losses (32 B) and fold the tight ones that are reached (P <= 1;
// 2.0 = not yet).  Chain per item: in-edges -> (tight, change bytes) ->
// gather, the own losses loaded beside the in-edges; marks from registers.
__global__ __launch_bounds__(FR_WAVES * 64) FR_OCC void fr_loss_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V, uint32_t NB, uint64_t E,
    const uint8_t *__restrict__ tight, const uint2 *__restrict__ ce, const uint32_t *__restrict__ tcnt, float *P, const uint8_t *__restrict__ sb_cur, uint8_t *sb_next,
    uint32_t *act, uint32_t *last, uint32_t t, bool sym, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, uint32_t *ctl, uint32_t dense_min, uint32_t nomark_min, unsigned long long *cnt) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * FR_WAVES + (threadIdx.x >> 6), nwaves = gridDim.x * FR_WAVES;
    const uint32_t cpb = (V + 63) / 64, nchunks = cpb * NB;
    bool any_imp = false;
    uint32_t n_imp = 0;
    const SweepMode md = sweep_mode(ctl, t, dense_min, nomark_min);
#if FR_COUNT
    uint32_t c_items = 0, c_work = 0, c_imp = 0, c_gath = 0;  // SRT_FR_COUNT (diagnostic builds)
#endif
    for (uint32_t c = __builtin_amdgcn_readfirstlane(wave); c < nchunks; c += nwaves) {
        const uint32_t b = c / cpb, v0 = (c % cpb) * 64;
        uint32_t *act_b = act + (uint64_t)b * V;
        const uint32_t a = v0 + lane < V && !md.dense ? act_b[v0 + lane] : 0u;
        uint64_t items = __ballot(md.dense ? v0 + lane < V : a >= t);
        float4 *Pb = reinterpret_cast<float4 *>(P + (uint64_t)b * V * FR_SRC);
        const uint8_t *tb = tight + (uint64_t)b * E * 64 + lane;
        const uint2 *cb = ce + (uint64_t)b * E;
        const uint32_t *cnb = tcnt + (uint64_t)b * V;
        const uint8_t *sbc = sb_cur + (uint64_t)b * V * 64 + lane;
        uint8_t *sbn = sb_next + (uint64_t)b * V * 64 + lane;
        if (!items) continue;
        // items are software-pipelined: the next item's in-edge head (row
        // bounds and first 64 in-edges) is loaded while the current one's
        // change bytes are in flight
        uint32_t v = v0 + __builtin_ctzll(items);
        items &= items - 1;
        uint64_t e0 = in_ptr[v], f1 = in_ptr[v + 1];  // [e0, e1): tight, [e0, f1): all in-edges
        uint64_t e1 = e0 + cnb[v];
        uint32_t eu = 0;
        float eeb = 0.f;
        if (e0 + lane < e1) {
            const uint2 e = cb[e0 + lane];
            eu = e.x;
            eeb = __uint_as_float(e.y);
        }
        for (;;) {
            const bool more = items != 0;
            const uint32_t vn = more ? v0 + __builtin_ctzll(items) : v;
            if (more) items &= items - 1;
            float4 *pv = Pb + (uint64_t)v * 128 + 2 * lane;
            // candidates; the own row is read only by the lanes with a tight,
            // changed parent, beside their first gathers (2 KB an item a
            // sweep for every lane otherwise)
            float best[8] = {2.f, 2.f, 2.f, 2.f, 2.f, 2.f, 2.f, 2.f};
            float4 o0 = make_float4(2.f, 2.f, 2.f, 2.f), o1 = o0;
            bool own = false;
            uint64_t ne0 = 0, ne1 = 0, nf1 = 0;
            uint32_t neu = 0;
            float neeb = 0.f;
            bool pre = !more;
            for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
                if (c0 != e0) {  // chunks past the head
                    const uint64_t k = c0 + lane;
                    eu = 0;
                    eeb = 0.f;
                    if (k < e1) {
                        const uint2 e = cb[k];
                        eu = e.x;
                        eeb = __uint_as_float(e.y);
                    }
                }
                const uint32_t n = e1 - c0 < 64 ? (uint32_t)(e1 - c0) : 64u;
                // groups of FR_MG in-edges: every lane's tight & changed mask of
                // the group in one round of loads, then gathers along the edges
                // some lane needs only (the masks of a group packed 4 a register)
                for (uint32_t j0 = 0; j0 < n; j0 += FR_MG) {
                    uint32_t mk[FR_MG / 4];
                    uint32_t amask = 0;  // wave-uniform: the group's edges some lane needs
                    {
                        uint32_t mq[FR_MG];
#pragma unroll
                        for (int q = 0; q < FR_MG; ++q) {
                            mq[q] = 0;
                            if (j0 + q < n) {
                                const uint32_t u = __builtin_amdgcn_readlane(eu, j0 + q);
                                mq[q] = tb[(c0 + j0 + q) * 64] & (sbc[(uint64_t)u * 64] | sbn[(uint64_t)u * 64]);
                            }
                        }
#pragma unroll
                        for (int q = 0; q < FR_MG; ++q) amask |= __ballot(mq[q] != 0) ? 1u << q : 0u;
#pragma unroll
                        for (int r = 0; r < FR_MG / 4; ++r)
                            mk[r] = mq[4 * r] | mq[4 * r + 1] << 8 | mq[4 * r + 2] << 16 | mq[4 * r + 3] << 24;
                    }
                    if (!own) {
                        uint32_t any = 0;
#pragma unroll
                        for (int r = 0; r < FR_MG / 4; ++r) any |= mk[r];
                        if (any) {
                            o0 = pv[0];
                            o1 = pv[1];
                            own = true;
                        }
                    }
                    if (!pre) {  // the next item's head, behind this group's loads
                        pre = true;
                        ne0 = in_ptr[vn];
                        nf1 = in_ptr[vn + 1];
                        ne1 = ne0 + cnb[vn];
                        if (ne0 + lane < ne1) {
                            const uint2 e = cb[ne0 + lane];
                            neu = e.x;
                            neeb = __uint_as_float(e.y);
                        }
                    }
                    while (amask) {
                        uint32_t m[FR_EBL];
                        float eb[FR_EBL];
                        float4 x0[FR_EBL], x1[FR_EBL];
#pragma unroll
                        for (int q = 0; q < FR_EBL; ++q) {
                            m[q] = 0;
                            eb[q] = 0.f;
                            x0[q] = x1[q] = make_float4(2.f, 2.f, 2.f, 2.f);
                            if (amask) {
                                const uint32_t jq = __builtin_ctz(amask);
                                amask &= amask - 1;
                                uint32_t w = mk[0];
#pragma unroll
                                for (int r = 1; r < FR_MG / 4; ++r) w = jq / 4 == (uint32_t)r ? mk[r] : w;
                                m[q] = (w >> (8 * (jq % 4))) & 0xffu;
                                const uint32_t u = __builtin_amdgcn_readlane(eu, j0 + jq);
                                eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j0 + jq));
#if FR_COUNT
                                ++c_gath;
#endif
                                if (m[q]) {
                                    x0[q] = Pb[(uint64_t)u * 128 + 2 * lane];
                                    x1[q] = Pb[(uint64_t)u * 128 + 2 * lane + 1];
                                }
                            }
                        }
#pragma unroll
                        for (int q = 0; q < FR_EBL; ++q) {
                            const float xs[8] = {x0[q].x, x0[q].y, x0[q].z, x0[q].w,
                                                 x1[q].x, x1[q].y, x1[q].z, x1[q].w};
#pragma unroll
                            for (int i = 0; i < 8; ++i)
                                if (((m[q] >> i) & 1u) && xs[i] <= 1.0f) {  // u reached (not the 2.0 init)
                                    const float cnd = fold(xs[i], eb[q]);
                                    best[i] = cnd < best[i] ? cnd : best[i];
                                }
                        }
                    }
                }
            }
            if (!pre) {  // v has no tight in-edge
                ne0 = in_ptr[vn];
                nf1 = in_ptr[vn + 1];
                ne1 = ne0 + cnb[vn];
                if (ne0 + lane < ne1) {
                    const uint2 e = cb[ne0 + lane];
                    neu = e.x;
                    neeb = __uint_as_float(e.y);
                }
            }
            uint32_t ib = 0;  // the lane's improved sources
#if FR_COUNT
            ++c_items;
            c_work += __ballot(own) != 0;
#endif
            if (own) {
                const float ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (best[i] < ov[i]) ib |= 1u << i;
                    else best[i] = ov[i];
                }
            }
            if (__ballot(ib != 0)) {
                any_imp = true;
                ++n_imp;
#if FR_COUNT
                ++c_imp;
#endif
                if (ib) {
                    pv[0] = make_float4(best[0], best[1], best[2], best[3]);
                    pv[1] = make_float4(best[4], best[5], best[6], best[7]);
                    sbn[(uint64_t)v * 64] = (uint8_t)ib;  // only this wave writes v's byte this sweep
                }
                if (md.mark) mark_rows(act_b, v, t, sym, in_edge, e0, f1, row_ptr, col, lane);
            }
            if (!more) break;
            v = vn;
            e0 = ne0;
            e1 = ne1;
            f1 = nf1;
            eu = neu;
            eeb = neeb;
        }
    }
#if FR_COUNT
    if (cnt && lane == 0) {
        atomicAdd(&cnt[0], (unsigned long long)c_items);
        atomicAdd(&cnt[1], (unsigned long long)c_work);
        atomicAdd(&cnt[2], (unsigned long long)c_imp);
        atomicAdd(&cnt[3], (unsigned long long)c_gath);
    }
#else
    (void)cnt;
#endif
    note_improved(last, t, any_imp, lane);
    count_improved(ctl, t, n_imp, lane);
}

// ---------------------------------------------------------------- emit
// Table rows of the launch: slot q -> row perm[q0 + q].  A 64 x 64 (slots x
// columns) tile through LDS: each column's 64 slots are one 128-B run of L
// and one 256-B run of P; the rows are stored coalesced.  Diagonal = the raw
// self-loop (mod.rs:210-217); min latency (mod.rs:474-476) and unreachable
// count (the assert at mod.rs:219) block-reduced into stats.
__global__ __launch_bounds__(256) void fr_emit_kernel(const uint16_t *__restrict__ L, const float *__restrict__ P,
                                                      uint32_t V, const uint32_t *__restrict__ nodes,
                                                      const uint32_t *__restrict__ perm, uint32_t n, uint32_t q0,
                                                      uint32_t nsrc, uint64_t gunit,
                                                      const uint64_t *__restrict__ sl_lat,
                                                      const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat,
                                                      float *__restrict__ out_loss, unsigned long long *stats) {
    __shared__ uint16_t tl[64][66];  // [column][slot]
    __shared__ float tp[64][65];
    __shared__ uint32_t rows[64], cols[64];
    __shared__ unsigned long long red_min[4], red_cnt[4];
    const uint32_t s0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    const uint32_t b = s0 / FR_SRC, o = s0 % FR_SRC;
    const int tid = threadIdx.x;
    if (tid < 64) {
        const uint32_t j = j0 + tid, q = s0 + tid;
        cols[tid] = j < n ? nodes[j] : ~0u;
        rows[tid] = q < nsrc ? (perm ? perm[q0 + q] : q0 + q) : ~0u;
    }
    __syncthreads();
    // 1. each column's 64 slots: 128 B of L (8 x 16 B) and 256 B of P (16 x 16 B)
    for (int idx = tid; idx < 64 * 8; idx += 256) {
        const int jj = idx / 8, part = idx % 8;
        uint4 x = make_uint4(~0u, ~0u, ~0u, ~0u);
        if (cols[jj] != ~0u)
            x = *reinterpret_cast<const uint4 *>(L + ((uint64_t)b * V + cols[jj]) * FR_SRC + o + part * 8);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            tl[jj][part * 8 + 2 * h] = (uint16_t)w[h];
            tl[jj][part * 8 + 2 * h + 1] = (uint16_t)(w[h] >> 16);
        }
    }
    for (int idx = tid; idx < 64 * 16; idx += 256) {
        const int jj = idx / 16, part = idx % 16;
        float4 x = make_float4(1.f, 1.f, 1.f, 1.f);
        if (cols[jj] != ~0u)
            x = *reinterpret_cast<const float4 *>(P + ((uint64_t)b * V + cols[jj]) * FR_SRC + o + part * 4);
        tp[jj][part * 4] = x.x;
        tp[jj][part * 4 + 1] = x.y;
        tp[jj][part * 4 + 2] = x.z;
        tp[jj][part * 4 + 3] = x.w;
    }
    __syncthreads();
    // 2. rows: latency as 2 columns (16 B) a lane, loss as 4 (16 B) a lane
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
    for (int idx = tid; idx < 64 * 32; idx += 256) {
        const int s = idx / 32, jj = (idx % 32) * 2;
        const uint32_t row = rows[s];
        if (row == ~0u || j0 + jj >= n) continue;
        uint64_t v2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t j = j0 + jj + k;
            const uint16_t l = tl[jj + k][s];
            uint64_t lat = row == j ? sl_lat[j] : l == L16_INF ? ~0ull : (uint64_t)l * gunit;
            if (j >= n) lat = ~0ull;
            else {
                unreach += (row != j && l == L16_INF);
                mn = lat < mn ? lat : mn;
            }
            v2[k] = lat;
        }
        uint64_t *dst = out_lat + (uint64_t)row * n + j0 + jj;
        if (j0 + jj + 1 < n && ((uintptr_t)dst & 15) == 0) {
            *reinterpret_cast<ulonglong2 *>(dst) = make_ulonglong2(v2[0], v2[1]);
        } else {
            dst[0] = v2[0];
            if (j0 + jj + 1 < n) dst[1] = v2[1];
        }
    }
    for (int idx = tid; idx < 64 * 16; idx += 256) {
        const int s = idx / 16, jj = (idx % 16) * 4;
        const uint32_t row = rows[s];
        if (row == ~0u || j0 + jj >= n) continue;
        float v4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = j0 + jj + k;
            v4[k] = j >= n ? 1.0f : row == j ? sl_loss[j] : tl[jj + k][s] == L16_INF ? 1.0f : tp[jj + k][s];
        }
        float *dst = out_loss + (uint64_t)row * n + j0 + jj;
        if (j0 + jj + 3 < n && ((uintptr_t)dst & 15) == 0) {
            *reinterpret_cast<float4 *>(dst) = make_float4(v4[0], v4[1], v4[2], v4[3]);
        } else {
            for (int k = 0; k < 4 && j0 + jj + k < n; ++k) dst[k] = v4[k];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t x = __shfl_xor(mn, off);
        mn = x < mn ? x : mn;
        unreach += __shfl_xor(unreach, off);
    }
    const int w = tid >> 6;
    if ((tid & 63) == 0) {
        red_min[w] = mn;
        red_cnt[w] = unreach;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], cnt = red_cnt[0];
        for (int k = 1; k < 4; ++k) {
            m = red_min[k] < m ? red_min[k] : m;
            cnt += red_cnt[k];
        }
        atomicMin(&stats[0], m);
        if (cnt) atomicAdd(&stats[1], cnt);
    }
}

__global__ void fr_stats_init_kernel(unsigned long long *stats) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
}

srt_status hip_err(srt_err *err, hipError_t e, const char *what) {
    if (err) {
        err->code = SRT_ERR_HIP;
        std::snprintf(err->msg, sizeof err->msg, "%s: %s", what, hipGetErrorString(e));
    }
    return SRT_ERR_HIP;
}

// Sweeps t0 + 1, t0 + 2, ... of one phase until one improves nothing.  The
// host reads the phase's last-improvement stamp after each chunk of sweeps
// (sweeps past convergence find no marked item and cost one act scan).
// Returns the last sweep enqueued in *t_end and the productive count in *n.
template <typename F>
srt_status run_phase(srt_plan *p, uint32_t t0, uint32_t chunk, F sweep, uint32_t *t_end, uint32_t *n, srt_err *err) {
    hipStream_t M = p->stream;
    uint32_t t = t0;
    for (;;) {
        for (uint32_t c = 0; c < chunk; ++c) sweep(++t);
        hipError_t e = hipMemcpyAsync(p->h_fimp, p->d_fimp, 4, hipMemcpyDeviceToHost, M);
        if (e == hipSuccess) e = hipStreamSynchronize(M);
        if (e != hipSuccess) return hip_err(err, e, "sparse frontier sweep");
        const uint32_t last = *p->h_fimp;
        if (last < t) {  // sweep t improved nothing (nor did any later than `last`)
            *t_end = t;
            *n = last > t0 ? last - t0 : 0;
            return SRT_OK;
        }
        if (t - t0 > p->sssp_tmax) {  // Bellman-Ford bound: cannot happen with positive latencies
            if (err) {
                err->code = SRT_ERR_INVALID;
                std::snprintf(err->msg, sizeof err->msg, "sssp did not converge after %u sweeps", t - t0);
            }
            return SRT_ERR_INVALID;
        }
        chunk = 2;
    }
}

}  // namespace

// One pass over this rank's table rows [row0, row1), fr_nb blocks of 512
// sources a launch.  Returns with the stream drained up to the last emit.
srt_status frontier_run(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    const uint64_t E = p->n_in_edges;
    Chg *chg = reinterpret_cast<Chg *>(p->d_fchg);
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->sssp_sweeps = 0;
    p->fr_lat_sweeps = p->fr_loss_sweeps = 0;
    hipError_t e;
    const uint32_t rows = p->row1 - p->row0;
    // symmetric seeding needs every block of this rank's rows resident
    const bool sym = p->fr_sym && p->fr_lblocks * FR_SRC >= rows;
    // the BFS source order of this rank's rows and, per vertex, the block in
    // which it is a source (built once per row range), uploaded on the plan's
    // stream from host copies the plan keeps
    // launches: blocks of 512 rows in equal shares of at most fr_nb blocks;
    // with symmetric seeding optionally a smaller first launch (fr_first
    // blocks: the only launch whose latency phase starts from the sources
    // alone)
    std::vector<uint32_t> lblk;
    {
        const uint32_t blocks = (rows + FR_SRC - 1) / FR_SRC;
        uint32_t rest = blocks;
        if (sym && p->fr_first && p->fr_first < blocks) {
            lblk.push_back(p->fr_first);
            rest -= p->fr_first;
        }
        const uint32_t k = (rest + p->fr_nb - 1) / p->fr_nb;
        for (uint32_t i = 0; i < k; ++i) lblk.push_back(rest / k + (i < rest % k));
    }
    const uint32_t *perm = nullptr;
    if (p->row1 > p->row0 && (!p->d_fdone || p->sperm_r0 != p->row0 || p->sperm_r1 != p->row1)) {
        const bool bfs = !p->h_bfs_rank.empty();
        if (bfs) {
            p->h_sperm.resize(p->n);
            for (uint32_t i = 0; i < p->n; ++i) p->h_sperm[i] = i;
            std::stable_sort(p->h_sperm.begin() + p->row0, p->h_sperm.begin() + p->row1, [&](uint32_t a, uint32_t b) {
                return p->h_bfs_rank[p->nodes[a]] < p->h_bfs_rank[p->nodes[b]];
            });
            // within each launch: shortest-latency-tree level order (srt_api.cpp
            // spt_rank), so a lane's and a line's sources change together
            if (!p->h_spt_rank.empty())
                for (uint32_t li = 0, q = 0; li < lblk.size(); q += lblk[li++] * FR_SRC) {
                    auto b0 = p->h_sperm.begin() + p->row0 + q;
                    auto b1 = p->h_sperm.begin() + p->row0 + std::min<uint32_t>(rows, q + lblk[li] * FR_SRC);
                    std::stable_sort(b0, b1, [&](uint32_t a, uint32_t b) {
                        return p->h_spt_rank[p->nodes[a]] < p->h_spt_rank[p->nodes[b]];
                    });
                }
        }
        p->h_fdone.assign(V, ~0u);
        for (uint32_t q = 0; q < rows; ++q)
            p->h_fdone[p->h_fnodes[bfs ? p->h_sperm[p->row0 + q] : p->row0 + q]] = q / FR_SRC;
        e = hipSuccess;
        if (bfs && !p->d_sperm) e = hipMalloc(&p->d_sperm, (size_t)p->n * 4);
        if (e == hipSuccess && !p->d_fdone) e = hipMalloc(&p->d_fdone, (size_t)std::max<uint32_t>(V, 1) * 4);
        if (e == hipSuccess && bfs)
            e = hipMemcpyAsync(p->d_sperm, p->h_sperm.data(), (size_t)p->n * 4, hipMemcpyHostToDevice, M);
        if (e == hipSuccess) e = hipMemcpyAsync(p->d_fdone, p->h_fdone.data(), (size_t)V * 4, hipMemcpyHostToDevice, M);
        if (e != hipSuccess) return hip_err(err, e, "sssp source order");
        p->sperm_r0 = p->row0;
        p->sperm_r1 = p->row1;
    }
    if (!p->h_bfs_rank.empty()) perm = p->d_sperm;
    // sweep stamps: start over (zeroed) long before they wrap
    if (p->fr_t > (1u << 30)) {
        if ((e = hipMemsetAsync(p->d_fchg, 0, (size_t)p->fr_nb * V * sizeof(Chg), M)) != hipSuccess ||
            (e = hipMemsetAsync(p->d_fact, 0, (size_t)p->fr_nb * V * 4, M)) != hipSuccess)
            return hip_err(err, e, "sssp stamps");
        p->fr_t = 1;
    }
    hipLaunchKernelGGL(fr_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats);
    const uint32_t launches = (uint32_t)lblk.size();
    while (p->ev.size() < 2 * (size_t)launches) {
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, 0);
        p->ev.push_back(ev);
    }
    const dim3 sgrid(p->fr_grid), sblk(FR_WAVES * 64);
    uint32_t chunk_lat = 12, chunk_loss = 12;
    // dense sweeps past half the launch's items improved, no marks past three
    // quarters (C4: 0.511 s without, 0.490 with; thresholds 30/60, 25/50 and
    // 60/85 % measured within 0.5%).  Knob SRT_FR_DENSE=0 (A/B, tests).
    const char *kd = std::getenv("SRT_FR_DENSE");
    const bool dense_on = !(kd && std::atoi(kd) == 0);
    for (uint32_t li = 0, B0 = 0; li < launches; B0 += lblk[li++]) {
        const uint32_t q0 = p->row0 + B0 * FR_SRC;
        const uint32_t nsrc = std::min<uint32_t>(lblk[li] * FR_SRC, p->row1 - q0);
        const uint32_t NB = (nsrc + FR_SRC - 1) / FR_SRC;
        uint16_t *L = p->d_fl + (sym ? (uint64_t)B0 * V * FR_SRC : 0);
        const dim3 seed_grid((nsrc + 255) / 256);
        (void)hipEventRecord(p->ev[2 * li], M);
        // 1. latency: INF, the exact columns of earlier launches (symmetric
        //    graphs), the sources
        if ((e = hipMemsetAsync(L, 0xff, (size_t)NB * V * FR_SRC * 2, M)) != hipSuccess)
            return hip_err(err, e, "sssp init");
        const uint64_t items = (uint64_t)NB * V;
        const uint32_t dmin = dense_on ? (uint32_t)std::min<uint64_t>(items / 2, ~0u) : ~0u;
        const uint32_t nmin = dense_on ? (uint32_t)std::min<uint64_t>(items * 3 / 4, ~0u) : ~0u;
        if ((e = hipMemsetAsync(p->d_fctl, 0, 8 * 4, M)) != hipSuccess) return hip_err(err, e, "sssp init");
        uint32_t t0 = ++p->fr_t;
        if (sym && B0 > 0) {
            hipLaunchKernelGGL(fr_sym_copy_kernel, dim3(NB * 8, B0 * 8), dim3(256), 0, M, p->d_fl, p->d_fnodes, perm, V,
                               p->row0, p->row1, B0);
            hipLaunchKernelGGL(fr_sym_act_kernel, dim3(2048), dim3(256), 0, M, p->d_fact, p->d_ffin, chg, p->d_fdone, V,
                               NB, B0, t0);
        } else if ((e = hipMemsetAsync(p->d_fact, 0, (size_t)NB * V * 4, M)) != hipSuccess ||
                   (e = hipMemsetAsync(p->d_ffin, 0, (size_t)NB * V, M)) != hipSuccess) {
            return hip_err(err, e, "sssp init");
        }
        hipLaunchKernelGGL(fr_seed_kernel, seed_grid, dim3(256), 0, M, L, nullptr, nullptr, chg, p->d_fact, p->d_fnodes,
                           perm, V, q0, nsrc, t0, p->d_frow_ptr, p->d_fcol);
        uint32_t t_end = 0, nsw = 0;
        srt_status st = run_phase(p, t0, chunk_lat, [&](uint32_t t) {
            hipLaunchKernelGGL(fr_lat_sweep_kernel, sgrid, sblk, 0, M, p->d_in_ptr, p->d_in_edge, V, NB, L, chg,
                               p->d_fact, p->d_ffin, p->d_fimp, t, p->fr_symg, p->d_frow_ptr, p->d_fcol, p->d_fctl, dmin, nmin);
        }, &t_end, &nsw, err);
        if (st != SRT_OK) return st;
        p->fr_lat_sweeps += nsw;
        p->sssp_sweeps += nsw;
        chunk_lat = std::max<uint32_t>(nsw + 1, 4);
        // 2. tight masks
        hipLaunchKernelGGL(fr_tight_kernel, sgrid, sblk, 0, M, p->d_in_ptr, p->d_in_edge, V, NB, E, L, p->d_ftight,
                           p->d_fce, p->d_fcnt, p->d_fp);
        // 3. loss (P = 2.0 stored by the tight pass; activity cleared of the
        //    final marks; change bits double-buffered)
        const size_t sbytes = (size_t)NB * V * 64;
        if ((e = hipMemsetAsync(p->d_fact, 0, (size_t)NB * V * 4, M)) != hipSuccess ||
            (e = hipMemsetAsync(p->d_fsb, 0, sbytes, M)) != hipSuccess ||
            (e = hipMemsetAsync(p->d_fctl, 0, 8 * 4, M)) != hipSuccess)
            return hip_err(err, e, "sssp loss init");
        t0 = t_end + 2;
        hipLaunchKernelGGL(fr_seed_kernel, seed_grid, dim3(256), 0, M, nullptr, p->d_fp, p->d_fsb, chg, p->d_fact,
                           p->d_fnodes, perm, V, q0, nsrc, t0, p->d_frow_ptr, p->d_fcol);
        // SRT_FR_COUNT=1 in a diagnostic build (-DFR_COUNT=1): per loss sweep,
        // items processed / with work / improved / edge gathers, printed after
        // the phase (the counters cost the kernel registers, so they are not in
        // the default build)
        static unsigned long long *dcnt_s = nullptr;
        unsigned long long *dcnt = nullptr;
        if (FR_COUNT && std::getenv("SRT_FR_COUNT")) {
            if (!dcnt_s) (void)hipMalloc(&dcnt_s, 4 * 256 * 8);
            dcnt = dcnt_s;
            (void)hipMemsetAsync(dcnt, 0, 4 * 256 * 8, M);
        }
        st = run_phase(p, t0, chunk_loss, [&](uint32_t t) {
            // sweep t reads the bits of sweep t - 1 (slot (t - t0 - 1) & 1; the
            // seeds are slot 0) and writes slot (t - t0) & 1, cleared first
            uint8_t *cur = p->d_fsb + ((t - t0 - 1) & 1) * sbytes, *nxt = p->d_fsb + ((t - t0) & 1) * sbytes;
            (void)hipMemsetAsync(nxt, 0, sbytes, M);
            hipLaunchKernelGGL(fr_loss_sweep_kernel, sgrid, sblk, 0, M, p->d_in_ptr, p->d_in_edge, V, NB, E,
                               p->d_ftight, p->d_fce, p->d_fcnt, p->d_fp, cur, nxt, p->d_fact, p->d_fimp, t, p->fr_symg, p->d_frow_ptr,
                               p->d_fcol, p->d_fctl, dmin, nmin,
                               dcnt ? dcnt + 4 * std::min<uint32_t>(t - t0, 255) : nullptr);
        }, &t_end, &nsw, err);
        if (st != SRT_OK) return st;
        p->fr_loss_sweeps += nsw;
        if (dcnt) {
            unsigned long long h[4 * 256];
            (void)hipMemcpy(h, dcnt, sizeof h, hipMemcpyDeviceToHost);
            std::fprintf(stderr, "[srt] loss sweeps of launch %u (items/work/improved/gathers):", li);
            for (uint32_t k = 1; k <= std::min<uint32_t>(t_end - t0, 255); ++k)
                std::fprintf(stderr, " %llu/%llu/%llu/%llu", h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]);
            std::fprintf(stderr, "\n");
        }
        p->sssp_sweeps += nsw;
        chunk_loss = std::max<uint32_t>(nsw + 1, 4);
        p->fr_t = t_end + 2;
        (void)hipEventRecord(p->ev[2 * li + 1], M);
        p->p3_launches++;
        hipLaunchKernelGGL(fr_emit_kernel, dim3((p->n + 63) / 64, (nsrc + 63) / 64), dim3(256), 0, M, L, p->d_fp, V,
                           p->d_fnodes, perm, p->n, q0, nsrc, p->sssp_g, p->d_sl_lat, p->d_sl_loss, p->d_out_lat,
                           p->d_out_loss, d_stats);
    }
    // algorithmic bytes: 12 B per in-edge + 12 B per vertex, per source
    p->p3_work = (double)rows * 12.0 * ((double)E + (double)V);
    return SRT_OK;
}

// device bytes of one 512-source block in flight: L (1 KB) + P (2 KB) + change
// record (16 B) + 2 x per-source change bits (128 B) + activity (4 B) + tight
// count (4 B) per vertex, the tight masks (64 B) and compacted edge (8 B) per
// in-edge
uint64_t frontier_block_bytes(uint32_t V, uint64_t E) { return (uint64_t)V * (1024 + 2048 + 152) + E * 72; }
size_t frontier_chg_bytes() { return sizeof(Chg); }

}  // namespace srt
