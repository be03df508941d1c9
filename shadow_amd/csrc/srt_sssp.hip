// srt_sssp.hip -- batched multi-source label-correcting SSSP for sparse graphs, gfx950.
//
// Replaces NetworkGraph::compute_shortest_paths (src/main/network/graph/mod.rs:183-228)
// when the graph is sparse (config C4: 100k-node AS-like graph, average degree 8):
// one petgraph Dijkstra per in-use source on a rayon pool becomes batches of 64
// sources swept together, one source per lane of a wave64.
//
// Path state: one u64 per (vertex, source)
//     key = (latency_ns / g) << 32  |  f32 bits of packet_loss
// Latency first, then loss, compared as one unsigned integer == the reference's
// lexicographic PathProperties order (mod.rs:305-313): losses are non-negative
// f32, whose bit patterns order like their values.  The relaxation is the
// reference's Add (mod.rs:322-331) verbatim: latency + edge latency, and
// 1 - (1 - loss) * (1 - edge loss) in f32, one rounding per op (no FMA).  So,
// unlike the dense closure (srt_fw.hip), the loss here is BIT-EXACT: petgraph's
// label-setting Dijkstra and this label-correcting fixpoint both return, for
// every target, the lexicographic minimum over all paths of (sum latency,
// left-fold loss) -- latencies are > 0 and the f32 fold is monotone in the
// path-prefix loss, so the minimum extends a minimal prefix.
// The host proves V * max_edge_latency / g < 2^32 - 1 (no carry into the tag).
//
// Layout in HBM (one "group" of nb batches in flight):
//   D[b][v][lane]      u64 keys, 64 sources contiguous per vertex row (512 B);
//   mask[2][b][v]      u64: lanes whose D[b][v][lane] improved in the previous
//                      sweep (double-buffered, every sweep rewrites every entry);
//   flag[3][b]         "something improved in sweep t" (ring of 3, see sweep).
// Sweep t (one launch per t): one wave per target v.  The wave loads 64 of v's
// in-edges at a time (one per lane, with the source vertex's change mask),
// ballots the edges whose source changed, and walks them 8 at a time: lane s
// gathers D[b][u][s] only where bit s of u's mask is set, relaxes, keeps the
// minimum, and finally stores the improved lanes and their ballot as v's next
// mask.  Gauss-Seidel in place: a wave may already see a value written in the
// same sweep (fine: every write also sets the writer's next mask, so readers
// re-read it in sweep t+1).  The group has converged when a sweep improves
// nothing; sweeps of converged batches exit at their first instruction.
#include <algorithm>
#include <cstdio>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr int SWP_WAVES = 4;  // waves (target vertices) per sweep workgroup
constexpr uint64_t SKEY_INF = ~0ull;

__device__ __forceinline__ uint64_t relax(uint64_t du, uint32_t w, float eb) {
    // eb = 1 - edge loss (rounded once, as the reference's (1f32 - other.packet_loss))
    const uint32_t lat = (uint32_t)(du >> 32) + w;
    const float a = __uint_as_float((uint32_t)du);
    const float loss = 1.0f - __fmul_rn(1.0f - a, eb);
    return ((uint64_t)lat << 32) | (uint64_t)__float_as_uint(loss);
}

// D, masks and flags of G groups of R batches (R*64 sources per group)
__global__ void sssp_init_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask, uint32_t *flag,
                                 uint32_t V, uint32_t nbat, uint32_t G) {
    const uint64_t nD = (uint64_t)nbat * V * 64, nM = 2ull * nbat * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < nD;
         e += (uint64_t)gridDim.x * blockDim.x) {
        D[e] = SKEY_INF;
        if (e < nM) mask[e] = 0;
        if (e < 3ull * G) flag[e] = 0;
    }
}

// source row row0 + q (q = (g*R + r)*64 + s) -> group g, word r, lane s:
// D[g][v][r][s], mask[g][v][r]
__global__ void sssp_seed_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask,
                                 const uint32_t *__restrict__ nodes, uint32_t V, uint32_t row0,
                                 uint32_t row1, uint32_t nbat, uint32_t R) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nbat * 64) return;
    const uint32_t g = q / (64 * R), r = (q / 64) % R, s = q % 64;
    if (row0 + q >= row1) return;
    const uint32_t src = nodes[row0 + q];
    const uint64_t row = (uint64_t)g * V + src;
    D[(row * R + r) * 64 + s] = 0ull;  // (0 ns, 0.0 loss): petgraph's zero score
    mask[row * R + r] = 1ull << s;     // sources within a word are distinct nodes
}

// Sweep t over G groups (blockIdx.y): one wave per target vertex v handles the
// R*64 sources of its group.  Per chunk of 64 in-edges every lane loads one
// edge and the R change masks of its source vertex; edges whose source changed
// are walked 4 at a time with up to 4*R predicated gathers in flight.
//
// Target activation (tail sweeps, act_mode != 0): act[3][g][v] is a byte ring.
// With ACT_SET a wave that improved v marks v's out-neighbours (CSR row v,
// self-loop skipped) in act[(t+1)%3] with plain byte stores (all writers write
// 1); with ACT_USE sweep t skips every target not marked in act[t%3] -- none of
// its in-neighbours changed in sweep t-1, so processing it would find no active
// edge -- and only stores its all-zero next masks.  Sweep t clears
// act[(t+2)%3], the slot sweep t+1 marks (read in t-1, so free in t).
constexpr uint32_t ACT_USE = 1, ACT_SET = 2;
// act_mode bit 2: the sweep visits the targets in reverse order (alternating
// directions let Gauss-Seidel carry a value along paths whose vertex indices
// fall as well as rise within one sweep)
constexpr uint32_t ACT_REV = 4;
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void sssp_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V,
    uint64_t *D, const uint64_t *__restrict__ mask_cur, uint64_t *__restrict__ mask_next,
    uint32_t *flag, uint32_t t, const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
    uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * G + g] = 0;  // for sweep t+1
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;                     // converged
    const int lane = threadIdx.x & 63;
    // Plain block order on purpose: an XCD-contiguous remap (each XCD sweeping
    // its own run of vertices) measured 2x slower on C4 (1.52 -> 2.9 s) -- all
    // XCDs on neighbouring vertices keep the gathered rows in the Infinity Cache.
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = (act_mode & ACT_REV) ? V - 1 - vi : vi;
    const uint64_t base = (uint64_t)g * V;  // first vertex row of the group
    const uint64_t aslot = (uint64_t)G * V;  // bytes per ring slot
    if (act_mode & (ACT_USE | ACT_SET)) {
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            if (lane < R) mask_next[(base + v) * R + lane] = 0;
            return;
        }
    }
    const uint64_t *Dg = D + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    uint64_t best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) best[r] = SKEY_INF;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = 0;
        float eeb = 0.f;
        uint64_t em[R];
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) em[r] = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w;
            eeb = e.eb;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                em[r] = mc[(uint64_t)eu * R + r];
                any |= em[r] != 0;
            }
        }
        uint64_t act = __ballot(any);
        while (act) {
            uint64_t du[4][R];
            uint32_t w[4];
            float eb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = 0;
                eb[q] = 0.f;
#pragma unroll
                for (int r = 0; r < R; ++r) du[q][r] = SKEY_INF;
                if (act) {
                    const int j = __builtin_ctzll(act);
                    act &= act - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    w[q] = __builtin_amdgcn_readlane(ew, j);
                    eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j));
                    const uint64_t *Du = Dg + (uint64_t)u * R * 64 + lane;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em[r], j);
                        const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em[r] >> 32), j);
                        const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                        if (bit & 1u) du[q][r] = Du[r * 64];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (du[q][r] != SKEY_INF) {
                        const uint64_t c = relax(du[q][r], w[q], eb[q]);
                        best[r] = c < best[r] ? c : best[r];
                    }
                }
            }
        }
    }
    uint64_t *Dv = D + ((base + v) * R) * 64 + lane;
    bool imp_any = false;
    uint64_t m_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool imp = false;
        if (best[r] != SKEY_INF && best[r] < Dv[r * 64]) {
            Dv[r * 64] = best[r];
            imp = true;
        }
        m_out[r] = __ballot(imp);
        imp_any |= m_out[r] != 0;
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) mask_next[(base + v) * R + r] = m_out[r];
        if (imp_any) flag[(t % 3) * G + g] = 1;  // idempotent store, no atomic
    }
    if ((act_mode & ACT_SET) && imp_any) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w != v) nxt[w] = 1;
        }
    }
}

// ------------------------------------------------------------ compact lists
// The fused sweep above gathers D[u][s] for every changed lane s of u: with
// 16 keys per 128-B line, a row whose changed lanes are scattered costs up to
// 4 lines for a handful of keys (C4: 475k lines per source per build; a line
// holds ~1.9 useful keys).  Here every wave that improves v also writes the
// improved keys of each 64-source word COMPACTLY, in lane order, into a
// parity slot CL[t+1 & 1][v][r][0..63]: key i of the slot belongs to the i-th
// set bit of v's next change mask.  A reader of in-edge u -> v takes lane s's
// key from slot index popcount(mask_u & lanes below s) -- the changed keys of
// a word sit in ceil(c / 16) lines (C4, simulated: 265k lines per source).
// The slot holds sweep t-1's values (Jacobi for the propagation; simulated:
// the same 28 sweeps as in-place Gauss-Seidel reads).  Nobody but v's own
// wave reads v's state any more, so it is kept as two planes -- latency u32
// and loss f32 bits -- and the closing compare reads the loss plane only on
// a latency tie: lexicographic (latency, loss) order, the same decisions as
// the u64 key compare.  Layout in d_sD: Lat[b][v][lane] then Loss[b][v][lane].
// Measured (C4, one 8,192-source launch; profiles/r02c4_*): FETCH 323 -> 220
// GB, time unchanged (1.52 s per build): in the heavy sweeps most lanes of a
// word have changed, so a list is as long as the row (peak-sweep FETCH only
// -8%, and those sweeps run at the ~5.8 TB/s random-line ceiling: TCC misses
// x 128 B), while the light sweeps are bound by each wave's chain of dependent
// loads (SQ: 63% of wave cycles waiting on memory, VALU 27% busy).  Variants
// that skipped idle words per edge or loaded the own latencies early, and 512
// sources per wave, measured 5-20% slower.  Opt-in (SRT_SSSP_CL=1): it needs
// 3x the state memory for no gain.
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void sssp_cl_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V,
    uint32_t *__restrict__ Lat, uint32_t *__restrict__ Loss, const uint64_t *__restrict__ cl_cur,
    uint64_t *__restrict__ cl_next, const uint64_t *__restrict__ mask_cur, uint64_t *__restrict__ mask_next,
    uint32_t *flag, uint32_t t, const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
    uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * G + g] = 0;  // for sweep t+1
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;                     // converged
    const int lane = threadIdx.x & 63;
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = (act_mode & ACT_REV) ? V - 1 - vi : vi;
    const uint64_t base = (uint64_t)g * V;
    const uint64_t aslot = (uint64_t)G * V;
    if (act_mode & (ACT_USE | ACT_SET)) {
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            if (lane < R) mask_next[(base + v) * R + lane] = 0;
            return;
        }
    }
    const uint64_t *clg = cl_cur + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    uint64_t best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) best[r] = SKEY_INF;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = 0;
        float eeb = 0.f;
        uint64_t em[R];
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) em[r] = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w;
            eeb = e.eb;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                em[r] = mc[(uint64_t)eu * R + r];
                any |= em[r] != 0;
            }
        }
        uint64_t actv = __ballot(any);
        while (actv) {
            uint64_t du[4][R];
            uint32_t w[4];
            float eb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = 0;
                eb[q] = 0.f;
#pragma unroll
                for (int r = 0; r < R; ++r) du[q][r] = SKEY_INF;
                if (actv) {
                    const int j = __builtin_ctzll(actv);
                    actv &= actv - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    w[q] = __builtin_amdgcn_readlane(ew, j);
                    eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j));
                    const uint64_t *Cu = clg + (uint64_t)u * R * 64;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em[r], j);
                        const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em[r] >> 32), j);
                        const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                        const uint32_t idx = __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
                        if (bit & 1u) du[q][r] = Cu[r * 64 + idx];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (du[q][r] != SKEY_INF) {
                        const uint64_t c = relax(du[q][r], w[q], eb[q]);
                        best[r] = c < best[r] ? c : best[r];
                    }
                }
            }
        }
    }
    const uint64_t vrow = (base + v) * R;
    bool imp_any = false;
    uint64_t m_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t e = (vrow + r) * 64 + lane;
        bool imp = false;
        if (best[r] != SKEY_INF) {
            // lexicographic (latency, loss) compare; the loss plane only on a tie
            const uint32_t bl = (uint32_t)(best[r] >> 32), cl = Lat[e];
            imp = bl < cl || (bl == cl && (uint32_t)best[r] < Loss[e]);
            if (imp) {
                Lat[e] = bl;
                Loss[e] = (uint32_t)best[r];
            }
        }
        m_out[r] = __ballot(imp);
        imp_any |= m_out[r] != 0;
        if (imp) {
            const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(m_out[r] >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m_out[r], 0u));
            cl_next[(vrow + r) * 64 + idx] = best[r];
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) mask_next[vrow + r] = m_out[r];
        if (imp_any) flag[(t % 3) * G + g] = 1;
    }
    if ((act_mode & ACT_SET) && imp_any) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w != v) nxt[w] = 1;
        }
    }
}

// planes + compact lists of G groups: latency INF, change masks and flags 0
// (the loss plane is read only on a latency tie, so INF latency needs no loss)
__global__ void sssp_cl_init_kernel(uint32_t *__restrict__ Lat, uint64_t *__restrict__ mask, uint32_t *flag,
                                    uint32_t V, uint32_t nbat, uint32_t G) {
    const uint64_t nD = (uint64_t)nbat * V * 64, nM = 2ull * nbat * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < nD;
         e += (uint64_t)gridDim.x * blockDim.x) {
        Lat[e] = 0xffffffffu;
        if (e < nM) mask[e] = 0;
        if (e < 3ull * G) flag[e] = 0;
    }
}

// sources: (0, 0.0) in the planes, their change bit, and the key in slot 0 of
// the parity-0 compact list (sources within a word are distinct vertices, so
// a seeded (vertex, word) has exactly one changed lane)
__global__ void sssp_cl_seed_kernel(uint32_t *__restrict__ Lat, uint32_t *__restrict__ Loss,
                                    uint64_t *__restrict__ cl0, uint64_t *__restrict__ mask,
                                    const uint32_t *__restrict__ nodes, uint32_t V, uint32_t row0, uint32_t row1,
                                    uint32_t nbat, uint32_t R) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nbat * 64) return;
    const uint32_t g = q / (64 * R), r = (q / 64) % R, s = q % 64;
    if (row0 + q >= row1) return;
    const uint64_t row = (uint64_t)g * V + nodes[row0 + q];
    Lat[(row * R + r) * 64 + s] = 0;
    Loss[(row * R + r) * 64 + s] = 0;
    cl0[(row * R + r) * 64] = 0ull;
    mask[row * R + r] = 1ull << s;
}

// Table rows of the group: row = row0 + (g*R + r)*64 + s for lane s of word r.
// A 64 x 64 (sources x columns) tile goes through LDS so both the gather from
// D (64 sources of one vertex) and the row-major table stores are coalesced.
// Diagonal = the raw self-loop (mod.rs:210-217); min latency (mod.rs:474-476)
// and unreachable count (the assert at mod.rs:219) are block-reduced into
// stats[0] (min) / stats[1] (count).  blockIdx.y = g*R + r.
// PL: the state is the compact-list sweep's two planes (D = Lat, then Loss
// nbat * V * 64 words further on), else u64 keys.
template <bool PL>
__global__ __launch_bounds__(256) void sssp_emit_kernel(
    const uint64_t *__restrict__ D, uint32_t V, uint32_t R, const uint32_t *__restrict__ nodes, uint32_t n,
    uint32_t row0, uint32_t row1, uint64_t gunit, const uint64_t *__restrict__ sl_lat,
    const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat, float *__restrict__ out_loss,
    unsigned long long *stats, uint64_t plane_words) {
    __shared__ uint64_t tile[64][65];
    __shared__ unsigned long long red_min[4], red_cnt[4];
    const uint32_t b = blockIdx.y, g = b / R, r = b % R, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x;
    const uint64_t off = (uint64_t)g * V * R * 64 + (uint64_t)r * 64;
    const uint32_t *Lat = reinterpret_cast<const uint32_t *>(D), *Loss = Lat + plane_words;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int jj = idx / 64, s = idx % 64;
        const uint32_t j = j0 + jj;
        uint64_t k = SKEY_INF;
        if (j < n) {
            const uint64_t e = off + (uint64_t)nodes[j] * R * 64 + s;
            if (PL) {
                const uint32_t l = Lat[e];
                if (l != 0xffffffffu) k = ((uint64_t)l << 32) | Loss[e];
            } else {
                k = D[e];
            }
        }
        tile[jj][s] = k;
    }
    __syncthreads();
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int s = idx / 64, jj = idx % 64;
        const uint32_t j = j0 + jj, row = row0 + b * 64 + s;
        if (j >= n || row >= row1) continue;
        uint64_t lat;
        float loss;
        if (row == j) {
            lat = sl_lat[j];
            loss = sl_loss[j];
        } else {
            const uint64_t k = tile[jj][s];
            if (k == SKEY_INF) {
                ++unreach;
                lat = ~0ull;
                loss = 1.0f;
            } else {
                lat = (k >> 32) * gunit;
                loss = __uint_as_float((uint32_t)k);
            }
        }
        out_lat[(uint64_t)row * n + j] = lat;
        out_loss[(uint64_t)row * n + j] = loss;
        mn = lat < mn ? lat : mn;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mn, off);
        mn = o < mn ? o : mn;
        unreach += __shfl_xor(unreach, off);
    }
    const int w = tid >> 6;
    if ((tid & 63) == 0) {
        red_min[w] = mn;
        red_cnt[w] = unreach;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], c = red_cnt[0];
        for (int k = 1; k < 4; ++k) {
            m = red_min[k] < m ? red_min[k] : m;
            c += red_cnt[k];
        }
        atomicMin(&stats[0], m);
        if (c) atomicAdd(&stats[1], c);
    }
}

// ------------------------------------------------------------------ split
// Split sweep (knob SRT_SSSP_SPLIT=1; measured slower on C4, 1.88 vs 1.51 s:
// the loss sweeps need as many sweeps as the latency ones -- the depth of
// the tight DAG in hops -- so halving the latency gathers does not pay for
// a second pass): latency first, loss second.
//   Phase A: u16 latency state, one 128-B line per (vertex, 64-source word)
//     instead of four -- saturating adds at L16_INF, so every latency below
//     L16_INF is exact and a saturated pair reads as "unreachable"; the host
//     then reruns the rank's rows with the fused u64 sweep above (which also
//     tells a disconnected graph from a long one).
//   Phase B: f32 loss state over the converged latencies: a source's loss
//     moves along an in-edge u -> v only where L(u) + w == L(v) (a tight
//     edge of that source), and v keeps the minimum of the reference's f32
//     Add -- the left fold over the tight DAG, the same fixpoint as the
//     lexicographic sweep, in as many sweeps as the DAG is
//     deep.
// Layout: L16[b][v][lane] u16, then LS[b][v][lane] f32 bits, inside d_sD.
constexpr uint32_t L16_INF = 0xffffu;
constexpr uint32_t LOSS_INF_BITS = 0x7f800000u;  // +inf: no loss value yet

__global__ void split_init_kernel(uint16_t *__restrict__ L, uint32_t *__restrict__ LS, uint64_t *__restrict__ mask,
                                  uint32_t *flag, uint32_t V, uint32_t nbat, uint32_t G) {
    const uint64_t nD = (uint64_t)nbat * V * 64, nM = 2ull * nbat * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < nD;
         e += (uint64_t)gridDim.x * blockDim.x) {
        L[e] = (uint16_t)L16_INF;
        LS[e] = LOSS_INF_BITS;
        if (e < nM) mask[e] = 0;
        if (e < 3ull * G) flag[e] = 0;
    }
}

// sources of the launch: latency 0 and loss 0 (petgraph's zero score), and
// their change bit in mask (both phases start from the sources)
__global__ void split_seed_kernel(uint16_t *__restrict__ L, uint32_t *__restrict__ LS, uint64_t *__restrict__ mask,
                                  const uint32_t *__restrict__ nodes, uint32_t V, uint32_t row0, uint32_t row1,
                                  uint32_t nbat, uint32_t R) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nbat * 64) return;
    const uint32_t g = q / (64 * R), r = (q / 64) % R, s = q % 64;
    if (row0 + q >= row1) return;
    const uint64_t row = (uint64_t)g * V + nodes[row0 + q];
    L[(row * R + r) * 64 + s] = 0;
    LS[(row * R + r) * 64 + s] = 0u;
    atomicOr((unsigned long long *)&mask[row * R + r], 1ull << s);
}

// Phase A sweep: sssp_sweep_kernel with u16 latency state (see there)
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void lat16_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V, uint16_t *L,
    const uint64_t *__restrict__ mask_cur, uint64_t *__restrict__ mask_next, uint32_t *flag, uint32_t t,
    const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col, uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * G + g] = 0;  // for sweep t+1
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;                     // converged
    const int lane = threadIdx.x & 63;
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = (act_mode & ACT_REV) ? V - 1 - vi : vi;
    const uint64_t base = (uint64_t)g * V;
    const uint64_t aslot = (uint64_t)G * V;
    if (act_mode & (ACT_USE | ACT_SET)) {
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            if (lane < R) mask_next[(base + v) * R + lane] = 0;
            return;
        }
    }
    const uint16_t *Lg = L + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    uint32_t best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) best[r] = L16_INF;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = 0;
        uint64_t em[R];
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) em[r] = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w < L16_INF ? e.w : L16_INF;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                em[r] = mc[(uint64_t)eu * R + r];
                any |= em[r] != 0;
            }
        }
        uint64_t actv = __ballot(any);
        while (actv) {
            uint32_t du[4][R], w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) du[q][r] = L16_INF;
                if (actv) {
                    const int j = __builtin_ctzll(actv);
                    actv &= actv - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    w[q] = __builtin_amdgcn_readlane(ew, j);
                    const uint16_t *Lu = Lg + (uint64_t)u * R * 64 + lane;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em[r], j);
                        const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em[r] >> 32), j);
                        const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                        if (bit & 1u) du[q][r] = Lu[r * 64];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    uint32_t c = du[q][r] + w[q];  // <= 2 L16_INF: no wrap
                    c = c < L16_INF ? c : L16_INF;
                    best[r] = c < best[r] ? c : best[r];
                }
            }
        }
    }
    uint16_t *Lv = L + ((base + v) * R) * 64 + lane;
    bool imp_any = false;
    uint64_t m_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool imp = false;
        if (best[r] < (uint32_t)Lv[r * 64]) {
            Lv[r * 64] = (uint16_t)best[r];
            imp = true;
        }
        m_out[r] = __ballot(imp);
        imp_any |= m_out[r] != 0;
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) mask_next[(base + v) * R + r] = m_out[r];
        if (imp_any) flag[(t % 3) * G + g] = 1;
    }
    if ((act_mode & ACT_SET) && imp_any) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w != v) nxt[w] = 1;
        }
    }
}

// Phase B sweep: one wave per target v; the edges whose source's loss changed
// last sweep, and for each lane (source) only where the edge is tight for it
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void loss_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V,
    const uint16_t *__restrict__ L, uint32_t *LS, const uint64_t *__restrict__ mask_cur,
    uint64_t *__restrict__ mask_next, uint32_t *flag, uint32_t t, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * G + g] = 0;
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;
    const int lane = threadIdx.x & 63;
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = (act_mode & ACT_REV) ? V - 1 - vi : vi;
    const uint64_t base = (uint64_t)g * V;
    const uint64_t aslot = (uint64_t)G * V;
    if (act_mode & (ACT_USE | ACT_SET)) {  // target activation, as lat16_sweep_kernel
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            if (lane < R) mask_next[(base + v) * R + lane] = 0;
            return;
        }
    }
    const uint16_t *Lg = L + base * R * 64;
    const uint32_t *LSg = LS + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    uint32_t lv[R], best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        lv[r] = Lg[((uint64_t)v * R + r) * 64 + lane];
        best[r] = LOSS_INF_BITS;
    }
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = 0;
        float eeb = 0.f;
        uint64_t em[R];
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) em[r] = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w;
            eeb = e.eb;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                em[r] = mc[(uint64_t)eu * R + r];
                any |= em[r] != 0;
            }
        }
        uint64_t actv = __ballot(any);
        while (actv) {
            uint32_t lu[4][R], lsu[4][R], w[4];
            float eb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = L16_INF;
                eb[q] = 0.f;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    lu[q][r] = L16_INF;
                    lsu[q][r] = LOSS_INF_BITS;
                }
                if (actv) {
                    const int j = __builtin_ctzll(actv);
                    actv &= actv - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    w[q] = __builtin_amdgcn_readlane(ew, j);
                    eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j));
                    const uint64_t row = (uint64_t)u * R * 64 + lane;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em[r], j);
                        const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em[r] >> 32), j);
                        const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                        // tight for this source: L(u) + w == L(v) (L(v) < INF)
                        if ((bit & 1u) && w[q] <= lv[r] && lv[r] < L16_INF) {
                            lu[q][r] = Lg[row + r * 64];
                            lsu[q][r] = LSg[row + r * 64];
                        }
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (lsu[q][r] != LOSS_INF_BITS && lu[q][r] + w[q] == lv[r]) {
                        // the reference's Add: 1 - (1 - a)(1 - e), one rounding per op
                        const float c = 1.0f - __fmul_rn(1.0f - __uint_as_float(lsu[q][r]), eb[q]);
                        const uint32_t cb = __float_as_uint(c);
                        best[r] = cb < best[r] ? cb : best[r];
                    }
                }
            }
        }
    }
    uint32_t *LSv = LS + ((base + v) * R) * 64 + lane;
    bool imp_any = false;
    uint64_t m_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool imp = false;
        if (best[r] < LSv[r * 64]) {
            LSv[r * 64] = best[r];
            imp = true;
        }
        m_out[r] = __ballot(imp);
        imp_any |= m_out[r] != 0;
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) mask_next[(base + v) * R + r] = m_out[r];
        if (imp_any) flag[(t % 3) * G + g] = 1;
    }
    if ((act_mode & ACT_SET) && imp_any) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w != v) nxt[w] = 1;
        }
    }
}

// Tight-edge bits of the group's sources after phase A: tb[(g E + e) R + r]
// bit s = in-edge e (u -> v) is tight for source s of word r, i.e.
// L(u) + w == L(v) < L16_INF.  One wave per target v.
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void tight_bits_kernel(const uint64_t *__restrict__ in_ptr,
                                                                    const InEdge *__restrict__ in_edge, uint32_t V,
                                                                    uint64_t E, const uint16_t *__restrict__ L,
                                                                    uint64_t *__restrict__ tb) {
    const uint32_t g = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const uint32_t v = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (v >= V) return;
    const uint64_t base = (uint64_t)g * V;
    const uint16_t *Lg = L + base * R * 64;
    uint32_t lv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) lv[r] = Lg[((uint64_t)v * R + r) * 64 + lane];
    uint64_t *tg = tb + (uint64_t)g * E * R;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = L16_INF;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w;
        }
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(64, e1 - c0);
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t u = __builtin_amdgcn_readlane(eu, j), w = __builtin_amdgcn_readlane(ew, j);
            const uint16_t *Lu = Lg + (uint64_t)u * R * 64 + lane;
            uint64_t bits[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t lu = Lu[r * 64];
                bits[r] = __ballot(lv[r] < L16_INF && w <= lv[r] && lu == lv[r] - w);
            }
            if (lane < R) {
                uint64_t b = bits[0];
#pragma unroll
                for (int r = 1; r < R; ++r)
                    if (lane == r) b = bits[r];
                tg[(c0 + j) * R + lane] = b;
            }
        }
    }
}

// Phase B sweep over precomputed tight bits: an edge is active for the lanes
// whose source's loss changed AND for which the edge is tight -- one f32
// gather, no latency reads
template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void loss_tb_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V, uint64_t E,
    const uint64_t *__restrict__ tb, uint32_t *LS, const uint64_t *__restrict__ mask_cur,
    uint64_t *__restrict__ mask_next, uint32_t *flag, uint32_t t, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * G + g] = 0;
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;
    const int lane = threadIdx.x & 63;
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = (act_mode & ACT_REV) ? V - 1 - vi : vi;
    const uint64_t base = (uint64_t)g * V;
    const uint64_t aslot = (uint64_t)G * V;
    if (act_mode & (ACT_USE | ACT_SET)) {
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            if (lane < R) mask_next[(base + v) * R + lane] = 0;
            return;
        }
    }
    const uint32_t *LSg = LS + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    const uint64_t *tg = tb + (uint64_t)g * E * R;
    uint32_t best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) best[r] = LOSS_INF_BITS;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0;
        float eeb = 0.f;
        uint64_t em[R];
        bool any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) em[r] = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            eeb = e.eb;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                em[r] = mc[(uint64_t)eu * R + r];
                if (em[r]) em[r] &= tg[k * R + r];
                any |= em[r] != 0;
            }
        }
        uint64_t actv = __ballot(any);
        while (actv) {
            uint32_t lsu[4][R];
            float eb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                eb[q] = 0.f;
#pragma unroll
                for (int r = 0; r < R; ++r) lsu[q][r] = LOSS_INF_BITS;
                if (actv) {
                    const int j = __builtin_ctzll(actv);
                    actv &= actv - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j));
                    const uint32_t *Pu = LSg + (uint64_t)u * R * 64 + lane;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em[r], j);
                        const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em[r] >> 32), j);
                        const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                        if (bit & 1u) lsu[q][r] = Pu[r * 64];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (lsu[q][r] != LOSS_INF_BITS) {
                        const float c = 1.0f - __fmul_rn(1.0f - __uint_as_float(lsu[q][r]), eb[q]);
                        const uint32_t cb = __float_as_uint(c);
                        best[r] = cb < best[r] ? cb : best[r];
                    }
                }
            }
        }
    }
    uint32_t *LSv = LS + ((base + v) * R) * 64 + lane;
    bool imp_any = false;
    uint64_t m_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool imp = false;
        if (best[r] < LSv[r * 64]) {
            LSv[r * 64] = best[r];
            imp = true;
        }
        m_out[r] = __ballot(imp);
        imp_any |= m_out[r] != 0;
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) mask_next[(base + v) * R + r] = m_out[r];
        if (imp_any) flag[(t % 3) * G + g] = 1;
    }
    if ((act_mode & ACT_SET) && imp_any) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
            const uint32_t w = col[k];
            if (w != v) nxt[w] = 1;
        }
    }
}

// Phase B's first sweep needs only the sources' out-neighbours: mark them in
// act slot 0 (one thread per source; byte stores, all writers write 1)
__global__ void split_seed_act_kernel(uint8_t *__restrict__ act, const uint32_t *__restrict__ nodes, uint32_t V,
                                      uint32_t row0, uint32_t row1, uint32_t nbat, uint32_t R,
                                      const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nbat * 64 || row0 + q >= row1) return;
    const uint32_t g = q / (64 * R), src = nodes[row0 + q];
    uint8_t *a = act + (uint64_t)g * V;
    for (uint64_t k = row_ptr[src]; k < row_ptr[src + 1]; ++k)
        if (col[k] != src) a[col[k]] = 1;
}

// sssp_emit_kernel for the split state
__global__ __launch_bounds__(256) void split_emit_kernel(
    const uint16_t *__restrict__ L, const uint32_t *__restrict__ LS, uint32_t V, uint32_t R,
    const uint32_t *__restrict__ nodes, uint32_t n, uint32_t row0, uint32_t row1, uint64_t gunit,
    const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat,
    float *__restrict__ out_loss, unsigned long long *stats) {
    __shared__ uint32_t tl[64][65], tp[64][65];
    __shared__ unsigned long long red_min[4], red_cnt[4];
    const uint32_t b = blockIdx.y, g = b / R, r = b % R, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x;
    const uint64_t off = (uint64_t)g * V * R * 64 + (uint64_t)r * 64;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int jj = idx / 64, s = idx % 64;
        const uint32_t j = j0 + jj;
        const uint64_t e = off + (j < n ? (uint64_t)nodes[j] * R * 64 : 0) + s;
        tl[jj][s] = j < n ? L[e] : L16_INF;
        tp[jj][s] = j < n ? LS[e] : LOSS_INF_BITS;
    }
    __syncthreads();
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int s = idx / 64, jj = idx % 64;
        const uint32_t j = j0 + jj, row = row0 + b * 64 + s;
        if (j >= n || row >= row1) continue;
        uint64_t lat;
        float loss;
        if (row == j) {
            lat = sl_lat[j];
            loss = sl_loss[j];
        } else if (tl[jj][s] >= L16_INF) {
            ++unreach;  // unreachable -- or saturated: the host reruns the rows
            lat = ~0ull;
            loss = 1.0f;
        } else {
            lat = (uint64_t)tl[jj][s] * gunit;
            loss = __uint_as_float(tp[jj][s]);
        }
        out_lat[(uint64_t)row * n + j] = lat;
        out_loss[(uint64_t)row * n + j] = loss;
        mn = lat < mn ? lat : mn;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = __shfl_xor(mn, o);
        mn = x < mn ? x : mn;
        unreach += __shfl_xor(unreach, o);
    }
    const int w = tid >> 6;
    if ((tid & 63) == 0) {
        red_min[w] = mn;
        red_cnt[w] = unreach;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], c = red_cnt[0];
        for (int k = 1; k < 4; ++k) {
            m = red_min[k] < m ? red_min[k] : m;
            c += red_cnt[k];
        }
        atomicMin(&stats[0], m);
        if (c) atomicAdd(&stats[1], c);
    }
}

__global__ void sssp_stats_init_kernel(unsigned long long *stats) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
}

// stats = (min over ranks of the min latency, sum over ranks of unreachable pairs)
__global__ void reduce_rank_stats_kernel(const unsigned long long *rstats, int nranks, unsigned long long *stats) {
    unsigned long long m = ~0ull, c = 0;
    for (int r = 0; r < nranks; ++r) {
        m = rstats[2 * r] < m ? rstats[2 * r] : m;
        c += rstats[2 * r + 1];
    }
    stats[0] = m;
    stats[1] = c;
}

}  // namespace

template <int R>
void launch_sweep(dim3 grid, hipStream_t s, srt_plan *p, uint64_t *mc, uint64_t *mn, uint32_t t, uint32_t act_mode) {
    hipLaunchKernelGGL(sssp_sweep_kernel<R>, grid, dim3(SWP_WAVES * 64), 0, s, p->d_in_ptr, p->d_in_edge, p->V,
                       p->d_sD, mc, mn, p->d_sflag, t, p->d_row_ptr, p->d_col, p->d_sact, act_mode);
}

template <int R>
void launch_cl_sweep(dim3 grid, hipStream_t s, srt_plan *p, uint64_t plane_words, uint64_t *mc, uint64_t *mn,
                     uint32_t t, uint32_t act_mode) {
    uint32_t *Lat = reinterpret_cast<uint32_t *>(p->d_sD);
    const uint64_t par = plane_words;  // one parity slot of the compact lists = one plane of keys
    hipLaunchKernelGGL(sssp_cl_sweep_kernel<R>, grid, dim3(SWP_WAVES * 64), 0, s, p->d_in_ptr, p->d_in_edge, p->V,
                       Lat, Lat + plane_words, p->d_scl + (t & 1) * par, p->d_scl + ((t + 1) & 1) * par, mc, mn,
                       p->d_sflag, t, p->d_row_ptr, p->d_col, p->d_sact, act_mode);
}

template <int R>
void launch_lat16(dim3 grid, hipStream_t s, srt_plan *p, uint64_t *mc, uint64_t *mn, uint32_t t, uint32_t act_mode) {
    hipLaunchKernelGGL(lat16_sweep_kernel<R>, grid, dim3(SWP_WAVES * 64), 0, s, p->d_in_ptr, p->d_in_edge, p->V,
                       reinterpret_cast<uint16_t *>(p->d_sD), mc, mn, p->d_sflag, t, p->d_row_ptr, p->d_col,
                       p->d_sact, act_mode);
}

template <int R>
void launch_loss(dim3 grid, hipStream_t s, srt_plan *p, const uint32_t *LS_off, uint64_t *mc, uint64_t *mn,
                 uint32_t t, uint32_t act_mode) {
    hipLaunchKernelGGL(loss_sweep_kernel<R>, grid, dim3(SWP_WAVES * 64), 0, s, p->d_in_ptr, p->d_in_edge, p->V,
                       reinterpret_cast<const uint16_t *>(p->d_sD), const_cast<uint32_t *>(LS_off), mc, mn,
                       p->d_sflag, t, p->d_row_ptr, p->d_col, p->d_sact, act_mode);
}

namespace {
// Sweeps t = 0, 1, ... of the launch's G groups until a sweep improves
// nothing; the host polls the convergence flags after each chunk of sweeps.
// sweep(t) enqueues sweep t.  Returns the sweep count in *t_out.
template <typename F>
srt_status sweep_until_converged(srt_plan *p, uint32_t G, uint32_t chunk, F sweep, uint32_t *t_out, srt_err *err) {
    hipStream_t M = p->stream;
    uint32_t t = 0;
    for (;;) {
        for (uint32_t c = 0; c < chunk; ++c, ++t) sweep(t);
        hipError_t e = hipMemcpyAsync(p->h_sflag, p->d_sflag + ((t - 1) % 3) * G, G * sizeof(uint32_t),
                                      hipMemcpyDeviceToHost, M);
        if (e == hipSuccess) e = hipStreamSynchronize(M);
        if (e != hipSuccess) {
            if (err) {
                err->code = SRT_ERR_HIP;
                std::snprintf(err->msg, sizeof err->msg, "sssp sweep: %s", hipGetErrorString(e));
            }
            return SRT_ERR_HIP;
        }
        bool any = false;
        for (uint32_t b = 0; b < G; ++b) any |= p->h_sflag[b] != 0;
        if (!any) break;
        if (t > p->V + 2) {  // Bellman-Ford bound: cannot happen with positive latencies
            if (err) {
                err->code = SRT_ERR_INVALID;
                std::snprintf(err->msg, sizeof err->msg, "sssp did not converge after %u sweeps", t);
            }
            return SRT_ERR_INVALID;
        }
        chunk = 4;
    }
    *t_out = t;
    return SRT_OK;
}

// One pass over this rank's table rows [row0, row1), G groups of R*64
// sources at a time: the fused u64 sweep, or (split) the u16 latency sweep
// then the loss sweep.  Returns with the stream drained up to the last emit.
srt_status sssp_pass(srt_plan *p, unsigned long long *d_stats, bool split, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, R = p->sssp_r, GMAX = p->sssp_nb / p->sssp_r;
    const uint32_t per_launch = 64 * R * GMAX;
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->sssp_sweeps = 0;
    p->sssp_loss_sweeps = 0;
    hipLaunchKernelGGL(sssp_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats);
    const uint32_t launches = (p->row1 - p->row0 + per_launch - 1) / per_launch;
    while (p->ev.size() < 2 * (size_t)launches) {
        hipEvent_t e;
        (void)hipEventCreateWithFlags(&e, 0);
        p->ev.push_back(e);
    }
    uint16_t *L16 = reinterpret_cast<uint16_t *>(p->d_sD);
    uint32_t *LS = reinterpret_cast<uint32_t *>(L16 + (uint64_t)p->sssp_nb * V * 64);
    const bool cl = !split && p->sssp_cl && p->d_scl;
    uint32_t chunk = 8, t_prev = 0, chunk_b = 8;
    for (uint32_t li = 0; li < launches; ++li) {
        const uint32_t g0 = p->row0 + li * per_launch;
        const uint32_t rows = std::min<uint32_t>(per_launch, p->row1 - g0);
        const uint32_t nbat = (rows + 63) / 64;           // 64-source words with work
        const uint32_t G = (nbat + R - 1) / R;            // groups in this launch
        const uint64_t plane_words = (uint64_t)G * R * V * 64;  // compact-list layout: plane / parity slot
        if (split) {
            hipLaunchKernelGGL(split_init_kernel, dim3(4096), dim3(256), 0, M, L16, LS, p->d_smask, p->d_sflag, V,
                               G * R, G);
            hipLaunchKernelGGL(split_seed_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, L16, LS,
                               p->d_smask, p->d_nodes, V, g0, g0 + rows, nbat, R);
        } else if (cl) {
            uint32_t *Lat = reinterpret_cast<uint32_t *>(p->d_sD);
            hipLaunchKernelGGL(sssp_cl_init_kernel, dim3(4096), dim3(256), 0, M, Lat, p->d_smask, p->d_sflag, V,
                               G * R, G);
            hipLaunchKernelGGL(sssp_cl_seed_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, Lat,
                               Lat + plane_words, p->d_scl, p->d_smask, p->d_nodes, V, g0, g0 + rows, nbat, R);
        } else {
            hipLaunchKernelGGL(sssp_init_kernel, dim3(4096), dim3(256), 0, M, p->d_sD, p->d_smask, p->d_sflag, V,
                               G * R, G);
            hipLaunchKernelGGL(sssp_seed_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, p->d_sD,
                               p->d_smask, p->d_nodes, V, g0, g0 + rows, nbat, R);
        }
        if (p->sssp_act_on) (void)hipMemsetAsync(p->d_sact, 0, 3ull * G * V, M);
        (void)hipEventRecord(p->ev[2 * li], M);
        const dim3 grid((V + SWP_WAVES - 1) / SWP_WAVES, G);
        // activation starts where the previous launch's sweeps thinned out
        // (SRT_SSSP_ACT: knob; the first launch has no history)
        uint32_t t_on = 0;
        if (p->sssp_act_on) t_on = p->sssp_act_from ? p->sssp_act_from : (t_prev ? std::max<uint32_t>(1, t_prev * 5 / 8) : 0);
        auto masks = [&](uint32_t t, uint64_t **mc, uint64_t **mn) {
            *mc = p->d_smask + (uint64_t)(t & 1) * G * R * V;
            *mn = p->d_smask + (uint64_t)((t + 1) & 1) * G * R * V;
        };
        uint32_t t = 0;
        srt_status st = sweep_until_converged(p, G, chunk, [&](uint32_t tt) {
            uint64_t *mc, *mn;
            masks(tt, &mc, &mn);
            // target activation from sweep t_on (the tail; sweep t_on-1 marks)
            const uint32_t am = ((t_on && tt + 1 >= t_on) ? (ACT_SET | (tt >= t_on ? ACT_USE : 0u)) : 0u) |
                                ((p->sssp_alt && (tt & 1)) ? ACT_REV : 0u);
            if (split) {
                if (R == 4) launch_lat16<4>(grid, M, p, mc, mn, tt, am);
                else if (R == 2) launch_lat16<2>(grid, M, p, mc, mn, tt, am);
                else launch_lat16<1>(grid, M, p, mc, mn, tt, am);
            } else if (cl) {
                if (R == 4) launch_cl_sweep<4>(grid, M, p, plane_words, mc, mn, tt, am);
                else if (R == 2) launch_cl_sweep<2>(grid, M, p, plane_words, mc, mn, tt, am);
                else launch_cl_sweep<1>(grid, M, p, plane_words, mc, mn, tt, am);
            } else {
                if (R == 4) launch_sweep<4>(grid, M, p, mc, mn, tt, am);
                else if (R == 2) launch_sweep<2>(grid, M, p, mc, mn, tt, am);
                else launch_sweep<1>(grid, M, p, mc, mn, tt, am);
            }
        }, &t, err);
        if (st != SRT_OK) return st;
        p->sssp_sweeps += t;
        // the next launch starts with as many sweeps as this one needed
        chunk = std::max<uint32_t>(t, 4);
        t_prev = t;
        if (split) {
            // phase B from the sources again: fresh masks and flags
            (void)hipMemsetAsync(p->d_smask, 0, 2ull * G * R * V * 8, M);
            (void)hipMemsetAsync(p->d_sflag, 0, 3ull * G * 4, M);
            hipLaunchKernelGGL(split_seed_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, L16, LS,
                               p->d_smask, p->d_nodes, V, g0, g0 + rows, nbat, R);
            // target activation from the first loss sweep (its active set:
            // the sources' out-neighbours), knob SRT_SSSP_LOSS_ACT=0 off
            const bool lact = p->sssp_act_on && p->sssp_loss_act;
            if (lact) {
                (void)hipMemsetAsync(p->d_sact, 0, 3ull * G * V, M);
                hipLaunchKernelGGL(split_seed_act_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, p->d_sact,
                                   p->d_nodes, V, g0, g0 + rows, nbat, R, p->d_row_ptr, p->d_col);
            }
            const uint32_t lam = lact ? (ACT_SET | ACT_USE) : 0u;
            // tight bits of every (in-edge, source) when they fit the spare
            // quarter of the path-state buffer (knob SRT_SSSP_TB=0: off)
            const uint64_t E = p->n_in_edges;
            uint64_t *TB = reinterpret_cast<uint64_t *>(LS + (uint64_t)p->sssp_nb * V * 64);
            const bool use_tb = p->sssp_tb && (uint64_t)G * R * E * 8 <= (uint64_t)p->sssp_nb * V * 128;
            if (use_tb) {
                if (R == 4) hipLaunchKernelGGL(tight_bits_kernel<4>, grid, dim3(SWP_WAVES * 64), 0, M, p->d_in_ptr, p->d_in_edge, V, E, L16, TB);
                else if (R == 2) hipLaunchKernelGGL(tight_bits_kernel<2>, grid, dim3(SWP_WAVES * 64), 0, M, p->d_in_ptr, p->d_in_edge, V, E, L16, TB);
                else hipLaunchKernelGGL(tight_bits_kernel<1>, grid, dim3(SWP_WAVES * 64), 0, M, p->d_in_ptr, p->d_in_edge, V, E, L16, TB);
            }
            uint32_t tb = 0;
            st = sweep_until_converged(p, G, chunk_b, [&](uint32_t tt0) {
                uint64_t *mc, *mn;
                masks(tt0, &mc, &mn);
                const uint32_t tt = tt0;
                const uint32_t lam_t = lam | ((p->sssp_alt && (tt & 1)) ? ACT_REV : 0u);
                if (use_tb) {
                    auto k4 = loss_tb_sweep_kernel<4>;
                    auto k2 = loss_tb_sweep_kernel<2>;
                    auto k1 = loss_tb_sweep_kernel<1>;
                    hipLaunchKernelGGL(R == 4 ? k4 : R == 2 ? k2 : k1, grid, dim3(SWP_WAVES * 64), 0, M, p->d_in_ptr,
                                       p->d_in_edge, V, E, (const uint64_t *)TB, LS, mc, mn, p->d_sflag, tt,
                                       p->d_row_ptr, p->d_col, p->d_sact, lam_t);
                } else if (R == 4) {
                    launch_loss<4>(grid, M, p, LS, mc, mn, tt, lam_t);
                } else if (R == 2) {
                    launch_loss<2>(grid, M, p, LS, mc, mn, tt, lam_t);
                } else {
                    launch_loss<1>(grid, M, p, LS, mc, mn, tt, lam_t);
                }
            }, &tb, err);
            if (st != SRT_OK) return st;
            p->sssp_loss_sweeps += tb;
            chunk_b = std::max<uint32_t>(tb, 4);
            if (std::getenv("SRT_TRACE")) std::fprintf(stderr, "[srt] sssp launch %u: %u latency sweeps, %u loss sweeps\n", li, t, tb);
        }
        (void)hipEventRecord(p->ev[2 * li + 1], M);
        p->p3_launches++;
        if (split)
            hipLaunchKernelGGL(split_emit_kernel, dim3((p->n + 63) / 64, G * R), dim3(256), 0, M, L16, LS, V, R,
                               p->d_nodes, p->n, g0, g0 + rows, p->sssp_g, p->d_sl_lat, p->d_sl_loss, p->d_out_lat,
                               p->d_out_loss, d_stats);
        else if (cl)
            hipLaunchKernelGGL(sssp_emit_kernel<true>, dim3((p->n + 63) / 64, G * R), dim3(256), 0, M, p->d_sD, V,
                               R, p->d_nodes, p->n, g0, g0 + rows, p->sssp_g, p->d_sl_lat, p->d_sl_loss,
                               p->d_out_lat, p->d_out_loss, d_stats, plane_words);
        else
            hipLaunchKernelGGL(sssp_emit_kernel<false>, dim3((p->n + 63) / 64, G * R), dim3(256), 0, M, p->d_sD,
                               V, R, p->d_nodes, p->n, g0, g0 + rows, p->sssp_g, p->d_sl_lat, p->d_sl_loss,
                               p->d_out_lat, p->d_out_loss, d_stats, 0ull);
    }
    // algorithmic bytes: 12 B per in-edge + 12 B per vertex, per source
    p->p3_work = (double)(p->row1 - p->row0) * 12.0 * ((double)p->n_in_edges + (double)V);
    return SRT_OK;
}
}  // namespace

// Whole build for this rank's table rows.  Split first (when enabled); a pair
// it leaves at the u16 limit is unreachable or saturated, and then the rows
// are rebuilt by the fused u64 sweep, which tells the two apart.
srt_status sssp_run(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    p->sssp_used_split = false;
    if (p->sssp_split) {
        srt_status st = sssp_pass(p, d_stats, true, err);
        if (st != SRT_OK) return st;
        unsigned long long h[2];
        hipError_t e = hipMemcpyAsync(h, d_stats, sizeof h, hipMemcpyDeviceToHost, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) {
            if (err) {
                err->code = SRT_ERR_HIP;
                std::snprintf(err->msg, sizeof err->msg, "sssp stats: %s", hipGetErrorString(e));
            }
            return SRT_ERR_HIP;
        }
        if (h[1] == 0) {
            p->sssp_used_split = true;
            return SRT_OK;
        }
    }
    return sssp_pass(p, d_stats, false, err);
}

void reduce_rank_stats(srt_plan *p, int nranks) {
    hipLaunchKernelGGL(reduce_rank_stats_kernel, dim3(1), dim3(1), 0, p->stream,
                       (const unsigned long long *)p->d_rstats, nranks, p->d_stats);
}

// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_sssp() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sssp_init_kernel));
}

}  // namespace srt
