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
// Sources enter the words in BFS order over the graph (srt_api.cpp bfs_rank),
// so a word's 64 sources are neighbours / siblings whose keys change at the
// same vertices in the same sweeps (fewer 128-B lines per change; C4 1.61 ->
// 1.56 s); optional delta-stepping (below) gates which keys move on.
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
__global__ void sssp_init_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask, uint64_t *__restrict__ pend,
                                 uint32_t *flag, uint32_t V, uint32_t nbat, uint32_t G) {
    const uint64_t nD = (uint64_t)nbat * V * 64, nM = 2ull * nbat * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < nD;
         e += (uint64_t)gridDim.x * blockDim.x) {
        D[e] = SKEY_INF;
        if (e < nM) mask[e] = 0;
        if (e < nM / 2) pend[e] = 0;
        // flags, thresholds and prop flags 0, pending minima ~0 (srt_sweep_kernel)
        if (e < 12ull * G) flag[e] = (e >= 6ull * G && e < 9ull * G) ? ~0u : 0u;
    }
}

// source row row0 + q (q = (g*R + r)*64 + s) -> group g, word r, lane s:
// D[g][v][r][s], mask[g][v][r]
// (perm: sweep slot -> table row, the BFS source order; null = identity)
__global__ void sssp_seed_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask,
                                 const uint32_t *__restrict__ nodes, const uint32_t *__restrict__ perm, uint32_t V,
                                 uint32_t row0, uint32_t row1, uint32_t nbat, uint32_t R) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nbat * 64) return;
    const uint32_t g = q / (64 * R), r = (q / 64) % R, s = q % 64;
    if (row0 + q >= row1) return;
    const uint32_t src = nodes[perm ? perm[row0 + q] : row0 + q];
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
//
// Delta-stepping (delta > 0, in latency units g): sweep t propagates only keys
// whose latency is below the threshold theta_t (theta_0 = 2 delta, then + delta
// a sweep, or at least the smallest pending latency + delta after a sweep that
// moved nothing; see below) -- the buckets are settled in order, so a key is
// far more often final when it moves on (C4: fewer re-relaxations per
// (vertex, source) and fewer gathered lines).  A wave whose closing compare
// leaves a key at or above the next threshold (improved now, or pending from
// an earlier sweep) keeps it in pend[g][v][r] instead of the next change mask
// and marks its own vertex active; the sweep where the threshold passes the
// key moves it to the change mask.  The fixpoint -- and so every key -- is
// the one of the ungated sweep: a key still pending keeps the group's flag
// set, and the threshold grows without bound.
//
// Empty buckets are skipped: flag[] holds, after the 3 convergence slots, per
// ring slot and group the threshold the sweep used (theta), the smallest
// pending latency it left (pmin, one atomicMin a wave) and whether it moved
// any key on (prop).  theta_0 = 2 delta; theta_t = theta_{t-1} + delta, or, if
// sweep t-1 moved nothing, at least pmin_{t-1} + delta -- so the next pending
// key moves at once instead of after (pmin - theta) / delta idle sweeps.  Every
// wave derives theta_t from the same slot values; block 0 stores it.

template <int R>
__global__ __launch_bounds__(SWP_WAVES * 64) void sssp_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V,
    uint64_t *D, const uint64_t *__restrict__ mask_cur, uint64_t *__restrict__ mask_next, uint64_t *__restrict__ pend,
    uint32_t *flag, uint32_t t, uint32_t delta, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, uint8_t *act, uint32_t act_mode) {
    const uint32_t g = blockIdx.y, G = gridDim.y;
    uint32_t *theta = flag + 3 * G, *pmin = flag + 6 * G, *prop = flag + 9 * G;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // slots of sweep t+1
        flag[((t + 1) % 3) * G + g] = 0;
        pmin[((t + 1) % 3) * G + g] = ~0u;
        prop[((t + 1) % 3) * G + g] = 0;
    }
    if (t > 0 && flag[((t + 2) % 3) * G + g] == 0) return;  // converged
    // this sweep's threshold (see above); saturates below the u32 latency range
    uint64_t th = ~0ull;
    if (delta) {
        if (t == 0) {
            th = 2ull * delta;
        } else {
            const uint32_t ps = ((t + 2) % 3) * G + g;
            th = (uint64_t)theta[ps] + delta;
            if (prop[ps] == 0 && pmin[ps] != ~0u) th = th > (uint64_t)pmin[ps] + delta ? th : (uint64_t)pmin[ps] + delta;
            th = th < 0xFFFFFFFFull ? th : 0xFFFFFFFFull;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) theta[(t % 3) * G + g] = (uint32_t)th;
    }
    const int lane = threadIdx.x & 63;
    // Plain block order on purpose: an XCD-contiguous remap (each XCD sweeping
    // its own run of vertices) measured 2x slower on C4 (1.52 -> 2.9 s) -- all
    // XCDs on neighbouring vertices keep the gathered rows in the Infinity Cache.
    const uint32_t vi = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (vi >= V) return;
    const uint32_t v = vi;
    const uint64_t base = (uint64_t)g * V;  // first vertex row of the group
    const uint64_t aslot = (uint64_t)G * V;  // bytes per ring slot
    bool skip_walk = false;
    if (act_mode & (ACT_USE | ACT_SET)) {
        if (lane == 0) act[((t + 2) % 3) * aslot + base + v] = 0;
        if ((act_mode & ACT_USE) && act[(t % 3) * aslot + base + v] == 0) {
            // no in-neighbour changed: only pending keys (delta-stepping) can
            // move on, which needs no in-edge walk
            bool pend_only = false;
            if (delta) {
                uint64_t pw = lane < R ? pend[(base + v) * R + lane] : 0ull;
                pend_only = __ballot(pw != 0) != 0;
            }
            if (!pend_only) {
                if (lane < R) mask_next[(base + v) * R + lane] = 0;
                return;
            }
            skip_walk = true;
        }
    }
    const uint64_t *Dg = D + base * R * 64;
    const uint64_t *mc = mask_cur + base * R;
    uint64_t best[R];
#pragma unroll
    for (int r = 0; r < R; ++r) best[r] = SKEY_INF;
    const uint64_t e0 = in_ptr[v], e1 = skip_walk ? e0 : in_ptr[v + 1];
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
    bool prop_any = false, pend_any = false;
    uint32_t pl = ~0u;  // smallest pending latency of this lane
    uint64_t m_out[R], p_out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bool imp = false;
        // pending keys of this word (one broadcast load; none without delta)
        const uint64_t pw = delta ? pend[(base + v) * R + r] : 0ull;
        const bool pb = (pw >> lane) & 1ull;
        // own key: only lanes with a candidate or a pending key read it
        uint64_t cur = SKEY_INF;
        if (best[r] != SKEY_INF || pb) cur = Dv[r * 64];
        if (best[r] != SKEY_INF && best[r] < cur) {
            Dv[r * 64] = best[r];
            cur = best[r];
            imp = true;
        }
        const bool cand = imp || pb;
        const bool go = cand && (cur >> 32) < th;
        m_out[r] = __ballot(go);
        p_out[r] = __ballot(cand && !go);
        if (cand && !go) pl = (uint32_t)(cur >> 32) < pl ? (uint32_t)(cur >> 32) : pl;
        prop_any |= m_out[r] != 0;
        pend_any |= p_out[r] != 0;
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            mask_next[(base + v) * R + r] = m_out[r];
            if (delta) pend[(base + v) * R + r] = p_out[r];
        }
        // idempotent stores, no atomics; every wave of the group hits the same
        // word, so read first and write only while it is still 0 (a hot line
        // written by every wave serialises in its L2 channel)
        uint32_t *fl = &flag[(t % 3) * G + g], *pr = &prop[(t % 3) * G + g];
        if ((prop_any || pend_any) && __builtin_nontemporal_load(fl) == 0) *fl = 1;
        if (prop_any && __builtin_nontemporal_load(pr) == 0) *pr = 1;
    }
    if (pend_any) {
        for (int off = 32; off > 0; off >>= 1) {
            const uint32_t o = __shfl_xor(pl, off);
            pl = o < pl ? o : pl;
        }
        uint32_t *pm = &pmin[(t % 3) * G + g];
        if (lane == 0 && pl < __builtin_nontemporal_load(pm)) atomicMin(pm, pl);
    }
    if (act_mode & ACT_SET) {
        uint8_t *nxt = act + ((t + 1) % 3) * aslot + base;
        if (prop_any) {
            for (uint64_t k = row_ptr[v] + lane; k < row_ptr[v + 1]; k += 64) {
                const uint32_t w = col[k];
                if (w != v && nxt[w] == 0) nxt[w] = 1;  // hubs: read before the store (hot lines)
            }
        }
    }
}

// Table rows of the group: row = row0 + (g*R + r)*64 + s for lane s of word r.
// A 64 x 64 (sources x columns) tile goes through LDS so both the gather from
// D (64 sources of one vertex) and the row-major table stores are coalesced.
// Diagonal = the raw self-loop (mod.rs:210-217); min latency (mod.rs:474-476)
// and unreachable count (the assert at mod.rs:219) are block-reduced into
// stats[0] (min) / stats[1] (count).  blockIdx.y = g*R + r.
__global__ __launch_bounds__(256) void sssp_emit_kernel(
    const uint64_t *__restrict__ D, uint32_t V, uint32_t R, const uint32_t *__restrict__ nodes,
    const uint32_t *__restrict__ perm, uint32_t n, uint32_t row0, uint32_t row1, uint64_t gunit,
    const uint64_t *__restrict__ sl_lat,
    const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat, float *__restrict__ out_loss,
    unsigned long long *stats) {
    __shared__ uint64_t tile[64][65];
    __shared__ unsigned long long red_min[4], red_cnt[4];
    const uint32_t b = blockIdx.y, g = b / R, r = b % R, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x;
    const uint64_t off = (uint64_t)g * V * R * 64 + (uint64_t)r * 64;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int jj = idx / 64, s = idx % 64;
        const uint32_t j = j0 + jj;
        uint64_t k = SKEY_INF;
        if (j < n) k = D[off + (uint64_t)nodes[j] * R * 64 + s];
        tile[jj][s] = k;
    }
    __syncthreads();
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int s = idx / 64, jj = idx % 64;
        const uint32_t j = j0 + jj, q = row0 + b * 64 + s;
        if (j >= n || q >= row1) continue;
        const uint32_t row = perm ? perm[q] : q;
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
                       p->d_sD, mc, mn, p->d_spend, p->d_sflag, t, p->sssp_delta, p->d_row_ptr, p->d_col, p->d_sact,
                       act_mode);
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
        if (t > p->sssp_tmax) {  // Bellman-Ford + bucket bound: cannot happen with positive latencies
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
// sources at a time.  Returns with the stream drained up to the last emit.
srt_status sssp_pass(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, R = p->sssp_r, GMAX = p->sssp_nb / p->sssp_r;
    const uint32_t per_launch = 64 * R * GMAX;
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->sssp_sweeps = 0;
    // the BFS source order of this rank's rows (built once per row range)
    const uint32_t *perm = nullptr;
    if (!p->h_bfs_rank.empty() && p->row1 > p->row0) {
        if (!p->d_sperm || p->sperm_r0 != p->row0 || p->sperm_r1 != p->row1) {
            // the host copy stays alive in the plan; the upload is ordered on
            // the plan's stream after the previous pass's emit (which reads it)
            std::vector<uint32_t> &pm = p->h_sperm;
            pm.resize(p->n);
            for (uint32_t i = 0; i < p->n; ++i) pm[i] = i;
            std::stable_sort(pm.begin() + p->row0, pm.begin() + p->row1, [&](uint32_t a, uint32_t b) {
                return p->h_bfs_rank[p->nodes[a]] < p->h_bfs_rank[p->nodes[b]];
            });
            hipError_t e = p->d_sperm ? hipSuccess : hipMalloc(&p->d_sperm, (size_t)p->n * 4);
            if (e == hipSuccess) e = hipStreamSynchronize(M);  // the previous emit is done with the old order
            if (e == hipSuccess)
                e = hipMemcpyAsync(p->d_sperm, pm.data(), (size_t)p->n * 4, hipMemcpyHostToDevice, M);
            if (e != hipSuccess) {
                if (err) {
                    err->code = SRT_ERR_HIP;
                    std::snprintf(err->msg, sizeof err->msg, "sssp source order: %s", hipGetErrorString(e));
                }
                return SRT_ERR_HIP;
            }
            p->sperm_r0 = p->row0;
            p->sperm_r1 = p->row1;
        }
        perm = p->d_sperm;
    }
    hipLaunchKernelGGL(sssp_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats);
    const uint32_t launches = (p->row1 - p->row0 + per_launch - 1) / per_launch;
    while (p->ev.size() < 2 * (size_t)launches) {
        hipEvent_t e;
        (void)hipEventCreateWithFlags(&e, 0);
        p->ev.push_back(e);
    }
    uint32_t chunk = 8, t_prev = 0;
    for (uint32_t li = 0; li < launches; ++li) {
        const uint32_t g0 = p->row0 + li * per_launch;
        const uint32_t rows = std::min<uint32_t>(per_launch, p->row1 - g0);
        const uint32_t nbat = (rows + 63) / 64;  // 64-source words with work
        const uint32_t G = (nbat + R - 1) / R;   // groups in this launch
        hipLaunchKernelGGL(sssp_init_kernel, dim3(4096), dim3(256), 0, M, p->d_sD, p->d_smask, p->d_spend, p->d_sflag,
                           V, G * R, G);
        hipLaunchKernelGGL(sssp_seed_kernel, dim3((nbat * 64 + 255) / 256), dim3(256), 0, M, p->d_sD, p->d_smask,
                           p->d_nodes, perm, V, g0, g0 + rows, nbat, R);
        if (p->sssp_act_on) (void)hipMemsetAsync(p->d_sact, 0, 3ull * G * V, M);
        (void)hipEventRecord(p->ev[2 * li], M);
        const dim3 grid((V + SWP_WAVES - 1) / SWP_WAVES, G);
        // activation starts where the previous launch's sweeps thinned out
        // (SRT_SSSP_ACT: knob; the first launch has no history)
        uint32_t t_on = 0;
        if (p->sssp_act_on) t_on = p->sssp_act_from ? p->sssp_act_from : (t_prev ? std::max<uint32_t>(1, t_prev * 5 / 8) : 0);
        uint32_t t = 0;
        srt_status st = sweep_until_converged(p, G, chunk, [&](uint32_t tt) {
            uint64_t *mc = p->d_smask + (uint64_t)(tt & 1) * G * R * V;
            uint64_t *mn = p->d_smask + (uint64_t)((tt + 1) & 1) * G * R * V;
            // target activation from sweep t_on (the tail; sweep t_on-1 marks)
            const uint32_t am = (t_on && tt + 1 >= t_on) ? (ACT_SET | (tt >= t_on ? ACT_USE : 0u)) : 0u;
            if (R == 4) launch_sweep<4>(grid, M, p, mc, mn, tt, am);
            else if (R == 2) launch_sweep<2>(grid, M, p, mc, mn, tt, am);
            else launch_sweep<1>(grid, M, p, mc, mn, tt, am);
        }, &t, err);
        if (st != SRT_OK) return st;
        p->sssp_sweeps += t;
        // the next launch starts with as many sweeps as this one needed
        chunk = std::max<uint32_t>(t, 4);
        t_prev = t;
        (void)hipEventRecord(p->ev[2 * li + 1], M);
        p->p3_launches++;
        hipLaunchKernelGGL(sssp_emit_kernel, dim3((p->n + 63) / 64, G * R), dim3(256), 0, M, p->d_sD, V, R,
                           p->d_nodes, perm, p->n, g0, g0 + rows, p->sssp_g, p->d_sl_lat, p->d_sl_loss, p->d_out_lat,
                           p->d_out_loss, d_stats);
    }
    // algorithmic bytes: 12 B per in-edge + 12 B per vertex, per source
    p->p3_work = (double)(p->row1 - p->row0) * 12.0 * ((double)p->n_in_edges + (double)V);
    return SRT_OK;
}
}  // namespace

// Whole build for this rank's table rows.
srt_status sssp_run(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    return p->sssp_frontier ? frontier_run(p, d_stats, err) : sssp_pass(p, d_stats, err);
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
