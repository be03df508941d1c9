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

__global__ void sssp_init_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask, uint32_t *flag,
                                 uint32_t V, uint32_t nb) {
    const uint64_t nD = (uint64_t)nb * V * 64, nM = 2ull * nb * V;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < nD;
         e += (uint64_t)gridDim.x * blockDim.x) {
        D[e] = SKEY_INF;
        if (e < nM) mask[e] = 0;
        if (e < 3ull * nb) flag[e] = 0;
    }
}

// batch b, lane s: source = nodes[row0 + b*64 + s] when that row is < row1
__global__ void sssp_seed_kernel(uint64_t *__restrict__ D, uint64_t *__restrict__ mask,
                                 const uint32_t *__restrict__ nodes, uint32_t V, uint32_t row0,
                                 uint32_t row1, uint32_t nb) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nb * 64) return;
    const uint32_t b = t / 64, s = t % 64, r = row0 + t;
    if (r >= row1) return;
    const uint32_t src = nodes[r];
    D[((uint64_t)b * V + src) * 64 + s] = 0ull;  // (0 ns, 0.0 loss): petgraph's zero score
    mask[(uint64_t)b * V + src] = 1ull << s;     // sources within a batch are distinct nodes
}

__global__ __launch_bounds__(SWP_WAVES * 64) void sssp_sweep_kernel(
    const uint64_t *__restrict__ in_ptr, const InEdge *__restrict__ in_edge, uint32_t V,
    uint64_t *D, const uint64_t *__restrict__ mask_cur, uint64_t *__restrict__ mask_next,
    uint32_t *flag, uint32_t t) {
    const uint32_t b = blockIdx.y, nb = gridDim.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[((t + 1) % 3) * nb + b] = 0;  // for sweep t+1
    if (t > 0 && flag[((t + 2) % 3) * nb + b] == 0) return;                     // converged
    const int lane = threadIdx.x & 63;
    const uint32_t v = __builtin_amdgcn_readfirstlane(blockIdx.x * SWP_WAVES + (threadIdx.x >> 6));
    if (v >= V) return;
    const uint64_t base = (uint64_t)b * V;
    const uint64_t *Db = D + base * 64;
    const uint64_t *mc = mask_cur + base;
    uint64_t best = SKEY_INF;
    const uint64_t e0 = in_ptr[v], e1 = in_ptr[v + 1];
    for (uint64_t c0 = e0; c0 < e1; c0 += 64) {
        const uint64_t k = c0 + lane;
        uint32_t eu = 0, ew = 0;
        float eeb = 0.f;
        uint64_t em = 0;
        if (k < e1) {
            const InEdge e = in_edge[k];
            eu = e.u;
            ew = e.w;
            eeb = e.eb;
            em = mc[eu];
        }
        uint64_t act = __ballot(em != 0);
        while (act) {
            uint64_t du[8];
            uint32_t w[8];
            float eb[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                du[q] = SKEY_INF;
                w[q] = 0;
                eb[q] = 0.f;
                if (act) {
                    const int j = __builtin_ctzll(act);
                    act &= act - 1;
                    const uint32_t u = __builtin_amdgcn_readlane(eu, j);
                    const uint32_t mlo = __builtin_amdgcn_readlane((uint32_t)em, j);
                    const uint32_t mhi = __builtin_amdgcn_readlane((uint32_t)(em >> 32), j);
                    w[q] = __builtin_amdgcn_readlane(ew, j);
                    eb[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eeb), j));
                    const uint32_t bit = lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32));
                    if (bit & 1u) du[q] = Db[(uint64_t)u * 64 + lane];
                }
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (du[q] != SKEY_INF) {
                    const uint64_t c = relax(du[q], w[q], eb[q]);
                    best = c < best ? c : best;
                }
            }
        }
    }
    bool imp = false;
    if (best != SKEY_INF) {
        uint64_t *dv = D + (base + v) * 64 + lane;
        if (best < *dv) {
            *dv = best;
            imp = true;
        }
    }
    const uint64_t m_out = __ballot(imp);
    if (lane == 0) {
        mask_next[base + v] = m_out;
        if (m_out) flag[(t % 3) * nb + b] = 1;  // idempotent store, no atomic
    }
}

// Table rows of the group: row = row0 + b*64 + s for source lane s of batch b.
// A 64 x 64 (sources x columns) tile goes through LDS so both the gather from
// D (64 sources of one vertex) and the row-major table stores are coalesced.
// Diagonal = the raw self-loop (mod.rs:210-217); min latency (mod.rs:474-476)
// and unreachable count (the assert at mod.rs:219) are block-reduced into
// stats[0] (min) / stats[1] (count).
__global__ __launch_bounds__(256) void sssp_emit_kernel(
    const uint64_t *__restrict__ D, uint32_t V, const uint32_t *__restrict__ nodes, uint32_t n, uint32_t row0,
    uint32_t row1, uint64_t g, const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss,
    uint64_t *__restrict__ out_lat, float *__restrict__ out_loss, unsigned long long *stats) {
    __shared__ uint64_t tile[64][65];
    __shared__ unsigned long long red_min[4], red_cnt[4];
    const uint32_t b = blockIdx.y, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x;
    const uint64_t *Db = D + (uint64_t)b * V * 64;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int jj = idx / 64, s = idx % 64;
        const uint32_t j = j0 + jj;
        tile[jj][s] = j < n ? Db[(uint64_t)nodes[j] * 64 + s] : SKEY_INF;
    }
    __syncthreads();
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int s = idx / 64, jj = idx % 64;
        const uint32_t j = j0 + jj, r = row0 + b * 64 + s;
        if (j >= n || r >= row1) continue;
        uint64_t lat;
        float loss;
        if (r == j) {
            lat = sl_lat[j];
            loss = sl_loss[j];
        } else {
            const uint64_t k = tile[jj][s];
            if (k == SKEY_INF) {
                ++unreach;
                lat = ~0ull;
                loss = 1.0f;
            } else {
                lat = (k >> 32) * g;
                loss = __uint_as_float((uint32_t)k);
            }
        }
        out_lat[(uint64_t)r * n + j] = lat;
        out_loss[(uint64_t)r * n + j] = loss;
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

// Whole build for this rank's table rows [row0, row1), group by group.  The
// host polls the convergence flags after each chunk of sweeps, so this call
// returns with the stream drained up to the last group's emit.
srt_status sssp_run(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, NB = p->sssp_nb;
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->sssp_sweeps = 0;
    hipLaunchKernelGGL(sssp_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats);
    const uint32_t groups = (p->row1 - p->row0 + 64 * NB - 1) / (64 * NB);
    while (p->ev.size() < 2 * (size_t)groups) {
        hipEvent_t e;
        hipEventCreateWithFlags(&e, 0);
        p->ev.push_back(e);
    }
    uint32_t chunk = 8;
    for (uint32_t gi = 0; gi < groups; ++gi) {
        const uint32_t g0 = p->row0 + gi * 64 * NB;
        const uint32_t rows = std::min<uint32_t>(64 * NB, p->row1 - g0);
        const uint32_t nb = (rows + 63) / 64;
        hipLaunchKernelGGL(sssp_init_kernel, dim3(4096), dim3(256), 0, M, p->d_sD, p->d_smask, p->d_sflag, V, nb);
        hipLaunchKernelGGL(sssp_seed_kernel, dim3((nb * 64 + 255) / 256), dim3(256), 0, M, p->d_sD, p->d_smask,
                           p->d_nodes, V, g0, g0 + rows, nb);
        hipEventRecord(p->ev[2 * gi], M);
        const dim3 grid((V + SWP_WAVES - 1) / SWP_WAVES, nb);
        uint32_t t = 0;
        for (;;) {
            for (uint32_t c = 0; c < chunk; ++c, ++t) {
                uint64_t *mc = p->d_smask + (uint64_t)(t & 1) * nb * V;
                uint64_t *mn = p->d_smask + (uint64_t)((t + 1) & 1) * nb * V;
                hipLaunchKernelGGL(sssp_sweep_kernel, grid, dim3(SWP_WAVES * 64), 0, M, p->d_in_ptr, p->d_in_edge,
                                   V, p->d_sD, mc, mn, p->d_sflag, t);
            }
            // flags of the last sweep (t-1): all zero == converged
            hipError_t e = hipMemcpyAsync(p->h_sflag, p->d_sflag + ((t - 1) % 3) * nb, nb * sizeof(uint32_t),
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
            for (uint32_t b = 0; b < nb; ++b) any |= p->h_sflag[b] != 0;
            if (!any) break;
            if (t > V + 2) {  // Bellman-Ford bound: cannot happen with positive latencies
                if (err) {
                    err->code = SRT_ERR_INVALID;
                    std::snprintf(err->msg, sizeof err->msg, "sssp did not converge after %u sweeps", t);
                }
                return SRT_ERR_INVALID;
            }
            chunk = 4;
        }
        hipEventRecord(p->ev[2 * gi + 1], M);
        p->p3_launches++;
        p->sssp_sweeps += t;
        // the next group starts with as many sweeps as this one needed
        chunk = std::max<uint32_t>(t, 4);
        hipLaunchKernelGGL(sssp_emit_kernel, dim3((p->n + 63) / 64, nb), dim3(256), 0, M, p->d_sD, V, p->d_nodes,
                           p->n, g0, g0 + rows, p->sssp_g, p->d_sl_lat, p->d_sl_loss, p->d_out_lat,
                           p->d_out_loss, d_stats);
    }
    // algorithmic bytes: 12 B per in-edge + 12 B per vertex, per source
    p->p3_work = (double)(p->row1 - p->row0) * 12.0 * ((double)p->n_in_edges + (double)V);
    return SRT_OK;
}

void reduce_rank_stats(srt_plan *p, int nranks) {
    hipLaunchKernelGGL(reduce_rank_stats_kernel, dim3(1), dim3(1), 0, p->stream,
                       (const unsigned long long *)p->d_rstats, nranks, p->d_stats);
}

}  // namespace srt
