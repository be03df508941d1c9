// srt_fw.hip -- blocked min-plus Floyd-Warshall over packed path keys, gfx950.
//
// Replaces NetworkGraph::compute_shortest_paths (src/main/network/graph/mod.rs:183-228):
// instead of one petgraph Dijkstra per in-use source on a rayon pool, the whole
// graph is closed in HBM with a three-phase blocked Floyd-Warshall:
//   round kb:  phase 1+2 (one launch): close the B x B pivot block, then relax
//              the pivot block-row and block-column through it;
//              phase 3: every other block C(i,j) = min(C, A(i,kb) (+) B(kb,j)),
//              a min-plus rank-B update -- the N^3 hot loop.
// Keys are u64 (see KeyParams in srt_internal.h): integer add + unsigned min
// implement the lexicographic (latency, loss) algebra of PathProperties.
#include "srt_internal.h"

namespace srt {

namespace {

constexpr int B = FW_B;       // 64
constexpr int NT = 256;       // threads per workgroup (4 waves)
constexpr int TPR = 16;       // threads per row of the 16x16 thread grid
constexpr int RPT = B / TPR;  // 4 rows / cols per thread

__device__ __forceinline__ uint64_t kmin(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ------------------------------------------------------------------ init
__global__ void fill_kernel(uint64_t *__restrict__ D, uint32_t Vp) {
    const uint64_t total = (uint64_t)Vp * Vp;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(e / Vp), c = (uint32_t)(e % Vp);
        D[e] = (r == c) ? 0ull : KEY_INF;
    }
}

__device__ __forceinline__ uint64_t edge_key(uint64_t lat, float loss, const KeyParams &kp) {
    const uint64_t lq = lat / kp.g;
    uint64_t q = 0;
    if (kp.qb) {
        const double nl = -log1p(-(double)loss);  // -ln(1 - loss) >= 0
        q = (nl >= kp.nlr_cap) ? kp.q_cap : (uint64_t)llrint(nl * kp.scale);
    }
    return (lq << kp.qb) | q;
}

// One wave per graph node row: D[u][v] = min over parallel edges u->v.  The
// diagonal keeps 0 (a self-loop never shortens a path; it is written into the
// table verbatim by the extract kernel, mod.rs:210-217).
__global__ void scatter_edges_kernel(uint64_t *__restrict__ D, uint32_t Vp,
                                     const uint64_t *__restrict__ row_ptr,
                                     const uint32_t *__restrict__ col,
                                     const uint64_t *__restrict__ lat,
                                     const float *__restrict__ loss, uint32_t V, KeyParams kp) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            const uint32_t v = col[k];
            if (v == u) continue;
            atomicMin((unsigned long long *)&D[(uint64_t)u * Vp + v],
                      (unsigned long long)edge_key(lat[k], loss[k], kp));
        }
    }
}

// ------------------------------------------------------- phase 1 + phase 2
// Block 0 closes the pivot block and writes it back; every other block closes
// the pivot block redundantly in LDS (64 short steps, far cheaper than an extra
// launch) and then relaxes one block of the pivot row (blockIdx < nblk) or
// pivot column through it.
__global__ __launch_bounds__(NT) void fw_phase12_kernel(uint64_t *__restrict__ D, uint32_t Vp,
                                                        uint32_t kb, uint32_t nblk) {
    __shared__ uint64_t P[B][B + 1];  // pivot block
    __shared__ uint64_t O[B][B + 1];  // own block
    const int tid = threadIdx.x, tx = tid % TPR, ty = tid / TPR;
    const uint64_t kb0 = (uint64_t)kb * B;

    for (int e = tid; e < B * B; e += NT) {
        const int r = e / B, c = e % B;
        P[r][c] = D[(kb0 + r) * Vp + kb0 + c];
    }
    __syncthreads();
    for (int k = 0; k < B; ++k) {
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const int r = ty + TPR * i, c = tx + TPR * j;
                P[r][c] = kmin(P[r][c], P[r][k] + P[k][c]);
            }
        __syncthreads();
    }
    if (blockIdx.x == 0) {
        for (int e = tid; e < B * B; e += NT) {
            const int r = e / B, c = e % B;
            D[(kb0 + r) * Vp + kb0 + c] = P[r][c];
        }
        return;
    }
    // which block: 1..nblk-1 -> row blocks (skipping kb), nblk..2*nblk-2 -> column blocks
    uint32_t idx = blockIdx.x - 1;
    const bool is_row = idx < nblk - 1;
    if (!is_row) idx -= nblk - 1;
    const uint32_t other = idx < kb ? idx : idx + 1;
    const uint64_t r0 = is_row ? kb0 : (uint64_t)other * B;
    const uint64_t c0 = is_row ? (uint64_t)other * B : kb0;
    for (int e = tid; e < B * B; e += NT) {
        const int r = e / B, c = e % B;
        O[r][c] = D[(r0 + r) * Vp + c0 + c];
    }
    __syncthreads();
    for (int k = 0; k < B; ++k) {
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const int r = ty + TPR * i, c = tx + TPR * j;
                const uint64_t cand = is_row ? P[r][k] + O[k][c] : O[r][k] + P[k][c];
                O[r][c] = kmin(O[r][c], cand);
            }
        __syncthreads();
    }
    for (int e = tid; e < B * B; e += NT) {
        const int r = e / B, c = e % B;
        D[(r0 + r) * Vp + c0 + c] = O[r][c];
    }
}

// ------------------------------------------------------------- phase 3
// C(i,j) = min(C(i,j), min_k A(i,k) + B(k,j)) for all blocks i,j != kb.
// grid = (nblk-1)^2 blocks; the pivot row/column are skipped by index remap.
__global__ __launch_bounds__(NT) void fw_phase3_kernel(uint64_t *__restrict__ D, uint32_t Vp,
                                                       uint32_t kb, uint32_t nblk) {
    __shared__ uint64_t As[B][B + 1];  // As[r][k] = D[i-block row r][pivot col k]
    __shared__ uint64_t Bs[B][B];      // Bs[k][c] = D[pivot row k][j-block col c]
    const int tid = threadIdx.x, tx = tid % TPR, ty = tid / TPR;
    const uint32_t m = nblk - 1;
    uint32_t bi = blockIdx.x / m, bj = blockIdx.x % m;
    bi += bi >= kb;
    bj += bj >= kb;
    const uint64_t i0 = (uint64_t)bi * B, j0 = (uint64_t)bj * B, k0 = (uint64_t)kb * B;

    for (int e = tid; e < B * B; e += NT) {
        const int r = e / B, c = e % B;
        As[r][c] = D[(i0 + r) * Vp + k0 + c];
        Bs[r][c] = D[(k0 + r) * Vp + j0 + c];
    }
    uint64_t acc[RPT][RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < RPT; ++j) acc[i][j] = D[(i0 + ty + TPR * i) * Vp + j0 + tx + TPR * j];
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < B; ++k) {
        uint64_t a[RPT], b[RPT];
#pragma unroll
        for (int i = 0; i < RPT; ++i) a[i] = As[ty + TPR * i][k];
#pragma unroll
        for (int j = 0; j < RPT; ++j) b[j] = Bs[k][tx + TPR * j];
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
            for (int j = 0; j < RPT; ++j) acc[i][j] = kmin(acc[i][j], a[i] + b[j]);
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int j = 0; j < RPT; ++j) D[(i0 + ty + TPR * i) * Vp + j0 + tx + TPR * j] = acc[i][j];
}

// ------------------------------------------------------------- extract
// table[i][j] = decode(D[nodes[i]][nodes[j]]); diagonal = the raw self-loop
// edge (mod.rs:210-217); min latency over the whole table (mod.rs:474-476);
// count of unreachable pairs (the reference's assert at mod.rs:219).
__global__ void extract_kernel(const uint64_t *__restrict__ D, uint32_t Vp,
                               const uint32_t *__restrict__ nodes, uint32_t n, KeyParams kp,
                               const uint64_t *__restrict__ sl_lat,
                               const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat,
                               float *__restrict__ out_loss, unsigned long long *stats) {
    const uint32_t cb = (n + blockDim.x - 1) / blockDim.x;  // column blocks per row
    const uint32_t i = blockIdx.x / cb;
    const uint32_t j = (blockIdx.x % cb) * blockDim.x + threadIdx.x;
    uint64_t lat = ~0ull;
    unsigned unreach = 0;
    if (j < n) {
        float loss;
        if (i == j) {
            lat = sl_lat[i];
            loss = sl_loss[i];
        } else {
            const uint64_t k = D[(uint64_t)nodes[i] * Vp + nodes[j]];
            if (k >= KEY_INF) {
                unreach = 1;
                lat = ~0ull;
                loss = 1.0f;
            } else {
                lat = (k >> kp.qb) * kp.g;
                const uint64_t q = kp.qb ? (k & ((1ull << kp.qb) - 1)) : 0ull;
                loss = (float)(-expm1(-(double)q * kp.inv_scale));
            }
        }
        out_lat[(uint64_t)i * n + j] = lat;
        out_loss[(uint64_t)i * n + j] = loss;
    }
    // wave reductions then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(lat, off);
        lat = o < lat ? o : lat;
        unreach += __shfl_xor(unreach, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&stats[0], (unsigned long long)lat);
        if (unreach) atomicAdd(&stats[1], (unsigned long long)unreach);
    }
}

__global__ void init_stats_kernel(unsigned long long *stats) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
}

__global__ void pack_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss,
                            srt_path *__restrict__ out, uint64_t total) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        srt_path p;
        p.latency_ns = lat[e];
        p.packet_loss = loss[e];
        p._pad = 0;
        out[e] = p;
    }
}

}  // namespace

void fw_init(srt_plan *p) {
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, p->stream, p->d_D, p->Vp);
    hipLaunchKernelGGL(scatter_edges_kernel, dim3(2048), dim3(256), 0, p->stream, p->d_D, p->Vp,
                       p->d_row_ptr, p->d_col, p->d_lat, p->d_loss, p->V, p->kp);
}

void fw_rounds(srt_plan *p) {
    const uint32_t nblk = p->Vp / B;
    p->p3_launches = 0;
    const size_t need = 2 * (size_t)nblk;
    while (p->ev.size() < need) {
        hipEvent_t e;
        hipEventCreate(&e);
        p->ev.push_back(e);
    }
    for (uint32_t kb = 0; kb < nblk; ++kb) {
        hipLaunchKernelGGL(fw_phase12_kernel, dim3(nblk > 1 ? 2 * nblk - 1 : 1), dim3(NT), 0,
                           p->stream, p->d_D, p->Vp, kb, nblk);
        if (nblk > 1) {
            hipEventRecord(p->ev[2 * kb], p->stream);
            hipLaunchKernelGGL(fw_phase3_kernel, dim3((nblk - 1) * (nblk - 1)), dim3(NT), 0,
                               p->stream, p->d_D, p->Vp, kb, nblk);
            hipEventRecord(p->ev[2 * kb + 1], p->stream);
            p->p3_launches++;
        }
    }
}

void fw_extract(srt_plan *p) {
    hipLaunchKernelGGL(init_stats_kernel, dim3(1), dim3(1), 0, p->stream, p->d_stats);
    const uint32_t cb = (p->n + 255) / 256;
    dim3 grid(cb * p->n);
    hipLaunchKernelGGL(extract_kernel, grid, dim3(256), 0, p->stream, p->d_D, p->Vp, p->d_nodes,
                       p->n, p->kp, p->d_sl_lat, p->d_sl_loss, p->d_out_lat, p->d_out_loss,
                       p->d_stats);
}

void pack_paths(srt_plan *p) {
    const uint64_t total = (uint64_t)p->n * p->n;
    hipLaunchKernelGGL(pack_kernel, dim3(4096), dim3(256), 0, p->stream, p->d_out_lat,
                       p->d_out_loss, p->d_pack, total);
}

}  // namespace srt
