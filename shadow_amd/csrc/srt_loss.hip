// srt_loss.hip -- exact packet_loss of the dense routing build ("K5"), gfx950.
//
// The blocked Floyd-Warshall (srt_fw.hip) closes LATENCIES only.  The
// reference's path cost is lexicographic (latency, loss) with loss folded from
// the source, one f32 rounding per op (graph/mod.rs:305-331):
//     l_0 = 0,  l_{k+1} = 1f32 - (1f32 - l_k) * (1f32 - e_k).
// petgraph's Dijkstra (strict `<`, visited set) returns for every target the
// lexicographic minimum over all paths; with latencies > 0 and the fold
// monotone in the prefix loss that is
//     loss[s][v] = min over tight in-edges (u -> v, e) of fold(loss[s][u], e),
//     tight: lat[s][u] + lat_e == lat[s][v],
// evaluated in increasing lat[s][.], loss[s][s] = 0.  Every tight predecessor
// has a strictly smaller latency, so it is final before v is read -- exactly
// what Dijkstra's settle order guarantees -- and the result is bit-identical.
//
// Two steps per build, after the closure:
//  1. tight-edge CSR.  An edge u -> v can be tight for some source only if its
//     own latency equals the closure's D[u][v] (else D[s][u] + D[u][v] would
//     beat it).  One pass over the adjacency flags those entries and counts
//     them per target, a scan and a fill build their pull CSR
//     {u, lat_e / g, 1f32 - e}.  On the 16k complete graph ~100 of the 16k
//     in-edges per vertex survive.
//  2. fold.  One workgroup per table row (source s) keeps lat[s][.] and
//     loss[s][.] in LDS (8 B per vertex: 16k vertices = 128 KiB), buckets the
//     vertices by latency (counting sort: bucket = lat >> shift, shift chosen so
//     the row's range fits NBK buckets) and processes the buckets in increasing
//     order, LPT lanes per target scanning its tight in-edges.  Bucket width 1
//     (shift 0) needs one pass per bucket: a tight predecessor is always in an
//     earlier bucket.  Wider buckets repeat the bucket until a pass changes
//     nothing (monotone fixpoint of the same fold, so the same bits).  The row
//     is then written out: latency = lat * g, loss, the raw self-loop on the
//     diagonal (mod.rs:210-217), min latency and unreachable count reduced into
//     stats (mod.rs:219, 474-476).
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr int NBK = 2048;        // latency buckets per row
constexpr int LOSS_NT = 1024;    // threads of the fold workgroup (16 waves)
constexpr size_t LDS_BUDGET = 160 * 1024 - 1024;

template <typename K>
struct KeyLat;
template <>
struct KeyLat<double> {
    static __device__ __forceinline__ bool inf(double k) { return !(k < 9007199254740992.0); }
    static __device__ __forceinline__ uint64_t lat(double k) { return (uint64_t)k; }
};
template <>
struct KeyLat<uint32_t> {
    static __device__ __forceinline__ bool inf(uint32_t k) { return k >= KEY32_INF; }
    static __device__ __forceinline__ uint64_t lat(uint32_t k) { return k; }
};
template <>
struct KeyLat<uint64_t> {
    static __device__ __forceinline__ bool inf(uint64_t k) { return k >= KEY_INF; }
    static __device__ __forceinline__ uint64_t lat(uint64_t k) { return k; }
};

// ---------------------------------------------------------- tight-edge CSR
// Pass 1 (one wave per adjacency row u): flag entry k (u -> v = col[k], not a
// self-loop) when lat[k] == D[u][v] * g, and count it for v.
template <typename K>
__global__ void tight_flag_kernel(const K *__restrict__ D, uint32_t Vp, uint32_t V,
                                  const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                                  const uint64_t *__restrict__ lat, uint64_t g, uint8_t *__restrict__ flag,
                                  uint32_t *__restrict__ cnt) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const K *Du = D + (uint64_t)u * Vp;
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            const uint32_t v = col[k];
            uint8_t f = 0;
            if (v != u) {
                const K d = Du[v];
                if (!KeyLat<K>::inf(d) && KeyLat<K>::lat(d) * g == lat[k]) {
                    f = 1;
                    atomicAdd(&cnt[v], 1u);
                }
            }
            flag[k] = f;
        }
    }
}

// Single workgroup: ptr = exclusive scan of cnt (ptr[V] = total), cnt reset
// to 0 (the fill cursor).
__global__ __launch_bounds__(1024) void tight_scan_kernel(uint32_t *__restrict__ cnt, uint64_t *__restrict__ ptr,
                                                          uint32_t V) {
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x, per = (V + 1023) / 1024;
    const uint32_t b = std::min<uint32_t>(V, t * per), e = std::min<uint32_t>(V, b + per);
    uint64_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += cnt[i];
    // inclusive scan of s over the block
    const int lane = t & 63, w = t >> 6;
    uint64_t x = s;
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int k = 0; k < 16; ++k) {
        if (k < w) before += wsum[k];
        all += wsum[k];
    }
    uint64_t run = before + x - s;
    for (uint32_t i = b; i < e; ++i) {
        ptr[i] = run;
        run += cnt[i];
        cnt[i] = 0;
    }
    if (t == 0) ptr[V] = all;
}

// Pass 2: place every flagged entry into its target's pull row.
template <typename LatT>
__global__ void tight_fill_kernel(uint32_t V, const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                                  const uint64_t *__restrict__ lat, const float *__restrict__ loss, uint64_t g,
                                  const uint8_t *__restrict__ flag, const uint64_t *__restrict__ ptr,
                                  uint32_t *__restrict__ cur, uint32_t *__restrict__ tu, LatT *__restrict__ tw,
                                  float *__restrict__ teb) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            if (!flag[k]) continue;
            const uint32_t v = col[k];
            const uint64_t pos = ptr[v] + atomicAdd(&cur[v], 1u);
            tu[pos] = u;
            tw[pos] = (LatT)(lat[k] / g);
            teb[pos] = 1.0f - loss[k];  // the reference's (1f32 - other.packet_loss), mod.rs:328
        }
    }
}

// ------------------------------------------------------------------- fold
__device__ __forceinline__ uint32_t lds_bytes_hist() { return ((NBK + 1) * 4 + 15) & ~15u; }

template <typename K, typename LatT, bool LROWS, int LPT>
__global__ __launch_bounds__(LOSS_NT) void tight_loss_kernel(
    const K *__restrict__ D, uint32_t Vp, uint32_t V, const uint32_t *__restrict__ nodes, uint32_t n,
    uint32_t row0, uint32_t row1, const uint64_t *__restrict__ tptr, const uint32_t *__restrict__ tu,
    const LatT *__restrict__ tw, const float *__restrict__ teb, uint64_t g, const uint64_t *__restrict__ sl_lat,
    const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat, float *__restrict__ out_loss,
    unsigned long long *stats, uint32_t *__restrict__ ord_all, LatT *lat_all, float *loss_all) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint64_t red[16];
    __shared__ unsigned long long red_min[16], red_cnt[16];
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem);
    LatT *lrow;
    float *prow;
    if constexpr (LROWS) {
        lrow = reinterpret_cast<LatT *>(smem + lds_bytes_hist());
        prow = reinterpret_cast<float *>(smem + lds_bytes_hist() + (((size_t)V * sizeof(LatT) + 15) & ~(size_t)15));
    } else {
        lrow = lat_all + (size_t)blockIdx.x * V;
        prow = loss_all + (size_t)blockIdx.x * V;
    }
    uint32_t *ord = ord_all + (size_t)blockIdx.x * V;
    const LatT LINF = (LatT)~(LatT)0;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const uint32_t grp = tid / LPT, sub = tid % LPT, ngrp = nt / LPT;
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;

    for (uint32_t i = row0 + blockIdx.x; i < row1; i += gridDim.x) {
        const uint32_t s = nodes[i];
        const K *Drow = D + (uint64_t)s * Vp;
        // 1. the row's latencies (units of g) and its largest finite one
        uint64_t mx = 0;
        for (uint32_t v = tid; v < V; v += nt) {
            const K k = Drow[v];
            const LatT l = KeyLat<K>::inf(k) ? LINF : (LatT)KeyLat<K>::lat(k);
            lrow[v] = l;
            prow[v] = __builtin_inff();
            if (l != LINF && (uint64_t)l > mx) mx = l;
        }
        for (uint32_t b = tid; b <= (uint32_t)NBK; b += nt) hist[b] = 0;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(mx, off);
            mx = o > mx ? o : mx;
        }
        if (lane == 0) red[wv] = mx;
        __syncthreads();
        mx = 0;
        for (int k = 0; k < nw; ++k) mx = red[k] > mx ? red[k] : mx;
        int shift = 0;
        while ((mx >> shift) >= (uint64_t)NBK) ++shift;
        // 2. counting sort of the reachable vertices (s excluded) by bucket
        for (uint32_t v = tid; v < V; v += nt) {
            const LatT l = lrow[v];
            if (v != s && l != LINF) atomicAdd(&hist[(uint64_t)l >> shift], 1u);
        }
        if (tid == 0) prow[s] = 0.0f;  // petgraph's zero score (0 ns, 0.0)
        __syncthreads();
        {  // exclusive scan of hist[0, NBK): each thread a contiguous run
            const uint32_t per = (NBK + nt - 1) / nt, b0 = std::min<uint32_t>(NBK, tid * per),
                           b1 = std::min<uint32_t>(NBK, b0 + per);
            uint32_t sum = 0;
            for (uint32_t b = b0; b < b1; ++b) sum += hist[b];
            uint32_t x = sum;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            __syncthreads();  // everyone has read hist before it is rewritten
            if (lane == 63) red[wv] = x;
            __syncthreads();
            uint32_t run = x - sum;
            for (int k = 0; k < wv; ++k) run += (uint32_t)red[k];
            for (uint32_t b = b0; b < b1; ++b) {
                const uint32_t c = hist[b];
                hist[b] = run;
                run += c;
            }
        }
        __syncthreads();
        for (uint32_t v = tid; v < V; v += nt) {
            const LatT l = lrow[v];
            if (v != s && l != LINF) ord[atomicAdd(&hist[(uint64_t)l >> shift], 1u)] = v;
        }
        __syncthreads();
        // hist[b] is now the end of bucket b (its start: hist[b-1], or 0)
        // 3. buckets in increasing latency
        const uint32_t nb = (uint32_t)(mx >> shift) + 1;
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t m0 = b ? hist[b - 1] : 0u, m1 = hist[b];
            if (m0 == m1) continue;  // uniform
            for (;;) {
                int changed = 0;
                for (uint32_t base = m0; base < m1; base += ngrp) {
                    const uint32_t m = base + grp;
                    const bool act = m < m1;
                    uint32_t v = 0;
                    float best = __builtin_inff();
                    if (act) {
                        v = ord[m];
                        const LatT lv = lrow[v];
                        const uint64_t e1 = tptr[v + 1];
                        for (uint64_t e = tptr[v] + sub; e < e1; e += 2 * LPT) {
                            const uint64_t e2 = e + LPT;
                            const bool h2 = e2 < e1;
                            const LatT w1 = tw[e], w2 = h2 ? tw[e2] : LINF;
                            const uint32_t u1 = tu[e], u2 = h2 ? tu[e2] : 0u;
                            const float b1 = teb[e], b2 = h2 ? teb[e2] : 0.0f;
                            if (w1 <= lv && lrow[u1] == lv - w1)
                                best = fminf(best, 1.0f - __fmul_rn(1.0f - prow[u1], b1));
                            if (w2 <= lv && lrow[u2] == lv - w2)
                                best = fminf(best, 1.0f - __fmul_rn(1.0f - prow[u2], b2));
                        }
                    }
#pragma unroll
                    for (int off = LPT / 2; off > 0; off >>= 1) best = fminf(best, __shfl_xor(best, off));
                    if (act && sub == 0 && best < prow[v]) {
                        prow[v] = best;
                        changed = 1;
                    }
                }
                const int any = __syncthreads_or(changed);
                if (shift == 0 || !any) break;  // width-1 buckets: one pass is exact
            }
        }
        // 4. table row i
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        for (uint32_t j = tid; j < n; j += nt) {
            uint64_t latv;
            float lossv;
            if (j == i) {
                latv = sl_lat[j];
                lossv = sl_loss[j];
            } else {
                const uint32_t v = nodes[j];
                const LatT l = lrow[v];
                if (l == LINF) {
                    ++unreach;
                    latv = ~0ull;
                    lossv = 1.0f;
                } else {
                    latv = (uint64_t)l * g;
                    lossv = prow[v];
                }
            }
            ol[j] = latv;
            op[j] = lossv;
            mn = latv < mn ? latv : mn;
        }
        __syncthreads();  // the next row rewrites the LDS rows
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mn, off);
        mn = o < mn ? o : mn;
        unreach += __shfl_xor(unreach, off);
    }
    if (lane == 0) {
        red_min[wv] = mn;
        red_cnt[wv] = unreach;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], c = red_cnt[0];
        for (int k = 1; k < nw; ++k) {
            m = red_min[k] < m ? red_min[k] : m;
            c += red_cnt[k];
        }
        atomicMin(&stats[0], m);
        if (c) atomicAdd(&stats[1], c);
    }
}

__global__ void loss_stats_init_kernel(unsigned long long *stats) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
}

template <typename T>
srt_status grow(T **p, uint64_t *cap, uint64_t need, srt_err *err, const char *what) {
    if (need <= *cap && *p) return SRT_OK;
    hipFree(*p);
    *p = nullptr;
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, std::max<uint64_t>(need, 1) * sizeof(T));
    if (e != hipSuccess) {
        if (err) {
            err->code = e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "hipMalloc(%s): %s", what, hipGetErrorString(e));
        }
        return e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
    }
    *p = (T *)q;
    *cap = need;
    return SRT_OK;
}

int cu_count(int dev) {
    static int cached[64] = {0};
    if (dev >= 0 && dev < 64 && cached[dev]) return cached[dev];
    int c = 256;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    if (dev >= 0 && dev < 64) cached[dev] = c;
    return c;
}

template <typename K, typename LatT, bool LROWS, int LPT>
srt_status launch_fold(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    const uint32_t V = p->V, rows = p->row1 - p->row0;
    const uint32_t nt = V >= 2048 ? LOSS_NT : 256;
    const size_t hist_b = ((NBK + 1) * 4 + 15) & ~(size_t)15;
    const size_t lds = LROWS ? hist_b + (((size_t)V * sizeof(LatT) + 15) & ~(size_t)15) + (size_t)V * 4 : hist_b;
    const int per_cu_threads = 2048 / (int)nt;
    int per_cu_lds = (int)std::max<size_t>(1, (160 * 1024) / (lds + 2048));
    const int per_cu = std::max(1, std::min(per_cu_threads, per_cu_lds));
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(rows, (uint32_t)(cu_count(p->device) * per_cu)));
    auto up16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t ord_b = up16((size_t)grid * V * 4), lat_b = LROWS ? 0 : up16((size_t)grid * V * sizeof(LatT)),
                 loss_b = LROWS ? 0 : up16((size_t)grid * V * 4);
    uint64_t cap = p->lscratch_cap;
    srt_status st = grow(reinterpret_cast<uint8_t **>(&p->d_lscratch), &cap, ord_b + lat_b + loss_b + 64, err,
                         "loss scratch");
    if (st != SRT_OK) return st;
    p->lscratch_cap = cap;
    uint8_t *base = reinterpret_cast<uint8_t *>(p->d_lscratch);
    uint32_t *ord = reinterpret_cast<uint32_t *>(base);
    LatT *lat_all = reinterpret_cast<LatT *>(base + ord_b);
    float *loss_all = reinterpret_cast<float *>(base + ord_b + lat_b);
    auto kern = tight_loss_kernel<K, LatT, LROWS, LPT>;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (rows)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, p->stream, reinterpret_cast<const K *>(p->d_D), p->Vp, V,
                           p->d_nodes, p->n, p->row0, p->row1, p->d_tptr, p->d_tu,
                           reinterpret_cast<const LatT *>(p->d_tw), p->d_teb, p->kp.g, p->d_sl_lat, p->d_sl_loss,
                           p->d_out_lat, p->d_out_loss, d_stats, ord, lat_all, loss_all);
    return SRT_OK;
}

template <typename K, typename LatT, bool LROWS>
srt_status launch_fold_lpt(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    // lanes per target ~ the average tight in-degree (a group walks a
    // target's in-edges two per lane per step)
    const double avg = p->V ? (double)p->t_edges / p->V : 0.0;
    if (avg > 48.0) return launch_fold<K, LatT, LROWS, 32>(p, d_stats, err);
    if (avg > 10.0) return launch_fold<K, LatT, LROWS, 8>(p, d_stats, err);
    return launch_fold<K, LatT, LROWS, 2>(p, d_stats, err);
}

template <typename K>
srt_status fw_loss_t(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    srt_status st;
    uint64_t cap_flag = p->d_tflag ? p->n_adj : 0, cap_cnt = p->d_tcnt ? V : 0, cap_ptr = p->d_tptr ? V + 1ull : 0;
    if ((st = grow(&p->d_tflag, &cap_flag, p->n_adj, err, "tight flags")) != SRT_OK ||
        (st = grow(&p->d_tcnt, &cap_cnt, V, err, "tight counts")) != SRT_OK ||
        (st = grow(&p->d_tptr, &cap_ptr, V + 1ull, err, "tight ptr")) != SRT_OK)
        return st;
    if (!p->h_tcount) {
        const hipError_t e = hipHostMalloc((void **)&p->h_tcount, sizeof(uint64_t), 0);
        if (e != hipSuccess) {
            if (err) {
                err->code = SRT_ERR_HIP;
                std::snprintf(err->msg, sizeof err->msg, "hipHostMalloc: %s", hipGetErrorString(e));
            }
            return SRT_ERR_HIP;
        }
    }
    if (!p->ev_loss0) {
        hipEventCreate(&p->ev_loss0);
        hipEventCreate(&p->ev_loss1);
    }
    hipEventRecord(p->ev_loss0, M);
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats);
    hipMemsetAsync(p->d_tcnt, 0, (size_t)V * 4, M);
    const K *D = reinterpret_cast<const K *>(p->d_D);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    if (V) {
        hipLaunchKernelGGL(tight_flag_kernel<K>, dim3(blocks), dim3(256), 0, M, D, p->Vp, V, p->d_row_ptr, p->d_col,
                           p->d_lat, p->kp.g, p->d_tflag, p->d_tcnt);
        hipLaunchKernelGGL(tight_scan_kernel, dim3(1), dim3(1024), 0, M, p->d_tcnt, p->d_tptr, V);
        hipMemcpyAsync(p->h_tcount, p->d_tptr + V, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
    } else {
        *p->h_tcount = 0;
    }
    hipError_t e = hipStreamSynchronize(M);
    if (e != hipSuccess) {
        if (err) {
            err->code = SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "tight-edge count: %s", hipGetErrorString(e));
        }
        return SRT_ERR_HIP;
    }
    p->t_edges = *p->h_tcount;
    const size_t wsz = p->kp.lat32 ? 4 : 8;
    if (p->t_edges > p->t_cap || !p->d_tu) {
        // grow all three arrays together (25% headroom)
        const uint64_t cap = std::max<uint64_t>(p->t_edges + p->t_edges / 4, 1024);
        hipFree(p->d_tu);
        hipFree(p->d_tw);
        hipFree(p->d_teb);
        p->d_tu = nullptr;
        p->d_tw = nullptr;
        p->d_teb = nullptr;
        p->t_cap = 0;
        void *a = nullptr, *b = nullptr, *c = nullptr;
        e = hipMalloc(&a, cap * 4);
        if (e == hipSuccess) e = hipMalloc(&b, cap * wsz);
        if (e == hipSuccess) e = hipMalloc(&c, cap * 4);
        if (e != hipSuccess) {
            hipFree(a);
            hipFree(b);
            if (err) {
                err->code = e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
                std::snprintf(err->msg, sizeof err->msg, "hipMalloc(tight edges): %s", hipGetErrorString(e));
            }
            return e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
        }
        p->d_tu = (uint32_t *)a;
        p->d_tw = b;
        p->d_teb = (float *)c;
        p->t_cap = cap;
    }
    if (V) {
        if (p->kp.lat32)
            hipLaunchKernelGGL(tight_fill_kernel<uint32_t>, dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr, p->d_col,
                               p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt, p->d_tu,
                               (uint32_t *)p->d_tw, p->d_teb);
        else
            hipLaunchKernelGGL(tight_fill_kernel<uint64_t>, dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr, p->d_col,
                               p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt, p->d_tu,
                               (uint64_t *)p->d_tw, p->d_teb);
    }
    const size_t hist_b = ((NBK + 1) * 4 + 15) & ~(size_t)15;
    if (p->kp.lat32) {
        if (hist_b + (size_t)V * 8 + 16 <= LDS_BUDGET) st = launch_fold_lpt<K, uint32_t, true>(p, d_stats, err);
        else st = launch_fold_lpt<K, uint32_t, false>(p, d_stats, err);
    } else {
        st = launch_fold_lpt<K, uint64_t, false>(p, d_stats, err);
    }
    if (st != SRT_OK) return st;
    hipEventRecord(p->ev_loss1, M);
    return SRT_OK;
}

}  // namespace

srt_status fw_loss(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    if (p->key_type == KEY_U32) return fw_loss_t<uint32_t>(p, d_stats, err);
    return p->key_type == KEY_F64 ? fw_loss_t<double>(p, d_stats, err) : fw_loss_t<uint64_t>(p, d_stats, err);
}

}  // namespace srt
