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
//     them per target, a scan and a fill build their pull CSR.  On the 16k
//     complete graph ~155 of the 16k in-edges per vertex survive.  When the
//     vertex index and the largest tight latency fit 32 bits together, an
//     entry is ONE u64, (1f32 - e) bits << 32 | (w << ubits) | u, and every
//     target's row is sorted by w (rocPRIM segmented radix sort on the w bits)
//     so a scan stops at the first w > lat[s][v].
//  2. fold.  One workgroup per table row (source s) keeps lat[s][.] and
//     loss[s][.] in LDS (8 B per vertex: 16k vertices = 128 KiB), buckets the
//     vertices by latency (counting sort: bucket = lat >> shift, shift chosen so
//     the row's range fits NBK buckets; wave-aggregated LDS atomics when the
//     row has few buckets; the sorted order holds 16-B records {v, first and
//     end in-edge, lat[s][v]}) and processes the buckets in increasing order,
//     LPT lanes per target scanning its tight in-edges, candidates min-ed into
//     loss[s][v] by LDS atomics on the f32 bits.  Bucket width 1 (shift 0)
//     needs one pass per bucket: a tight predecessor is always in an earlier
//     bucket.  Wider buckets repeat the bucket until a pass changes nothing
//     (monotone fixpoint of the same fold, so the same bits).  The row is then
//     written out: latency = lat * g, loss, the raw self-loop on the diagonal
//     (mod.rs:210-217), min latency and unreachable count reduced into stats
//     (mod.rs:219, 474-476).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr int NBK = 2048;        // latency buckets per row
constexpr int LOSS_NT = 1024;    // threads of the fold workgroup (16 waves)
constexpr size_t LDS_BUDGET = 160 * 1024 - 1024;

template <typename K>
struct KeyLat;
template <>
struct KeyLat<uint32_t> {
    static __device__ __forceinline__ bool inf(uint32_t k) { return k >= KEY32_INF; }
    static __device__ __forceinline__ uint64_t lat(uint32_t k) { return k; }
};
template <>
struct KeyLat<double> {
    static __device__ __forceinline__ bool inf(double k) { return !(k < 9007199254740992.0); }
    static __device__ __forceinline__ uint64_t lat(double k) { return (uint64_t)k; }
};
template <>
struct KeyLat<uint64_t> {
    static __device__ __forceinline__ bool inf(uint64_t k) { return k >= KEY_INF; }
    static __device__ __forceinline__ uint64_t lat(uint64_t k) { return k; }
};

// latency (units of g) of closure entry idx; kt = srt_plan::key_type (uniform)
__device__ __forceinline__ uint64_t closure_lat(const void *D, uint64_t idx, int kt, bool &inf) {
    if (kt == KEY_U32) {
        const uint32_t k = reinterpret_cast<const uint32_t *>(D)[idx];
        inf = KeyLat<uint32_t>::inf(k);
        return k;
    }
    if (kt == KEY_F64) {
        const double k = reinterpret_cast<const double *>(D)[idx];
        inf = KeyLat<double>::inf(k);
        return inf ? 0 : KeyLat<double>::lat(k);
    }
    const uint64_t k = reinterpret_cast<const uint64_t *>(D)[idx];
    inf = KeyLat<uint64_t>::inf(k);
    return k;
}

// ---------------------------------------------------------- tight-edge CSR
// Pass 1 (one wave per adjacency row u): flag entry k (u -> v = col[k], not a
// self-loop) when lat[k] == D[u][v] * g, count it for v, track the largest
// tight latency.
template <typename K>
__global__ void tight_flag_kernel(const K *__restrict__ D, uint32_t Vp, uint32_t V,
                                  const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                                  const uint64_t *__restrict__ lat, uint64_t g, uint8_t *__restrict__ flag,
                                  uint32_t *__restrict__ cnt, unsigned long long *maxw) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    uint64_t mw = 0;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const K *Du = D + (uint64_t)u * Vp;
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            const uint32_t v = col[k];
            uint8_t f = 0;
            if (v != u) {
                const K d = Du[v];
                const uint64_t w = KeyLat<K>::lat(d);
                if (!KeyLat<K>::inf(d) && w * g == lat[k]) {
                    f = 1;
                    atomicAdd(&cnt[v], 1u);
                    mw = w > mw ? w : mw;
                }
            }
            flag[k] = f;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mw, off);
        mw = o > mw ? o : mw;
    }
    if (lane == 0 && mw) atomicMax(maxw, (unsigned long long)mw);
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

// Pass 2: place every flagged entry into its target's pull row; PACKED: one
// u64 per entry, (1f32 - e) bits << 32 | (w << ubits) | u, else separate
// u / w / 1-e arrays.
template <typename LatT, bool PACKED>
__global__ void tight_fill_kernel(uint32_t V, const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                                  const uint64_t *__restrict__ lat, const float *__restrict__ loss, uint64_t g,
                                  const uint8_t *__restrict__ flag, const uint64_t *__restrict__ ptr,
                                  uint32_t *__restrict__ cur, uint32_t *__restrict__ tu, LatT *__restrict__ tw,
                                  float *__restrict__ teb, uint64_t *__restrict__ tpk, uint32_t ubits) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            if (!flag[k]) continue;
            const uint32_t v = col[k];
            const uint64_t pos = ptr[v] + atomicAdd(&cur[v], 1u);
            const uint64_t w = lat[k] / g;
            const float eb = 1.0f - loss[k];  // the reference's (1f32 - other.packet_loss), mod.rs:328
            if constexpr (PACKED) {
                tpk[pos] = ((uint64_t)__float_as_uint(eb) << 32) | (((uint32_t)w << ubits) | u);
            } else {
                tu[pos] = u;
                tw[pos] = (LatT)w;
                teb[pos] = eb;
            }
        }
    }
}

// ------------------------------------------------------------------- fold
// The whole wave calls this (uniform trip counts): for every active lane,
// the old value of hist[b] + its rank among the wave's lanes with the same b,
// and hist[b] incremented by their count -- one LDS atomic per distinct b.
__device__ __forceinline__ uint32_t agg_inc(uint32_t *hist, uint32_t b, bool active) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t todo = __ballot(active);
    uint32_t res = 0;
    while (todo) {
        const int leader = __builtin_ctzll(todo);
        const uint32_t lb = __builtin_amdgcn_readlane(b, leader);
        const uint64_t m = __ballot(active && b == lb) & todo;
        uint32_t base = 0;
        if (lane == (uint32_t)leader) base = atomicAdd(&hist[lb], (uint32_t)__popcll(m));
        base = __builtin_amdgcn_readlane(base, leader);
        if ((m >> lane) & 1ull) res = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        todo &= ~m;
    }
    return res;
}

constexpr uint32_t HIST_BYTES = ((NBK + 1) * 4 + 15) & ~15u;

// One pass over the members ord[m0, m1) of a bucket, packed form: LPT lanes
// per target, UNR in-edges per lane per step (loads in flight: the scan is
// latency bound).  The edge array is padded past its end, so the UNR loads of
// a step are unconditional (one 8-B load each:
// {word, 1-e}); a slot counts only if it is inside the row and its w <= lv
// (rows are sorted by w).  Tight
// candidates go into prow[v] by LDS atomic min on the f32 bits (non-negative
// floats order like their bits); a tight edge with w == lv can only start at
// s (every other vertex has latency >= 1), and those were pushed from s's
// adjacency row beforehand, so a lane stops at w >= lv.  ITER (buckets wider
// than one latency) also
// reports whether any value dropped.  The next target's record is loaded
// while the current one is scanned.
template <typename LatT, int LPT, int UNR, bool ITER>
__device__ __forceinline__ int scan_bucket_packed(const uint4 *__restrict__ ord, uint32_t m0, uint32_t m1,
                                                  uint32_t grp, uint32_t sub, uint32_t ngrp,
                                                  const uint64_t *__restrict__ tpk, const LatT *lrow, float *prow,
                                                  uint32_t ubits, uint32_t umask) {
    int changed = 0;
    uint32_t m = m0 + grp;
    uint4 rec = m < m1 ? ord[m] : make_uint4(0, 0, 0, 0);
    for (; m < m1; m += ngrp) {
        const uint4 cur = rec;
        if (m + ngrp < m1) rec = ord[m + ngrp];
        const uint32_t v = cur.x, e1 = cur.z;
        const LatT lv = (LatT)cur.w;
        const uint64_t *wp = tpk + cur.y + sub;
        uint32_t *dst = reinterpret_cast<uint32_t *>(prow) + v;
        for (uint32_t e = cur.y + sub; e < e1; e += UNR * LPT, wp += UNR * LPT) {
            uint64_t wd[UNR];
#pragma unroll
            for (int q = 0; q < UNR; ++q) wd[q] = wp[q * LPT];
            bool ok[UNR];
            uint32_t u[UNR];
            LatT need[UNR], lu[UNR];
#pragma unroll
            for (int q = 0; q < UNR; ++q) {
                const uint32_t lo = (uint32_t)wd[q], w = lo >> ubits;
                ok[q] = e + q * LPT < e1 && (LatT)w < lv;  // w == lv: only from s (pushed)
                u[q] = ok[q] ? lo & umask : 0u;
                need[q] = lv - (LatT)w;
            }
#pragma unroll
            for (int q = 0; q < UNR; ++q) lu[q] = lrow[u[q]];
#pragma unroll
            for (int q = 0; q < UNR; ++q) {
                if (ok[q] && lu[q] == need[q]) {
                    const float c = 1.0f - __fmul_rn(1.0f - prow[u[q]], __uint_as_float((uint32_t)(wd[q] >> 32)));
                    if constexpr (ITER) changed |= __float_as_uint(c) < atomicMin(dst, __float_as_uint(c));
                    else atomicMin(dst, __float_as_uint(c));
                }
            }
            if (!ok[UNR - 1]) break;
        }
    }
    return changed;
}

template <typename LatT, bool LROWS, int LPT, bool PACKED>
__global__ __launch_bounds__(LOSS_NT) void tight_loss_kernel(
    const void *__restrict__ D, int key_type, uint32_t Vp, uint32_t V, const uint32_t *__restrict__ nodes,
    uint32_t n, uint32_t row0, uint32_t row1, const uint64_t *__restrict__ tptr, const uint32_t *__restrict__ tu,
    const LatT *__restrict__ tw, const float *__restrict__ teb, const uint64_t *__restrict__ tpk, uint32_t ubits,
    uint64_t g, const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss,
    uint64_t *__restrict__ out_lat, float *__restrict__ out_loss, unsigned long long *stats,
    uint4 *__restrict__ ord_all, LatT *lat_all, float *loss_all, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, const uint64_t *__restrict__ elat, const float *__restrict__ eloss,
    uint32_t diag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint64_t red[16];
    __shared__ unsigned long long red_min[16], red_cnt[16];
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem);
    LatT *lrow;
    float *prow;
    if constexpr (LROWS) {
        lrow = reinterpret_cast<LatT *>(smem + HIST_BYTES);
        prow = reinterpret_cast<float *>(smem + HIST_BYTES + (((size_t)V * sizeof(LatT) + 15) & ~(size_t)15));
    } else {
        lrow = lat_all + (size_t)blockIdx.x * V;
        prow = loss_all + (size_t)blockIdx.x * V;
    }
    // ord[pos] = {v, first tight in-edge, end, lat[s][v]} in bucket order: the
    // member loop needs one 16-B load per target, no tptr / lrow lookups
    uint4 *ord = ord_all + (size_t)blockIdx.x * V;
    const LatT LINF = (LatT)~(LatT)0;
    const uint32_t umask = (1u << ubits) - 1u;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const uint32_t grp = tid / LPT, sub = tid % LPT, ngrp = nt / LPT;
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;

    for (uint32_t i = row0 + blockIdx.x; i < row1; i += gridDim.x) {
        const uint32_t s = nodes[i];
        // 1. the row's latencies (units of g) and its largest finite one
        uint64_t mx = 0;
        for (uint32_t v = tid; v < V; v += nt) {
            bool inf;
            const uint64_t l64 = closure_lat(D, (uint64_t)s * Vp + v, key_type, inf);
            const LatT l = inf ? LINF : (LatT)l64;
            lrow[v] = l;
            prow[v] = __builtin_inff();
            if (!inf && l64 > mx) mx = l64;
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
        // diag (timing-only knob SRT_LOSS_DIAG, wrong tables): bit 0 skips the
        // bucket scans, bit 1 the row output, bit 2 the counting sort
        const uint32_t nb = (diag & 5u) ? 0u : (uint32_t)(mx >> shift) + 1;
        const bool few = nb <= 64;  // uniform: aggregate the LDS atomics per wave
        // 2. counting sort of the reachable vertices (s excluded) by bucket
        for (uint32_t base = 0; base < ((diag & 4u) ? 0u : V); base += nt) {
            const uint32_t v = base + tid;
            const LatT l = v < V ? lrow[v] : LINF;
            const bool ok = v < V && v != s && l != LINF;
            const uint32_t b = ok ? (uint32_t)((uint64_t)l >> shift) : 0u;
            if (few) agg_inc(hist, b, ok);
            else if (ok) atomicAdd(&hist[b], 1u);
        }
        if (tid == 0) prow[s] = 0.0f;  // petgraph's zero score (0 ns, 0.0)
        __syncthreads();
        // the one-hop tight paths: s's own edges s -> v with lat == lat[s][v]
        // (fold(0, e) = 1 - (1 - 0) (1 - e)); the bucket scans then skip
        // every in-edge with w == lat[s][v], whose tail can only be s
        for (uint64_t k = row_ptr[s] + tid; k < row_ptr[s + 1]; k += nt) {
            const uint32_t v = col[k];
            const LatT l = lrow[v];
            if (v != s && l != LINF && (uint64_t)l * g == elat[k]) {
                const float c = 1.0f - __fmul_rn(1.0f - 0.0f, 1.0f - eloss[k]);
                atomicMin(reinterpret_cast<uint32_t *>(prow) + v, __float_as_uint(c));
            }
        }
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
            __syncthreads();  // everyone has read red (max) before it is rewritten
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
        for (uint32_t base = 0; base < ((diag & 4u) ? 0u : V); base += nt) {
            const uint32_t v = base + tid;
            const LatT l = v < V ? lrow[v] : LINF;
            const bool ok = v < V && v != s && l != LINF;
            const uint32_t b = ok ? (uint32_t)((uint64_t)l >> shift) : 0u;
            uint32_t pos = 0;
            if (few) pos = agg_inc(hist, b, ok);
            else if (ok) pos = atomicAdd(&hist[b], 1u);
            if (ok) ord[pos] = make_uint4(v, (uint32_t)tptr[v], (uint32_t)tptr[v + 1], (uint32_t)l);
        }
        __syncthreads();
        // hist[b] is now the end of bucket b (its start: hist[b-1], or 0)
        // 3. buckets in increasing latency
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t m0 = b ? hist[b - 1] : 0u, m1 = hist[b];
            if (m0 == m1) continue;  // uniform
            for (;;) {
                int changed = 0;
                if constexpr (PACKED) {
                    if (shift)
                        changed = scan_bucket_packed<LatT, LPT, 8, true>(ord, m0, m1, grp, sub, ngrp, tpk, lrow, prow,
                                                                      ubits, umask);
                    else
                        scan_bucket_packed<LatT, LPT, 8, false>(ord, m0, m1, grp, sub, ngrp, tpk, lrow, prow, ubits,
                                                             umask);
                } else {
                    for (uint32_t base = m0; base < m1; base += ngrp) {
                        const uint32_t m = base + grp;
                        const bool act = m < m1;
                        uint32_t v = 0;
                        float best = __builtin_inff();
                        if (act) {
                            const uint4 rec = ord[m];
                            v = rec.x;
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
                }
                const int any = __syncthreads_or(changed);
                if (shift == 0 || !any) break;  // width-1 buckets: one pass is exact
            }
        }
        // 4. table row i
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        for (uint32_t j = tid; j < ((diag & 2u) ? 0u : n); j += nt) {
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

__global__ void loss_stats_init_kernel(unsigned long long *stats, unsigned long long *maxw) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
    *maxw = 0ull;
}

srt_status fail(srt_err *err, hipError_t e, const char *what) {
    const srt_status st = e == hipErrorOutOfMemory ? SRT_ERR_OOM : SRT_ERR_HIP;
    if (err) {
        err->code = st;
        std::snprintf(err->msg, sizeof err->msg, "%s: %s", what, hipGetErrorString(e));
    }
    return st;
}

template <typename T>
srt_status grow(T **p, uint64_t *cap, uint64_t need, srt_err *err, const char *what) {
    if (need <= *cap && *p) return SRT_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, std::max<uint64_t>(need, 1) * sizeof(T));
    if (e != hipSuccess) return fail(err, e, what);
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

int bits_of(uint64_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

template <typename LatT, bool LROWS, int LPT, bool PACKED>
srt_status launch_fold(srt_plan *p, unsigned long long *d_stats, uint32_t ubits, srt_err *err) {
    const uint32_t V = p->V, rows = p->row1 - p->row0;
    const uint32_t nt = V >= 2048 ? LOSS_NT : 256;
    const size_t lds = LROWS ? HIST_BYTES + (((size_t)V * sizeof(LatT) + 15) & ~(size_t)15) + (size_t)V * 4
                             : HIST_BYTES;
    const int per_cu_threads = 2048 / (int)nt;
    const int per_cu_lds = (int)std::max<size_t>(1, (160 * 1024) / (lds + 2048));
    const int per_cu = std::max(1, std::min(per_cu_threads, per_cu_lds));
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(rows, (uint32_t)(cu_count(p->device) * per_cu)));
    auto up16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t ord_b = up16((size_t)grid * V * 16), lat_b = LROWS ? 0 : up16((size_t)grid * V * sizeof(LatT)),
                 loss_b = LROWS ? 0 : up16((size_t)grid * V * 4);
    uint64_t cap = p->lscratch_cap;
    srt_status st = grow(reinterpret_cast<uint8_t **>(&p->d_lscratch), &cap, ord_b + lat_b + loss_b + 64, err,
                         "hipMalloc(loss scratch)");
    p->lscratch_cap = cap;
    if (st != SRT_OK) return st;
    uint8_t *base = reinterpret_cast<uint8_t *>(p->d_lscratch);
    uint4 *ord = reinterpret_cast<uint4 *>(base);
    LatT *lat_all = reinterpret_cast<LatT *>(base + ord_b);
    float *loss_all = reinterpret_cast<float *>(base + ord_b + lat_b);
    auto kern = tight_loss_kernel<LatT, LROWS, LPT, PACKED>;
    static bool lds_attr_set = false;  // per instantiation
    if (LROWS && !lds_attr_set) {
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(LDS_BUDGET - 4096));
        lds_attr_set = true;
    }
    if (rows)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, p->stream, (const void *)p->d_D, p->key_type, p->Vp, V,
                           p->d_nodes, p->n, p->row0, p->row1, p->d_tptr, p->d_tu,
                           reinterpret_cast<const LatT *>(p->d_tw), p->d_teb, p->d_tpk, ubits, p->kp.g, p->d_sl_lat,
                           p->d_sl_loss, p->d_out_lat, p->d_out_loss, d_stats, ord, lat_all, loss_all, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, std::getenv("SRT_LOSS_DIAG") ? (uint32_t)std::atoi(std::getenv("SRT_LOSS_DIAG")) : 0u);
    return SRT_OK;
}

template <typename LatT, bool LROWS, bool PACKED>
srt_status launch_fold_lpt(srt_plan *p, unsigned long long *d_stats, uint32_t ubits, srt_err *err) {
    // lanes per target ~ the average tight in-degree (a group walks a target's
    // in-edges 2-4 per lane per step)
    const double avg = p->V ? (double)p->t_edges / p->V : 0.0;
    if constexpr (PACKED) {
        // 4 lanes x 8 edges per target (C3, same box: 4 / 8 / 16 lanes ->
        // 31.9 / 33.0 / 36.5 ms for the pass; knob SRT_LOSS_LPT = 8 / 16)
        const char *k = std::getenv("SRT_LOSS_LPT");
        if (k && std::atoi(k) == 8) return launch_fold<LatT, LROWS, 8, PACKED>(p, d_stats, ubits, err);
        if (k && std::atoi(k) == 16) return launch_fold<LatT, LROWS, 16, PACKED>(p, d_stats, ubits, err);
        if (avg > 10.0) return launch_fold<LatT, LROWS, 4, PACKED>(p, d_stats, ubits, err);
        return launch_fold<LatT, LROWS, 2, PACKED>(p, d_stats, ubits, err);
    }
    if (avg > 48.0) return launch_fold<LatT, LROWS, 32, PACKED>(p, d_stats, ubits, err);
    if (avg > 10.0) return launch_fold<LatT, LROWS, 8, PACKED>(p, d_stats, ubits, err);
    return launch_fold<LatT, LROWS, 2, PACKED>(p, d_stats, ubits, err);
}

template <typename K>
srt_status tight_csr_t(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    srt_status st;
    uint64_t cap_flag = p->d_tflag ? p->n_adj : 0, cap_cnt = p->d_tcnt ? V : 0, cap_ptr = p->d_tptr ? V + 1ull : 0,
             cap_mw = p->d_tmaxw ? 1 : 0;
    if ((st = grow(&p->d_tflag, &cap_flag, p->n_adj, err, "hipMalloc(tight flags)")) != SRT_OK ||
        (st = grow(&p->d_tcnt, &cap_cnt, V, err, "hipMalloc(tight counts)")) != SRT_OK ||
        (st = grow(&p->d_tptr, &cap_ptr, V + 1ull, err, "hipMalloc(tight ptr)")) != SRT_OK ||
        (st = grow(&p->d_tmaxw, &cap_mw, 1, err, "hipMalloc(tight max)")) != SRT_OK)
        return st;
    if (!p->h_tcount) {
        const hipError_t e = hipHostMalloc((void **)&p->h_tcount, 2 * sizeof(uint64_t), 0);
        if (e != hipSuccess) return fail(err, e, "hipHostMalloc");
    }
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats,
                       (unsigned long long *)p->d_tmaxw);
    (void)hipMemsetAsync(p->d_tcnt, 0, (size_t)V * 4, M);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    p->h_tcount[0] = p->h_tcount[1] = 0;
    if (V) {
        hipLaunchKernelGGL(tight_flag_kernel<K>, dim3(blocks), dim3(256), 0, M, reinterpret_cast<const K *>(p->d_D),
                           p->Vp, V, p->d_row_ptr, p->d_col, p->d_lat, p->kp.g, p->d_tflag, p->d_tcnt,
                           (unsigned long long *)p->d_tmaxw);
        hipLaunchKernelGGL(tight_scan_kernel, dim3(1), dim3(1024), 0, M, p->d_tcnt, p->d_tptr, V);
        (void)hipMemcpyAsync(p->h_tcount, p->d_tptr + V, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
        (void)hipMemcpyAsync(p->h_tcount + 1, p->d_tmaxw, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
    }
    hipError_t e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(err, e, "tight-edge count");
    p->t_edges = p->h_tcount[0];
    const uint64_t maxw = p->h_tcount[1];
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    // packed form: u and w share one word, rows sorted by w (knob
    // SRT_LOSS_UNPACKED=1 forces the 3-array form for A/B and parity tests)
    p->t_packed = p->kp.lat32 && ubits + bits_of(maxw) <= 32 && p->t_edges < (1ull << 32) &&
                  !std::getenv("SRT_LOSS_UNPACKED");
    const size_t wsz = p->kp.lat32 ? 4 : 8;
    if (p->t_edges + 1024 > p->t_cap || !p->d_tu) {
        // grow every edge array together (25% headroom)
        // (+1024: the packed scan reads up to (UNR - 1) * LPT entries past a row's end)
        const uint64_t cap = std::max<uint64_t>(p->t_edges + p->t_edges / 4 + 1024, 2048);
        for (void *q : {(void *)p->d_tu, p->d_tw, (void *)p->d_teb, (void *)p->d_tpk, (void *)p->d_tpk2})
            (void)hipFree(q);
        p->d_tu = nullptr;
        p->d_tw = nullptr;
        p->d_teb = nullptr;
        p->d_tpk = p->d_tpk2 = nullptr;
        p->t_cap = 0;
        void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr, *f = nullptr;
        e = hipMalloc(&a, cap * 4);
        if (e == hipSuccess) e = hipMalloc(&b, cap * wsz);
        if (e == hipSuccess) e = hipMalloc(&c, cap * 4);
        if (e == hipSuccess) e = hipMalloc(&d, cap * 8);
        if (e == hipSuccess) e = hipMalloc(&f, cap * 8);
        if (e != hipSuccess) {
            for (void *q : {a, b, c, d}) (void)hipFree(q);
            return fail(err, e, "hipMalloc(tight edges)");
        }
        p->d_tu = (uint32_t *)a;
        p->d_tw = b;
        p->d_teb = (float *)c;
        p->d_tpk = (uint64_t *)d;
        p->d_tpk2 = (uint64_t *)f;
        p->t_cap = cap;
    }
    if (!V) return SRT_OK;
    if (p->t_packed) {
        hipLaunchKernelGGL((tight_fill_kernel<uint32_t, true>), dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt,
                           (uint32_t *)nullptr, (uint32_t *)nullptr, (float *)nullptr, p->d_tpk2, ubits);
        // every target's row sorted by w (bits ubits .. of the low word) into d_tpk
        const unsigned end_bit = ubits + (unsigned)std::max(1, bits_of(maxw));
        size_t need = 0;
        e = rocprim::segmented_radix_sort_keys(nullptr, need, p->d_tpk2, p->d_tpk, (unsigned)p->t_edges, V,
                                               p->d_tptr, p->d_tptr + 1, ubits, end_bit, M);
        if (e != hipSuccess) return fail(err, e, "segmented sort (size)");
        uint64_t tcap = p->tsort_tmp_cap;
        st = grow(reinterpret_cast<uint8_t **>(&p->d_tsort_tmp), &tcap, need + 256, err, "hipMalloc(sort scratch)");
        p->tsort_tmp_cap = tcap;
        if (st != SRT_OK) return st;
        size_t have = p->tsort_tmp_cap;
        e = rocprim::segmented_radix_sort_keys(p->d_tsort_tmp, have, p->d_tpk2, p->d_tpk, (unsigned)p->t_edges, V,
                                               p->d_tptr, p->d_tptr + 1, ubits, end_bit, M);
        if (e != hipSuccess) return fail(err, e, "segmented sort");
    } else if (p->kp.lat32) {
        hipLaunchKernelGGL((tight_fill_kernel<uint32_t, false>), dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt, p->d_tu,
                           (uint32_t *)p->d_tw, p->d_teb, (uint64_t *)nullptr, 0u);
    } else {
        hipLaunchKernelGGL((tight_fill_kernel<uint64_t, false>), dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt, p->d_tu,
                           (uint64_t *)p->d_tw, p->d_teb, (uint64_t *)nullptr, 0u);
    }
    return SRT_OK;
}

srt_status fold(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    const uint32_t V = p->V;
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    const bool lds_rows = HIST_BYTES + (size_t)V * 8 + 16 <= LDS_BUDGET - 4096;
    if (p->kp.lat32) {
        if (p->t_packed)
            return lds_rows ? launch_fold_lpt<uint32_t, true, true>(p, d_stats, ubits, err)
                            : launch_fold_lpt<uint32_t, false, true>(p, d_stats, ubits, err);
        return lds_rows ? launch_fold_lpt<uint32_t, true, false>(p, d_stats, 0, err)
                        : launch_fold_lpt<uint32_t, false, false>(p, d_stats, 0, err);
    }
    return launch_fold_lpt<uint64_t, false, false>(p, d_stats, 0, err);
}

}  // namespace

srt_status fw_loss(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    if (!p->ev_loss0) {
        (void)hipEventCreate(&p->ev_loss0);
        (void)hipEventCreate(&p->ev_loss1);
    }
    (void)hipEventRecord(p->ev_loss0, p->stream);
    srt_status st;
    if (p->key_type == KEY_U32) st = tight_csr_t<uint32_t>(p, d_stats, err);
    else if (p->key_type == KEY_F64) st = tight_csr_t<double>(p, d_stats, err);
    else st = tight_csr_t<uint64_t>(p, d_stats, err);
    if (st != SRT_OK) return st;
    if ((st = fold(p, d_stats, err)) != SRT_OK) return st;
    (void)hipEventRecord(p->ev_loss1, p->stream);
    return SRT_OK;
}

}  // namespace srt
