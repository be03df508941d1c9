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

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr int NBK = 2048;        // latency buckets per row
constexpr int LOSS_NT = 1024;    // threads of the fold workgroup (16 waves)
// push scan: edges a lane loads per step (C3: 2 / 4 / 8 / 16 -> 24.8 / 20.7 /
// 21.7 / 25.7 ms for the pass: a member's edges below its bound are few, so
// wider steps fetch past the bound and narrower ones expose the latency)
constexpr int PUNR = 4;
constexpr size_t LDS_BUDGET = 160 * 1024 - 1024;

template <typename K>
struct KeyLat;
template <>
struct KeyLat<uint16_t> {
    static __device__ __forceinline__ bool inf(uint16_t k) { return k >= KEY16_INF; }
    static __device__ __forceinline__ uint64_t lat(uint16_t k) { return k; }
};
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
    if (kt == KEY_U16) {
        const uint16_t k = reinterpret_cast<const uint16_t *>(D)[idx];
        inf = KeyLat<uint16_t>::inf(k);
        return k;
    }
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
__global__ void tight_flag_kernel(const K *__restrict__ D, uint32_t Vp, uint32_t u0, uint32_t u1,
                                  const uint64_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                                  const uint64_t *__restrict__ lat, uint64_t g, uint8_t *__restrict__ flag,
                                  uint32_t *__restrict__ cnt, unsigned long long *maxw,
                                  unsigned long long *total) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    uint64_t mw = 0, tot = 0;
    for (uint32_t u = u0 + wave; u < u1; u += nwaves) {
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
                    if (cnt) atomicAdd(&cnt[v], 1u);
                    mw = w > mw ? w : mw;
                    ++tot;
                }
            }
            flag[k] = f;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mw, off);
        mw = o > mw ? o : mw;
        tot += __shfl_xor(tot, off);
    }
    if (lane == 0 && mw) atomicMax(maxw, (unsigned long long)mw);
    if (lane == 0 && total && tot) atomicAdd(total, (unsigned long long)tot);
}

// Sharded tail: the flagged entries of the rank's own adjacency rows [u0, u1)
// as records {v, u, w, 1f32 - e bits} at list[cursor..): a wave counts its
// row's flags, takes the row's range with one atomic (one per chunk would
// serialise ~10^6 atomics on the cursor), then writes them in order.
__global__ void tight_list_kernel(uint32_t u0, uint32_t u1, const uint64_t *__restrict__ row_ptr,
                                  const uint32_t *__restrict__ col, const uint64_t *__restrict__ lat,
                                  const float *__restrict__ loss, uint64_t g, const uint8_t *__restrict__ flag,
                                  uint4 *__restrict__ list, unsigned long long *cursor) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = u0 + wave; u < u1; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        uint32_t cnt = 0;
        for (uint64_t k = b + lane; k < e; k += 64) cnt += flag[k];
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
        if (!cnt) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(cursor, (unsigned long long)cnt);
        base = __shfl(base, 0);
        for (uint64_t k0 = b; k0 < e; k0 += 64) {
            const uint64_t k = k0 + lane;
            const bool f = k < e && flag[k];
            const uint64_t m = __ballot(f);
            if (f) {
                const uint64_t pos = base + __popcll(m & ((1ull << lane) - 1ull));
                const float eb = 1.0f - loss[k];  // the reference's (1f32 - other.packet_loss), mod.rs:328
                list[pos] = make_uint4(col[k], u, (uint32_t)(lat[k] / g), __float_as_uint(eb));
            }
            base += __popcll(m);
        }
    }
}

// One GPU, packed forms: the tight edges of adjacency rows [0, V) straight
// into the list, one wave per row in two passes -- pass 1 tests each 64-entry
// chunk (w * g == lat and w == D[u][v]) and keeps its ballot in LDS (chunks
// past TR_CH are tested again in pass 2), one atomic takes the row's range,
// pass 2 writes the records of the set lanes.  No flag array: against the
// flag + list kernels (1.16 + 0.74 ms on C3) the adjacency is read once and
// the second pass touches only the tight entries.  Writes only when the whole
// row fits below cap (list slots); total and max w are always counted, so a
// run with cap 0 (or too small a list) counts and the caller runs it again.
constexpr uint32_t TR_CH = 256;  // chunks (64 entries) a wave keeps in LDS: rows up to 16,384 entries
template <typename K>
__global__ __launch_bounds__(256) void tight_rows_kernel(const K *__restrict__ D, uint32_t Vp, uint32_t V,
                                                         const uint64_t *__restrict__ row_ptr,
                                                         const uint32_t *__restrict__ col,
                                                         const uint64_t *__restrict__ lat,
                                                         const float *__restrict__ loss, uint64_t g,
                                                         uint4 *__restrict__ list, uint64_t cap,
                                                         unsigned long long *cursor, unsigned long long *maxw,
                                                         unsigned long long *total) {
    __shared__ uint64_t bal[4][TR_CH];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    uint64_t mw = 0, tot = 0, mnw = ~0ull;
    auto test = [&](uint32_t u, const K *Du, uint64_t k, uint64_t e) -> bool {
        if (k >= e) return false;
        const uint32_t v = col[k];
        if (v == u) return false;
        const K d = Du[v];
        const uint64_t w = KeyLat<K>::lat(d);
        return !KeyLat<K>::inf(d) && w * g == lat[k];
    };
    for (uint32_t u = wave; u < V; u += nwaves) {
        const K *Du = D + (uint64_t)u * Vp;
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        const uint32_t nch = (uint32_t)((e - b + 63) / 64);
        uint32_t cnt = 0;
        // 4 chunks per step: their col / lat loads, then their D loads, in flight together
        for (uint32_t c0 = 0; c0 < nch; c0 += 4) {
            uint32_t v[4];
            uint64_t l[4];
            K d[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t k = b + 64ull * (c0 + q) + lane;
                v[q] = k < e ? col[k] : u;
                l[q] = k < e ? lat[k] : 0;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = Du[v[q]];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t w = KeyLat<K>::lat(d[q]);
                const bool f = v[q] != u && !KeyLat<K>::inf(d[q]) && w * g == l[q];
                const uint64_t m = __ballot(f);
                if (f) {
                    mw = w > mw ? w : mw;
                    mnw = w < mnw ? w : mnw;
                }
                if (c0 + q < TR_CH && lane == 0) bal[wv][c0 + q] = m;
                cnt += (uint32_t)__popcll(m);
            }
        }
        if (!cnt) continue;
        tot += cnt;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(cursor, (unsigned long long)cnt);
        base = __shfl(base, 0);
        if (base + cnt > cap) continue;  // uniform: the caller grows the list and runs again
        for (uint32_t c = 0; c < nch; ++c) {
            const uint64_t k = b + 64ull * c + lane;
            const uint64_t m = c < TR_CH ? bal[wv][c] : __ballot(test(u, Du, k, e));
            if (!m) continue;  // uniform
            if ((m >> lane) & 1ull) {
                const uint64_t pos = base + __popcll(m & ((1ull << lane) - 1ull));
                const float eb = 1.0f - loss[k];  // the reference's (1f32 - other.packet_loss), mod.rs:328
                list[pos] = make_uint4(col[k], u, (uint32_t)(lat[k] / g), __float_as_uint(eb));
            }
            base += __popcll(m);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mw, off);
        mw = o > mw ? o : mw;
        const uint64_t o2 = __shfl_xor(mnw, off);
        mnw = o2 < mnw ? o2 : mnw;
    }
    // tot is uniform per wave (ballot counts); total[1]: max of ~min w (zeroed by the caller)
    if (lane == 0 && mw) atomicMax(maxw, (unsigned long long)mw);
    if (lane == 0 && tot) {
        atomicAdd(total, (unsigned long long)tot);
        atomicMax(total + 1, (unsigned long long)~mnw);
    }
}

// Level solve (the closure-free dense path, see level_solve_kernel): the
// class CSRs of the edges u -> v (v != u) of latency <= wmax units, straight
// from the adjacency.  Out-rows: one wave per adjacency row u (whose entries
// ARE u's out-edges), two passes -- pass 1 tests each 64-entry chunk (the
// latency first; the column is loaded only for the lanes that pass: C3 ~2% of
// the entries), counts the hits per class by LDS atomics and stages each hit
// (its place in the row, 16 bits, and its weight in units, 16 bits, or a mark
// that pass 2 reads the latency again) in LDS at its ballot rank; one
// global atomic takes the row's range, the row's class offsets are written
// (slot k: start of class k + 1; slot CLS - 1: the row's end), and pass 2
// deals the staged hits, OUT_PL a lane at once (their loss / column gathers in
// flight together), writing each (1f32 - e bits << 32 | v; 0 bits
// without losses) at its class's running position and counting it for the
// in-row of (v, class).  A row with more than OUT_SCAP hits, or of more than
// 65,536 entries, is tested again chunk by chunk in pass 2.  No global atomic per entry on the out side, where
// a row's ~50 entries of a class would all hit one counter.  Entries past
// `cap` are counted, not written (the caller sizes and runs again).
constexpr uint32_t OUT_SCAP = 1024;  // hits a wave stages in LDS (C3: ~330 a row at the bound, more in the probes)
#ifndef SRT_OUT_PL
#define SRT_OUT_PL 4
#endif
constexpr int OUT_PL = SRT_OUT_PL;  // staged hits a lane places at once (pass 2)
#ifndef SRT_OUT_UNR
#define SRT_OUT_UNR 8
#endif
constexpr int OUT_UNR = SRT_OUT_UNR;  // chunks of a row in flight a lane (pass 1)
#ifndef SRT_OUT_UNR16
#define SRT_OUT_UNR16 8
#endif
constexpr int OUT_UNR16 = SRT_OUT_UNR16;  // ... of the u16 copy: 256-entry chunks (8 B a lane)
template <bool WITH_LOSS, bool IN = true, bool IDENT = false, bool L16 = false>
__global__ __launch_bounds__(256) void lvl_out_kernel(uint32_t u0, uint32_t V, const uint64_t *__restrict__ row_ptr,
                                                      const uint32_t *__restrict__ col,
                                                      const uint64_t *__restrict__ lat, const float *__restrict__ loss,
                                                      uint64_t g, double inv_g, uint64_t wmax_ns, uint32_t cls,
                                                      uint32_t q, uint32_t vb,
                                                      uint32_t *__restrict__ off_out, uint32_t *__restrict__ in_cnt,
                                                      uint64_t *__restrict__ ce_out, uint64_t cap,
                                                      unsigned long long *cursor, unsigned long long *maxw,
                                                      const uint16_t *__restrict__ lat16 = nullptr) {
    static_assert(!L16 || (IDENT && !IN), "the u16 copy: identity rows of symmetric plans");
    __shared__ uint32_t stage[4][OUT_SCAP];  // per wave: place in the row | units << 16 (0xffff: read again) of hit j
    __shared__ uint32_t ccnt[4][64];      // per wave: hits per class (pass 1), running positions (pass 2)
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t mw = 0;
    // l = w * g exactly; the class: w / q (q = 0: the exact weight)
    auto units_of = [&](uint64_t l) -> uint64_t { return (uint64_t)((double)l * inv_g + 0.5); };
    auto cls_of_units = [&](uint64_t wu) -> uint32_t { return (uint32_t)(q ? wu / q : wu); };
    for (uint32_t u = u0 + wave; u < V; u += nwaves) {  // rows [u0, V)
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        const uint32_t nch = (uint32_t)((e - b + 63) / 64);
        ccnt[wv][lane] = 0;
        uint32_t cnt = 0;
        const uint32_t wmax_u = (uint32_t)(wmax_ns / g);  // L16: the bound in units (wmax_ns = wmax_u g, < 0xffff)
        if (L16) {  // u16 units, 4 a lane a 256-entry chunk (identity rows of V % 4 == 0 entries)
            const uint2 *row = reinterpret_cast<const uint2 *>(lat16 + b);
            const uint32_t len = (uint32_t)(e - b), nq = (len + 255) / 256;
            for (uint32_t c0 = 0; c0 < nq; c0 += OUT_UNR16) {
                uint2 x[OUT_UNR16];
#pragma unroll
                for (int r = 0; r < OUT_UNR16; ++r) {
                    const uint32_t o = 256 * (c0 + r) + 4 * lane;
                    x[r] = o < len ? row[64 * (c0 + r) + lane] : make_uint2(~0u, ~0u);
                }
#pragma unroll
                for (int r = 0; r < OUT_UNR16; ++r) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t w = ((i < 2 ? x[r].x : x[r].y) >> (16 * (i & 1))) & 0xffffu;
                        const uint32_t o = 256 * (c0 + r) + 4 * lane + i;
                        const bool f = w <= wmax_u && o != u;
                        const uint64_t m = __ballot(f);
                        if (f) {
                            const uint32_t c = cls_of_units(w);
                            atomicAdd(&ccnt[wv][c - 1], 1u);
                            mw = c > mw ? c : mw;
                            const uint32_t j = cnt + (uint32_t)__popcll(m & below);
                            if (j < OUT_SCAP) stage[wv][j] = o | w << 16;
                        }
                        cnt += (uint32_t)__popcll(m);
                    }
                }
            }
        }
        for (uint32_t c0 = 0; c0 < (L16 ? 0u : nch); c0 += OUT_UNR) {
            uint64_t l[OUT_UNR];
#pragma unroll
            for (int r = 0; r < OUT_UNR; ++r) {
                const uint64_t k = b + 64ull * (c0 + r) + lane;
                l[r] = k < e ? lat[k] : ~0ull;
            }
#pragma unroll
            for (int r = 0; r < OUT_UNR; ++r) {
                const uint64_t k = b + 64ull * (c0 + r) + lane;
                // col only where the latency passes; identity rows (IDENT): the
                // column is the entry's place in its row
                const bool f = l[r] <= wmax_ns && (IDENT ? (uint32_t)(k - b) != u : col[k] != u);
                const uint64_t m = __ballot(f);
                if (f) {
                    const uint64_t wu = units_of(l[r]);
                    const uint32_t c = cls_of_units(wu);
                    atomicAdd(&ccnt[wv][c - 1], 1u);
                    mw = c > mw ? c : mw;
                    const uint32_t j = cnt + (uint32_t)__popcll(m & below);
                    if (j < OUT_SCAP) stage[wv][j] = (uint32_t)(k - b) | (wu < 0xffffu ? (uint32_t)wu : 0xffffu) << 16;
                }
                cnt += (uint32_t)__popcll(m);
            }
        }
        // cnt is uniform (ballot counts); ccnt complete for this wave's lanes
        unsigned long long base = 0;
        if (cnt && lane == 0) base = atomicAdd(cursor, (unsigned long long)cnt);
        base = __shfl(base, 0);
        const bool fits = base + cnt <= cap;
        // class offsets of row u: exclusive prefix of the class counts (lanes < cls)
        uint32_t x = lane < cls ? ccnt[wv][lane] : 0u, incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t start = (uint32_t)base + incl - x;
        if (lane < cls) off_out[(uint64_t)u * cls + lane] = fits ? (lane == cls - 1 ? (uint32_t)(base + cnt) : start) : 0u;
        ccnt[wv][lane] = start;  // running positions
        if (!cnt || !fits) continue;  // uniform
        const bool staged = cnt <= OUT_SCAP && e - b <= 65536;
        auto put = [&](uint32_t v, uint64_t wu, float ls) {
            const uint32_t cl = cls_of_units(wu);
            const uint32_t pos = atomicAdd(&ccnt[wv][cl - 1], 1u);
            const float eb = WITH_LOSS ? 1.0f - ls : 0.0f;  // (1f32 - other.packet_loss), mod.rs:328
            // q > 0 (quantized classes): the weight's remainder w - c q rides
            // along, (1 - e) in bits 34.. (a loss in [0, 1]: its bits are < 2^30)
            ce_out[pos] = q ? ((uint64_t)__float_as_uint(eb) << 34) | ((wu - (uint64_t)cl * q) << vb) | v
                            : ((uint64_t)__float_as_uint(eb) << 32) | v;
            if (IN) atomicAdd(&in_cnt[(uint64_t)v * cls + cl - 1], 1u);  // symmetric plans: no in-rows
        };
        if (staged) {  // uniform: the staged hits, OUT_PL a lane at once
            for (uint32_t j0 = 0; j0 < cnt; j0 += 64 * OUT_PL) {
                uint32_t o[OUT_PL], v[OUT_PL];
                uint64_t wu[OUT_PL];
                float ls[OUT_PL];
#pragma unroll
                for (int r = 0; r < OUT_PL; ++r) {
                    const uint32_t j = j0 + 64 * r + lane;
                    const uint32_t h = j < cnt ? stage[wv][j] : 0u;
                    o[r] = h & 0xffffu;
                    wu[r] = h >> 16;
                }
#pragma unroll
                for (int r = 0; r < OUT_PL; ++r) {
                    const bool ok = j0 + 64 * r + lane < cnt;
                    v[r] = IDENT ? o[r] : ok ? col[b + o[r]] : 0u;
                    ls[r] = WITH_LOSS && ok ? loss[b + o[r]] : 0.0f;
                    if (ok && wu[r] == 0xffffu) wu[r] = units_of(lat[b + o[r]]);  // wide weights
                }
#pragma unroll
                for (int r = 0; r < OUT_PL; ++r)
                    if (j0 + 64 * r + lane < cnt) put(v[r], wu[r], ls[r]);
            }
        } else if (L16) {  // rows of more hits: tested again
            for (uint64_t k = b + lane; k < e; k += 64) {
                const uint32_t w = lat16[k];
                if (w <= wmax_u && (uint32_t)(k - b) != u) put((uint32_t)(k - b), w, WITH_LOSS ? loss[k] : 0.0f);
            }
        } else {  // rows of more hits: tested again, chunk by chunk
            for (uint32_t c = 0; c < nch; ++c) {
                const uint64_t k = b + 64ull * c + lane;
                const uint64_t l = k < e ? lat[k] : ~0ull;
                if (l <= wmax_ns && (IDENT ? (uint32_t)(k - b) != u : col[k] != u))
                    put(IDENT ? (uint32_t)(k - b) : col[k], units_of(l), WITH_LOSS ? loss[k] : 0.0f);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = __shfl_xor(mw, off);
        mw = o > mw ? o : mw;
    }
    if (lane == 0 && mw) atomicMax(maxw, (unsigned long long)mw);
}

// In-rows of the level solve's class CSRs: every out-entry u -> v of class c
// (walked per out-row, one wave a row) placed at its (v, c) slot's cursor
// (in_off: the exclusive scan of lvl_out_kernel's counts), its head v (the
// bits of vmask) replaced by the tail u.
__global__ __launch_bounds__(256) void lvl_in_kernel(uint32_t V, uint32_t cls, uint64_t vmask,
                                                     const uint32_t *__restrict__ off_out,
                                                     const uint64_t *__restrict__ ce_out,
                                                     const uint32_t *__restrict__ in_off, uint32_t *__restrict__ in_cur,
                                                     uint64_t *__restrict__ ce_in) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint32_t *ou = off_out + (uint64_t)u * cls;
        const uint32_t e0 = ou[0], e1 = ou[cls - 1];
        for (uint32_t k = e0 + lane; k < e1; k += 64) {
            uint32_t c = 1;  // the class of entry k: the last class whose start is <= k
            while (c + 1 < cls && ou[c] <= k) ++c;
            const uint64_t w = ce_out[k];
            const uint32_t v = (uint32_t)(w & vmask);
            const uint64_t slot = (uint64_t)v * cls + c - 1;
            const uint32_t pos = in_off[slot] + atomicAdd(&in_cur[slot], 1u);
            ce_in[pos] = (w & ~vmask) | u;
        }
    }
}

// a latency in units of g for the u16 adjacency copy (exact: g divides every
// edge latency; 0xffff: longer than any class bound)
__device__ __forceinline__ uint16_t units16(uint64_t l, double inv_g) {
    const uint64_t u = (uint64_t)((double)l * inv_g + 0.5);
    return (uint16_t)(u < 0xffffu ? u : 0xffffu);
}

// Exact check that a level plan's class in-rows equal its out-rows, so the
// run builds only the out-rows (lvl_sym): the adjacency is V identity rows
// (proved by the host scan, CsrStats::ident: entry (u, v) at u * V + v) and
// every pair of latency <= wmax_ns has its mirror with the same latency (and,
// loss != nullptr, the same loss bits) -- then the class-c in-entries of x are
// the class-c out-entries of x, entry for entry.  Triangle tile pairs (bi <=
// bj) of 64 x 64: tile (bj, bi) staged in LDS, tile (bi, bj) compared with it
// transposed; a wave reads 64 consecutive latencies of a row a step (512 B),
// losses only where a latency is short enough to matter.  Any difference
// clears *ok.
__global__ __launch_bounds__(256) void lvl_sym_tile_kernel(uint32_t V, const uint64_t *__restrict__ lat,
                                                           const float *__restrict__ loss, uint64_t wmax_ns,
                                                           uint32_t *ok, uint16_t *__restrict__ lat16, double inv_g) {
    __shared__ uint64_t tl[64][65];
    __shared__ uint32_t tp[64][65];
    const uint32_t nb = (V + 63) / 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const uint64_t ntri = (uint64_t)nb * (nb + 1) / 2;
    bool bad = false;
    for (uint64_t t = blockIdx.x; t < ntri; t += gridDim.x) {
        // triangle index -> (bi, bj), bi <= bj: row bi starts at bi * nb - bi (bi - 1) / 2
        const double nn = 2.0 * nb + 1.0;
        uint32_t bi = (uint32_t)((nn - sqrt(nn * nn - 8.0 * (double)t)) * 0.5);
        auto row0 = [&](uint64_t r) { return r * nb - r * (r - 1) / 2; };
        while (bi > 0 && row0(bi) > t) --bi;
        while (row0(bi + 1) <= t) ++bi;
        const uint32_t bj = bi + (uint32_t)(t - row0(bi));
        // a wave's 16 rows of a tile in flight at once (latency and loss
        // together: 12 B a lane a row), then through LDS
        const uint32_t v_a = bi * 64 + tx;  // staged tile (bj, bi): column bi * 64 + tx
        uint64_t la[16];
        uint32_t pa[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t u = bj * 64 + ty + 4 * i;
            const bool in = u < V && v_a < V;
            const uint64_t k = (uint64_t)u * V + v_a;
            la[i] = in ? lat[k] : 0ull;
            pa[i] = in && loss ? __float_as_uint(loss[k]) : 0u;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            tl[ty + 4 * i][tx] = la[i];
            tp[ty + 4 * i][tx] = pa[i];
        }
        __syncthreads();
        // the u16-unit copy of the adjacency (V % 4 == 0): every tile, the
        // triangle's and its mirror's, out of the LDS tile 4 entries (8 B) a store
        auto put16 = [&](uint32_t r0, uint32_t c0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t gi = threadIdx.x + 256 * i, r = gi >> 4, c = (gi & 15) * 4;
                if (r0 + r < V && c0 + c < V) {
                    const uint32_t lo = units16(tl[r][c], inv_g) | (uint32_t)units16(tl[r][c + 1], inv_g) << 16;
                    const uint32_t hi = units16(tl[r][c + 2], inv_g) | (uint32_t)units16(tl[r][c + 3], inv_g) << 16;
                    *reinterpret_cast<uint2 *>(lat16 + (uint64_t)(r0 + r) * V + c0 + c) = make_uint2(lo, hi);
                }
            }
        };
        const uint32_t v_b = bj * 64 + tx;  // compared tile (bi, bj)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t u = bi * 64 + ty + 4 * i;
            const bool in = u < V && v_b < V;
            const uint64_t k = (uint64_t)u * V + v_b;
            la[i] = in ? lat[k] : 0ull;
            pa[i] = in && loss ? __float_as_uint(loss[k]) : 0u;
        }
        if (lat16) put16(bj * 64, bi * 64);  // the staged tile's, behind the compared tile's loads
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t r = ty + 4 * i, u = bi * 64 + r;
            if (u < V && v_b < V && u != v_b) {
                const uint64_t l = la[i], lm = tl[tx][r];
                if (l <= wmax_ns || lm <= wmax_ns) bad |= l != lm || pa[i] != tp[tx][r];
            }
        }
        __syncthreads();
        if (lat16 && bi != bj) {  // the compared tile through the same LDS tile
#pragma unroll
            for (int i = 0; i < 16; ++i) tl[ty + 4 * i][tx] = la[i];
            __syncthreads();
            put16(bi * 64, bj * 64);
            __syncthreads();
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicAnd(ok, 0u);
}

// The adjacency indices of the entries a level plan's class CSRs read
// (latency <= wmax_ns, not a self-loop), for the one-call build's loss upload
// (only those losses cross PCIe).  One wave per row: pass 1 keeps the chunks'
// ballots in LDS, one atomic reserves the row's range, pass 2 writes the
// indices in row order.  Past `cap` entries are counted, not written.
template <bool IDENT>
__global__ __launch_bounds__(256) void lvl_index_kernel(uint32_t V, const uint64_t *__restrict__ row_ptr,
                                                        const uint32_t *__restrict__ col,
                                                        const uint64_t *__restrict__ lat, uint64_t wmax_ns,
                                                        uint32_t *__restrict__ idx, uint64_t cap,
                                                        unsigned long long *cursor) {
    __shared__ uint64_t bal[4][TR_CH];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        const uint32_t nch = (uint32_t)((e - b + 63) / 64);
        auto test = [&](uint32_t c) -> uint64_t {
            const uint64_t k = b + 64ull * c + lane;
            const uint64_t l = k < e ? lat[k] : ~0ull;
            return __ballot(l <= wmax_ns && (IDENT ? (uint32_t)(k - b) != u : col[k] != u));
        };
        uint32_t cnt = 0;
        for (uint32_t c0 = 0; c0 < nch; c0 += 4) {
            uint64_t m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) m[q] = c0 + q < nch ? test(c0 + q) : 0ull;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (c0 + q < TR_CH && lane == 0) bal[wv][c0 + q] = m[q];
                cnt += (uint32_t)__popcll(m[q]);
            }
        }
        unsigned long long base = 0;
        if (cnt && lane == 0) base = atomicAdd(cursor, (unsigned long long)cnt);
        base = __shfl(base, 0);
        if (!cnt || base + cnt > cap) continue;  // uniform
        for (uint32_t c = 0; c < nch; ++c) {
            const uint64_t m = c < TR_CH ? bal[wv][c] : test(c);
            if (!m) continue;  // uniform
            if ((m >> lane) & 1ull) idx[base + (uint64_t)__popcll(m & below)] = (uint32_t)(b + 64ull * c + lane);
            base += (uint64_t)__popcll(m);
        }
    }
}

// symmetric plans' one-call build: every uploaded loss equals its mirror's
// (identity rows: entry u * V + v <-> v * V + u; the mirror is uploaded too,
// having the same latency); any difference clears *ok
__global__ void loss_mirror_check_kernel(const uint32_t *__restrict__ idx, uint64_t count, uint64_t V,
                                         const float *__restrict__ loss, uint32_t *ok) {
    bool bad = false;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = idx[i];
        bad |= __float_as_uint(loss[k]) != __float_as_uint(loss[(k % V) * V + k / V]);
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicAnd(ok, 0u);
}

__global__ void loss_scatter_kernel(const uint32_t *__restrict__ idx, const float *__restrict__ val, uint64_t count,
                                    float *__restrict__ loss) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x)
        loss[idx[i]] = val[i];
}

// Per-row counts of a tight-edge list (v = ~0: padding): rows by target v
// (pull CSR) or, BY_SRC, by source u (push CSR)
template <bool BY_SRC>
__global__ void tight_list_count_kernel(const uint4 *__restrict__ list, uint64_t slots, uint32_t *__restrict__ cnt,
                                        uint32_t nv) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < slots; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = list[e];
        if (r.x != ~0u && r.x < nv && r.y < nv) atomicAdd(&cnt[BY_SRC ? r.y : r.x], 1u);
    }
}

// ... and the packed CSR entries of the list: (1-e) bits << 32 | w << ubits |
// the other endpoint (u for pull rows, v for push rows)
template <bool BY_SRC>
__global__ void tight_list_fill_kernel(const uint4 *__restrict__ list, uint64_t slots,
                                       const uint64_t *__restrict__ ptr, uint32_t *__restrict__ cur,
                                       uint64_t *__restrict__ tpk, uint32_t ubits, uint32_t nv) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < slots; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = list[e];
        if (r.x == ~0u || r.x >= nv || r.y >= nv) continue;  // padding (or a record the transport damaged)
        const uint32_t row = BY_SRC ? r.y : r.x, other = BY_SRC ? r.x : r.y;
        const uint64_t pos = ptr[row] + atomicAdd(&cur[row], 1u);
        tpk[pos] = ((uint64_t)r.w << 32) | ((r.z << ubits) | other);
    }
}

// Sharded tail: every rank's staged rows into the table.  slot s = r * lrow_max
// + k holds table row lrows[s] (~0: padding) as latency units (~0:
// unreachable) and loss.
// Dfull (u16 keys, the symmetric sharded closure on every rank): the staging
// holds only the loss; latencies come from D (the diagonal: the self-loop).
__global__ void expand_rows_kernel(const uint32_t *__restrict__ lrows, uint32_t slots, uint32_t n,
                                   const void *__restrict__ slat, bool lat16, const float *__restrict__ sloss,
                                   uint64_t g, uint64_t *__restrict__ out_lat, float *__restrict__ out_loss,
                                   const uint16_t *__restrict__ Dfull, uint32_t Vp, const uint32_t *__restrict__ nodes,
                                   const uint64_t *__restrict__ sl_lat) {
    for (uint32_t sl = blockIdx.x; sl < slots; sl += gridDim.x) {
        const uint32_t i = lrows[sl];
        if (i == ~0u) continue;
        const uint16_t *s16 = reinterpret_cast<const uint16_t *>(slat) + (uint64_t)sl * n;
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(slat) + (uint64_t)sl * n;
        const float *sp = sloss + (uint64_t)sl * n;
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        const uint16_t *Drow = Dfull ? Dfull + (uint64_t)nodes[i] * Vp : nullptr;
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
            uint64_t l;
            if (j == i) {
                l = sl_lat[i];  // the raw self-loop: need not fit the staged latency field
            } else if (Drow) {
                const uint32_t x = Drow[nodes[j]];
                l = x >= KEY16_INF ? ~0ull : (uint64_t)x * g;
            } else if (lat16) {
                const uint32_t x = s16[j];
                l = x == 0xffffu ? ~0ull : (uint64_t)x * g;
            } else {
                const uint32_t x = s32[j];
                l = x == ~0u ? ~0ull : (uint64_t)x * g;
            }
            ol[j] = l;
            op[j] = sp[j];
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

// Push form (the default when the tight out-edge CSR is built): ord's members
// are the sources u of the bucket, record {u, first tight out-edge, end, lim}
// with lim = max latency of the row + 1 - lat(u); u's final loss goes along
// each out-edge u -> v with w < lim (no target of the row is further away)
// where lat(v) == lat(u) + w, by LDS atomic min on prow[v].  Against the pull
// form's per-target bound (w < lat(v)) the row-wide bound scans far fewer
// edges on the dense configs (C3: a vertex two units away pushes only its
// one-unit edges).
template <typename LatT, int LPT, int UNR, bool ITER>
__device__ __forceinline__ int scan_bucket_push(const uint4 *__restrict__ ord, uint32_t m0, uint32_t m1,
                                                uint32_t grp, uint32_t sub, uint32_t ngrp,
                                                const uint64_t *__restrict__ tpk, const LatT *lrow, float *prow,
                                                uint32_t ubits, uint32_t umask, LatT maxp1) {
    int changed = 0;
    uint32_t m = m0 + grp;
    uint4 rec = m < m1 ? ord[m] : make_uint4(0, 0, 0, 0);
    for (; m < m1; m += ngrp) {
        const uint4 cur = rec;
        if (m + ngrp < m1) rec = ord[m + ngrp];
        const uint32_t e1 = cur.z;
        const LatT lim = (LatT)cur.w, lu = maxp1 - lim;
        const float onem = 1.0f - prow[cur.x];
        const uint64_t *wp = tpk + cur.y + sub;
        for (uint32_t e = cur.y + sub; e < e1; e += UNR * LPT, wp += UNR * LPT) {
            uint64_t wd[UNR];
#pragma unroll
            for (int q = 0; q < UNR; ++q) wd[q] = wp[q * LPT];
            bool ok[UNR];
            uint32_t v[UNR];
            LatT want[UNR], lv[UNR];
#pragma unroll
            for (int q = 0; q < UNR; ++q) {
                const uint32_t lo = (uint32_t)wd[q], w = lo >> ubits;
                ok[q] = e + q * LPT < e1 && (LatT)w < lim;
                v[q] = ok[q] ? lo & umask : 0u;
                want[q] = lu + (LatT)w;
            }
#pragma unroll
            for (int q = 0; q < UNR; ++q) lv[q] = lrow[v[q]];
#pragma unroll
            for (int q = 0; q < UNR; ++q) {
                if (ok[q] && lv[q] == want[q]) {
                    const float c = 1.0f - __fmul_rn(onem, __uint_as_float((uint32_t)(wd[q] >> 32)));
                    uint32_t *dst = reinterpret_cast<uint32_t *>(prow) + v[q];
                    if constexpr (ITER) changed |= __float_as_uint(c) < atomicMin(dst, __float_as_uint(c));
                    else atomicMin(dst, __float_as_uint(c));
                }
            }
            if (!ok[UNR - 1]) break;
        }
    }
    return changed;
}

template <typename LatT, bool LROWS, int LPT, bool PACKED, bool PUSH>
__global__ __launch_bounds__(LOSS_NT) void tight_loss_kernel(
    const void *__restrict__ D, int key_type, uint32_t Vp, uint32_t V, const uint32_t *__restrict__ nodes,
    uint32_t n, uint32_t row0, uint32_t row1, const uint64_t *__restrict__ tptr, const uint32_t *__restrict__ tu,
    const LatT *__restrict__ tw, const float *__restrict__ teb, const uint64_t *__restrict__ tpk, uint32_t ubits,
    uint64_t g, const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss,
    uint64_t *__restrict__ out_lat, float *__restrict__ out_loss, unsigned long long *stats,
    uint4 *__restrict__ ord_all, LatT *lat_all, float *loss_all, const uint64_t *__restrict__ row_ptr,
    const uint32_t *__restrict__ col, const uint64_t *__restrict__ elat, const float *__restrict__ eloss,
    const uint32_t *__restrict__ row_list, void *__restrict__ out32, float *__restrict__ out32_loss, bool stage16) {
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

    // rows: [row0, row1) of the table, or (sharded tail) row_list[0, row1) --
    // then the row goes to slot k of the u32 staging (latency units, ~0 =
    // unreachable) instead of the table
    const uint32_t nrows = row_list ? row1 : row1 - row0;
    for (uint32_t k = blockIdx.x; k < nrows; k += gridDim.x) {
        const uint32_t i = row_list ? row_list[k] : row0 + k;
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
        const uint32_t nb = (uint32_t)(mx >> shift) + 1;
        const bool few = nb <= 64;  // uniform: aggregate the LDS atomics per wave
        // 2. counting sort of the reachable vertices (s excluded) by bucket
        for (uint32_t base = 0; base < V; base += nt) {
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
        // (fold(0, e) = 1 - (1 - 0) (1 - e)); the pull scans then skip every
        // in-edge with w == lat[s][v], whose tail can only be s.  Push: s's
        // tight out-edges (w <= the row's max latency), else its adjacency row.
        if constexpr (PUSH) {
            const uint64_t p0 = tptr[s], p1 = tptr[s + 1];
            for (uint64_t k = p0 + tid; k < p1; k += nt) {
                const uint64_t wd = tpk[k];
                const uint32_t lo = (uint32_t)wd, w = lo >> ubits, v = lo & umask;
                if ((uint64_t)w <= mx && lrow[v] == (LatT)w) {
                    const float c = 1.0f - __fmul_rn(1.0f - 0.0f, __uint_as_float((uint32_t)(wd >> 32)));
                    atomicMin(reinterpret_cast<uint32_t *>(prow) + v, __float_as_uint(c));
                }
            }
        } else {
            for (uint64_t k = row_ptr[s] + tid; k < row_ptr[s + 1]; k += nt) {
                const uint32_t v = col[k];
                const LatT l = lrow[v];
                if (v != s && l != LINF && (uint64_t)l * g == elat[k]) {
                    const float c = 1.0f - __fmul_rn(1.0f - 0.0f, 1.0f - eloss[k]);
                    atomicMin(reinterpret_cast<uint32_t *>(prow) + v, __float_as_uint(c));
                }
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
        for (uint32_t base = 0; base < V; base += nt) {
            const uint32_t v = base + tid;
            const LatT l = v < V ? lrow[v] : LINF;
            const bool ok = v < V && v != s && l != LINF;
            const uint32_t b = ok ? (uint32_t)((uint64_t)l >> shift) : 0u;
            uint32_t pos = 0;
            if (few) pos = agg_inc(hist, b, ok);
            else if (ok) pos = atomicAdd(&hist[b], 1u);
            if (ok)
                ord[pos] = make_uint4(v, (uint32_t)tptr[v], (uint32_t)tptr[v + 1],
                                      PUSH ? (uint32_t)(mx + 1 - (uint64_t)l) : (uint32_t)l);
        }
        __syncthreads();
        // hist[b] is now the end of bucket b (its start: hist[b-1], or 0)
        // 3. buckets in increasing latency
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t m0 = b ? hist[b - 1] : 0u, m1 = hist[b];
            if (m0 == m1) continue;  // uniform
            for (;;) {
                int changed = 0;
                if constexpr (PUSH) {
                    if (shift)
                        changed = scan_bucket_push<LatT, LPT, PUNR, true>(ord, m0, m1, grp, sub, ngrp, tpk, lrow, prow,
                                                                    ubits, umask, (LatT)(mx + 1));
                    else
                        scan_bucket_push<LatT, LPT, PUNR, false>(ord, m0, m1, grp, sub, ngrp, tpk, lrow, prow, ubits,
                                                           umask, (LatT)(mx + 1));
                } else if constexpr (PACKED) {
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
        // 4. table row i (or staging slot k)
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        // staging slot k: latency units as u16 (stage16: u16 keys, < 0x7fff)
        // or u32, ~0 = unreachable
        uint32_t *o32 = out32 && !stage16 ? reinterpret_cast<uint32_t *>(out32) + (uint64_t)k * n : nullptr;
        uint16_t *o16 = out32 && stage16 ? reinterpret_cast<uint16_t *>(out32) + (uint64_t)k * n : nullptr;
        float *o32p = out32_loss ? out32_loss + (uint64_t)k * n : nullptr;  // staging (loss only if !out32)
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
            if (o32p) {
                if (o16) o16[j] = latv == ~0ull ? (uint16_t)0xffffu : (uint16_t)(latv / g);
                else if (o32) o32[j] = latv == ~0ull ? ~0u : (uint32_t)(latv / g);
                o32p[j] = lossv;
            } else {
                ol[j] = latv;
                op[j] = lossv;
            }
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

// --------------------------------------------------------------- level fold
// The pull form scans, for every target v of a row, its tight in-edges with
// w < lat[s][v]; the push form scans, for every u, its tight out-edges up to
// the row's largest latency.  Both walk ~10x more edges than end up tight for
// the row (C3: ~1.9M edge tests a row for ~0.27M tight ones).  With the
// vertices grouped by latency level (N_l = {v : lat[s][v] = l}, N_0 = {s})
// the candidates of level l are exactly the edges u -> v, u in N_j, v in N_l,
// of weight w = l - j, and for each weight class w that set can be walked
// from either end: push from N_j along class-w out-edges, or pull into N_l
// along class-w in-edges -- whichever level is smaller (a class's out- and
// in-degrees are alike).  C3: ~0.26M edge tests a row.  Every candidate is
// the same fold(loss[s][u], e) either way, min-ed into loss[s][v] by LDS
// atomics, and level j < l is final before level l starts (one barrier per
// level), so the result is the same bits as the single-direction scans.
//
// Class CSRs (built from the tight-edge list, no sort): out-rows and in-rows
// grouped by exact weight w = 1..WC; tcls[x*cls + w-1] .. tcls[x*cls + w] is
// class w of vertex x.  Applies when every tight edge has w <= WC, every
// closure latency is < NBK units (proof bound lmax), V < 65536 (u16 member
// lists) and the row fits LDS: lat u16 + loss f32 + members u16 (8 B/vertex).
constexpr uint32_t WC = 31;   // weight classes at most (exact weights, or quantized: floor(w / q))
// offsets per vertex (p->t_cls: classes 1..cls-1, then the end): 16 when
// every class is <= 15 (C3: half the offset arrays of 32, 6.8 vs 7.0 ms), else 32

// class of a tight weight w: w itself (q = 1), else floor(w / q) (quantized
// levels, q = the smallest tight weight)
__device__ __forceinline__ uint32_t wclass(uint32_t w, uint32_t q) { return q == 1 ? w : w / q; }

__global__ void tcls_count_kernel(const uint4 *__restrict__ list, uint64_t slots, uint32_t *__restrict__ cnt,
                                  uint64_t vc1, uint32_t q, uint32_t cls) {
    const uint64_t nv = (vc1 - 1) / cls;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < slots; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = list[e];
        if (r.x == ~0u) continue;
        const uint32_t c = wclass(r.z, q);
        if (r.x >= nv || r.y >= nv || c == 0 || c >= cls) continue;  // a record the transport damaged
        atomicAdd(&cnt[(uint64_t)r.y * cls + c - 1], 1u);        // out-row of u
        atomicAdd(&cnt[vc1 + (uint64_t)r.x * cls + c - 1], 1u);  // in-row of v
    }
}

__global__ void tcls_fill_kernel(const uint4 *__restrict__ list, uint64_t slots, const uint32_t *__restrict__ off,
                                 uint32_t *__restrict__ cur, uint64_t *__restrict__ ce_out,
                                 uint64_t *__restrict__ ce_in, uint64_t vc1, uint32_t q, uint32_t *__restrict__ cw,
                                 uint64_t cw_in, uint32_t cls) {
    const uint64_t nv = (vc1 - 1) / cls;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < slots; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = list[e];
        if (r.x == ~0u) continue;
        const uint32_t c = wclass(r.z, q);
        if (r.x >= nv || r.y >= nv || c == 0 || c >= cls) continue;
        const uint64_t a = (uint64_t)r.y * cls + c - 1, b = vc1 + (uint64_t)r.x * cls + c - 1;
        const uint64_t ia = off[a] + atomicAdd(&cur[a], 1u), ib = off[b] + atomicAdd(&cur[b], 1u);
        ce_out[ia] = ((uint64_t)r.w << 32) | r.x;
        ce_in[ib] = ((uint64_t)r.w << 32) | r.y;
        if (cw) {  // quantized classes: the exact weight beside each entry
            cw[ia] = r.z;
            cw[cw_in + ib] = r.z;
        }
    }
}

// One workgroup per table row, 16 waves.  LDS: hist (level ends), lat u16
// (0xffff: unreachable), loss f32 bits, members u16 (the vertices in level
// order, counting sort).  Output as tight_loss_kernel.
// QUANT (level width qw > 1, see level_q): lrow holds floor(L / qw); a class-c
// edge's tail lies in level l - c or l - c - 1, and a candidate is taken only
// when L(s,u) + w == L(s,v) exactly (the closure row's exact values, read from
// D; the class entries' weights from cw).  The output latencies come from D.
#ifndef LOSS_COUNT
#define LOSS_COUNT 0
#endif
#if LOSS_COUNT
__device__ unsigned long long loss_cnt[9];  // diagnostic builds: items, edge visits, hits, levels, phase ticks x4, push hits
__device__ unsigned long long lvl_cnt[8][5];  // level solve, per level (<= 7): ticks plan+compact / walk / collect, items, rows
__constant__ uint32_t lvl_diag;                // level solve ablations (SRT_LVL_DIAG)
#endif
template <int LPT, int UNR, bool QUANT, uint32_t CLSN, int VW>
__global__ __launch_bounds__(LOSS_NT) void level_loss_kernel(
    const void *__restrict__ D, int key_type, uint32_t Vp, uint32_t V, const uint32_t *__restrict__ nodes, uint32_t n,
    uint32_t row0, uint32_t row1, const uint32_t *__restrict__ tcls, uint64_t vc1,
    const uint64_t *__restrict__ ce_out, const uint64_t *__restrict__ ce_in, uint64_t g,
    const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat,
    float *__restrict__ out_loss, unsigned long long *stats, const uint32_t *__restrict__ row_list,
    void *__restrict__ out32, float *__restrict__ out32_loss, bool stage16, uint32_t qw,
    const uint32_t *__restrict__ cw, uint64_t cw_in) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint64_t red[16];
    __shared__ unsigned long long red_min[16], red_cnt[16];
    constexpr uint32_t WCN = CLSN - 1;
    __shared__ uint32_t plan_end[WCN + 1];  // inclusive prefix of the class item counts
    __shared__ uint32_t wcnt[16][32];      // few-level sort: per-wave level counts, then bases
    __shared__ uint32_t plan_push;         // bit w: class w pushes from N_{l-w}
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem);
    uint16_t *lrow = reinterpret_cast<uint16_t *>(smem + HIST_BYTES);
    const size_t lat_b = ((size_t)V * 2 + 15) & ~(size_t)15;
    uint32_t *prow = reinterpret_cast<uint32_t *>(smem + HIST_BYTES + lat_b);
    uint16_t *mem = reinterpret_cast<uint16_t *>(smem + HIST_BYTES + lat_b + (size_t)V * 4);
    const uint16_t LINF = 0xffffu;
    const uint32_t FINF = 0x7f800000u;  // +inf bits
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const uint32_t grp = tid / LPT, sub = tid % LPT, ngrp = nt / LPT;
    const uint32_t *cls_out = tcls, *cls_in = tcls + vc1;
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0;
#if LOSS_COUNT
    uint32_t c_vis = 0, c_hit = 0, c_phit = 0;
#endif
    const uint32_t nrows = row_list ? row1 : row1 - row0;
    for (uint32_t k = blockIdx.x; k < nrows; k += gridDim.x) {
        const uint32_t i = row_list ? row_list[k] : row0 + k;
        const uint32_t s = nodes[i];
#if LOSS_COUNT
        unsigned long long tk0 = wall_clock64();
#define LOSS_TICK(slot)                                                          \
    if (tid == 0) {                                                              \
        const unsigned long long tk1 = wall_clock64();                           \
        atomicAdd(&loss_cnt[slot], tk1 - tk0);                                   \
        tk0 = tk1;                                                               \
    }
#else
#define LOSS_TICK(slot)
#endif
        // 1. the row's latencies (units of g, < NBK by the host's proof bound)
        uint32_t mx = 0;
        auto put = [&](uint32_t v, bool inf, uint64_t l64) {
            const uint16_t l = inf ? LINF : v == s ? (uint16_t)0 : (uint16_t)(QUANT ? l64 / qw : l64);
            lrow[v] = l;
            prow[v] = v == s ? 0u : FINF;  // petgraph's zero score (0 ns, 0.0) at s
            if (l != LINF && l > mx) mx = l;
        };
        if (key_type == KEY_U16 && (Vp & 7u) == 0) {
            // 2-byte keys: 8 a thread in one 16-byte load (C3: 2 loads a
            // thread instead of 16 dependent round trips; the row is padded to Vp)
            const uint16_t *Dr = reinterpret_cast<const uint16_t *>(D) + (uint64_t)s * Vp;
            for (uint32_t v8 = tid * 8; v8 < V; v8 += nt * 8) {
                const uint4 raw = *reinterpret_cast<const uint4 *>(Dr + v8);
                auto put2 = [&](uint32_t v, uint32_t wd) {
                    const uint16_t k0 = (uint16_t)wd, k1 = (uint16_t)(wd >> 16);
                    if (v < V) put(v, k0 >= KEY16_INF, k0);
                    if (v + 1 < V) put(v + 1, k1 >= KEY16_INF, k1);
                };
                put2(v8, raw.x);
                put2(v8 + 2, raw.y);
                put2(v8 + 4, raw.z);
                put2(v8 + 6, raw.w);
            }
        } else {
            for (uint32_t v = tid; v < V; v += nt) {
                bool inf;
                const uint64_t l64 = closure_lat(D, (uint64_t)s * Vp + v, key_type, inf);
                put(v, inf, l64);
            }
        }
        for (uint32_t b = tid; b <= (uint32_t)NBK; b += nt) hist[b] = 0;
        for (int off = 32; off > 0; off >>= 1) {
            const uint32_t o = __shfl_xor(mx, off);
            mx = o > mx ? o : mx;
        }
        if (lane == 0) red[wv] = mx;
        __syncthreads();
        mx = 0;
        for (int q = 0; q < nw; ++q) mx = red[q] > mx ? (uint32_t)red[q] : mx;
        LOSS_TICK(4)
        // 2. counting sort of the reachable vertices (s at level 0) by level.
        // Few levels (mx < 32, C3: ~6): one ballot per level and 64-vertex
        // chunk, a wave's count of level l in lane l; the per-wave counts are
        // scanned level-major, so every wave places its chunks' vertices at
        // its own bases without atomics.  Else LDS atomics per distinct level.
        if (mx < 32) {
            uint32_t mine = 0;  // lane l: this wave's vertices at level l
            for (uint32_t base = 0; base < V; base += nt) {
                const uint32_t v = base + tid;
                const uint16_t l = v < V ? lrow[v] : LINF;
                for (uint32_t q = 0; q <= mx; ++q) {
                    const uint64_t m = __ballot(l == q);
                    if (lane == (int)q) mine += (uint32_t)__popcll(m);
                }
            }
            if (lane < 32) wcnt[wv][lane] = lane <= (int)mx ? mine : 0u;
            __syncthreads();
            if (wv == 0 && lane < 32) {
                uint32_t tot = 0;
                for (int q = 0; q < nw; ++q) tot += wcnt[q][lane];
                uint32_t x = tot;  // inclusive scan over the levels (lanes 0..31)
                for (int off = 1; off < 32; off <<= 1) {
                    const uint32_t y = __shfl_up(x, off, 32);
                    if (lane >= off) x += y;
                }
                uint32_t run = x - tot;  // start of level `lane`
                for (int q = 0; q < nw; ++q) {
                    const uint32_t c = wcnt[q][lane];
                    wcnt[q][lane] = run;
                    run += c;
                }
                if (lane <= (int)mx) hist[lane] = x;  // end of level `lane`
            }
            __syncthreads();
            uint32_t at = wcnt[wv][lane & 31];  // lane l: where this wave's next level-l vertex goes
            for (uint32_t base = 0; base < V; base += nt) {
                const uint32_t v = base + tid;
                const uint16_t l = v < V ? lrow[v] : LINF;
                for (uint32_t q = 0; q <= mx; ++q) {
                    const uint64_t m = __ballot(l == q);
                    if (!m) continue;  // uniform
                    const uint32_t b = __builtin_amdgcn_readlane(at, q);
                    if (l == q) mem[b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)v;
                    if (lane == (int)q) at += (uint32_t)__popcll(m);
                }
            }
            __syncthreads();
        } else {
        for (uint32_t base = 0; base < V; base += nt) {
            const uint32_t v = base + tid;
            const uint16_t l = v < V ? lrow[v] : LINF;
            const bool ok = l != LINF;
            if (ok) atomicAdd(&hist[l], 1u);
        }
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
            __syncthreads();  // everyone has read red (max) before it is rewritten
            if (lane == 63) red[wv] = x;
            __syncthreads();
            uint32_t run = x - sum;
            for (int q = 0; q < wv; ++q) run += (uint32_t)red[q];
            for (uint32_t b = b0; b < b1; ++b) {
                const uint32_t c = hist[b];
                hist[b] = run;
                run += c;
            }
        }
        __syncthreads();
        for (uint32_t base = 0; base < V; base += nt) {
            const uint32_t v = base + tid;
            const uint16_t l = v < V ? lrow[v] : LINF;
            const bool ok = l != LINF;
            if (ok) mem[atomicAdd(&hist[l], 1u)] = (uint16_t)v;
        }
        __syncthreads();
        }
        // hist[l] is now the end of level l (its start: hist[l-1], or 0)
        LOSS_TICK(5)
        // 3. levels in increasing latency, every weight class from its smaller end
        for (uint32_t l = 1; l <= mx; ++l) {
            const uint32_t lo = hist[l - 1], cnt_l = hist[l] - lo;
            if (!cnt_l) continue;  // uniform
            if (tid == 0) {
                uint32_t run = 0, pm = 0;
                for (uint32_t w = 1; w <= WCN; ++w) {
                    uint32_t items = 0;
                    if (w <= l) {
                        // the tails' levels: l - w (and, quantized, l - w - 1)
                        const uint32_t j = l - w, jl = QUANT && j ? j - 1 : j;
                        const uint32_t nj = hist[j] - (jl ? hist[jl - 1] : 0u);
                        if (nj <= cnt_l) pm |= 1u << w;
                        items = nj < cnt_l ? nj : cnt_l;
                    }
                    run += items;
                    plan_end[w] = run;
                }
                plan_push = pm;
            }
            __syncthreads();
            const uint32_t T = plan_end[WCN], pm = plan_push;
            // item t -> (class w, member x, its edge range); the next item's
            // range is loaded while the current one is walked
            auto item = [&](uint32_t t, uint32_t &w, uint32_t &x, uint32_t &e0, uint32_t &e1) {
                w = 1;
                while (t >= plan_end[w]) ++w;
                const uint32_t m = t - (w > 1 ? plan_end[w - 1] : 0u), j = l - w, jl = QUANT && j ? j - 1 : j;
                const bool push = (pm >> w) & 1u;
                x = mem[(push ? (jl ? hist[jl - 1] : 0u) : lo) + m];
                const uint32_t *cl = push ? cls_out : cls_in;
                e0 = cl[(uint64_t)x * CLSN + w - 1];
                e1 = cl[(uint64_t)x * CLSN + w];
            };
            uint32_t nw_ = 1, nx = 0, ne0 = 0, ne1 = 0;
#if LOSS_COUNT
            if (tid == 0) { atomicAdd(&loss_cnt[0], (unsigned long long)T); atomicAdd(&loss_cnt[3], 1ull); }
#endif
            if (grp < T) item(grp, nw_, nx, ne0, ne1);
            for (uint32_t t = grp; t < T; t += ngrp) {
                const uint32_t w = nw_, x = nx, e0 = ne0, e1 = ne1, j = l - w;
                if (t + ngrp < T) item(t + ngrp, nw_, nx, ne0, ne1);
                const bool push = (pm >> w) & 1u;
                const uint64_t *ce = push ? ce_out : ce_in;
                // push: x in N_j, its class-w out-edges x -> v, v in N_l;
                // pull: x in N_l, its class-w in-edges u -> x, u in N_j
                const uint16_t want = (uint16_t)(push ? l : j);
                const float onem = push ? 1.0f - __uint_as_float(prow[x]) : 0.0f;
                // exact closure values of the quantized fold (2- or 4-byte keys, level_q)
                auto exact = [&](uint32_t y) -> uint32_t {
                    const uint64_t idx = (uint64_t)s * Vp + y;
                    return key_type == KEY_U16 ? (uint32_t)reinterpret_cast<const uint16_t *>(D)[idx]
                                               : reinterpret_cast<const uint32_t *>(D)[idx];
                };
                const uint32_t Lx = QUANT ? exact(x) : 0u;
                const uint32_t *cwp = QUANT ? cw + (push ? 0 : cw_in) : nullptr;
                // VW = 2: a lane loads 2 adjacent entries (16 B) at a time from
                // the even entry at or below e0, masking the entries outside [e0, e1)
                constexpr int NE = UNR * VW;  // entries a lane an iteration
                for (uint32_t b = VW == 2 ? e0 & ~1u : e0; b < e1; b += UNR * LPT * VW) {
                    uint64_t wd[NE];
                    uint32_t ei[NE];
#pragma unroll
                    for (int q = 0; q < UNR; ++q) {
                        const uint32_t at = b + (sub + q * LPT) * VW;  // padded past the end
                        if (VW == 2) {
                            const uint4 r2 = *reinterpret_cast<const uint4 *>(ce + at);
                            wd[2 * q] = ((uint64_t)r2.y << 32) | r2.x;
                            wd[2 * q + 1] = ((uint64_t)r2.w << 32) | r2.z;
                            ei[2 * q] = at;
                            ei[2 * q + 1] = at + 1;
                        } else {
                            wd[q] = ce[at];
                            ei[q] = at;
                        }
                    }
                    uint32_t o[NE];
                    bool ok[NE];
#pragma unroll
                    for (int q = 0; q < NE; ++q) {
                        ok[q] = ei[q] < e1 && (VW == 1 || ei[q] >= e0);
                        o[q] = ok[q] ? (uint32_t)wd[q] : 0u;
                    }
                    uint16_t lo_[NE];
#pragma unroll
                    for (int q = 0; q < NE; ++q) lo_[q] = lrow[o[q]];
                    bool hit[NE];
#pragma unroll
                    for (int q = 0; q < NE; ++q) {
                        if (!QUANT) {
                            hit[q] = ok[q] && lo_[q] == want;
                        } else {
                            // the tail's level (j or j - 1) or the head's (l), then exact
                            hit[q] = ok[q] && (push ? lo_[q] == want : lo_[q] == want || lo_[q] + 1 == want);
                            if (hit[q]) {
                                const uint32_t Lo = exact(o[q]), wq = cwp[ei[q]];
                                hit[q] = push ? Lx + wq == Lo : Lo + wq == Lx;  // finite: no wrap below 2^31
                            }
                        }
                    }
#if LOSS_COUNT
                    for (int q = 0; q < NE; ++q) {
                        c_vis += ok[q];
                        c_hit += hit[q];
                        c_phit += push && hit[q];
                    }
#endif
#pragma unroll
                    for (int q = 0; q < NE; ++q) {
                        if (hit[q]) {
                            const float r = __uint_as_float((uint32_t)(wd[q] >> 32));
                            if (push) {
                                const float c = 1.0f - __fmul_rn(onem, r);
                                atomicMin(&prow[o[q]], __float_as_uint(c));
                            } else {
                                const float c = 1.0f - __fmul_rn(1.0f - __uint_as_float(prow[o[q]]), r);
                                atomicMin(&prow[x], __float_as_uint(c));
                            }
                        }
                    }
                }
            }
            __syncthreads();  // level l final; plan_end rewritten by the next level
        }
        LOSS_TICK(6)
        // 4. table row i (or staging slot k)
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        uint32_t *o32 = out32 && !stage16 ? reinterpret_cast<uint32_t *>(out32) + (uint64_t)k * n : nullptr;
        uint16_t *o16 = out32 && stage16 ? reinterpret_cast<uint16_t *>(out32) + (uint64_t)k * n : nullptr;
        float *o32p = out32_loss ? out32_loss + (uint64_t)k * n : nullptr;  // staging (loss only if !out32)
        // (4 node ids loaded ahead a thread; the staged latency is the
        // closure's unit count, no division by g)
        for (uint32_t j0 = tid; j0 < n; j0 += 4 * nt) {
            uint32_t vv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = j0 + q * nt < n ? nodes[j0 + q * nt] : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = j0 + q * nt;
                if (j >= n) break;
                uint64_t latv, lu;
                float lossv;
                if (j == i) {
                    latv = sl_lat[j];
                    lossv = sl_loss[j];
                    lu = latv == ~0ull ? ~0ull : latv / g;
                } else {
                    const uint32_t v = vv[q];
                    const uint16_t l = lrow[v];
                    if (l == LINF) {
                        ++unreach;
                        latv = lu = ~0ull;
                        lossv = 1.0f;
                    } else {
                        bool vinf;
                        lu = QUANT ? closure_lat(D, (uint64_t)s * Vp + v, key_type, vinf) : (uint64_t)l;
                        latv = lu * g;
                        lossv = __uint_as_float(prow[v]);
                    }
                }
                if (o32p) {
                    if (o16) o16[j] = latv == ~0ull ? (uint16_t)0xffffu : (uint16_t)lu;
                    else if (o32) o32[j] = latv == ~0ull ? ~0u : (uint32_t)lu;
                    o32p[j] = lossv;
                } else {
                    ol[j] = latv;
                    op[j] = lossv;
                }
                mn = latv < mn ? latv : mn;
            }
        }
        __syncthreads();  // the next row rewrites the LDS rows
        LOSS_TICK(7)
    }
#if LOSS_COUNT
    atomicAdd(&loss_cnt[1], (unsigned long long)c_vis);
    atomicAdd(&loss_cnt[2], (unsigned long long)c_hit);
    atomicAdd(&loss_cnt[8], (unsigned long long)c_phit);
#endif
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
        for (int q = 1; q < nw; ++q) {
            m = red_min[q] < m ? red_min[q] : m;
            c += red_cnt[q];
        }
        atomicMin(&stats[0], m);
        if (c) atomicAdd(&stats[1], c);
    }
}

// ------------------------------------------------------------ level solve
constexpr size_t SOLVE_HIST = 256;  // level ends, levels <= LWC
constexpr uint32_t LWC = 63;        // the level solve's classes / levels at most (CLSN 64)
// Closure-free dense build (SRT_ALGO_LEVEL): petgraph's Dijkstra per source
// (mod.rs:195-198) as a bucket queue with unit-wide buckets -- Dial's
// algorithm -- over the graph's edges of latency <= B units, where B bounds
// every shortest path (the create-time probe: out- plus in-eccentricity of one
// in-use node, level_probe).  No edge longer than B can lie on a shortest
// path, so the pruned graph has the same distances and the same tight edges.
// Latencies are integers in units of g >= 1, so the bucket of level l holds
// exactly N_l = {v : L(s,v) = l}, final once every level j < l is: its members
// are the heads of the class-(l - j) edges out of N_j.  For each class w the
// candidates of level l are walked from the smaller end, as in the level fold
// above: push along class-w out-edges of N_{l-w}, or -- when the still
// unsettled set U_l is smaller -- pull along class-w in-edges of every u in
// U_l, testing the tail's level.  A hit sets the head's level to l (a plain
// store: every writer stores l) and min-folds the loss candidate
// 1 - (1 - loss[u]) (1 - e) into it by an LDS atomic on the f32 bits: the tails
// are final, so the result is the min over tight in-edges, the same bits as the
// reference's lexicographic (latency, loss) Dijkstra (the level fold's
// argument).  One workgroup per table row; LDS: level u16, loss f32, and
// the settled vertices in level order u16 (8 B a vertex, as the level fold).
// C3 (16k complete graph, latencies 1-300 ms): B = 8, levels of ~1 / 60 /
// 3,000 / 13,000 / few vertices, ~175k edge visits a row against 16,384^2 / 2
// relaxations a row for the triangle Floyd-Warshall.
// probe != nullptr: no table; probe[2 + k] = the largest level over the
// in-use columns of row k (0xffff if one is unreached by level lcap), the u64
// at probe[0] += the edges walked.
// SP (VW = 2): the class lists walked as one stream of chunks a lane group,
// software-pipelined (see the walk below).
template <int LPT, int UNR, uint32_t CLSN, int VW, bool NT, bool SP = false>
__global__ __launch_bounds__(LOSS_NT) void level_solve_kernel(
    uint32_t V, const uint32_t *__restrict__ nodes, uint32_t n, uint32_t row0, uint32_t row1,
    const uint32_t *__restrict__ cls_out, const uint32_t *__restrict__ cls_in, const uint64_t *__restrict__ ce_out,
    const uint64_t *__restrict__ ce_in, uint32_t lcap, uint64_t g, const uint64_t *__restrict__ sl_lat,
    const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat, float *__restrict__ out_loss,
    unsigned long long *stats, const uint32_t *__restrict__ row_list, void *__restrict__ out32,
    float *__restrict__ out32_loss, bool stage16, uint32_t *__restrict__ probe,
    unsigned long long *__restrict__ visit_cnt, bool idn, unsigned long long *row_ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ unsigned long long red_min[16], red_cnt[16], red_vis[16];
    __shared__ uint32_t dyn_k;
    __shared__ uint32_t red_max[16];
    constexpr uint32_t WCN = CLSN - 1;
    __shared__ uint32_t plan_end[WCN + 1];
    __shared__ uint64_t plan_push;
    __shared__ uint32_t plan_pull;
    __shared__ uint32_t cur[2][2];  // [level parity]: unsettled compaction, level collection
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem);  // hist[l]: end of level l in mem (l <= 31)
    uint16_t *lrow = reinterpret_cast<uint16_t *>(smem + SOLVE_HIST);
    const size_t lat_b = ((size_t)V * 2 + 15) & ~(size_t)15, mem_b = ((size_t)V * 2 + 15) & ~(size_t)15;
    uint32_t *prow = reinterpret_cast<uint32_t *>(smem + SOLVE_HIST + lat_b);
    uint16_t *mem = reinterpret_cast<uint16_t *>(smem + SOLVE_HIST + lat_b + (size_t)V * 4);
    (void)mem_b;
    const uint16_t LINF = 0xffffu;
    const uint32_t FINF = 0x7f800000u;  // +inf bits
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const uint32_t grp = tid / LPT, sub = tid % LPT, ngrp = nt / LPT;
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0, visits = 0;
    const uint32_t nrows = row_list ? row1 : row1 - row0;
    // rows dealt by a counter (row_ctr != nullptr; else statically, row k to
    // workgroup k mod grid): a workgroup takes its next row one row ahead (the
    // atomic's latency behind the row's work), so a CU whose rows ran long
    // takes fewer; every workgroup makes exactly one fetch past the last row
    unsigned long long kn = 0;
    auto fetch = [&]() -> uint32_t {
        if (tid == 0) dyn_k = (uint32_t)(kn < nrows ? kn : nrows);
        __syncthreads();
        return dyn_k;
    };
    if (row_ctr && tid == 0) kn = atomicAdd(&row_ctr[0], 1ull);
    uint32_t k0 = blockIdx.x;
    if (row_ctr) k0 = fetch();
    for (uint32_t k = k0; k < nrows; k = row_ctr ? fetch() : k + gridDim.x) {
        if (row_ctr && tid == 0) kn = atomicAdd(&row_ctr[0], 1ull);  // the next row
        const uint32_t i = row_list ? row_list[k] : row0 + k;
        const uint32_t s = nodes[i];
#if LOSS_COUNT
        unsigned long long tk0 = wall_clock64();
#endif
        // 1. every vertex unreached, s at level 0 (petgraph's zero score);
        // four vertices a thread a step (8-B level and 16-B loss stores)
        for (uint32_t v4 = 4 * tid; v4 < V; v4 += 4 * nt) {
            if (v4 + 3 < V) {
                uint2 lw = make_uint2(0xffffffffu, 0xffffffffu);
                uint4 pw = make_uint4(FINF, FINF, FINF, FINF);
                if (s - v4 < 4u) {  // s among them: level 0, loss 0 (selects, no indexed lvalue)
                    const uint32_t q = s - v4;
                    lw.x &= q == 0 ? 0xffff0000u : q == 1 ? 0x0000ffffu : 0xffffffffu;
                    lw.y &= q == 2 ? 0xffff0000u : q == 3 ? 0x0000ffffu : 0xffffffffu;
                    pw.x = q == 0 ? 0u : pw.x;
                    pw.y = q == 1 ? 0u : pw.y;
                    pw.z = q == 2 ? 0u : pw.z;
                    pw.w = q == 3 ? 0u : pw.w;
                }
                *reinterpret_cast<uint2 *>(lrow + v4) = lw;
                *reinterpret_cast<uint4 *>(prow + v4) = pw;
            } else {
                for (uint32_t v = v4; v < V; ++v) {
                    lrow[v] = v == s ? (uint16_t)0 : LINF;
                    prow[v] = v == s ? 0u : FINF;
                }
            }
        }
        if (tid == 0) {
            hist[0] = 1;
            mem[0] = (uint16_t)s;
            cur[1][0] = cur[1][1] = 0;
        }
        __syncthreads();
        LOSS_TICK(4)
        uint32_t settled = 1;
        // the vertices v with lrow[v] == want appended to mem[at + cur[par][ci]
        // ...) in any order: four a thread a step (one 8-B level read), one
        // LDS atomic a wave a step
        auto compact = [&](uint16_t want, uint32_t at, uint32_t par, int ci) {
            for (uint32_t v4 = 4 * tid; v4 < V; v4 += 4 * nt) {
                uint32_t fm = 0;
                if (v4 + 3 < V) {
                    const uint2 w = *reinterpret_cast<const uint2 *>(lrow + v4);
                    fm = (uint32_t)((w.x & 0xffffu) == want) | (uint32_t)((w.x >> 16) == want) << 1 |
                         (uint32_t)((w.y & 0xffffu) == want) << 2 | (uint32_t)((w.y >> 16) == want) << 3;
                } else {
                    for (uint32_t q = 0; q < 4; ++q)
                        if (v4 + q < V && lrow[v4 + q] == want) fm |= 1u << q;
                }
                uint32_t tot = 0, bel = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint64_t m = __ballot((fm >> q) & 1u);
                    tot += (uint32_t)__popcll(m);
                    bel += (uint32_t)__popcll(m & below);
                }
                if (!tot) continue;  // uniform
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(&cur[par][ci], tot);
                b = __shfl(b, 0);
                uint32_t pos = at + b + bel;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if ((fm >> q) & 1u) mem[pos++] = (uint16_t)(v4 + q);
            }
        };
        // 2. levels in increasing latency
        for (uint32_t l = 1; l <= lcap && settled < V; ++l) {
            const uint32_t U = V - settled, par = l & 1u;
            if (tid == 0) {
                uint32_t run = 0, pl = 0;
                uint64_t pm = 0;
                for (uint32_t w = 1; w <= WCN; ++w) {
                    uint32_t items = 0;
                    if (w <= l) {
                        const uint32_t j = l - w, nj = hist[j] - (j ? hist[j - 1] : 0u);
                        if (nj && nj <= U) {
                            pm |= 1ull << w;
                            items = nj;
                        } else if (nj) {
                            pl = 1;
                            items = U;
                        }
                    }
                    run += items;
                    plan_end[w] = run;
                }
                plan_push = pm;
                plan_pull = pl;
                cur[par][0] = cur[par][1] = 0;
            }
            __syncthreads();
            const uint32_t T = plan_end[WCN];
            const uint64_t pm = plan_push;
            // no tail level l - w (w <= WCN, every class) holds a vertex: the
            // levels >= l are all empty (uniform)
            if (T == 0) break;
#if LOSS_COUNT
            unsigned long long lt0 = wall_clock64();
#define LVL_TICK(q)                                                                    \
    if (tid == 0 && l < 8) {                                                           \
        const unsigned long long lt1 = wall_clock64();                                 \
        atomicAdd(&lvl_cnt[l][q], lt1 - lt0);                                          \
        lt0 = lt1;                                                                     \
    }
            if (tid == 0 && l < 8) {
                atomicAdd(&lvl_cnt[l][3], (unsigned long long)T);
                atomicAdd(&lvl_cnt[l][4], 1ull);
            }
#else
#define LVL_TICK(q)
#endif
            if (plan_pull) {
                // the unsettled vertices into mem[settled, V) (any order)
                compact(LINF, settled, par, 0);
                __syncthreads();
            }
            LVL_TICK(0)
            // item t: its class w (searched up from the w passed in -- a lane
            // group's items come in increasing t, so from its last item's:
            // one LDS read, not up to WCN dependent ones), vertex and list
            auto item = [&](uint32_t t, uint32_t &w, uint32_t &x, uint32_t &e0, uint32_t &e1) {
                while (t >= plan_end[w]) ++w;
                const uint32_t m = t - (w > 1 ? plan_end[w - 1] : 0u), j = l - w;
                const bool push = (pm >> w) & 1ull;
                x = mem[push ? (j ? hist[j - 1] : 0u) + m : settled + m];
                const uint32_t *cl = push ? cls_out : cls_in;
                e0 = cl[(uint64_t)x * CLSN + w - 1];
                e1 = cl[(uint64_t)x * CLSN + w];
            };
            if constexpr (SP) {
                // The level's items as one stream of chunks a lane group (CH
                // entries of one item's class list, UNR pairs a lane): the next
                // chunk's entry loads go out before this chunk's level probes
                // and folds, so their latency hides behind the LDS work, and an
                // item's offsets are read one item ahead.  Push and pull chunks
                // run apart (push is uniform in an item and, but at a class
                // boundary, in a wave), without a per-entry direction test.
                static_assert(VW == 2, "the pipelined walk loads entry pairs");
                constexpr uint32_t CH = UNR * LPT * 2;
                constexpr int NE = UNR * 2;
                auto load = [&](uint4 *d, uint32_t w, uint32_t b) {
                    const uint64_t *ce = ((pm >> w) & 1ull) ? ce_out : ce_in;
#pragma unroll
                    for (int q = 0; q < UNR; ++q) d[q] = *reinterpret_cast<const uint4 *>(ce + b + (sub + q * LPT) * 2);
                };
                // a small level (2 T <= lane groups) in a workgroup alone on its
                // CU (1,024 threads: nothing else hides its latency): K groups an
                // item, group g taking item g mod T's chunks g div T, + K, + 2K,
                // ... (one item a group), so its few lists are walked in one or
                // two steps instead of one chunk a step by one group (C3 4.40 ->
                // 4.26 ms; C2's 4 workgroups a CU: 0.334 -> 0.351 ms, so not there)
                const uint32_t K = nt == LOSS_NT && 2 * T <= ngrp ? ngrp / T : 1u;
                const uint32_t CHS = K * CH;  // a group's chunk stride in an item
                uint32_t ct = K > 1 ? (grp < T * K ? grp % T : T) : grp, cw = 1, cx = 0, ce0 = 0, ce1 = 0;
                uint32_t pw = 1, px = 0, pe0 = 0, pe1 = 0;  // the group's next item
                if (ct < T) item(ct, cw, cx, ce0, ce1);
                pw = cw;
                if (ct + ngrp < T) item(ct + ngrp, pw, px, pe0, pe1);
                uint32_t cb = (ce0 & ~1u) + (K > 1 ? grp / T : 0u) * CH;
                uint4 cur[UNR];
                if (ct < T && cb < ce1) load(cur, cw, cb);  // (a chunk past a short list: nothing to load)
                while (ct < T) {
                    // the next chunk: this item's next one, or the next item's first
                    uint32_t nt2 = ct, nw2 = cw, nx2 = cx, ne02 = ce0, ne12 = ce1, nb = cb + CHS;
                    const bool adv = nb >= ce1;
                    if (adv) {
                        nt2 = ct + ngrp;
                        nw2 = pw;
                        nx2 = px;
                        ne02 = pe0;
                        ne12 = pe1;
                        nb = pe0 & ~1u;
                    }
                    uint4 nxt[UNR];
                    if (nt2 < T) load(nxt, nw2, nb);
                    if (adv && nt2 + ngrp < T) item(nt2 + ngrp, pw, px, pe0, pe1);
                    if (cb < ce1) {
                        uint64_t wd[NE];
                        uint32_t o[NE];
                        bool ok[NE];
#pragma unroll
                        for (int q = 0; q < UNR; ++q) {
                            wd[2 * q] = ((uint64_t)cur[q].y << 32) | cur[q].x;
                            wd[2 * q + 1] = ((uint64_t)cur[q].w << 32) | cur[q].z;
                            const uint32_t at = cb + (sub + q * LPT) * 2;
                            ok[2 * q] = at < ce1 && at >= ce0;
                            ok[2 * q + 1] = at + 1 < ce1;  // at + 1 >= ce0: at >= ce0 & ~1
                        }
#pragma unroll
                        for (int q = 0; q < NE; ++q) o[q] = ok[q] ? (uint32_t)wd[q] : 0u;
                        uint16_t lo_[NE];
#pragma unroll
                        for (int q = 0; q < NE; ++q) lo_[q] = lrow[o[q]];
#pragma unroll
                        for (int q = 0; q < NE; ++q) visits += ok[q];
                        if ((pm >> cw) & 1ull) {
                            // push: x in N_j, its class-w out-edges x -> v, v
                            // unsettled or at l: v enters level l (stored once),
                            // its loss min-folded by an LDS atomic
                            const float onem = 1.0f - __uint_as_float(prow[cx]);
#pragma unroll
                            for (int q = 0; q < NE; ++q)
                                if (ok[q] && lo_[q] >= (uint16_t)l) {
                                    const float r = __uint_as_float((uint32_t)(wd[q] >> 32));
#if LOSS_COUNT
                                    if (!(lvl_diag & 2) && lo_[q] > (uint16_t)l) lrow[o[q]] = (uint16_t)l;
                                    if (!(lvl_diag & 1))
                                        atomicMin(&prow[o[q]], __float_as_uint(1.0f - __fmul_rn(onem, r)));
#else
                                    if (lo_[q] > (uint16_t)l) lrow[o[q]] = (uint16_t)l;
                                    atomicMin(&prow[o[q]], __float_as_uint(1.0f - __fmul_rn(onem, r)));
#endif
                                }
                        } else {
                            // pull: x unsettled, its class-w in-edges u -> x, u in N_j
                            const uint32_t j = l - cw;
#pragma unroll
                            for (int q = 0; q < NE; ++q)
                                if (ok[q] && lo_[q] == (uint16_t)j) {
                                    const float r = __uint_as_float((uint32_t)(wd[q] >> 32));
                                    lrow[cx] = (uint16_t)l;
                                    const float c = 1.0f - __fmul_rn(1.0f - __uint_as_float(prow[o[q]]), r);
                                    atomicMin(&prow[cx], __float_as_uint(c));
                                }
                        }
                    }
                    ct = nt2;
                    cw = nw2;
                    cx = nx2;
                    ce0 = ne02;
                    ce1 = ne12;
                    cb = nb;
#pragma unroll
                    for (int q = 0; q < UNR; ++q) cur[q] = nxt[q];
                }
            } else {
                uint32_t nw_ = 1, nx = 0, ne0 = 0, ne1 = 0;
                if (grp < T) item(grp, nw_, nx, ne0, ne1);
                for (uint32_t t = grp; t < T; t += ngrp) {
                    const uint32_t w = nw_, x = nx, e0 = ne0, e1 = ne1, j = l - w;
                    if (t + ngrp < T) item(t + ngrp, nw_, nx, ne0, ne1);
                    const bool push = (pm >> w) & 1ull;
                    const uint64_t *ce = push ? ce_out : ce_in;
                    // push: x in N_j, its class-w out-edges x -> v, v unsettled or at l;
                    // pull: x unsettled, its class-w in-edges u -> x, u in N_j
                    const float onem = push ? 1.0f - __uint_as_float(prow[x]) : 0.0f;
                    constexpr int NE = UNR * VW;
                    for (uint32_t b = VW == 2 ? e0 & ~1u : e0; b < e1; b += UNR * LPT * VW) {
                        uint64_t wd[NE];
                        uint32_t ei[NE];
#pragma unroll
                        for (int q = 0; q < UNR; ++q) {
                            const uint32_t at = b + (sub + q * LPT) * VW;  // padded past the end
                            if (VW == 2) {
                                const uint4 r2 = *reinterpret_cast<const uint4 *>(ce + at);
                                wd[2 * q] = ((uint64_t)r2.y << 32) | r2.x;
                                wd[2 * q + 1] = ((uint64_t)r2.w << 32) | r2.z;
                                ei[2 * q] = at;
                                ei[2 * q + 1] = at + 1;
                            } else {
                                wd[q] = ce[at];
                                ei[q] = at;
                            }
                        }
                        uint32_t o[NE];
                        bool ok[NE];
#pragma unroll
                        for (int q = 0; q < NE; ++q) {
                            ok[q] = ei[q] < e1 && (VW == 1 || ei[q] >= e0);
                            o[q] = ok[q] ? (uint32_t)wd[q] : 0u;
                        }
                        uint16_t lo_[NE];
#pragma unroll
                        for (int q = 0; q < NE; ++q) lo_[q] = lrow[o[q]];
#pragma unroll
                        for (int q = 0; q < NE; ++q) {
                            visits += ok[q];
                            const bool hit = ok[q] && (push ? lo_[q] >= (uint16_t)l : lo_[q] == (uint16_t)j);
                            if (hit) {
                                // the head enters level l (every writer stores l; a
                                // head already at l is not stored again), its loss
                                // min-folded by an LDS atomic (reading the loss first
                                // and skipping the atomic when it cannot lower it
                                // measured slower: C3 walk 49 -> 56 us a row)
                                const float r = __uint_as_float((uint32_t)(wd[q] >> 32));
                                if (push) {
#if LOSS_COUNT
                                    // diagnostic builds: lvl_diag bit 0 drops the loss atomics,
                                    // bit 1 the level stores (wrong tables; timing only)
                                    if (!(lvl_diag & 2) && lo_[q] != (uint16_t)l) lrow[o[q]] = (uint16_t)l;
                                    if (!(lvl_diag & 1))
                                        atomicMin(&prow[o[q]], __float_as_uint(1.0f - __fmul_rn(onem, r)));
#else
                                    if (lo_[q] != (uint16_t)l) lrow[o[q]] = (uint16_t)l;
                                    atomicMin(&prow[o[q]], __float_as_uint(1.0f - __fmul_rn(onem, r)));
#endif
                                } else {
                                    lrow[x] = (uint16_t)l;
                                    const float c = 1.0f - __fmul_rn(1.0f - __uint_as_float(prow[o[q]]), r);
                                    atomicMin(&prow[x], __float_as_uint(c));
                                }
                            }
                        }
                    }
                }
            }
            __syncthreads();  // every head of level l found
            LVL_TICK(1)
            // N_l (the vertices now at level l) -> mem[settled, ...)
            compact((uint16_t)l, settled, par, 1);
            __syncthreads();
            LVL_TICK(2)
            settled += cur[par][1];
            if (tid == 0) hist[l] = settled;
        }
        __syncthreads();  // hist / lrow final for the output
        LOSS_TICK(6)
        // 3. table row i (or staging slot k), or the probe's row maximum
        if (probe) {
            uint32_t rmax = 0;
            for (uint32_t j0 = tid; j0 < n; j0 += nt) {
                const uint32_t l = lrow[nodes[j0]];
                rmax = l > rmax ? l : rmax;
            }
            for (int off = 32; off > 0; off >>= 1) {
                const uint32_t o = __shfl_xor(rmax, off);
                rmax = o > rmax ? o : rmax;
            }
            if (lane == 0) red_max[wv] = rmax;
            __syncthreads();
            if (tid == 0) {
                uint32_t m = 0;
                for (int q = 0; q < nw; ++q) m = red_max[q] > m ? red_max[q] : m;
                probe[2 + k] = m;
            }
            __syncthreads();
            continue;
        }
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        uint32_t *o32 = out32 && !stage16 ? reinterpret_cast<uint32_t *>(out32) + (uint64_t)k * n : nullptr;
        uint16_t *o16 = out32 && stage16 ? reinterpret_cast<uint16_t *>(out32) + (uint64_t)k * n : nullptr;
        float *o32p = out32_loss ? out32_loss + (uint64_t)k * n : nullptr;
        if (idn) {
            // every node in use, in node order (nodes[j] = j, n = V, n % 4 == 0):
            // four columns a thread a step -- one 8-B level and one 16-B loss
            // read from LDS, 16-B non-temporal stores
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
            for (uint32_t j4 = 4 * tid; j4 < n; j4 += 4 * nt) {
                const uint2 lw = *reinterpret_cast<const uint2 *>(lrow + j4);
                const uint4 pw = *reinterpret_cast<const uint4 *>(prow + j4);
                const uint32_t lv[4] = {lw.x & 0xffffu, lw.x >> 16, lw.y & 0xffffu, lw.y >> 16};
                const uint32_t pv[4] = {pw.x, pw.y, pw.z, pw.w};
                uint64_t lu[4], latv[4];
                float lossv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (j4 + q == i) {
                        latv[q] = sl_lat[i];
                        lossv[q] = sl_loss[i];
                        lu[q] = latv[q] == ~0ull ? ~0ull : latv[q] / g;
                    } else if (lv[q] == LINF) {
                        ++unreach;
                        latv[q] = lu[q] = ~0ull;
                        lossv[q] = 1.0f;
                    } else {
                        lu[q] = lv[q];
                        latv[q] = lu[q] * g;
                        lossv[q] = __uint_as_float(pv[q]);
                    }
                    mn = latv[q] < mn ? latv[q] : mn;
                }
                const f32x4 lp = {lossv[0], lossv[1], lossv[2], lossv[3]};
                if (o32p) {
                    if (o16) {
                        const u16x4 lq = {(unsigned short)(latv[0] == ~0ull ? 0xffffu : lu[0]),
                                          (unsigned short)(latv[1] == ~0ull ? 0xffffu : lu[1]),
                                          (unsigned short)(latv[2] == ~0ull ? 0xffffu : lu[2]),
                                          (unsigned short)(latv[3] == ~0ull ? 0xffffu : lu[3])};
                        __builtin_nontemporal_store(lq, reinterpret_cast<u16x4 *>(o16 + j4));
                    } else if (o32) {
                        const u32x4 lq = {latv[0] == ~0ull ? ~0u : (unsigned)lu[0],
                                          latv[1] == ~0ull ? ~0u : (unsigned)lu[1],
                                          latv[2] == ~0ull ? ~0u : (unsigned)lu[2],
                                          latv[3] == ~0ull ? ~0u : (unsigned)lu[3]};
                        __builtin_nontemporal_store(lq, reinterpret_cast<u32x4 *>(o32 + j4));
                    }
                    __builtin_nontemporal_store(lp, reinterpret_cast<f32x4 *>(o32p + j4));
                } else if (NT) {
                    const u64x2 a = {latv[0], latv[1]}, c = {latv[2], latv[3]};
                    __builtin_nontemporal_store(a, reinterpret_cast<u64x2 *>(ol + j4));
                    __builtin_nontemporal_store(c, reinterpret_cast<u64x2 *>(ol + j4 + 2));
                    __builtin_nontemporal_store(lp, reinterpret_cast<f32x4 *>(op + j4));
                } else {
                    *reinterpret_cast<u64x2 *>(ol + j4) = u64x2{latv[0], latv[1]};
                    *reinterpret_cast<u64x2 *>(ol + j4 + 2) = u64x2{latv[2], latv[3]};
                    *reinterpret_cast<f32x4 *>(op + j4) = lp;
                }
            }
        } else
        for (uint32_t j0 = tid; j0 < n; j0 += 4 * nt) {
            uint32_t vv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = j0 + q * nt < n ? nodes[j0 + q * nt] : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = j0 + q * nt;
                if (j >= n) break;
                uint64_t latv, lu;
                float lossv;
                if (j == i) {
                    latv = sl_lat[j];
                    lossv = sl_loss[j];
                    lu = latv == ~0ull ? ~0ull : latv / g;
                } else {
                    const uint16_t l = lrow[vv[q]];
                    if (l == LINF) {
                        ++unreach;
                        latv = lu = ~0ull;
                        lossv = 1.0f;
                    } else {
                        lu = l;
                        latv = lu * g;
                        lossv = __uint_as_float(prow[vv[q]]);
                    }
                }
                // streamed out without allocating in the caches (NT): the
                // class CSRs the walks read stay resident
                if (o32p) {
                    if (o16) __builtin_nontemporal_store(latv == ~0ull ? (uint16_t)0xffffu : (uint16_t)lu, o16 + j);
                    else if (o32) __builtin_nontemporal_store(latv == ~0ull ? ~0u : (uint32_t)lu, o32 + j);
                    __builtin_nontemporal_store(lossv, o32p + j);
                } else if (NT) {
                    __builtin_nontemporal_store(latv, ol + j);
                    __builtin_nontemporal_store(lossv, op + j);
                } else {
                    ol[j] = latv;
                    op[j] = lossv;
                }
                mn = latv < mn ? latv : mn;
            }
        }
        __syncthreads();  // the next row rewrites the LDS rows
        LOSS_TICK(7)
    }
#if LOSS_COUNT
    if (!probe) atomicAdd(&loss_cnt[1], visits);
#endif
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mn, off);
        mn = o < mn ? o : mn;
        unreach += __shfl_xor(unreach, off);
        visits += __shfl_xor(visits, off);
    }
    if (lane == 0) {
        red_min[wv] = mn;
        red_cnt[wv] = unreach;
        red_vis[wv] = visits;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], c = red_cnt[0], vz = red_vis[0];
        for (int q = 1; q < nw; ++q) {
            m = red_min[q] < m ? red_min[q] : m;
            c += red_cnt[q];
            vz += red_vis[q];
        }
        if (probe) {
            if (vz) atomicAdd(reinterpret_cast<unsigned long long *>(probe), vz);
        } else {
            atomicMin(&stats[0], m);
            if (c) atomicAdd(&stats[1], c);
            if (visit_cnt && vz) atomicAdd(visit_cnt, vz);
        }
        // the last workgroup done (every fetch made) returns the counter to 0
        // for the next launch (memory-side atomics; the launch boundary orders it)
        if (row_ctr && atomicAdd(&row_ctr[1], 1ull) == gridDim.x - 1ull) {
            atomicExch(&row_ctr[0], 0ull);
            atomicExch(&row_ctr[1], 0ull);
        }
    }
}

// ------------------------------------------------- quantized level solve
// The level solve for latencies that are not small integers of g (Shadow
// reads any unit down to ns, units.rs:377-388: C3ns has g = 1 ns and edges of
// 1-301 ms).  Buckets of width q <= the shortest edge (units): bucket k holds
// the vertices of L(s, v) in [k q, (k + 1) q), classes c = floor(w / q) >= 1.
// A tight predecessor u of v has L(s, u) <= L(s, v) - q, so it lies in an
// earlier bucket, and an edge of class c out of bucket j reaches bucket j + c
// or j + c + 1.  Processing the pairs (j, c) with j + c = k at step k (push
// along class-c out-edges of N_j, or pull into the unsettled set along class-c
// in-edges from tails in bucket j, the smaller end as in level_solve_kernel)
// therefore leaves every vertex whose key lands in bucket k final once step k
// is done: its candidates come from steps k - 1 and k only.  A vertex's key is
// one u64, L units << 32 | loss bits, min-ed by an LDS atomic: the
// lexicographic (latency, loss) order of the reference's Dijkstra (mod.rs:
// 305-340), over tails that are final when read.  Candidates past dcap (the
// probe's bound B) are dropped, so every key stored is settled by the last
// bucket, B / q.  Class entries: v in bits [0, vb), the weight's remainder
// w - c q in [vb, vb + rb), (1f32 - e) bits in [34, 64).  LDS: 8 B a vertex;
// the settled vertices in bucket order live in a per-workgroup global scratch
// (mem_all + blockIdx.x * V, L2-resident).  stage_mode: 0 the table, 2 u32
// units + f32 loss staging (row k at k * n), 3 8-byte records {units, loss
// bits}.  probe != nullptr: probe[2 + k] = the largest L units over the in-use
// columns of row k (~0 if one is unreached), the u64 at probe[0] += visits.
template <int LPT, int UNR, uint32_t CLSN, int VW, bool NT>
__global__ __launch_bounds__(LOSS_NT) void level_q_kernel(
    uint32_t V, const uint32_t *__restrict__ nodes, uint32_t n, uint32_t row0, uint32_t row1,
    const uint32_t *__restrict__ cls_out, const uint32_t *__restrict__ cls_in, const uint64_t *__restrict__ ce_out,
    const uint64_t *__restrict__ ce_in, uint32_t kcap, uint32_t dcap, uint32_t qw, uint32_t rb, uint32_t vb, uint64_t g,
    const uint64_t *__restrict__ sl_lat, const float *__restrict__ sl_loss, uint64_t *__restrict__ out_lat,
    float *__restrict__ out_loss, unsigned long long *stats, const uint32_t *__restrict__ row_list,
    void *__restrict__ stage, float *__restrict__ stage_loss, uint32_t stage_mode, uint32_t *__restrict__ probe,
    unsigned long long *__restrict__ visit_cnt, uint16_t *__restrict__ mem_all) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ unsigned long long red_min[16], red_cnt[16], red_vis[16];
    __shared__ uint32_t red_max[16];
    constexpr uint32_t WCN = CLSN - 1;
    __shared__ uint32_t plan_end[WCN + 1];
    __shared__ uint64_t plan_push;
    __shared__ uint32_t plan_pull;
    __shared__ uint32_t cur[2][2];
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem);  // hist[k]: end of bucket k in mem (k <= 31)
    unsigned long long *key = reinterpret_cast<unsigned long long *>(smem + SOLVE_HIST);
    uint16_t *mem = mem_all + (uint64_t)blockIdx.x * V;
    const unsigned long long KINF = ~0ull;
    const uint64_t vmask = (1ull << vb) - 1ull, rmask = (1ull << rb) - 1ull;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const uint32_t grp = tid / LPT, sub = tid % LPT, ngrp = nt / LPT;
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t mn = ~0ull;
    unsigned long long unreach = 0, visits = 0;
    const uint32_t nrows = row_list ? row1 : row1 - row0;
    for (uint32_t k = blockIdx.x; k < nrows; k += gridDim.x) {
        const uint32_t i = row_list ? row_list[k] : row0 + k;
        const uint32_t s = nodes[i];
        for (uint32_t v = tid; v < V; v += nt) key[v] = v == s ? 0ull : KINF;
        if (tid == 0) {
            hist[0] = 1;
            mem[0] = (uint16_t)s;
            cur[1][0] = cur[1][1] = 0;
        }
        __syncthreads();
        uint32_t settled = 1;
        for (uint32_t b = 1; b <= kcap && settled < V; ++b) {
            const uint32_t U = V - settled, par = b & 1u;
            if (tid == 0) {
                uint32_t run = 0, pl = 0;
                uint64_t pm = 0;
                for (uint32_t c = 1; c <= WCN; ++c) {
                    uint32_t items = 0;
                    if (c <= b) {
                        const uint32_t j = b - c, nj = hist[j] - (j ? hist[j - 1] : 0u);
                        if (nj && nj <= U) {
                            pm |= 1ull << c;
                            items = nj;
                        } else if (nj) {
                            pl = 1;
                            items = U;
                        }
                    }
                    run += items;
                    plan_end[c] = run;
                }
                plan_push = pm;
                plan_pull = pl;
                cur[par][0] = cur[par][1] = 0;
            }
            __syncthreads();
            const uint32_t T = plan_end[WCN];
            const uint64_t pm = plan_push;
            const uint32_t lo = b * qw, hi = lo + qw;  // bucket b: latencies [lo, hi)
            if (T && plan_pull) {
                // the unsettled vertices (key at bucket >= b, or none) into mem[settled, V)
                for (uint32_t base = 0; base < V; base += nt) {
                    const uint32_t v = base + tid;
                    const bool f = v < V && (uint32_t)(key[v] >> 32) >= lo;
                    const uint64_t m = __ballot(f);
                    if (!m) continue;  // uniform
                    uint32_t o = 0;
                    if (lane == 0) o = atomicAdd(&cur[par][0], (uint32_t)__popcll(m));
                    o = __shfl(o, 0);
                    if (f) mem[settled + o + (uint32_t)__popcll(m & below)] = (uint16_t)v;
                }
                __syncthreads();
            }
            auto item = [&](uint32_t t, uint32_t &c, uint32_t &x, uint32_t &e0, uint32_t &e1) {
                c = 1;
                while (t >= plan_end[c]) ++c;
                const uint32_t m = t - (c > 1 ? plan_end[c - 1] : 0u), j = b - c;
                const bool push = (pm >> c) & 1ull;
                x = mem[push ? (j ? hist[j - 1] : 0u) + m : settled + m];
                const uint32_t *cl = push ? cls_out : cls_in;
                e0 = cl[(uint64_t)x * CLSN + c - 1];
                e1 = cl[(uint64_t)x * CLSN + c];
            };
            uint32_t nc_ = 1, nx = 0, ne0 = 0, ne1 = 0;
            if (grp < T) item(grp, nc_, nx, ne0, ne1);
            for (uint32_t t = grp; t < T; t += ngrp) {
                const uint32_t c = nc_, x = nx, e0 = ne0, e1 = ne1, j = b - c;
                if (t + ngrp < T) item(t + ngrp, nc_, nx, ne0, ne1);
                const bool push = (pm >> c) & 1ull;
                const uint64_t *ce = push ? ce_out : ce_in;
                const uint32_t cbase = c * qw, jlo = j * qw, jhi = jlo + qw;
                // push: x in bucket j (final), its class-c out-edges x -> v;
                // pull: x unsettled, its class-c in-edges u -> x from u in bucket j
                const unsigned long long kx = push ? key[x] : 0ull;
                const uint32_t dx = (uint32_t)(kx >> 32);
                const float onem = 1.0f - __uint_as_float((uint32_t)kx);
                unsigned long long best = KINF;
                constexpr int NE = UNR * VW;
                for (uint32_t e = VW == 2 ? e0 & ~1u : e0; e < e1; e += UNR * LPT * VW) {
                    uint64_t wd[NE];
                    uint32_t ei[NE];
#pragma unroll
                    for (int q = 0; q < UNR; ++q) {
                        const uint32_t at = e + (sub + q * LPT) * VW;  // padded past the end
                        if (VW == 2) {
                            const uint4 r2 = *reinterpret_cast<const uint4 *>(ce + at);
                            wd[2 * q] = ((uint64_t)r2.y << 32) | r2.x;
                            wd[2 * q + 1] = ((uint64_t)r2.w << 32) | r2.z;
                            ei[2 * q] = at;
                            ei[2 * q + 1] = at + 1;
                        } else {
                            wd[q] = ce[at];
                            ei[q] = at;
                        }
                    }
                    uint32_t o[NE];
                    bool ok[NE];
#pragma unroll
                    for (int q = 0; q < NE; ++q) {
                        ok[q] = ei[q] < e1 && (VW == 1 || ei[q] >= e0);
                        o[q] = ok[q] ? (uint32_t)(wd[q] & vmask) : 0u;
                    }
                    unsigned long long ko[NE];
#pragma unroll
                    for (int q = 0; q < NE; ++q) ko[q] = key[o[q]];
#pragma unroll
                    for (int q = 0; q < NE; ++q) {
                        visits += ok[q];
                        const uint32_t w = cbase + (uint32_t)((wd[q] >> vb) & rmask);
                        const float r = __uint_as_float((uint32_t)(wd[q] >> 34));
                        if (push) {
                            const uint32_t d = dx + w;
                            const unsigned long long ck =
                                ((unsigned long long)d << 32) | __float_as_uint(1.0f - __fmul_rn(onem, r));
                            if (ok[q] && d <= dcap && ck < ko[q]) atomicMin(&key[o[q]], ck);
                        } else {
                            const uint32_t du = (uint32_t)(ko[q] >> 32), d = du + w;
                            // tail in bucket j (an unreached tail's ~0 is past every bucket)
                            if (ok[q] && du >= jlo && du < jhi && d <= dcap) {
                                const float lu = __uint_as_float((uint32_t)ko[q]);
                                const unsigned long long ck =
                                    ((unsigned long long)d << 32) | __float_as_uint(1.0f - __fmul_rn(1.0f - lu, r));
                                best = ck < best ? ck : best;
                            }
                        }
                    }
                }
                if (!push && best != KINF) atomicMin(&key[x], best);
            }
            __syncthreads();  // every key of bucket b final
            // N_b (the keys now in bucket b) -> mem[settled, ...)
            for (uint32_t base = 0; base < V; base += nt) {
                const uint32_t v = base + tid;
                const unsigned long long kv = v < V ? key[v] : KINF;
                const uint32_t dv = (uint32_t)(kv >> 32);
                const bool f = kv != KINF && dv >= lo && dv < hi;
                const uint64_t m = __ballot(f);
                if (!m) continue;  // uniform
                uint32_t o = 0;
                if (lane == 0) o = atomicAdd(&cur[par][1], (uint32_t)__popcll(m));
                o = __shfl(o, 0);
                if (f) mem[settled + o + (uint32_t)__popcll(m & below)] = (uint16_t)v;
            }
            __syncthreads();
            const uint32_t got = cur[par][1];
            // no tail in buckets b - WCN .. b and bucket b empty: every later
            // bucket is empty (uniform)
            if (!T && !got) break;
            settled += got;
            if (tid == 0) hist[b] = settled;
        }
        __syncthreads();  // keys final for the output
        if (probe) {
            uint32_t rmax = 0;
            for (uint32_t j0 = tid; j0 < n; j0 += nt) {
                const unsigned long long kv = key[nodes[j0]];
                const uint32_t l = kv == KINF ? ~0u : (uint32_t)(kv >> 32);
                rmax = l > rmax ? l : rmax;
            }
            for (int off = 32; off > 0; off >>= 1) {
                const uint32_t o = __shfl_xor(rmax, off);
                rmax = o > rmax ? o : rmax;
            }
            if (lane == 0) red_max[wv] = rmax;
            __syncthreads();
            if (tid == 0) {
                uint32_t m = 0;
                for (int q = 0; q < nw; ++q) m = red_max[q] > m ? red_max[q] : m;
                probe[2 + k] = m;
            }
            __syncthreads();
            continue;
        }
        uint64_t *ol = out_lat + (uint64_t)i * n;
        float *op = out_loss + (uint64_t)i * n;
        uint32_t *o32 = stage_mode == 2 ? reinterpret_cast<uint32_t *>(stage) + (uint64_t)k * n : nullptr;
        float *o32p = stage_mode == 2 ? stage_loss + (uint64_t)k * n : nullptr;
        uint2 *orec = stage_mode == 3 ? reinterpret_cast<uint2 *>(stage) + (uint64_t)k * n : nullptr;
        for (uint32_t j0 = tid; j0 < n; j0 += 4 * nt) {
            uint32_t vv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = j0 + q * nt < n ? nodes[j0 + q * nt] : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = j0 + q * nt;
                if (j >= n) break;
                uint64_t latv, lu;
                float lossv;
                if (j == i) {
                    latv = sl_lat[j];
                    lossv = sl_loss[j];
                    lu = latv == ~0ull ? ~0ull : latv / g;
                } else {
                    const unsigned long long kv = key[vv[q]];
                    if (kv == KINF) {
                        ++unreach;
                        latv = lu = ~0ull;
                        lossv = 1.0f;
                    } else {
                        lu = kv >> 32;
                        latv = lu * g;
                        lossv = __uint_as_float((uint32_t)kv);
                    }
                }
                // a staged self-loop past the u32 field saturates; the
                // consumers rewrite the diagonal from the host's self-loops
                const uint32_t l32 = lu >= 0xffffffffull ? ~0u : (uint32_t)lu;
                if (orec) {
                    __builtin_nontemporal_store(((uint64_t)__float_as_uint(lossv) << 32) | l32,
                                                reinterpret_cast<uint64_t *>(orec) + j);
                } else if (o32) {
                    __builtin_nontemporal_store(l32, o32 + j);
                    __builtin_nontemporal_store(lossv, o32p + j);
                } else if (NT) {
                    __builtin_nontemporal_store(latv, ol + j);
                    __builtin_nontemporal_store(lossv, op + j);
                } else {
                    ol[j] = latv;
                    op[j] = lossv;
                }
                mn = latv < mn ? latv : mn;
            }
        }
        __syncthreads();  // the next row rewrites the LDS keys and the scratch
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(mn, off);
        mn = o < mn ? o : mn;
        unreach += __shfl_xor(unreach, off);
        visits += __shfl_xor(visits, off);
    }
    if (lane == 0) {
        red_min[wv] = mn;
        red_cnt[wv] = unreach;
        red_vis[wv] = visits;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long m = red_min[0], c = red_cnt[0], vz = red_vis[0];
        for (int q = 1; q < nw; ++q) {
            m = red_min[q] < m ? red_min[q] : m;
            c += red_cnt[q];
            vz += red_vis[q];
        }
        if (probe) {
            if (vz) atomicAdd(reinterpret_cast<unsigned long long *>(probe), vz);
        } else {
            atomicMin(&stats[0], m);
            if (c) atomicAdd(&stats[1], c);
            if (visit_cnt && vz) atomicAdd(visit_cnt, vz);
        }
    }
}

// The shortest non-self-loop edge latency (ns) min-ed into *out: one wave per
// adjacency row; the column is read only where the latency would lower the
// lane's minimum (the quantized level solve's bucket width)
__global__ __launch_bounds__(256) void edge_min_kernel(uint32_t V, const uint64_t *__restrict__ row_ptr,
                                                       const uint32_t *__restrict__ col,
                                                       const uint64_t *__restrict__ lat, unsigned long long *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    uint64_t m = ~0ull;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            const uint64_t l = lat[k];
            if (l < m && col[k] != u) m = l;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(m, off);
        m = o < m ? o : m;
    }
    if (lane == 0 && m != ~0ull) atomicMin(out, (unsigned long long)m);
}

__global__ void loss_stats_init_kernel(unsigned long long *stats, unsigned long long *maxw) {
    stats[0] = ~0ull;
    stats[1] = 0ull;
    *maxw = 0ull;
}

// the level build's per-run counters in one launch (small memsets are a
// ~4.6 us fill kernel each on the device timeline): stats, the class max,
// the visit count; or (stats == nullptr) the class-CSR pass's cursor and max
__global__ void level_zero_kernel(unsigned long long *stats, unsigned long long *a, unsigned long long *b) {
    if (stats) {
        stats[0] = ~0ull;
        stats[1] = 0ull;
    }
    if (a) *a = 0ull;
    if (b) *b = 0ull;
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

// rows: [row0, row1) of the table, or the sharded tail's row list (RowJob)
struct RowJob {
    const uint32_t *list = nullptr;  // device, count entries
    uint32_t count = 0;
    bool range = false;              // no list: table rows [r0, r1) instead of [row0, row1)
    uint32_t r0 = 0, r1 = 0;
    void *out32 = nullptr;           // staging row 0 (u16 or u32 latency units, see srt_plan::stage16)
    float *out32_loss = nullptr;
};

template <typename LatT, bool LROWS, int LPT, bool PACKED, bool PUSH>
srt_status launch_fold(srt_plan *p, unsigned long long *d_stats, uint32_t ubits, const RowJob &job, srt_err *err) {
    const uint32_t V = p->V, rows = job.list ? job.count : job.range ? job.r1 - job.r0 : p->row1 - p->row0;
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
    auto kern = tight_loss_kernel<LatT, LROWS, LPT, PACKED, PUSH>;
    // set on every launch (cheap): a once-per-process flag would miss a
    // second device and race between plans built concurrently
    if (LROWS)
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(LDS_BUDGET - 4096));
    if (rows)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, p->stream, (const void *)p->d_D, p->key_type, p->Vp, V,
                           p->d_nodes, p->n, job.list ? 0u : job.range ? job.r0 : p->row0,
                           job.list ? job.count : job.range ? job.r1 : p->row1, p->d_tptr, p->d_tu,
                           reinterpret_cast<const LatT *>(p->d_tw), p->d_teb, p->d_tpk, ubits, p->kp.g, p->d_sl_lat,
                           p->d_sl_loss, p->d_out_lat, p->d_out_loss, d_stats, ord, lat_all, loss_all, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, job.list, job.out32, job.out32_loss, p->stage16);
    return SRT_OK;
}

template <typename LatT, bool LROWS, bool PACKED>
srt_status launch_fold_lpt(srt_plan *p, unsigned long long *d_stats, uint32_t ubits, const RowJob &job,
                           srt_err *err) {
    // lanes per target ~ the average tight in-degree (a group walks a target's
    // in-edges 2-4 per lane per step)
    const double avg = p->V ? (double)p->t_edges / p->V : 0.0;
    if constexpr (PACKED) {
        if (p->t_push) {
            if (avg > 10.0) return launch_fold<LatT, LROWS, 4, true, true>(p, d_stats, ubits, job, err);
            return launch_fold<LatT, LROWS, 2, true, true>(p, d_stats, ubits, job, err);
        }
        // 4 lanes x 8 edges per target (C3, same box: 4 / 8 / 16 lanes ->
        // 31.9 / 33.0 / 36.5 ms for the pass)
        if (avg > 10.0) return launch_fold<LatT, LROWS, 4, PACKED, false>(p, d_stats, ubits, job, err);
        return launch_fold<LatT, LROWS, 2, PACKED, false>(p, d_stats, ubits, job, err);
    }
    if (avg > 48.0) return launch_fold<LatT, LROWS, 32, PACKED, false>(p, d_stats, ubits, job, err);
    if (avg > 10.0) return launch_fold<LatT, LROWS, 8, PACKED, false>(p, d_stats, ubits, job, err);
    return launch_fold<LatT, LROWS, 2, PACKED, false>(p, d_stats, ubits, job, err);
}

// tight edge arrays for p->t_edges entries (grown together, 25% headroom;
// +1024: the packed scan reads up to (UNR - 1) * LPT entries past a row's end)
srt_status ensure_edge_arrays(srt_plan *p, srt_err *err) {
    if (p->t_edges + 1024 <= p->t_cap && p->d_tu) return SRT_OK;
    const size_t wsz = p->kp.lat32 ? 4 : 8;
    const uint64_t cap = std::max<uint64_t>(p->t_edges + p->t_edges / 4 + 1024, 2048);
    for (void *q : {(void *)p->d_tu, p->d_tw, (void *)p->d_teb, (void *)p->d_tpk, (void *)p->d_tpk2}) (void)hipFree(q);
    p->d_tu = nullptr;
    p->d_tw = nullptr;
    p->d_teb = nullptr;
    p->d_tpk = p->d_tpk2 = nullptr;
    p->t_cap = 0;
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr, *f = nullptr;
    hipError_t e = hipMalloc(&a, cap * 4);
    if (e == hipSuccess) e = hipMalloc(&b, cap * wsz);
    if (e == hipSuccess) e = hipMalloc(&c, cap * 4);
    if (e == hipSuccess) e = hipMalloc(&d, cap * 8);
    if (e == hipSuccess) e = hipMalloc(&f, cap * 8);
    if (e != hipSuccess) {
        for (void *q : {a, b, c, d, f}) (void)hipFree(q);
        return fail(err, e, "hipMalloc(tight edges)");
    }
    p->d_tu = (uint32_t *)a;
    p->d_tw = b;
    p->d_teb = (float *)c;
    p->d_tpk = (uint64_t *)d;
    p->d_tpk2 = (uint64_t *)f;
    p->t_cap = cap;
    return SRT_OK;
}

// packed entries d_tpk2 (rows by d_tptr) -> d_tpk, every target's row sorted
// by w (bits ubits .. of the low word)
srt_status sort_packed(srt_plan *p, uint32_t ubits, uint64_t maxw, srt_err *err) {
    const unsigned end_bit = ubits + (unsigned)std::max(1, bits_of(maxw));
    size_t need = 0;
    hipError_t e = rocprim::segmented_radix_sort_keys(nullptr, need, p->d_tpk2, p->d_tpk, (unsigned)p->t_edges, p->V,
                                                      p->d_tptr, p->d_tptr + 1, ubits, end_bit, p->stream);
    if (e != hipSuccess) return fail(err, e, "segmented sort (size)");
    uint64_t tcap = p->tsort_tmp_cap;
    srt_status st = grow(reinterpret_cast<uint8_t **>(&p->d_tsort_tmp), &tcap, need + 256, err, "hipMalloc(sort scratch)");
    p->tsort_tmp_cap = tcap;
    if (st != SRT_OK) return st;
    size_t have = p->tsort_tmp_cap;
    e = rocprim::segmented_radix_sort_keys(p->d_tsort_tmp, have, p->d_tpk2, p->d_tpk, (unsigned)p->t_edges, p->V,
                                           p->d_tptr, p->d_tptr + 1, ubits, end_bit, p->stream);
    if (e != hipSuccess) return fail(err, e, "segmented sort");
    return SRT_OK;
}

// The tight-edge list buffer holds p->tlist_cap uint4 slots in every path
// (one GPU: the whole list; sharded and emulated: W per-rank chunks of C
// slots).  Grow to `cap` slots when fewer than `need` are allocated.
static srt_status ensure_tlist(srt_plan *p, uint64_t cap, uint64_t need, srt_err *err) {
    if (p->d_tlist && need <= p->tlist_cap) return SRT_OK;
    (void)hipFree(p->d_tlist);
    p->d_tlist = nullptr;
    p->tlist_cap = 0;
    hipError_t e = hipMalloc(&p->d_tlist, cap * sizeof(uint4));
    if (e != hipSuccess) return fail(err, e, "hipMalloc(tight list)");
    p->tlist_cap = cap;
    return SRT_OK;
}

// The level fold applies (see level_loss_kernel): every tight weight <= WC,
// every closure latency < NBK units, u16 member lists, the row in LDS.
// Returns the fold's level width q in units of g: 1 (exact levels) when every
// tight weight is its own class (w <= WC) and every closure latency < NBK;
// else, when the smallest tight weight minw is known (one-GPU tight pass),
// quantized levels floor(L / q) with q = minw: a tight edge then climbs at
// least one level, its class floor(w / q) <= WC places its tail in one of two
// levels, and an exact test L(s,u) + w == L(s,v) on the closure row picks the
// candidates (C3 with ns latencies: g = 1 ns, tight weights 1.0-16 ms).  0: no.
uint32_t level_q(const srt_plan *p, uint64_t maxw, uint64_t minw) {
    if (const char *e = std::getenv("SRT_LOSS_LEVEL"))  // A/B and parity tests of the scan folds
        if (std::atoi(e) == 0) return 0;
    const size_t lds = HIST_BYTES + (((size_t)p->V * 2 + 15) & ~(size_t)15) + (size_t)p->V * 4 + (size_t)p->V * 2;
    if (!(p->kp.lat32 && p->V < 65536 && lds + 16 <= LDS_BUDGET - 4096 && maxw >= 1)) return 0;
    if (maxw <= WC && p->kp.lmax < (uint64_t)NBK) return 1;
    if (minw >= 2 && minw <= maxw && maxw / minw <= WC && p->kp.lmax / minw < (uint64_t)NBK - 1 &&
        minw < (1ull << 32) && (p->key_type == srt::KEY_U16 || p->key_type == srt::KEY_U32) &&
        !std::getenv("SRT_LOSS_NOQ"))
        return (uint32_t)minw;
    return 0;
}

// The class CSRs of the list's slots (records {v, u, w, 1-e bits}, v = ~0:
// padding) at level width p->t_q: out-rows in d_tpk, in-rows in d_tpk2,
// grouped by (vertex, class floor(w / q)) -- no sort.
srt_status build_class_csr(srt_plan *p, uint64_t slots, uint64_t maxw, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    srt_status st;
    const uint32_t lblocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (slots + 255) / 256));
    const uint32_t q = p->t_q;
    if (q > 1 && p->tcw_cap < 2 * p->t_cap) {  // the exact weights beside the class entries
        (void)hipFree(p->d_tcw);
        p->d_tcw = nullptr;
        p->tcw_cap = 0;
        const hipError_t e = hipMalloc(&p->d_tcw, 2 * p->t_cap * sizeof(uint32_t));
        if (e != hipSuccess) return fail(err, e, "hipMalloc(class weights)");
        p->tcw_cap = 2 * p->t_cap;
    }
    const uint32_t mc = q == 1 ? (uint32_t)maxw : (uint32_t)(maxw / q);  // the largest class
    p->t_cls = mc < 16 ? 16 : 32;
    const uint32_t cls = p->t_cls;
    const uint64_t vc1 = (uint64_t)V * cls + 1;
    uint64_t c1 = p->tcls_cap, c2 = p->tcls_cap;
    if ((st = grow(&p->d_tcls, &c1, 2 * vc1, err, "hipMalloc(class offsets)")) != SRT_OK ||
        (st = grow(&p->d_tccnt, &c2, 2 * vc1, err, "hipMalloc(class counts)")) != SRT_OK)
        return st;
    p->tcls_cap = std::min(c1, c2);
    (void)hipMemsetAsync(p->d_tccnt, 0, 2 * vc1 * 4, M);
    hipLaunchKernelGGL(tcls_count_kernel, dim3(lblocks), dim3(256), 0, M, p->d_tlist, slots, p->d_tccnt, vc1, q,
                       cls);
    size_t need = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, need, p->d_tccnt, p->d_tcls, 0u, (size_t)vc1,
                                           rocprim::plus<uint32_t>(), M);
    if (e != hipSuccess) return fail(err, e, "class scan (size)");
    uint64_t tcap = p->tscan_tmp_cap;
    if ((st = grow(reinterpret_cast<uint8_t **>(&p->d_tscan_tmp), &tcap, need + 256, err,
                   "hipMalloc(scan scratch)")) != SRT_OK)
        return st;
    p->tscan_tmp_cap = tcap;
    for (int d = 0; d < 2; ++d) {
        size_t have = p->tscan_tmp_cap;
        e = rocprim::exclusive_scan(p->d_tscan_tmp, have, p->d_tccnt + d * vc1, p->d_tcls + d * vc1, 0u,
                                    (size_t)vc1, rocprim::plus<uint32_t>(), M);
        if (e != hipSuccess) return fail(err, e, "class scan");
    }
    (void)hipMemsetAsync(p->d_tccnt, 0, 2 * vc1 * 4, M);
    hipLaunchKernelGGL(tcls_fill_kernel, dim3(lblocks), dim3(256), 0, M, p->d_tlist, slots, p->d_tcls,
                       p->d_tccnt, p->d_tpk, p->d_tpk2, vc1, q, q > 1 ? p->d_tcw : nullptr, p->t_cap, cls);
    p->t_push = false;
    return SRT_OK;
}

// Rows of the tight-edge list (slots records, v = ~0: padding, p->t_edges
// real ones): the class CSRs when the level fold applies (no sort), else the
// packed push (rows by source) or pull rows sorted by w.
srt_status build_tight_rows(srt_plan *p, uint64_t slots, uint32_t ubits, uint64_t maxw, srt_err *err,
                            uint64_t minw = 0) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    const uint32_t lblocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192, (slots + 255) / 256));
    p->t_q = level_q(p, maxw, minw);
    p->t_level = p->t_q != 0;
    if (p->t_level) return build_class_csr(p, slots, maxw, err);
    (void)hipMemsetAsync(p->d_tcnt, 0, (size_t)V * 4, M);
    // push form: CSR over tight OUT-edges (the pull form over in-edges
    // measured slower and was removed)
    hipLaunchKernelGGL(tight_list_count_kernel<true>, dim3(lblocks), dim3(256), 0, M, p->d_tlist, slots, p->d_tcnt, V);
    hipLaunchKernelGGL(tight_scan_kernel, dim3(1), dim3(1024), 0, M, p->d_tcnt, p->d_tptr, V);
    hipLaunchKernelGGL(tight_list_fill_kernel<true>, dim3(lblocks), dim3(256), 0, M, p->d_tlist, slots, p->d_tptr,
                       p->d_tcnt, p->d_tpk2, ubits, V);
    p->t_push = true;
    return sort_packed(p, ubits, maxw, err);
}

template <int LPT>
srt_status launch_level(srt_plan *p, unsigned long long *d_stats, const RowJob &job) {
    const uint32_t V = p->V, rows = job.list ? job.count : job.range ? job.r1 - job.r0 : p->row1 - p->row0;
    if (!rows) return SRT_OK;
    const size_t lds = HIST_BYTES + (((size_t)V * 2 + 15) & ~(size_t)15) + (size_t)V * 4 + (size_t)V * 2;
    const uint32_t nt = V >= 2048 ? LOSS_NT : 256;
    const int per_cu = std::max(1, std::min(2048 / (int)nt, (int)std::max<size_t>(1, (160 * 1024) / (lds + 2048))));
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(rows, (uint32_t)(cu_count(p->device) * per_cu)));
    // exact forms: loads of 2 entries (16 B), 4 in flight a lane with 16
    // classes (C3 loss pass 6.5 -> 6.2 ms vs 8 single entries; 6 pairs 6.8,
    // 2 lanes an item 7.2), 2 with 32 (C2 ~2% faster than 4 single entries);
    // quantized: 3 (16 classes) or 2 (32) single entries (the exact weights
    // beside them leave no registers for pairs)
    auto kern = p->t_cls == 16 ? (p->t_q > 1 ? level_loss_kernel<LPT, 3, true, 16, 1> : level_loss_kernel<LPT, 4, false, 16, 2>)
                               : (p->t_q > 1 ? level_loss_kernel<LPT, 2, true, 32, 1> : level_loss_kernel<LPT, 2, false, 32, 2>);
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(LDS_BUDGET - 4096));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, p->stream, (const void *)p->d_D, p->key_type, p->Vp, V,
                       p->d_nodes, p->n, job.list ? 0u : job.range ? job.r0 : p->row0,
                       job.list ? job.count : job.range ? job.r1 : p->row1, p->d_tcls, (uint64_t)V * p->t_cls + 1,
                       p->d_tpk, p->d_tpk2, p->kp.g, p->d_sl_lat, p->d_sl_loss, p->d_out_lat, p->d_out_loss, d_stats,
                       job.list, job.out32, job.out32_loss, p->stage16, p->t_q, p->d_tcw, p->t_cap);
#if LOSS_COUNT
    {  // diagnostic builds (-DLOSS_COUNT=1): totals of every level fold so far
        unsigned long long c[9];
        (void)hipStreamSynchronize(p->stream);
        (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(loss_cnt), sizeof c);
        std::fprintf(stderr,
                     "[srt] level fold: items %llu visits %llu hits %llu (push %llu) levels %llu rows %u; us per row: "
                     "load %.2f sort %.2f levels %.2f out %.2f\n",
                     c[0], c[1], c[2], c[8], c[3], rows, c[4] * 0.01 / rows, c[5] * 0.01 / rows, c[6] * 0.01 / rows,
                     c[7] * 0.01 / rows);
    }
#endif
    return SRT_OK;
}

// Push-form tight CSR on one GPU: the flagged adjacency entries compacted
// per source row (tight_list_kernel), then rows by source u, packed with v and
// sorted by w.  *done = false: not packable, the caller builds the pull form.
template <typename K>
srt_status tight_csr_push_t(srt_plan *p, unsigned long long *d_stats, bool *done, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    *done = false;
    srt_status st;
    uint64_t cap_info = p->d_tinfo ? 2 : 0, cap_cur = p->d_tcursor ? 1 : 0;
    if ((st = grow(&p->d_tinfo, &cap_info, 2, err, "hipMalloc(tight info)")) != SRT_OK ||
        (st = grow(&p->d_tcursor, &cap_cur, 1, err, "hipMalloc(tight cursor)")) != SRT_OK)
        return st;
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats, (unsigned long long *)p->d_tmaxw);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    // the list straight from the adjacency (tight_rows_kernel) into the list
    // the last run sized; a first run (or a larger count) counts, grows the
    // list and runs again
    auto rows = [&]() {
        (void)hipMemsetAsync(p->d_tinfo, 0, 2 * sizeof(unsigned long long), M);
        (void)hipMemsetAsync(p->d_tcursor, 0, sizeof(unsigned long long), M);
        hipLaunchKernelGGL(tight_rows_kernel<K>, dim3(blocks), dim3(256), 0, M, reinterpret_cast<const K *>(p->d_D),
                           p->Vp, V, p->d_row_ptr, p->d_col, p->d_lat, p->d_loss, p->kp.g, p->d_tlist,
                           p->d_tlist ? p->tlist_cap : 0ull, p->d_tcursor, (unsigned long long *)p->d_tmaxw,
                           p->d_tinfo);
        (void)hipMemcpyAsync(p->h_tcount, p->d_tinfo, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
        (void)hipMemcpyAsync(p->h_tcount + 1, p->d_tmaxw, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
        (void)hipMemcpyAsync(p->h_tcount + 2, p->d_tinfo + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
        return hipStreamSynchronize(M);
    };
    if (!p->d_tlist) {
        // a plan's first run (every end-to-end build): a list of n_adj / 32
        // records up front (C3: 8.4M slots for the 2.5M tight edges), so the
        // pass runs once; a larger count grows the list and runs again
        const uint64_t guess = std::max<uint64_t>(1ull << 16, p->n_adj / 32);
        if ((st = ensure_tlist(p, guess, guess, err)) != SRT_OK) return st;
    }
    hipError_t e = rows();
    if (e != hipSuccess) return fail(err, e, "tight-edge list");
    const uint64_t total = p->h_tcount[0], maxw = p->h_tcount[1];
    const uint64_t minw = total ? ~p->h_tcount[2] : 0;  // the kernel kept max(~w)
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    // the level fold's class CSRs need no packed (u, w) word: wide weights
    // (ns units) still fold by levels when level_q allows
    const bool packable = p->kp.lat32 && ubits + bits_of(maxw) <= 32 && total < (1ull << 32);
    if (!packable && !(total && level_q(p, maxw, minw))) return SRT_OK;
    p->t_edges = total;
    if ((st = ensure_edge_arrays(p, err)) != SRT_OK) return st;
    const uint64_t C = std::max<uint64_t>(total, 1);
    if (!p->d_tlist || total > p->tlist_cap) {
        if ((st = ensure_tlist(p, C + C / 4 + 64, C, err)) != SRT_OK) return st;
        if ((e = rows()) != hipSuccess) return fail(err, e, "tight-edge list");
    }
    if ((st = build_tight_rows(p, total, ubits, maxw, err, minw)) != SRT_OK) return st;
    if (std::getenv("SRT_TRACE"))
        std::fprintf(stderr, "[srt] tight edges %llu, w in [%llu, %llu] units, lmax %llu: %s fold, level width %u\n",
                     (unsigned long long)total, (unsigned long long)minw, (unsigned long long)maxw,
                     (unsigned long long)p->kp.lmax, p->t_level ? "level" : "scan", p->t_q);
    p->t_packed = packable;
    *done = true;
    return SRT_OK;
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
        const hipError_t e = hipHostMalloc((void **)&p->h_tcount, 4 * sizeof(uint64_t), 0);
        if (e != hipSuccess) return fail(err, e, "hipHostMalloc");
    }
    p->t_push = false;
    p->t_level = false;
    if (V && !std::getenv("SRT_LOSS_UNPACKED")) {
        bool done = false;
        if ((st = tight_csr_push_t<K>(p, d_stats, &done, err)) != SRT_OK || done) return st;
    }
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats,
                       (unsigned long long *)p->d_tmaxw);
    (void)hipMemsetAsync(p->d_tcnt, 0, (size_t)V * 4, M);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    p->h_tcount[0] = p->h_tcount[1] = 0;
    if (V) {
        hipLaunchKernelGGL(tight_flag_kernel<K>, dim3(blocks), dim3(256), 0, M, reinterpret_cast<const K *>(p->d_D),
                           p->Vp, 0u, V, p->d_row_ptr, p->d_col, p->d_lat, p->kp.g, p->d_tflag, p->d_tcnt,
                           (unsigned long long *)p->d_tmaxw, (unsigned long long *)nullptr);
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
    if ((st = ensure_edge_arrays(p, err)) != SRT_OK) return st;
    if (!V) return SRT_OK;
    if (p->t_packed) {
        hipLaunchKernelGGL((tight_fill_kernel<uint32_t, true>), dim3(blocks), dim3(256), 0, M, V, p->d_row_ptr,
                           p->d_col, p->d_lat, p->d_loss, p->kp.g, p->d_tflag, p->d_tptr, p->d_tcnt,
                           (uint32_t *)nullptr, (uint32_t *)nullptr, (float *)nullptr, p->d_tpk2, ubits);
        if ((st = sort_packed(p, ubits, maxw, err)) != SRT_OK) return st;
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

srt_status fold(srt_plan *p, unsigned long long *d_stats, const RowJob &job, srt_err *err) {
    const uint32_t V = p->V;
    if (p->t_level) {
        return launch_level<4>(p, d_stats, job);  // 4 lanes per class walk (2 and 8 measured slower)
    }
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    const bool lds_rows = HIST_BYTES + (size_t)V * 8 + 16 <= LDS_BUDGET - 4096;
    if (p->kp.lat32) {
        if (p->t_packed)
            return lds_rows ? launch_fold_lpt<uint32_t, true, true>(p, d_stats, ubits, job, err)
                            : launch_fold_lpt<uint32_t, false, true>(p, d_stats, ubits, job, err);
        return lds_rows ? launch_fold_lpt<uint32_t, true, false>(p, d_stats, 0, job, err)
                        : launch_fold_lpt<uint32_t, false, false>(p, d_stats, 0, job, err);
    }
    return launch_fold_lpt<uint64_t, false, false>(p, d_stats, 0, job, err);
}

// Sharded tail (comm bound): the tight edges of this rank's own adjacency
// rows (its closure block-rows, final locally), the (count, max latency) of
// every rank exchanged, then -- when the packed form applies -- the edge
// lists all-gathered and the full pull CSR built from them on every rank.
// *sharded = false: not packable, the caller falls back to the key
// all-gather and the replicated CSR.
template <typename K>
srt_status tight_csr_shard_t(srt_plan *p, unsigned long long *d_stats, bool *sharded, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, W = (uint32_t)p->comm->nranks, r = (uint32_t)p->comm->rank;
    const uint32_t u0 = (uint32_t)std::min<uint64_t>((uint64_t)p->rb0 * FW_B, V);
    const uint32_t u1 = (uint32_t)std::min<uint64_t>((uint64_t)p->rb1 * FW_B, V);
    *sharded = false;
    srt_status st;
    uint64_t cap_flag = p->d_tflag ? p->n_adj : 0, cap_cnt = p->d_tcnt ? V : 0, cap_ptr = p->d_tptr ? V + 1ull : 0,
             cap_mw = p->d_tmaxw ? 1 : 0, cap_info = p->d_tinfo ? 2ull * W : 0, cap_cur = p->d_tcursor ? 1 : 0;
    if ((st = grow(&p->d_tflag, &cap_flag, std::max<uint64_t>(p->n_adj, 1), err, "hipMalloc(tight flags)")) != SRT_OK ||
        (st = grow(&p->d_tcnt, &cap_cnt, std::max<uint64_t>(V, 1), err, "hipMalloc(tight counts)")) != SRT_OK ||
        (st = grow(&p->d_tptr, &cap_ptr, V + 1ull, err, "hipMalloc(tight ptr)")) != SRT_OK ||
        (st = grow(&p->d_tmaxw, &cap_mw, 1, err, "hipMalloc(tight max)")) != SRT_OK ||
        (st = grow(&p->d_tinfo, &cap_info, 2ull * W, err, "hipMalloc(tight info)")) != SRT_OK ||
        (st = grow(&p->d_tcursor, &cap_cur, 1, err, "hipMalloc(tight cursor)")) != SRT_OK)
        return st;
    if (!p->h_tinfo) {
        const hipError_t e = hipHostMalloc((void **)&p->h_tinfo, 2 * sizeof(unsigned long long) * W, 0);
        if (e != hipSuccess) return fail(err, e, "hipHostMalloc");
    }
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats, (unsigned long long *)p->d_tmaxw);
    (void)hipMemsetAsync(p->d_tinfo, 0, 2 * sizeof(unsigned long long) * W, M);
    (void)hipMemsetAsync(p->d_tcursor, 0, sizeof(unsigned long long), M);
    const uint32_t own_rows = u1 > u0 ? u1 - u0 : 0;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (own_rows + 3) / 4));
    if (own_rows)
        hipLaunchKernelGGL(tight_flag_kernel<K>, dim3(blocks), dim3(256), 0, M, reinterpret_cast<const K *>(p->d_D),
                           p->Vp, u0, u1, p->d_row_ptr, p->d_col, p->d_lat, p->kp.g, p->d_tflag, (uint32_t *)nullptr,
                           p->d_tinfo + 2 * r + 1, p->d_tinfo + 2 * r);
    if ((st = comm_allgather_inplace(p->comm, p->d_tinfo, 2 * sizeof(unsigned long long), M, err)) != SRT_OK)
        return st;
    (void)hipMemcpyAsync(p->h_tinfo, p->d_tinfo, 2 * sizeof(unsigned long long) * W, hipMemcpyDeviceToHost, M);
    hipError_t e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(err, e, "tight-edge count exchange");
    uint64_t total = 0, maxw = 0, C = 1;
    for (uint32_t q = 0; q < W; ++q) {
        total += p->h_tinfo[2 * q];
        maxw = std::max<uint64_t>(maxw, p->h_tinfo[2 * q + 1]);
        C = std::max<uint64_t>(C, p->h_tinfo[2 * q]);
    }
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    if (!(p->kp.lat32 && ubits + bits_of(maxw) <= 32 && total < (1ull << 32) && !std::getenv("SRT_LOSS_UNPACKED")))
        return SRT_OK;
    if ((st = ensure_tlist(p, (C + C / 4 + 64) * W, C * W, err)) != SRT_OK) return st;
    // own chunk: the records, then v = ~0 padding up to C
    (void)hipMemsetAsync(p->d_tlist + (uint64_t)r * C, 0xff, C * sizeof(uint4), M);
    if (own_rows)
        hipLaunchKernelGGL(tight_list_kernel, dim3(blocks), dim3(256), 0, M, u0, u1, p->d_row_ptr, p->d_col, p->d_lat,
                           p->d_loss, p->kp.g, p->d_tflag, p->d_tlist + (uint64_t)r * C, p->d_tcursor);
    if ((st = comm_allgather_inplace(p->comm, p->d_tlist, C * sizeof(uint4), M, err)) != SRT_OK) return st;
    p->t_edges = total;
    p->t_packed = true;
    if ((st = ensure_edge_arrays(p, err)) != SRT_OK) return st;
    if ((st = build_tight_rows(p, C * W, ubits, maxw, err)) != SRT_OK) return st;
    *sharded = true;
    return SRT_OK;
}

// staged slots [s0, s0 + slots) into the table, on the main stream
void expand_slots(srt_plan *p, size_t s0, uint32_t slots) {
    if (!slots || !p->n) return;
    const size_t lb = p->stage16 ? 2 : 4;
    hipLaunchKernelGGL(expand_rows_kernel, dim3(std::min<uint32_t>(slots, 4096)), dim3(256), 0, p->stream,
                       p->d_lrows + s0, slots, p->n,
                       (const void *)(reinterpret_cast<const uint8_t *>(p->d_slat) + s0 * p->n * lb), p->stage16,
                       p->d_sloss + s0 * p->n, p->kp.g, p->d_out_lat, p->d_out_loss,
                       p->stage_loss_only ? reinterpret_cast<const uint16_t *>(p->d_D) : nullptr, p->Vp, p->d_nodes,
                       p->d_sl_lat);
}

// chunk c of the staging into the table as soon as its all-gather is done
// (ev_tail[q + c]): the expansion of chunk c overlaps the all-gathers of the
// later chunks (emulated C3, 8 ranks: the 1.4 ms expansion was serial after
// the last all-gather)
void expand_chunks_behind(srt_plan *p, uint32_t W) {
    const uint32_t q = p->tail_q, cr = p->tail_cr;
    for (uint32_t c = 0; c < q; ++c) {
        (void)hipStreamWaitEvent(p->stream, p->ev_tail[q + c], 0);
        expand_slots(p, (size_t)c * W * cr, W * cr);
    }
    p->tail_expanded = true;
}

template <typename K>
srt_status loss_sharded_t(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    bool sharded = false;
    srt_status st = tight_csr_shard_t<K>(p, d_stats, &sharded, err);
    if (st != SRT_OK) return st;
    if (!sharded) {
        // replicated fallback: every rank's closure rows, then the CSR of all rows
        if ((st = fw_gather_keys(p, err)) != SRT_OK) return st;
        if ((st = tight_csr_t<K>(p, d_stats, err)) != SRT_OK) return st;
        return fold(p, d_stats, RowJob{}, err);
    }
    const uint32_t W = (uint32_t)p->comm->nranks, r = (uint32_t)p->comm->rank;
    const size_t chunk = (size_t)p->lrow_max * p->n;
    p->stage16 = p->key_type == KEY_U16;
    // every rank holds the whole closure: exchange the loss only (knob
    // SRT_TAIL_LAT=1 stages the latencies too, for A/B)
    p->stage_loss_only = p->fw_full_d && p->stage16;
    const size_t lb = p->stage16 ? 2 : 4;  // bytes per staged latency
    if (!p->d_slat) {
        void *a = nullptr, *b = nullptr;
        hipError_t e = hipMalloc(&a, std::max<size_t>(chunk * W, 1) * 4);
        if (e == hipSuccess) e = hipMalloc(&b, std::max<size_t>(chunk * W, 1) * 4);
        if (e != hipSuccess) {
            (void)hipFree(a);
            return fail(err, e, "hipMalloc(row staging)");
        }
        p->d_slat = (uint32_t *)a;
        p->d_sloss = (float *)b;
    }
    // the fold in tail_q chunks of tail_cr rows; chunk c's rows go to every
    // rank on the comm stream while chunk c + 1 folds (collectives stay in
    // one order on every rank: the chunks, then -- on M, after the last
    // chunk -- the rank stats)
    const uint32_t q = p->tail_q, cr = p->tail_cr;
    const size_t cbytes = (size_t)cr * p->n * 4, lbytes = (size_t)cr * p->n * lb;
    hipStream_t M = p->stream, C = p->comm_stream;
    for (uint32_t c = 0; c < q; ++c) {
        const size_t slot = ((size_t)c * W + r) * cr;
        RowJob job;
        job.list = p->d_lrows + slot;
        job.count = p->lrow_cnt[r] > c * cr ? std::min(cr, p->lrow_cnt[r] - c * cr) : 0u;
        job.out32 = p->stage_loss_only ? nullptr : reinterpret_cast<uint8_t *>(p->d_slat) + slot * p->n * lb;
        job.out32_loss = p->d_sloss + slot * p->n;
        if ((st = fold(p, d_stats, job, err)) != SRT_OK) return st;
        (void)hipEventRecord(p->ev_tail[c], M);
        (void)hipStreamWaitEvent(C, p->ev_tail[c], 0);
        const size_t base = (size_t)c * W * cr * p->n;
        if ((!p->stage_loss_only &&
             (st = comm_allgather_inplace(p->comm, reinterpret_cast<uint8_t *>(p->d_slat) + base * lb, lbytes, C,
                                          err)) != SRT_OK) ||
            (st = comm_allgather_inplace(p->comm, p->d_sloss + base, cbytes, C, err)) != SRT_OK)
            return st;
        (void)hipEventRecord(p->ev_tail[q + c], C);
    }
    expand_chunks_behind(p, W);
    p->shard_tail = true;
    return SRT_OK;
}

// Measurement only (SRT_FW_EMULATE_RANKS = N, no comm): wait `ticks` of the
// constant wall clock on the stream -- stands in for a collective
__global__ void emu_wait_kernel(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// Emulated rank 0 of an N-rank sharded tail, on the closure the first run
// left in D: the flags of its own adjacency rows, the list over every row
// (the other rows' flags are the closing run's, of the same D), the count /
// scan / fill / sort of the full list, the fold of its own rows into the
// staging.  The three all-gathers are waits of SRT_FW_EMU_AG_US (default 25)
// + received bytes / SRT_FW_EMU_AG_GBPS (default 300).
template <typename K>
srt_status loss_emulated_t(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, W = p->emulate_ranks;
    const uint32_t u1 = (uint32_t)std::min<uint64_t>((uint64_t)std::max<uint32_t>(1, p->Vp / FW_B / W) * FW_B, V);
    srt_status st;
    uint64_t cap_info = p->d_tinfo ? 2 : 0, cap_cur = p->d_tcursor ? 1 : 0;
    if ((st = grow(&p->d_tinfo, &cap_info, 2, err, "hipMalloc(tight info)")) != SRT_OK ||
        (st = grow(&p->d_tcursor, &cap_cur, 1, err, "hipMalloc(tight cursor)")) != SRT_OK)
        return st;
    if (!p->h_tinfo) {
        const hipError_t e = hipHostMalloc((void **)&p->h_tinfo, 2 * sizeof(unsigned long long), 0);
        if (e != hipSuccess) return fail(err, e, "hipHostMalloc");
    }
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device);
    const double lat_us = std::getenv("SRT_FW_EMU_AG_US") ? std::atof(std::getenv("SRT_FW_EMU_AG_US")) : 25.0;
    const double gbps = std::getenv("SRT_FW_EMU_AG_GBPS") ? std::atof(std::getenv("SRT_FW_EMU_AG_GBPS")) : 300.0;
    auto allgather_on = [&](double bytes_per_rank, hipStream_t s) {
        const double us = lat_us + bytes_per_rank * (W - 1) / (gbps * 1e3);
        hipLaunchKernelGGL(emu_wait_kernel, dim3(1), dim3(64), 0, s, (long long)(us * khz / 1000.0));
    };
    auto allgather = [&](double bytes_per_rank) { allgather_on(bytes_per_rank, M); };
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, M, d_stats, (unsigned long long *)p->d_tmaxw);
    (void)hipMemsetAsync(p->d_tinfo, 0, 2 * sizeof(unsigned long long), M);
    (void)hipMemsetAsync(p->d_tcursor, 0, sizeof(unsigned long long), M);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (u1 + 3) / 4));
    hipLaunchKernelGGL(tight_flag_kernel<K>, dim3(blocks), dim3(256), 0, M, reinterpret_cast<const K *>(p->d_D), p->Vp,
                       0u, u1, p->d_row_ptr, p->d_col, p->d_lat, p->kp.g, p->d_tflag, (uint32_t *)nullptr,
                       p->d_tinfo + 1, p->d_tinfo);
    allgather(16.0);
    (void)hipMemcpyAsync(p->h_tinfo, p->d_tinfo, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, M);
    hipError_t e = hipStreamSynchronize(M);
    if (e != hipSuccess) return fail(err, e, "tight-edge count");
    const uint64_t total = p->emu_tight, maxw = p->emu_maxw;
    const uint64_t C = std::max<uint64_t>({1, p->h_tinfo[0], (total + W - 1) / W});
    const uint32_t ubits = (uint32_t)std::max(1, bits_of(V ? V - 1 : 0));
    if (!(p->kp.lat32 && ubits + bits_of(maxw) <= 32 && total < (1ull << 32)))
        return fail(err, hipErrorNotSupported, "rank emulation needs the packed tight-edge form");
    const uint64_t slots = C * W;
    if ((st = ensure_tlist(p, slots, slots, err)) != SRT_OK) return st;
    (void)hipMemsetAsync(p->d_tlist, 0xff, slots * sizeof(uint4), M);
    const uint32_t vblocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    hipLaunchKernelGGL(tight_list_kernel, dim3(vblocks), dim3(256), 0, M, 0u, V, p->d_row_ptr, p->d_col, p->d_lat,
                       p->d_loss, p->kp.g, p->d_tflag, p->d_tlist, p->d_tcursor);
    allgather((double)C * sizeof(uint4));
    p->t_edges = total;
    p->t_packed = true;
    if ((st = ensure_edge_arrays(p, err)) != SRT_OK) return st;
    if ((st = build_tight_rows(p, slots, ubits, maxw, err)) != SRT_OK) return st;
    const size_t chunk = (size_t)p->lrow_max * p->n;
    p->stage16 = p->key_type == KEY_U16;
    p->stage_loss_only = p->fw_full_d && p->stage16;
    const size_t lb = p->stage_loss_only ? 0 : p->stage16 ? 2 : 4;  // bytes per staged latency
    if (!p->d_slat) {
        void *a = nullptr, *b = nullptr;
        e = hipMalloc(&a, std::max<size_t>(chunk * W, 1) * 4);
        if (e == hipSuccess) e = hipMalloc(&b, std::max<size_t>(chunk * W, 1) * 4);
        if (e != hipSuccess) {
            (void)hipFree(a);
            return fail(err, e, "hipMalloc(row staging)");
        }
        p->d_slat = (uint32_t *)a;
        p->d_sloss = (float *)b;
    }
    const uint32_t q = p->tail_q, cr = p->tail_cr;
    hipStream_t Cs = p->comm_stream;
    for (uint32_t c = 0; c < q; ++c) {
        const size_t slot = (size_t)c * W * cr;  // rank 0's slots of chunk c
        RowJob job;
        job.list = p->d_lrows + slot;
        job.count = p->lrow_cnt[0] > c * cr ? std::min(cr, p->lrow_cnt[0] - c * cr) : 0u;
        job.out32 = p->stage_loss_only ? nullptr : reinterpret_cast<uint8_t *>(p->d_slat) + slot * p->n * lb;
        job.out32_loss = p->d_sloss + slot * p->n;
        if ((st = fold(p, d_stats, job, err)) != SRT_OK) return st;
        (void)hipEventRecord(p->ev_tail[c], M);
        (void)hipStreamWaitEvent(Cs, p->ev_tail[c], 0);
        allgather_on((double)cr * p->n * (4.0 + lb), Cs);  // latency units + loss
        (void)hipEventRecord(p->ev_tail[q + c], Cs);
    }
    expand_chunks_behind(p, W);  // emulation: the others' slots are stale (same volume)
    allgather(16.0);  // rank stats
    p->shard_tail = true;
    return SRT_OK;
}

}  // namespace

LevelCtx level_ctx(srt_plan *p) {
    LevelCtx c;
    c.device = p->device;
    c.stream = p->stream;
    c.V = p->V;
    c.n = p->n;
    c.g = p->kp.g;
    c.t_cls = p->t_cls;
    c.tcls = p->d_tcls;
    c.ce_out = p->d_tpk;
    c.ce_in = p->lvl_single ? p->d_tpk : p->d_tpk2;
    c.nodes = p->d_nodes;
    c.sl_lat = p->d_sl_lat;
    c.sl_loss = p->d_sl_loss;
    c.out_lat = p->d_out_lat;
    c.out_loss = p->d_out_loss;
    c.visits = p->d_lvisit;
    c.q = p->lvl_q;
    c.rb = p->lvl_rb;
    c.vb = p->lvl_vb;
    c.lmem = p->d_lmem;
    c.idn = p->ident_nodes && p->n == p->V && p->n % 4 == 0;
    // rows dealt by a counter (knob SRT_LVL_DYN=0: statically, A/B)
    static const bool dyn = !(std::getenv("SRT_LVL_DYN") && std::atoi(std::getenv("SRT_LVL_DYN")) == 0);
    if (dyn && !p->d_rowctr) {
        if (hipMalloc(&p->d_rowctr, 2 * sizeof(unsigned long long)) != hipSuccess ||
            hipMemsetAsync(p->d_rowctr, 0, 2 * sizeof(unsigned long long), p->stream) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(p->d_rowctr);
            p->d_rowctr = nullptr;
        }
    }
    c.row_ctr = dyn ? p->d_rowctr : nullptr;
    return c;
}

uint32_t level_vbits(uint32_t V) {
    uint32_t vb = 1;
    while ((1u << vb) < V) ++vb;
    return vb;
}

namespace {
// ------------------------------------------------------------ level solve
// The class CSRs of the graph's edges of latency <= wmax units (self-loops
// dropped), classes = exact weights 1..wmax <= WC: out-rows straight from the
// adjacency (lvl_out_kernel), in-rows by a scan of their counts and one walk
// of the out-rows (lvl_in_kernel).  The entry arrays hold p->lvl_cap entries:
// the first call (the create-time probe, wmax = min(31, max edge)) counts,
// sizes them and runs again; every later call prunes at the probe's bound <=
// that wmax, so its count fits and nothing waits for the host.
srt_status level_csr(srt_plan *p, uint64_t wmax, bool with_loss, srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V;
    const uint32_t q = p->lvl_q, vb = q ? p->lvl_vb : 32u;
    const uint64_t ncls = q ? wmax / q : wmax;
    const uint32_t cls = ncls < 16 ? 16 : ncls < 32 ? 32 : 64;
    const uint64_t vc1 = (uint64_t)V * cls + 1;
    srt_status st;
    uint64_t c1 = p->tcls_cap, c2 = p->tcls_cap, cap_cur = p->d_tcursor ? 1 : 0, cap_mw = p->d_tmaxw ? 1 : 0;
    if ((st = grow(&p->d_tcls, &c1, 2 * vc1, err, "hipMalloc(class offsets)")) != SRT_OK ||
        (st = grow(&p->d_tccnt, &c2, 2 * vc1, err, "hipMalloc(class counts)")) != SRT_OK ||
        (st = grow(&p->d_tcursor, &cap_cur, 1, err, "hipMalloc(level cursor)")) != SRT_OK ||
        (st = grow(&p->d_tmaxw, &cap_mw, 1, err, "hipMalloc(level max)")) != SRT_OK)
        return st;
    p->tcls_cap = std::min(c1, c2);
    if (!p->h_tcount) {
        const hipError_t e = hipHostMalloc((void **)&p->h_tcount, 4 * sizeof(uint64_t), 0);
        if (e != hipSuccess) return fail(err, e, "hipHostMalloc");
    }
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (V + 3) / 4));
    const uint64_t wns = wmax * p->kp.g;
    const double inv_g = 1.0 / (double)p->kp.g;
    // symmetric plans (lvl_sym_tile_kernel: identity rows, mirrored pairs --
    // their losses too when the entries carry them): out-rows only
    const bool single = with_loss ? p->lvl_sym : p->lvl_sym_lat;
    p->lvl_single = single;
    auto out_pass = [&]() {
        if (!single)  // in-row counts, then in-row cursors (out-rows-only plans count none)
            (void)hipMemsetAsync(p->d_tccnt, 0, 2 * vc1 * 4, M);
        hipLaunchKernelGGL(level_zero_kernel, dim3(1), dim3(1), 0, M, (unsigned long long *)nullptr,
                           (unsigned long long *)p->d_tcursor, (unsigned long long *)p->d_tmaxw);
        if (single && p->d_lat16 && with_loss)  // the u16-unit copy (symmetry check; wmax < 0xffff units)
            hipLaunchKernelGGL((lvl_out_kernel<true, false, true, true>), dim3(blocks), dim3(256), 0, M, 0u, V,
                               p->d_row_ptr, p->d_col, p->d_lat, p->d_loss, p->kp.g, inv_g, wns, cls, q, vb, p->d_tcls,
                               p->d_tccnt, p->d_tpk, p->lvl_cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw,
                               p->d_lat16);
        else if (single && p->d_lat16)
            hipLaunchKernelGGL((lvl_out_kernel<false, false, true, true>), dim3(blocks), dim3(256), 0, M, 0u, V,
                               p->d_row_ptr, p->d_col, p->d_lat, (const float *)nullptr, p->kp.g, inv_g, wns, cls, q, vb,
                               p->d_tcls, p->d_tccnt, p->d_tpk, p->lvl_cap, p->d_tcursor,
                               (unsigned long long *)p->d_tmaxw, p->d_lat16);
        else if (single && with_loss)  // symmetric plans have identity rows (lvl_sym_tile_kernel)
            hipLaunchKernelGGL((lvl_out_kernel<true, false, true>), dim3(blocks), dim3(256), 0, M, 0u, V, p->d_row_ptr,
                               p->d_col, p->d_lat, p->d_loss, p->kp.g, inv_g, wns, cls, q, vb, p->d_tcls, p->d_tccnt,
                               p->d_tpk, p->lvl_cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw);
        else if (single)
            hipLaunchKernelGGL((lvl_out_kernel<false, false, true>), dim3(blocks), dim3(256), 0, M, 0u, V, p->d_row_ptr,
                               p->d_col, p->d_lat, (const float *)nullptr, p->kp.g, inv_g, wns, cls, q, vb, p->d_tcls,
                               p->d_tccnt, p->d_tpk, p->lvl_cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw);
        else if (with_loss)
            hipLaunchKernelGGL(lvl_out_kernel<true>, dim3(blocks), dim3(256), 0, M, 0u, V, p->d_row_ptr, p->d_col,
                               p->d_lat, p->d_loss, p->kp.g, inv_g, wns, cls, q, vb, p->d_tcls, p->d_tccnt,
                               p->d_tpk, p->lvl_cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw);
        else
            hipLaunchKernelGGL(lvl_out_kernel<false>, dim3(blocks), dim3(256), 0, M, 0u, V, p->d_row_ptr, p->d_col,
                               p->d_lat, (const float *)nullptr, p->kp.g, inv_g, wns, cls, q, vb, p->d_tcls,
                               p->d_tccnt, p->d_tpk, p->lvl_cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw);
    };
    // first call (the create-time probe): entry arrays of the caller's
    // estimate (p->lvl_est; +1024: the solve's 2-entry loads read up to UNR *
    // LPT * 2 entries past a class's end), one pass, the count read back; an
    // estimate too small (or none) sizes them by the count and runs again.
    // lvl_cap = the count: every later call prunes at a bound <= this wmax
    auto size_arrays = [&](uint64_t entries) -> srt_status {
        uint64_t ca = 0, cb = 0;
        (void)hipFree(p->d_tpk);
        (void)hipFree(p->d_tpk2);
        p->d_tpk = p->d_tpk2 = nullptr;
        p->t_cap = 0;
        srt_status s2;
        // symmetric plans read the in-rows through the out-rows: no second array
        // (allocated below when a later run needs in-rows after all)
        if ((s2 = grow(&p->d_tpk, &ca, entries + 1024, err, "hipMalloc(level out-rows)")) != SRT_OK ||
            (!single && (s2 = grow(&p->d_tpk2, &cb, entries + 1024, err, "hipMalloc(level in-rows)")) != SRT_OK))
            return s2;
        p->lvl_cap = entries;
        return SRT_OK;
    };
    const bool first = !p->lvl_cap;
    if (first && p->lvl_est && (st = size_arrays(p->lvl_est)) != SRT_OK) return st;
    cspan_begin(p);
    out_pass();
    cspan_end(p);
    if (first) {
        hipError_t e = hipMemcpyAsync(p->h_tcount, p->d_tcursor, sizeof(uint64_t), hipMemcpyDeviceToHost, M);
        if (e == hipSuccess) e = hipStreamSynchronize(M);
        if (e != hipSuccess) return fail(err, e, "level edge count");
        const uint64_t count = std::max<uint64_t>(p->h_tcount[0], 1);
        if (count > p->lvl_cap) {
            if ((st = size_arrays(count)) != SRT_OK) return st;
            cspan_begin(p);
            out_pass();
            cspan_end(p);
        }
        p->lvl_cap = count;
    }
    if (single) {
        // symmetric plan (lvl_sym_tile_kernel): the in-rows are the out-rows;
        // their offsets copied, the entries read through the same array
        // (level_ctx)
        cspan_begin(p);
        const hipError_t e = hipMemcpyAsync(p->d_tcls + vc1, p->d_tcls, vc1 * 4, hipMemcpyDeviceToDevice, M);
        cspan_end(p);
        if (e != hipSuccess) return fail(err, e, "class offsets (symmetric)");
        p->t_cls = cls;
        p->t_q = 1;
        p->t_level = true;
        p->t_edges = p->lvl_cap;
        return SRT_OK;
    }
    if (!p->d_tpk2) {  // a symmetric plan whose run needs in-rows (its losses did not mirror)
        uint64_t cb = 0;
        if ((st = grow(&p->d_tpk2, &cb, p->lvl_cap + 1024, err, "hipMalloc(level in-rows)")) != SRT_OK) return st;
    }
    size_t need = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, need, p->d_tccnt, p->d_tcls + vc1, 0u, (size_t)vc1,
                                           rocprim::plus<uint32_t>(), M);
    if (e != hipSuccess) return fail(err, e, "class scan (size)");
    uint64_t tcap = p->tscan_tmp_cap;
    if ((st = grow(reinterpret_cast<uint8_t **>(&p->d_tscan_tmp), &tcap, need + 256, err,
                   "hipMalloc(scan scratch)")) != SRT_OK)
        return st;
    p->tscan_tmp_cap = tcap;
    size_t have = p->tscan_tmp_cap;
    cspan_begin(p);
    e = rocprim::exclusive_scan(p->d_tscan_tmp, have, p->d_tccnt, p->d_tcls + vc1, 0u, (size_t)vc1,
                                rocprim::plus<uint32_t>(), M);
    if (e != hipSuccess) return fail(err, e, "class scan");
    const uint64_t vmask = q ? (1ull << vb) - 1ull : 0xffffffffull;
    hipLaunchKernelGGL(lvl_in_kernel, dim3(blocks), dim3(256), 0, M, V, cls, vmask, p->d_tcls, p->d_tpk,
                       p->d_tcls + vc1, p->d_tccnt + vc1, p->d_tpk2);
    cspan_end(p);
    p->t_cls = cls;
    p->t_q = 1;
    p->t_level = true;
    p->t_edges = p->lvl_cap;  // the probe's count (an upper bound at the run's smaller wmax)
    return SRT_OK;
}

__global__ void set_u64_kernel(unsigned long long *p, unsigned long long v) { *p = v; }

// The class CSR of a symmetric level plan (identity rows, mirrored pairs:
// out-rows only) built sharded over W ranks: the fixed per-graph work of a
// row-sharded build, which every rank paid whole before (C3: 0.63 ms of an
// 8-rank share of ~1.4 ms).  Rank r builds the out-rows of vertices [r vr,
// (r + 1) vr) into entry slot r (entries [r C, (r + 1) C), its cursor starting
// at r C, so the class offsets it writes are absolute) and its offsets into
// offset slot r; one all-gather of each (in place, C entries and vr * cls
// offsets a rank -- C3, 8 ranks: ~5 MB + 128 KB a rank) and every rank holds
// the whole class CSR.  C = the largest slice's entry count, measured once (a
// counting pass per slice and an all-gather of the counts) at the first run.
// comm == nullptr: the measurement form (srt_plan_shard_rows with
// SRT_LVL_SHARD_EMU=1, one GPU): the first run builds every slice, later runs
// rebuild the own slice only and wait out a modelled all-gather
// (SRT_FW_EMU_AG_US + received bytes / SRT_FW_EMU_AG_GBPS, as the FW emulation).
srt_status level_csr_sharded(srt_plan *p, uint64_t wmax, bool with_loss, uint32_t W, uint32_t r, srt_comm *comm,
                             srt_err *err) {
    hipStream_t M = p->stream;
    const uint32_t V = p->V, vr = (V + W - 1) / W;
    const uint32_t cls = wmax < 16 ? 16 : wmax < 32 ? 32 : 64;
    const uint64_t vc1 = (uint64_t)V * cls + 1;
    srt_status st;
    uint64_t c1 = p->tcls_cap, c2 = p->tcls_cap, cap_cur = p->d_tcursor ? 1 : 0, cap_mw = p->d_tmaxw ? 1 : 0,
             cap_cnt = p->d_lvl_counts ? W : 0;
    if ((st = grow(&p->d_tcls, &c1, 2 * vc1, err, "hipMalloc(class offsets)")) != SRT_OK ||
        (st = grow(&p->d_tccnt, &c2, 2 * vc1, err, "hipMalloc(class counts)")) != SRT_OK ||
        (st = grow(&p->d_tcursor, &cap_cur, 1, err, "hipMalloc(level cursor)")) != SRT_OK ||
        (st = grow(&p->d_tmaxw, &cap_mw, 1, err, "hipMalloc(level max)")) != SRT_OK ||
        (st = grow(&p->d_lvl_offstage, &p->lvl_offstage_cap, (uint64_t)W * vr * cls, err,
                   "hipMalloc(class offset slots)")) != SRT_OK ||
        (st = grow(&p->d_lvl_counts, &cap_cnt, W, err, "hipMalloc(slice counts)")) != SRT_OK)
        return st;
    p->tcls_cap = std::min(c1, c2);
    const double inv_g = 1.0 / (double)p->kp.g;
    const uint64_t wns = wmax * p->kp.g;
    auto slice = [&](uint32_t s, uint64_t base, uint64_t cap, uint64_t *entries) {
        const uint32_t u0 = std::min(V, s * vr), u1 = std::min(V, (s + 1) * vr);
        const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (u1 - u0 + 3) / 4));
        hipLaunchKernelGGL(set_u64_kernel, dim3(1), dim3(1), 0, M, p->d_tcursor, (unsigned long long)base);
        if (with_loss)
            hipLaunchKernelGGL((lvl_out_kernel<true, false, true>), dim3(blocks), dim3(256), 0, M, u0, u1, p->d_row_ptr,
                               p->d_col, p->d_lat, p->d_loss, p->kp.g, inv_g, wns, cls, 0u, 32u, p->d_lvl_offstage,
                               p->d_tccnt, entries, cap, p->d_tcursor, (unsigned long long *)p->d_tmaxw);
        else
            hipLaunchKernelGGL((lvl_out_kernel<false, false, true>), dim3(blocks), dim3(256), 0, M, u0, u1,
                               p->d_row_ptr, p->d_col, p->d_lat, (const float *)nullptr, p->kp.g, inv_g, wns, cls, 0u,
                               32u, p->d_lvl_offstage, p->d_tccnt, entries, cap, p->d_tcursor,
                               (unsigned long long *)p->d_tmaxw);
    };
    const bool emu = comm == nullptr;
    if (!p->lvl_seg_cap) {
        // sizing: every slice counted (cap 0: nothing written); the measured
        // form counts all W here, a rank its own and all-gathers the counts
        std::vector<unsigned long long> cnt(W, 0);
        for (uint32_t s = 0; s < W; ++s) {
            if (!emu && s != r) continue;
            slice(s, 0, 0, p->d_tpk);
            const hipError_t e = hipMemcpyAsync(p->d_lvl_counts + s, p->d_tcursor, 8, hipMemcpyDeviceToDevice, M);
            if (e != hipSuccess) return fail(err, e, "slice count");
        }
        if (!emu && (st = comm_allgather_inplace(comm, p->d_lvl_counts, 8, M, err)) != SRT_OK) return st;
        hipError_t e = hipMemcpyAsync(cnt.data(), p->d_lvl_counts, 8ull * W, hipMemcpyDeviceToHost, M);
        if (e == hipSuccess) e = hipStreamSynchronize(M);
        if (e != hipSuccess) return fail(err, e, "slice counts");
        uint64_t C = 1;
        for (uint32_t s = 0; s < W; ++s) C = std::max<uint64_t>(C, cnt[s]);
        (void)hipFree(p->d_tpk);
        (void)hipFree(p->d_tpk2);
        p->d_tpk = p->d_tpk2 = nullptr;
        uint64_t ca = 0;
        if ((st = grow(&p->d_tpk, &ca, C * W + 1024, err, "hipMalloc(level out-rows)")) != SRT_OK) return st;
        p->lvl_seg_cap = C;
        p->lvl_cap = C * W;
        p->lvl_emu_built = false;
    }
    const uint64_t C = p->lvl_seg_cap;
    cspan_begin(p);
    if (emu && !p->lvl_emu_built) {  // the measured form's first run: every rank's slice
        for (uint32_t s = 0; s < W; ++s) slice(s, s * C, (s + 1) * C, p->d_tpk);
        p->lvl_emu_built = true;
    } else {
        slice(r, (uint64_t)r * C, (uint64_t)(r + 1) * C, p->d_tpk);
        if (emu) {
            int khz = 100000;
            (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device);
            const double lat_us = std::getenv("SRT_FW_EMU_AG_US") ? std::atof(std::getenv("SRT_FW_EMU_AG_US")) : 25.0;
            const double gbps = std::getenv("SRT_FW_EMU_AG_GBPS") ? std::atof(std::getenv("SRT_FW_EMU_AG_GBPS")) : 300.0;
            const double bytes = (double)C * 8 + (double)vr * cls * 4;
            const double us = lat_us + bytes * (W - 1) / (gbps * 1e3);
            hipLaunchKernelGGL(emu_wait_kernel, dim3(1), dim3(64), 0, M, (long long)(us * khz / 1000.0));
        } else if ((st = comm_allgather_inplace(comm, p->d_tpk, C * 8, M, err)) != SRT_OK ||
                   (st = comm_allgather_inplace(comm, p->d_lvl_offstage, (uint64_t)vr * cls * 4, M, err)) != SRT_OK) {
            return st;
        }
    }
    // the offsets, out-rows and (symmetric) in-rows alike
    hipError_t e = hipMemcpyAsync(p->d_tcls, p->d_lvl_offstage, (uint64_t)V * cls * 4, hipMemcpyDeviceToDevice, M);
    if (e == hipSuccess)
        e = hipMemcpyAsync(p->d_tcls + vc1, p->d_lvl_offstage, (uint64_t)V * cls * 4, hipMemcpyDeviceToDevice, M);
    cspan_end(p);
    if (e != hipSuccess) return fail(err, e, "class offsets (sharded)");
    p->lvl_single = true;
    p->t_cls = cls;
    p->t_q = 1;
    p->t_level = true;
    p->t_edges = C * W;
    return SRT_OK;
}

// Workgroups of a level solve launch over `rows` rows (one row per
// workgroup at a time; the LDS row decides how many fit a CU)
uint32_t level_grid(int device, uint32_t V, bool quant, uint32_t rows, uint32_t *nt_out) {
    const size_t lds = quant ? SOLVE_HIST + (size_t)V * 8
                             : SOLVE_HIST + (((size_t)V * 2 + 15) & ~(size_t)15) + (size_t)V * 4 +
                                   (((size_t)V * 2 + 15) & ~(size_t)15);
    // workgroups a CU's LDS holds, then the fewest threads a workgroup (256,
    // 512 or 1024) that still fill the CU's 2,048 thread slots: more rows in
    // flight a CU for small graphs (C2, 4k: 4 x 512 threads 0.39 ms a solve
    // against 2 x 1024 0.50 ms; 4 x 256 0.39), one 1,024-thread workgroup for
    // C3's 128 KB rows
    const int lds_cu = (int)std::max<size_t>(1, (160 * 1024) / (lds + 2048));
    uint32_t nt = 256;
    while (nt < LOSS_NT && (int)(2048 / nt) > lds_cu) nt *= 2;
    const int per_cu = std::max(1, std::min(2048 / (int)nt, lds_cu));
    if (nt_out) *nt_out = nt;
    return std::max<uint32_t>(1, std::min<uint32_t>(rows, (uint32_t)(cu_count(device) * per_cu)));
}

// level_solve_kernel (or level_q_kernel, c.q > 0) over rows [r0, r1) (or the
// row list) of the context c (probe: no table, reverse = in- and out-CSRs
// swapped: distances TO the row's node); lcap = the bound B in units.
// stage_mode 0: the table; 1: u16 latency units + f32 loss staging, row k of
// the job at k * n; 2: u32 units + loss; 3: 8-byte records (quantized only)
void launch_solve_ctx(const LevelCtx &c, unsigned long long *d_stats, const uint32_t *list, uint32_t r0, uint32_t r1,
                      uint32_t lcap, bool reverse, uint32_t *probe, void *stage, float *stage_loss,
                      uint32_t stage_mode) {
    const uint32_t V = c.V, rows = list ? r1 : r1 - r0;
    if (!rows) return;
    const bool quant = c.q != 0;
    uint32_t nt = 0;
    const uint32_t grid = level_grid(c.device, V, quant, rows, &nt);
    const size_t lds = quant ? SOLVE_HIST + (size_t)V * 8
                             : SOLVE_HIST + (((size_t)V * 2 + 15) & ~(size_t)15) + (size_t)V * 4 +
                                   (((size_t)V * 2 + 15) & ~(size_t)15);
    // table rows by non-temporal stores (knob SRT_LVL_NT=0/1: A/B measurement)
    static const bool nts = !(std::getenv("SRT_LVL_NT") && std::atoi(std::getenv("SRT_LVL_NT")) == 0);
    const uint64_t vc1 = (uint64_t)V * c.t_cls + 1;
    const uint32_t *co = c.tcls, *ci = c.tcls + vc1;
    const uint64_t *eo = c.ce_out, *ei = c.ce_in;
    if (reverse) {
        std::swap(co, ci);
        std::swap(eo, ei);
    }
    if (quant) {
        auto kern = c.t_cls == 16   ? (nts ? level_q_kernel<4, 4, 16, 2, true> : level_q_kernel<4, 4, 16, 2, false>)
                    : c.t_cls == 32 ? (nts ? level_q_kernel<4, 2, 32, 2, true> : level_q_kernel<4, 2, 32, 2, false>)
                                    : (nts ? level_q_kernel<4, 2, 64, 2, true> : level_q_kernel<4, 2, 64, 2, false>);
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(LDS_BUDGET - 4096));
        const uint32_t kcap = std::min<uint32_t>(lcap / c.q, LWC);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, c.stream, V, c.nodes, c.n, list ? 0u : r0, r1, co, ci,
                           eo, ei, kcap, lcap, c.q, c.rb, c.vb, c.g, c.sl_lat, c.sl_loss, c.out_lat, c.out_loss, d_stats,
                           list, stage, stage_loss, stage_mode, probe, c.visits, c.lmem);
        return;
    }
    // knob SRT_LVL_SP=0: the per-item walk (A/B).  Measured at C3 (same box):
    // branch-free hits through a per-lane dummy word 4.83 ms, the same as the
    // pipelined walk; lane groups x pairs in flight 4x4 (kept) 4.79, 2x4 5.22,
    // 8x2 5.50, 4x2 5.57, 2x2 6.09 ms
    static const bool sp = !(std::getenv("SRT_LVL_SP") && std::atoi(std::getenv("SRT_LVL_SP")) == 0);
    auto kern =
        sp ? (c.t_cls == 16   ? (nts ? level_solve_kernel<4, 4, 16, 2, true, true>
                                     : level_solve_kernel<4, 4, 16, 2, false, true>)
              : c.t_cls == 32 ? (nts ? level_solve_kernel<4, 2, 32, 2, true, true>
                                     : level_solve_kernel<4, 2, 32, 2, false, true>)
                              : (nts ? level_solve_kernel<4, 2, 64, 2, true, true>
                                     : level_solve_kernel<4, 2, 64, 2, false, true>))
           : (c.t_cls == 16   ? (nts ? level_solve_kernel<4, 4, 16, 2, true> : level_solve_kernel<4, 4, 16, 2, false>)
              : c.t_cls == 32 ? (nts ? level_solve_kernel<4, 2, 32, 2, true> : level_solve_kernel<4, 2, 32, 2, false>)
                              : (nts ? level_solve_kernel<4, 2, 64, 2, true> : level_solve_kernel<4, 2, 64, 2, false>));
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(LDS_BUDGET - 4096));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), lds, c.stream, V, c.nodes, c.n, list ? 0u : r0, r1, co, ci, eo, ei,
                       lcap, c.g, c.sl_lat, c.sl_loss, c.out_lat, c.out_loss, d_stats, list,
                       stage_mode ? stage : nullptr, stage_mode ? stage_loss : nullptr, stage_mode == 1, probe,
                       c.visits, c.idn, c.row_ctr);
}

// the per-workgroup scratch of the quantized solve (p->d_lmem): every
// workgroup a launch may have, V u16 each
srt_status level_scratch(srt_plan *p, srt_err *err) {
    if (!p->lvl_q) return SRT_OK;
    const uint64_t need = (uint64_t)level_grid(p->device, p->V, true, ~0u, nullptr) * p->V;
    return grow(&p->d_lmem, &p->lmem_cap, need, err, "hipMalloc(level scratch)");
}

srt_status launch_solve(srt_plan *p, unsigned long long *d_stats, const RowJob &job, uint32_t lcap, bool reverse,
                        uint32_t *probe, srt_err *err) {
    srt_status st = level_scratch(p, err);
    if (st != SRT_OK) return st;
    const uint32_t r0 = job.list ? 0u : job.range ? job.r0 : p->row0;
    const uint32_t r1 = job.list ? job.count : job.range ? job.r1 : p->row1;
    launch_solve_ctx(level_ctx(p), d_stats, job.list, r0, r1, lcap, reverse, probe, job.out32_loss ? job.out32 : nullptr,
                     job.out32_loss, job.out32_loss ? (p->stage16 ? 1u : 2u) : 0u);
    return SRT_OK;
}

}  // namespace

// Create-time proof for the level solve: the pruned graph's (edges <= wmax
// units) distances from and to K <= 8 in-use nodes s, spread over the node
// list, by probe rows.  Every in-use u, v has d(u, v) <= d(u, s) + d(s, v) <=
// in-ecc(s) + out-ecc(s) for each s (pruned distances bound the real ones from
// above), so *bound = the smallest such sum; ~0 when every s misses an in-use
// node within wmax levels one way or the other.  *visits: the edges a
// forward probe row walked on average (the AUTO price).  p->lvl_q > 0: the
// quantized solve's buckets of q units; the bound must keep every class and
// bucket <= 31 (B < 32 q).
srt_status level_probe(srt_plan *p, uint64_t wmax, uint32_t wc, uint64_t *bound, uint64_t *visits, srt_err *err) {
    *bound = ~0ull;
    *visits = 0;
    if (!p->n) return SRT_OK;
    p->lvl_cap = 0;  // a new bound: count and size the entry arrays again
    // the estimate: latencies spread evenly up to the longest edge, twice over
    {
        const uint64_t maxu = p->lvl_maxu ? p->lvl_maxu : wmax;
        const double f = std::min(1.0, 2.0 * (double)wmax / (double)std::max<uint64_t>(maxu, 1));
        p->lvl_est = (uint64_t)((double)p->n_adj * f) + 65536;
    }
    srt_status st = level_csr(p, wmax, false, err);
    if (st != SRT_OK) return st;
    const uint32_t K = std::min<uint32_t>(8, p->n);
    uint32_t rows[8];
    for (uint32_t k = 0; k < K; ++k) rows[k] = (uint32_t)((uint64_t)k * p->n / K);
    uint32_t *d_pr = nullptr;
    hipError_t e = hipMalloc(&d_pr, 48 * sizeof(uint32_t));  // fwd [0, 16), rev [16, 32), rows [32, 40)
    if (e != hipSuccess) return fail(err, e, "hipMalloc(level probe)");
    uint32_t h[32] = {};
    (void)hipMemsetAsync(d_pr, 0, 32 * sizeof(uint32_t), p->stream);
    e = hipMemcpyAsync(d_pr + 32, rows, K * sizeof(uint32_t), hipMemcpyHostToDevice, p->stream);
    RowJob job;
    job.list = d_pr + 32;
    job.count = K;
    const uint64_t LQ = (uint64_t)(wc + 1) * (p->lvl_q ? p->lvl_q : 1) - 1;  // the largest bound the solve takes
    // distances up to LQ (not only up to wmax: a path of short edges may be
    // longer than the longest edge)
    const uint32_t cap = (uint32_t)LQ;
    if (e == hipSuccess) {
        cspan_begin(p);
        st = launch_solve(p, nullptr, job, cap, false, d_pr, err);
        if (st == SRT_OK) st = launch_solve(p, nullptr, job, cap, true, d_pr + 16, err);
        cspan_end(p);
        if (st != SRT_OK) {
            (void)hipStreamSynchronize(p->stream);
            (void)hipFree(d_pr);
            return st;
        }
        e = hipMemcpyAsync(h, d_pr, sizeof h, hipMemcpyDeviceToHost, p->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    (void)hipFree(d_pr);
    if (e != hipSuccess) return fail(err, e, "level probe");
    uint64_t vis = 0;
    std::memcpy(&vis, h, 8);
    *visits = vis / K;
    for (uint32_t k = 0; k < K; ++k)
        if (h[2 + k] <= cap && h[18 + k] <= cap && (uint64_t)h[2 + k] + h[18 + k] <= LQ)  // classes <= wc
            *bound = std::min<uint64_t>(*bound, (uint64_t)h[2 + k] + h[18 + k]);
    if (std::getenv("SRT_TRACE"))
        std::fprintf(stderr,
                     "[srt] level probe: %llu edges <= %llu units, q %u, %u rows, bound %lld, %llu visits a row\n",
                     (unsigned long long)p->t_edges, (unsigned long long)wmax, p->lvl_q, K,
                     *bound == ~0ull ? -1ll : (long long)*bound, (unsigned long long)*visits);
    return SRT_OK;
}

// The level solve's build (SRT_ALGO_LEVEL): the class CSRs of the edges <=
// kp.lmax units (the probe's bound), then the rows -- in chunks of
// fold_chunk_rows when the one-call build downloads behind them (ev_fold), as
// fw_loss's fold.  A sharded plan solves its own rows [row0, row1).
namespace {
// Sharded level solve (comm bound): this rank's rows (d_lrows, by
// build_loss_rows) solved in tail_q chunks into the staging as u16 latency
// units + f32 loss (6 B a pair, half the table's 12), chunk c's rows
// all-gathered on the comm stream behind chunk c + 1's solve and expanded into
// every rank's table behind its all-gather -- the sharded FW tail's pipeline
// with the solve in place of the fold.
srt_status level_sharded(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    const uint32_t W = (uint32_t)p->comm->nranks, r = (uint32_t)p->comm->rank;
    const size_t chunk = (size_t)p->lrow_max * p->n;
    p->stage16 = p->lvl_q == 0;  // quantized: u32 units
    p->stage_loss_only = false;
    if (!p->d_slat) {
        void *a = nullptr, *b = nullptr;
        hipError_t e = hipMalloc(&a, std::max<size_t>(chunk * W, 1) * 4);
        if (e == hipSuccess) e = hipMalloc(&b, std::max<size_t>(chunk * W, 1) * 4);
        if (e != hipSuccess) {
            (void)hipFree(a);
            return fail(err, e, "hipMalloc(row staging)");
        }
        p->d_slat = (uint32_t *)a;
        p->d_sloss = (float *)b;
    }
    const uint32_t q = p->tail_q, cr = p->tail_cr, lcap = (uint32_t)p->kp.lmax;
    const size_t cbytes = (size_t)cr * p->n * 4, lbytes = (size_t)cr * p->n * (p->stage16 ? 2 : 4);
    hipStream_t M = p->stream, C = p->comm_stream;
    while (p->ev.size() < 2 * (size_t)q) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence) != hipSuccess)
            return fail(err, hipErrorUnknown, "event");
        p->ev.push_back(e);
    }
    srt_status st;
    for (uint32_t c = 0; c < q; ++c) {
        const size_t slot = ((size_t)c * W + r) * cr;
        RowJob job;
        job.list = p->d_lrows + slot;
        job.count = p->lrow_cnt[r] > c * cr ? std::min(cr, p->lrow_cnt[r] - c * cr) : 0u;
        job.out32 = reinterpret_cast<uint8_t *>(p->d_slat) + slot * p->n * (p->stage16 ? 2 : 4);
        job.out32_loss = p->d_sloss + slot * p->n;
        (void)hipEventRecord(p->ev[2 * c], M);
        if ((st = launch_solve(p, d_stats, job, lcap, false, nullptr, err)) != SRT_OK) return st;
        (void)hipEventRecord(p->ev[2 * c + 1], M);
        p->p3_launches++;
        p->p3_work += (double)job.count * p->n;
        (void)hipEventRecord(p->ev_tail[c], M);
        (void)hipStreamWaitEvent(C, p->ev_tail[c], 0);
        const size_t base = (size_t)c * W * cr * p->n;
        if ((st = comm_allgather_inplace(p->comm,
                                         reinterpret_cast<uint8_t *>(p->d_slat) + base * (p->stage16 ? 2 : 4), lbytes, C,
                                         err)) != SRT_OK ||
            (st = comm_allgather_inplace(p->comm, p->d_sloss + base, cbytes, C, err)) != SRT_OK)
            return st;
        (void)hipEventRecord(p->ev_tail[q + c], C);
    }
    expand_chunks_behind(p, W);
    p->shard_tail = true;
    return SRT_OK;
}
}  // namespace

srt_status level_prepare(srt_plan *p, srt_err *err) { return level_csr(p, p->kp.lmax, true, err); }

void level_solve_stage(const LevelCtx &c, uint32_t r0, uint32_t r1, uint32_t lmax, void *stage_lat,
                       float *stage_loss, uint32_t stage_mode, unsigned long long *d_stats) {
    launch_solve_ctx(c, d_stats, nullptr, r0, r1, lmax, false, nullptr, stage_lat, stage_loss, stage_mode);
}

size_t level_scratch_bytes(int device, uint32_t V, bool quant) {
    return quant ? (size_t)level_grid(device, V, true, ~0u, nullptr) * V * 2 : 0;
}

void level_loss_index(srt_plan *p, uint32_t *d_idx, uint64_t cap, unsigned long long *d_cnt, hipStream_t s) {
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (p->V + 3) / 4));
    (void)hipMemsetAsync(d_cnt, 0, sizeof *d_cnt, s);
    // identity rows: the column is the entry's place in its row (no column loads)
    if (p->ident_rows)
        hipLaunchKernelGGL(lvl_index_kernel<true>, dim3(blocks), dim3(256), 0, s, p->V, p->d_row_ptr, p->d_col,
                           p->d_lat, p->kp.lmax * p->kp.g, d_idx, cap, d_cnt);
    else
        hipLaunchKernelGGL(lvl_index_kernel<false>, dim3(blocks), dim3(256), 0, s, p->V, p->d_row_ptr, p->d_col,
                           p->d_lat, p->kp.lmax * p->kp.g, d_idx, cap, d_cnt);
}

void loss_scatter(const uint32_t *d_idx, const float *d_val, uint64_t count, float *d_loss, hipStream_t s) {
    if (count)
        hipLaunchKernelGGL(loss_scatter_kernel, dim3((uint32_t)std::min<uint64_t>(4096, (count + 255) / 256)),
                           dim3(256), 0, s, d_idx, d_val, count, d_loss);
}

void loss_mirror_check(const uint32_t *d_idx, uint64_t count, uint64_t V, const float *d_loss, uint32_t *d_ok,
                       hipStream_t s) {
    if (count)
        hipLaunchKernelGGL(loss_mirror_check_kernel, dim3((uint32_t)std::min<uint64_t>(4096, (count + 255) / 256)),
                           dim3(256), 0, s, d_idx, count, V, d_loss, d_ok);
}

srt_status level_sym_check(srt_plan *p, uint64_t wmax_units, bool with_loss, bool *sym, srt_err *err) {
    *sym = false;
    if (!p->V || p->n_adj != (uint64_t)p->V * p->V || !p->ident_rows) return SRT_OK;
    uint32_t *d_ok = nullptr;
    hipError_t e = hipMalloc(&d_ok, 4);
    if (e != hipSuccess) return fail(err, e, "hipMalloc(symmetry flag)");
    uint32_t one = 1;
    e = hipMemcpyAsync(d_ok, &one, 4, hipMemcpyHostToDevice, p->stream);
    const uint64_t nb = (p->V + 63) / 64;
    // every latency below 0xffff units and rows of a multiple of 4 entries: the
    // check also writes the adjacency's u16-unit copy, which the class-CSR
    // passes stream instead of the u64 latencies (a quarter of the bytes; C3
    // 16k: out-rows 538 -> 309 us a build, the check 542 -> 854 us once).  From
    // 8,192 vertices: at C2's 4k it measured 0.01-0.02 ms slower a build
    const char *k16 = std::getenv("SRT_LAT16");  // knob: 0 = never, 1 = at any size (A/B, tests)
    const int kv16 = k16 ? std::atoi(k16) : -1;
    const bool want16 = wmax_units < 0xffff && p->V % 4 == 0 && kv16 != 0 && (kv16 == 1 || p->V >= 8192);
    (void)hipFree(p->d_lat16);
    p->d_lat16 = nullptr;
    if (e == hipSuccess && want16 && hipMalloc(&p->d_lat16, p->n_adj * 2) != hipSuccess) {
        (void)hipGetLastError();
        p->d_lat16 = nullptr;  // no room: the u64 latencies are streamed
    }
    cspan_begin(p);
    if (e == hipSuccess)
        hipLaunchKernelGGL(lvl_sym_tile_kernel, dim3((uint32_t)std::min<uint64_t>(nb * (nb + 1) / 2, 8192)), dim3(256),
                           0, p->stream, p->V, p->d_lat, with_loss ? p->d_loss : nullptr, wmax_units * p->kp.g, d_ok,
                           p->d_lat16, 1.0 / (double)p->kp.g);
    cspan_end(p);
    uint32_t ok = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&ok, d_ok, 4, hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    (void)hipFree(d_ok);
    if (e != hipSuccess) return fail(err, e, "symmetry check");
    *sym = ok != 0;
    if (!*sym) {  // only symmetric plans' out-rows read it
        (void)hipFree(p->d_lat16);
        p->d_lat16 = nullptr;
    }
    return SRT_OK;
}

// The shortest non-self-loop edge of the plan's graph, ns (~0: none)
srt_status level_min_edge(srt_plan *p, uint64_t *min_ns, srt_err *err) {
    *min_ns = ~0ull;
    unsigned long long *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof *d);
    if (e != hipSuccess) return fail(err, e, "hipMalloc(edge min)");
    (void)hipMemsetAsync(d, 0xff, sizeof *d, p->stream);
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(8192, (p->V + 3) / 4));
    cspan_begin(p);
    hipLaunchKernelGGL(edge_min_kernel, dim3(blocks), dim3(256), 0, p->stream, p->V, p->d_row_ptr, p->d_col, p->d_lat,
                       d);
    cspan_end(p);
    e = hipMemcpyAsync(min_ns, d, sizeof *d, hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    (void)hipFree(d);
    return e == hipSuccess ? SRT_OK : fail(err, e, "edge min");
}

void level_stats_init(unsigned long long *d_stats, hipStream_t s) {
    hipLaunchKernelGGL(loss_stats_init_kernel, dim3(1), dim3(1), 0, s, d_stats, d_stats + 2);
}

srt_status level_run(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    if (!p->ev_loss0) {
        (void)hipEventCreate(&p->ev_loss0);
        (void)hipEventCreate(&p->ev_loss1);
    }
    (void)hipEventRecord(p->ev_loss0, p->stream);
    p->shard_tail = false;
    p->tail_expanded = false;
    p->stage16 = false;
    // symmetric integer-level plans sharded over ranks build the class CSR
    // sharded too (level_csr_sharded); the others build it whole
    const bool sym_int = p->lvl_sym && !p->lvl_q && p->ident_rows;
    srt_status st;
    if (sym_int && p->comm && p->comm->nranks > 1)
        st = level_csr_sharded(p, p->kp.lmax, true, (uint32_t)p->comm->nranks, (uint32_t)p->comm->rank, p->comm, err);
    else if (sym_int && p->row_shard && p->lvl_emu_ranks > 1)
        st = level_csr_sharded(p, p->kp.lmax, true, p->lvl_emu_ranks,
                               (uint32_t)((uint64_t)p->row0 * p->lvl_emu_ranks / std::max<uint32_t>(p->n, 1)), nullptr,
                               err);
    else
        st = level_csr(p, p->kp.lmax, true, err);
    if (st != SRT_OK) return st;
    if (!p->d_lvisit) {
        const hipError_t e = hipMalloc(&p->d_lvisit, sizeof(unsigned long long));
        if (e != hipSuccess) return fail(err, e, "hipMalloc(visit counter)");
    }
    hipLaunchKernelGGL(level_zero_kernel, dim3(1), dim3(1), 0, p->stream, d_stats, (unsigned long long *)p->d_tmaxw,
                       p->d_lvisit);
#if LOSS_COUNT
    {
        const uint32_t dg = std::getenv("SRT_LVL_DIAG") ? (uint32_t)std::atoi(std::getenv("SRT_LVL_DIAG")) : 0u;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(lvl_diag), &dg, sizeof dg);
    }
#endif
    if (p->comm) {
        p->p3_launches = 0;
        p->p3_work = 0.0;
        p->p3_tiles = 0;
        st = level_sharded(p, d_stats, err);
        (void)hipEventRecord(p->ev_loss1, p->stream);
        return st;
    }
    const uint32_t lcap = (uint32_t)p->kp.lmax;
    // the solve launches are the plan's timed dominant launches (event pairs,
    // srt_plan_kernel_stats; work = the table pairs they write)
    const uint32_t cr = p->fold_chunk_rows ? p->fold_chunk_rows : std::max<uint32_t>(1, p->row1 - p->row0);
    const uint32_t nc = (p->row1 - p->row0 + cr - 1) / cr;
    while (p->ev.size() < 2 * (size_t)nc) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence) != hipSuccess)
            return fail(err, hipErrorUnknown, "event");
        p->ev.push_back(e);
    }
    while (p->fold_chunk_rows && p->ev_fold.size() < nc) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(err, hipErrorUnknown, "event");
        p->ev_fold.push_back(e);
    }
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->p3_tiles = 0;
    for (uint32_t c = 0; c < nc; ++c) {
        RowJob job;
        job.range = true;
        job.r0 = p->row0 + c * cr;
        job.r1 = std::min(p->row1, job.r0 + cr);
        (void)hipEventRecord(p->ev[2 * c], p->stream);
        if ((st = launch_solve(p, d_stats, job, lcap, false, nullptr, err)) != SRT_OK) return st;
        (void)hipEventRecord(p->ev[2 * c + 1], p->stream);
        p->p3_launches++;
        p->p3_work += (double)(job.r1 - job.r0) * p->n;
        if (p->fold_chunk_rows) (void)hipEventRecord(p->ev_fold[c], p->stream);
    }
    (void)hipEventRecord(p->ev_loss1, p->stream);
#if LOSS_COUNT
    {  // diagnostic builds (-DLOSS_COUNT=1): totals of every level solve so far
        unsigned long long c[9];
        (void)hipStreamSynchronize(p->stream);
        (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(loss_cnt), sizeof c);
        const double rows = (double)(p->row1 - p->row0);
        std::fprintf(stderr, "[srt] level solve (cumulative): visits %llu, us per row per CU: init %.2f levels %.2f out %.2f\n",
                     c[1], c[4] * 0.01 / rows, c[6] * 0.01 / rows, c[7] * 0.01 / rows);
        unsigned long long lc[8][5];
        (void)hipMemcpyFromSymbol(lc, HIP_SYMBOL(lvl_cnt), sizeof lc);
        for (int l = 1; l < 8; ++l)
            if (lc[l][4])
                std::fprintf(stderr, "[srt]   level %d: rows %llu items/row %.0f us/row: plan %.2f walk %.2f collect %.2f\n", l,
                             lc[l][4], (double)lc[l][3] / lc[l][4], lc[l][0] * 0.01 / lc[l][4],
                             lc[l][1] * 0.01 / lc[l][4], lc[l][2] * 0.01 / lc[l][4]);
    }
#endif
    return SRT_OK;
}

void expand_shard_rows(srt_plan *p, int nranks) { expand_slots(p, 0, (uint32_t)nranks * p->lrow_max); }

srt_status fw_loss(srt_plan *p, unsigned long long *d_stats, srt_err *err) {
    if (p->algo == SRT_ALGO_LEVEL) return level_run(p, d_stats, err);
    if (!p->ev_loss0) {
        (void)hipEventCreate(&p->ev_loss0);
        (void)hipEventCreate(&p->ev_loss1);
    }
    (void)hipEventRecord(p->ev_loss0, p->stream);
    srt_status st;
    p->shard_tail = false;
    p->tail_expanded = false;
    if (p->comm) {
        if (p->key_type == KEY_U16) st = loss_sharded_t<uint16_t>(p, d_stats, err);
        else if (p->key_type == KEY_U32) st = loss_sharded_t<uint32_t>(p, d_stats, err);
        else if (p->key_type == KEY_F64) st = loss_sharded_t<double>(p, d_stats, err);
        else st = loss_sharded_t<uint64_t>(p, d_stats, err);
        if (st != SRT_OK) return st;
        (void)hipEventRecord(p->ev_loss1, p->stream);
        return SRT_OK;
    }
    if (p->emulate_ranks > 1 && p->emu_closed) {
        if (p->key_type == KEY_U16) st = loss_emulated_t<uint16_t>(p, d_stats, err);
        else if (p->key_type == KEY_U32) st = loss_emulated_t<uint32_t>(p, d_stats, err);
        else if (p->key_type == KEY_F64) st = loss_emulated_t<double>(p, d_stats, err);
        else st = loss_emulated_t<uint64_t>(p, d_stats, err);
        if (st != SRT_OK) return st;
        (void)hipEventRecord(p->ev_loss1, p->stream);
        return SRT_OK;
    }
    if (p->key_type == KEY_U16) st = tight_csr_t<uint16_t>(p, d_stats, err);
    else if (p->key_type == KEY_U32) st = tight_csr_t<uint32_t>(p, d_stats, err);
    else if (p->key_type == KEY_F64) st = tight_csr_t<double>(p, d_stats, err);
    else st = tight_csr_t<uint64_t>(p, d_stats, err);
    if (st != SRT_OK) return st;
    p->emu_tight = p->t_edges;
    p->emu_maxw = p->h_tcount[1];
    if (p->fold_chunk_rows) {
        // chunks of table rows, each followed by its event (the end-to-end
        // download of chunk c overlaps the fold of chunk c + 1)
        const uint32_t cr = p->fold_chunk_rows, nc = (p->row1 - p->row0 + cr - 1) / cr;
        while (p->ev_fold.size() < nc) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(err, hipErrorUnknown, "event");
            p->ev_fold.push_back(e);
        }
        for (uint32_t c = 0; c < nc; ++c) {
            RowJob job;
            job.range = true;
            job.r0 = p->row0 + c * cr;
            job.r1 = std::min(p->row1, job.r0 + cr);
            if ((st = fold(p, d_stats, job, err)) != SRT_OK) return st;
            (void)hipEventRecord(p->ev_fold[c], p->stream);
        }
    } else if ((st = fold(p, d_stats, RowJob{}, err)) != SRT_OK) {
        return st;
    }
    (void)hipEventRecord(p->ev_loss1, p->stream);
    return SRT_OK;
}

// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_loss() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&loss_stats_init_kernel));
}

}  // namespace srt
