// srt_scan.cpp -- one pass over the borrowed CSR at plan creation.
//
// The edge-attribute checks of ShadowEdge::try_from that the ABI cannot
// assume (src/main/network/graph/mod.rs:72-111: latency != 0, loss in [0, 1]),
// endpoints in range, the self-loops of every node (mod.rs:210-217, 256-293),
// and the statistics the key proofs need (gcd and max of the latencies,
// completeness, parallel edges), plus the symmetry fingerprint of the AUTO
// price.  Rows are split over host threads (the CPU share of the job:
// OMP_NUM_THREADS, else up to 32) by equal adjacency counts; it runs while the
// main thread sets up the device and uploads the CSR, and on big graphs it
// sets the pace of that upload (C3: 2.7e8 entries, 16 B read a entry), so the
// row loop is branch-free reductions the compiler vectorises (an AVX2 + FMA
// clone where the CPU has them): the gcd's divisibility test is
// rint(l / g) * g == l by the reciprocal (exact below 2^51), the first
// offending entry of an error is looked up only in a row that has one.  A row
// counts as free of parallel edges when its far endpoints are strictly
// monotone (petgraph lists a node's edges in reverse insertion order, so a GML
// graph written in node order is); any other row is treated as possibly
// parallel, which only costs the FW init an atomic min and the key proof its
// completeness shortcut.
#include "srt_scan.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>

namespace srt {

int host_threads(uint64_t work) {
    if (work < (1ull << 20)) return 1;
    int t = (int)std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) t = std::atoi(e);
    if (const char *e = std::getenv("SRT_HOST_THREADS")) t = std::atoi(e);
    return std::max(1, std::min(t, 32));
}

namespace {

// reductions of one row
struct RowAcc {
    uint64_t mx = 0;       // max latency
    uint64_t hi = 0;       // OR of latency >> 32 (u32 upload), and >> 51 below
    uint64_t hi51 = 0;
    uint32_t maxc = 0;     // max far endpoint
    uint32_t idx = 0;      // OR of col[k] ^ (k - b): 0 iff the row is 0 .. e-b-1
    uint32_t zero = 0;     // a zero latency
    uint32_t bad = 0;      // a loss outside [0, 1] (or NaN)
    uint32_t ndiv = 0;     // a latency the running gcd does not divide
    uint32_t self = 0;     // self-loop entries
    uint32_t fa = 0, fc = 0, fcl = 0;  // fingerprint: sum c*c + l, sum c, sum c*l (mod 2^32)
};

inline uint32_t loss_bad(uint32_t q) { return (q > 0x3f800000u) & (q != 0x80000000u); }

// FMA: the divisibility remainder in f64; else in integers
template <bool FMA, bool W, bool LOSS>
inline __attribute__((always_inline)) void row_body(const uint32_t *__restrict__ col, const uint64_t *__restrict__ lat,
                                                    const uint32_t *__restrict__ lossb, uint64_t n, uint32_t u,
                                                    double gd, double rcp, bool check_div,
                                                    uint32_t *__restrict__ out32, RowAcc &a) {
    uint64_t mx = 0, hi = 0, hi51 = 0;
    uint32_t maxc = 0, idx = 0, zero = 0, bad = 0, self = 0, fa = 0, fc = 0, fcl = 0;
    for (uint64_t k = 0; k < n; ++k) {
        const uint32_t c = col[k];
        const uint64_t l = lat[k];
        const uint32_t l32 = (uint32_t)l;
        maxc = c > maxc ? c : maxc;
        idx |= c ^ (uint32_t)k;
        zero |= l == 0;
        if (LOSS) bad |= loss_bad(lossb[k]);
        mx = l > mx ? l : mx;
        hi |= l >> 32;
        hi51 |= l >> 51;
        self += c == u;
        fa += c * c + l32;
        fc += c;
        fcl += c * l32;
        if (W) out32[k] = l32;
    }
    uint32_t ndiv = 0;
    if (check_div) {
        if (FMA) {
            // l as f64 by the exponent trick (exact below 2^52; larger rows take
            // the slow path through hi51); q = rint(l / g) exact for g | l below 2^51
            for (uint64_t k = 0; k < n; ++k) {
                uint64_t bits = lat[k] | 0x4330000000000000ull;
                double d;
                std::memcpy(&d, &bits, 8);
                d -= 4503599627370496.0;  // 2^52
                const double q = std::rint(d * rcp);
                ndiv |= std::fma(q, gd, -d) != 0.0;
            }
        } else {
            const uint64_t g = (uint64_t)gd;
            for (uint64_t k = 0; k < n; ++k) {
                const uint64_t l = lat[k];
                const uint64_t q = (uint64_t)std::rint((double)(int64_t)l * rcp);
                ndiv |= q * g != l;
            }
        }
    }
    a.mx = mx;
    a.hi = hi;
    a.hi51 = hi51;
    a.maxc = maxc;
    a.idx = idx;
    a.zero = zero;
    a.bad = bad;
    a.ndiv = ndiv;
    a.self = self;
    a.fa = fa;
    a.fc = fc;
    a.fcl = fcl;
}

using RowFn = void (*)(const uint32_t *, const uint64_t *, const uint32_t *, uint64_t, uint32_t, double, double, bool,
                       uint32_t *, RowAcc &);

template <bool W, bool LOSS>
__attribute__((target("avx2,fma"))) void row_avx2(const uint32_t *col, const uint64_t *lat, const uint32_t *lossb,
                                                  uint64_t n, uint32_t u, double gd, double rcp, bool cd,
                                                  uint32_t *out32, RowAcc &a) {
    row_body<true, W, LOSS>(col, lat, lossb, n, u, gd, rcp, cd, out32, a);
}
template <bool W, bool LOSS>
void row_generic(const uint32_t *col, const uint64_t *lat, const uint32_t *lossb, uint64_t n, uint32_t u, double gd,
                 double rcp, bool cd, uint32_t *out32, RowAcc &a) {
    row_body<false, W, LOSS>(col, lat, lossb, n, u, gd, rcp, cd, out32, a);
}

template <bool LOSS>
RowFn pick_row(bool w, bool simd) {
    return w ? (simd ? row_avx2<true, LOSS> : row_generic<true, LOSS>)
             : (simd ? row_avx2<false, LOSS> : row_generic<false, LOSS>);
}

bool have_avx2_fma() {
    static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    return ok;
}

}  // namespace

void scan_rows(const srt_csr *g, uint32_t r0, uint32_t r1, CsrStats &st, CsrStats *out, uint32_t *lat32,
               uint64_t k_base, bool *lat_over, bool *identity, bool check_loss) {
    const uint32_t V = g->n_nodes;
    const bool simd = have_avx2_fma();
    const RowFn fn = check_loss ? pick_row<true>(lat32 != nullptr, simd) : pick_row<false>(lat32 != nullptr, simd);
    const uint32_t *lossb = reinterpret_cast<const uint32_t *>(g->loss);
    uint64_t gcd = st.gcd, maxlat = st.maxlat, selfl = st.selfloops;
    uint32_t sa = (uint32_t)st.sym_a, sb = (uint32_t)st.sym_b;
    double gd = (double)gcd, rcp = gcd ? 1.0 / (double)gcd : 0.0;
    bool ident = true, over = false;
    for (uint32_t u = r0; u < r1; ++u) {
        const uint64_t b = g->row_ptr[u], e = g->row_ptr[u + 1], n = e - b;
        RowAcc a;
        // gcd 0 (nothing seen yet) or 1 needs no divisibility test
        fn(g->col + b, g->lat_ns + b, lossb + b, n, u, gd, rcp, gcd > 1, lat32 ? lat32 + (b - k_base) : nullptr, a);
        if (a.zero || a.bad || a.maxc >= V) {  // an invalid entry: its first index
            for (uint64_t k = b; k < e; ++k) {
                if (g->col[k] >= V && st.badcol_k == ~0ull) st.badcol_k = k;
                if (g->lat_ns[k] == 0 && st.zero_k == ~0ull) st.zero_k = k;
                if (check_loss && loss_bad(lossb[k]) && st.badloss_k == ~0ull) st.badloss_k = k;
            }
        }
        if (gcd != 1 && (gcd == 0 || a.ndiv || a.hi51)) {  // the gcd changes (or is not yet known)
            for (uint64_t k = b; k < e; ++k) {
                const uint64_t l = g->lat_ns[k];
                if (l && (gcd == 0 || l % gcd)) gcd = std::gcd(gcd, l);
            }
            gd = (double)gcd;
            rcp = gcd ? 1.0 / (double)gcd : 0.0;
        }
        maxlat = a.mx > maxlat ? a.mx : maxlat;
        over |= a.hi != 0;
        ident &= n == V && a.idx == 0;
        uint64_t first = ~0ull;
        if (a.self) first = (uint64_t)(std::find(g->col + b, g->col + e, u) - g->col);
        out->sl_cnt[u] = a.self;
        out->sl_first[u] = first;
        selfl += a.self;
        // fingerprint: sum u*(c*c + l) = u * fa; sum c*(u*u + l) = u*u * fc + fcl
        sa += u * a.fa;
        sb += u * u * a.fc + a.fcl;
        // strictly monotone far endpoints: no parallel edges in the row
        bool inc = true, dec = true;
        if (n > 1) {
            uint32_t vi = 0, vd = 0;
            const uint32_t *c = g->col + b;
            for (uint64_t k = 1; k < n; ++k) {
                vi |= c[k] <= c[k - 1];
                vd |= c[k] >= c[k - 1];
            }
            inc = !vi;
            dec = !vd;
        }
        const bool uniq = inc || dec;
        st.unique &= uniq;
        st.complete &= uniq && (n - a.self) == (uint64_t)V - 1;
    }
    st.gcd = gcd;
    st.maxlat = maxlat;
    st.selfloops = selfl;
    st.sym_a = sa;
    st.sym_b = sb;
    if (lat_over && over) *lat_over = true;
    if (identity && !ident) *identity = false;
    st.ident &= ident;
}

void merge_stats(const std::vector<CsrStats> &part, uint32_t V, CsrStats *out) {
    out->complete = V > 0;
    out->ident = V > 0;
    uint32_t sa = 0, sb = 0;
    for (const CsrStats &st : part) {
        out->gcd = std::gcd(out->gcd, st.gcd);
        out->maxlat = std::max(out->maxlat, st.maxlat);
        out->selfloops += st.selfloops;
        sa += (uint32_t)st.sym_a;
        sb += (uint32_t)st.sym_b;
        out->zero_k = std::min(out->zero_k, st.zero_k);
        out->badloss_k = std::min(out->badloss_k, st.badloss_k);
        out->badcol_k = std::min(out->badcol_k, st.badcol_k);
        out->unique &= st.unique;
        out->complete &= st.complete;
        out->ident &= st.ident;
    }
    out->sym_a = sa;
    out->sym_b = sb;
    if (out->gcd == 0) out->gcd = 1;
}

void csr_scan(const srt_csr *g, CsrStats *out, bool check_loss) {
    const uint32_t V = g->n_nodes;
    out->sl_cnt.assign(V, 0);
    out->sl_first.assign(V, ~0ull);
    const int T = host_threads(g->n_adj);
    std::vector<CsrStats> part(T);
    auto work = [&](int t, uint32_t r0, uint32_t r1) {
        scan_rows(g, r0, r1, part[t], out, nullptr, 0, nullptr, nullptr, check_loss);
    };
    // row ranges with about n_adj / T entries each
    std::vector<uint32_t> cut(T + 1, V);
    cut[0] = 0;
    for (int t = 1; t < T; ++t) {
        const uint64_t target = g->n_adj * (uint64_t)t / T;
        cut[t] = (uint32_t)(std::lower_bound(g->row_ptr, g->row_ptr + V + 1, target) - g->row_ptr);
        cut[t] = std::max(std::min(cut[t], V), cut[t - 1]);
    }
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work, t, cut[t], cut[t + 1]);
    work(0, cut[0], cut[1]);
    for (auto &th : pool) th.join();
    merge_stats(part, V, out);
}

uint64_t first_bad_loss(const srt_csr *g) {
    const uint64_t m = g->n_adj;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(g->loss);
    const int T = host_threads(m);
    std::vector<uint64_t> first(T, ~0ull);
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t)
        pool.emplace_back([&, t] {
            for (uint64_t k = m * t / T; k < m * (t + 1) / T; ++k)
                if (loss_bits_bad(q[k])) {
                    first[t] = k;
                    break;
                }
        });
    for (auto &th : pool) th.join();
    return *std::min_element(first.begin(), first.end());
}

}  // namespace srt
