// scan_bench.cpp -- CPU timing and cross-check of the plan-creation CSR scan
// (shadow_amd/csrc/srt_scan.cpp) on a C3-shaped CSR: the complete n-node
// graph with self-loops, rows 0 .. n-1 in order, latencies U{1..300} ms in ns,
// 6-decimal losses.  The r03 scan (one branchy pass, a f64 division per
// entry) is restated here as the reference; the stats and the u32 latency
// copy must match.  Also: a directed variant (fingerprint must differ) and
// planted errors (first offending entries must match).
//   g++ -O3 -std=c++17 -pthread -Iinclude tools/scan_bench.cpp shadow_amd/csrc/srt_scan.cpp -o /tmp/scan_bench
//   /tmp/scan_bench [n] [threads]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>

#include "../shadow_amd/csrc/srt_scan.h"

using srt::CsrStats;

static void ref_rows(const srt_csr *g, uint32_t r0, uint32_t r1, CsrStats &st, CsrStats *out, uint32_t *lat32) {
    const uint32_t V = g->n_nodes;
    for (uint32_t u = r0; u < r1; ++u) {
        const uint64_t b = g->row_ptr[u], e = g->row_ptr[u + 1];
        uint32_t cnt = 0, prev = 0;
        uint64_t first = ~0ull;
        bool inc = true, dec = true;
        for (uint64_t k = b; k < e; ++k) {
            const uint32_t c = g->col[k];
            const uint64_t l = g->lat_ns[k];
            const float q = g->loss[k];
            if (c >= V && st.badcol_k == ~0ull) st.badcol_k = k;
            if (l == 0 && st.zero_k == ~0ull) st.zero_k = k;
            if (!(q >= 0.0f && q <= 1.0f) && st.badloss_k == ~0ull) st.badloss_k = k;
            st.maxlat = std::max(st.maxlat, l);
            if (lat32) lat32[k] = (uint32_t)l;
            if (st.gcd != 1 && l) {  // r03: divisibility by the running gcd in f64
                bool divides;
                if (st.gcd && l < (1ull << 53) && st.gcd < (1ull << 53)) {
                    const uint64_t qi = (uint64_t)((double)l / (double)st.gcd);
                    divides = qi * st.gcd == l;
                } else {
                    divides = st.gcd && l % st.gcd == 0;
                }
                if (!divides) st.gcd = std::gcd(st.gcd, l);
            }
            if (c == u) {
                if (!cnt) first = k;
                ++cnt;
            }
            if (k > b) {
                inc &= c > prev;
                dec &= c < prev;
            }
            prev = c;
        }
        out->sl_cnt[u] = cnt;
        out->sl_first[u] = first;
        st.selfloops += cnt;
        const bool uniq = inc || dec;
        st.unique &= uniq;
        st.complete &= uniq && (e - b - cnt) == (uint64_t)V - 1;
    }
}

static uint64_t sm(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

struct Csr {
    std::vector<uint64_t> row_ptr, lat;
    std::vector<uint32_t> col;
    std::vector<float> loss;
    srt_csr g{};
};

// complete graph; directed: the two orientations of a pair get different latencies
static void make(Csr &c, uint32_t n, bool directed) {
    c.row_ptr.resize(n + 1);
    const uint64_t m = (uint64_t)n * n;
    c.col.resize(m);
    c.lat.resize(m);
    c.loss.resize(m);
    std::vector<std::thread> th;
    const int T = 8;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (uint32_t u = t; u < n; u += T) {
                c.row_ptr[u] = (uint64_t)u * n;
                for (uint32_t v = 0; v < n; ++v) {
                    const uint32_t a = std::min(u, v), b = std::max(u, v);
                    uint64_t s = ((uint64_t)a << 32 | b) ^ (directed && u > v ? 0x5555ull : 0);
                    const uint64_t r = sm(&s);
                    const uint64_t k = (uint64_t)u * n + v;
                    c.col[k] = v;
                    c.lat[k] = (1 + r % 300) * 1000000ull;
                    c.loss[k] = (float)((r >> 20) % 10001) / 1e6f;
                }
            }
        });
    for (auto &x : th) x.join();
    c.row_ptr[n] = m;
    c.g.n_nodes = n;
    c.g.n_adj = m;
    c.g.row_ptr = c.row_ptr.data();
    c.g.col = c.col.data();
    c.g.lat_ns = c.lat.data();
    c.g.loss = c.loss.data();
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// both scans on T threads by row ranges; returns (ref s, new s)
static void run(const srt_csr *g, int T, CsrStats *ref, CsrStats *nw, std::vector<uint32_t> *l_ref,
                std::vector<uint32_t> *l_new, double *t_ref, double *t_new) {
    const uint32_t V = g->n_nodes;
    for (int pass = 0; pass < 2; ++pass) {
        CsrStats *out = pass ? nw : ref;
        out->sl_cnt.assign(V, 0);
        out->sl_first.assign(V, ~0ull);
        std::vector<CsrStats> part(T);
        uint32_t *l32 = pass ? l_new->data() : l_ref->data();
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const uint32_t a = (uint32_t)((uint64_t)V * t / T), b = (uint32_t)((uint64_t)V * (t + 1) / T);
                bool ov = false, id = true;
                if (pass) srt::scan_rows(g, a, b, part[t], out, l32, 0, &ov, &id);
                else ref_rows(g, a, b, part[t], out, l32);
            });
        for (auto &x : th) x.join();
        srt::merge_stats(part, V, out);
        (pass ? *t_new : *t_ref) = now() - t0;
    }
}

static int check(const CsrStats &a, const CsrStats &b, const char *what) {
    int bad = 0;
#define CK(f)                                                                                     \
    if (a.f != b.f) {                                                                             \
        std::printf("  MISMATCH %s: %s ref %llu new %llu\n", what, #f, (unsigned long long)a.f, \
                    (unsigned long long)b.f);                                                     \
        bad = 1;                                                                                  \
    }
    CK(gcd) CK(maxlat) CK(selfloops) CK(zero_k) CK(badloss_k) CK(badcol_k) CK(unique) CK(complete)
#undef CK
    if (a.sl_cnt != b.sl_cnt || a.sl_first != b.sl_first) {
        std::printf("  MISMATCH %s: self-loops\n", what);
        bad = 1;
    }
    return bad;
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 16384;
    const int T = argc > 2 ? std::atoi(argv[2]) : 8;
    Csr c;
    make(c, n, false);
    const uint64_t m = c.g.n_adj;
    std::vector<uint32_t> l_ref(m), l_new(m);
    int bad = 0;
    for (int rep = 0; rep < 3; ++rep) {
        CsrStats a, b;
        double tr, tn;
        run(&c.g, T, &a, &b, &l_ref, &l_new, &tr, &tn);
        bad |= check(a, b, "complete");
        bad |= l_ref != l_new;
        std::printf("n=%u entries=%llu threads=%d: r03 scan %.1f ms, new %.1f ms (%.2f ns/entry/thread), sym fp %s\n",
                    n, (unsigned long long)m, T, tr * 1e3, tn * 1e3, tn * 1e9 * T / m,
                    b.sym_a == b.sym_b ? "equal" : "DIFFERENT");
        bad |= b.sym_a != b.sym_b;
    }
    // errors and a gcd change late in the graph
    c.lat[m / 3] = 0;
    c.loss[m / 2] = -0.5f;
    c.loss[m / 2 + 7] = -0.0f;  // valid
    c.col[m - 5] = n + 3;
    c.lat[m / 4] = 1000000ull * 7 + 500;  // gcd 500 ns from a quarter in
    {
        CsrStats a, b;
        double tr, tn;
        run(&c.g, T, &a, &b, &l_ref, &l_new, &tr, &tn);
        bad |= check(a, b, "planted errors");
        std::printf("planted: zero_k %llu badloss_k %llu badcol_k %llu gcd %llu\n", (unsigned long long)b.zero_k,
                    (unsigned long long)b.badloss_k, (unsigned long long)b.badcol_k, (unsigned long long)b.gcd);
    }
    Csr d;
    make(d, std::min<uint32_t>(n, 2048), true);
    {
        std::vector<uint32_t> a1(d.g.n_adj), a2(d.g.n_adj);
        CsrStats a, b;
        double tr, tn;
        run(&d.g, T, &a, &b, &a1, &a2, &tr, &tn);
        bad |= check(a, b, "directed");
        std::printf("directed: sym fp %s\n", b.sym_a == b.sym_b ? "EQUAL" : "different");
        bad |= b.sym_a == b.sym_b;
    }
    std::printf(bad ? "FAIL\n" : "OK\n");
    return bad;
}
