// srt_gml.cpp -- GML ingest straight into the petgraph-shaped CSR of srt.h.
//
// Grammar: src/lib/gml-parser/src/parser.rs:45-273 (nom combinators):
//   gml   := ws* "graph" sp* "[" NL item* "]"   (trailing text ignored)
//   item  := key ( node | edge | directed | value )
//   node/edge := sp* "[" NL (key value)* "]" NL
//   value := sp* ( int NL | float NL | string NL )      -- tried in that order
//   NL    := sp* [ \t\r\n]+ (must contain CR or LF) sp*
// Validation: ShadowNode/ShadowEdge::try_from (src/main/network/graph/mod.rs:28-111),
// edge endpoints looked up by GML id (mod.rs:164-175, last node with an id wins),
// Time units (src/main/utility/units.rs:405-439) converted to ns.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <string_view>
#include <sys/mman.h>
#include <unordered_map>
#include <vector>

#include "srt_internal.h"

namespace {
// vectors whose resize() leaves elements uninitialised: the big arrays of the
// ingest are written in full by the parallel phases, so their pages are first
// touched there, on every thread, instead of zeroed by one thread
// Big ones (>= 4 MiB) are mapped directly and advised onto transparent huge
// pages: an ingest at C3 scale allocates several GB, and 4-KiB page faults
// (each one a kernel zero-fill) were a large part of a cold parse.
template <typename T>
struct NoInit : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <typename U>
    NoInit(const NoInit<U> &) noexcept {}
    static constexpr size_t BIG = 4u << 20, HUGE = 2u << 20;
    T *allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < BIG) return std::allocator<T>::allocate(n);
        const size_t len = (bytes + HUGE - 1) & ~(HUGE - 1);
        void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, len, MADV_HUGEPAGE);
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t n) noexcept {
        const size_t bytes = n * sizeof(T);
        if (bytes < BIG) return std::allocator<T>::deallocate(p, n);
        munmap(p, (bytes + HUGE - 1) & ~(HUGE - 1));
    }
    template <typename U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <typename U, typename... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
};
template <typename T>
using uvec = std::vector<T, NoInit<T>>;
}  // namespace

struct srt_gml {
    bool directed = false;
    std::vector<uint32_t> ids;
    std::vector<uint64_t> row_ptr;
    uvec<uint32_t> col;
    uvec<uint64_t> lat;
    uvec<float> loss;
};

namespace {

struct Fail {
    std::string msg;
};

enum class VT { Int, Float, Str };
struct Val {
    VT t;
    int32_t i = 0;
    float f = 0.f;
    std::string_view s;
};
struct KV {
    std::string_view k;
    Val v;
};

class Lexer {
   public:
    explicit Lexer(std::string_view t) : p_(t.data()), e_(t.data() + t.size()), b_(t.data()) {}
    // sub-range [b, e) of t; error offsets stay relative to t
    Lexer(std::string_view t, size_t b, size_t e) : p_(t.data() + b), e_(t.data() + e), b_(t.data()) {}
    size_t pos() const { return (size_t)(p_ - b_); }

    [[noreturn]] void fail(const char *what) {
        throw Fail{std::string(what) + " at byte " + std::to_string(p_ - b_)};
    }
    static bool sp(char c) { return c == ' ' || c == '\t'; }
    static bool msp(char c) { return sp(c) || c == '\r' || c == '\n'; }
    static bool alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
    static bool digit(char c) { return c >= '0' && c <= '9'; }

    void sp0() { while (p_ < e_ && sp(*p_)) ++p_; }
    void msp0() { while (p_ < e_ && msp(*p_)) ++p_; }
    bool newline() {
        const char *s = p_;
        sp0();
        if (p_ >= e_ || !msp(*p_)) {
            p_ = s;
            return false;
        }
        while (p_ < e_ && msp(*p_)) ++p_;
        sp0();
        return true;
    }
    bool tag(char c) {
        if (p_ < e_ && *p_ == c) {
            ++p_;
            return true;
        }
        return false;
    }
    bool tag(std::string_view t) {
        if ((size_t)(e_ - p_) >= t.size() && std::memcmp(p_, t.data(), t.size()) == 0) {
            p_ += t.size();
            return true;
        }
        return false;
    }
    bool key(std::string_view *k) {
        if (p_ >= e_ || !(alpha(*p_) || *p_ == '_')) return false;
        const char *s = p_++;
        while (p_ < e_ && (alpha(*p_) || digit(*p_) || *p_ == '_')) ++p_;
        *k = std::string_view(s, (size_t)(p_ - s));
        return true;
    }
    // value := sp0 (int NL | float NL | string NL); false = no alternative matched
    bool value(Val *v) {
        sp0();
        const char *save = p_;
        if (p_ < e_ && digit(*p_)) {  // int: digit1 parsed as i32 (overflow -> next alt)
            int64_t x = 0;
            bool ovf = false;
            while (p_ < e_ && digit(*p_)) {
                x = x * 10 + (*p_ - '0');
                if (x > INT32_MAX) ovf = true, x = INT32_MAX + 1ll;
                ++p_;
            }
            // a '.', 'e' or 'E' right after the digits fails the int's newline:
            // straight to the float alternative
            const bool fl = p_ < e_ && (*p_ == '.' || *p_ == 'e' || *p_ == 'E');
            if (!ovf && !fl && newline()) {
                v->t = VT::Int;
                v->i = (int32_t)x;
                return true;
            }
            p_ = save;
        }
        {  // float: nom recognize_float, then correctly rounded f32 parse
            const char *q = p_;
            if (q < e_ && (*q == '+' || *q == '-')) ++q;
            bool ok = false;
            if (q < e_ && digit(*q)) {
                while (q < e_ && digit(*q)) ++q;
                if (q < e_ && *q == '.') {
                    ++q;
                    while (q < e_ && digit(*q)) ++q;
                }
                ok = true;
            } else if (q + 1 < e_ && *q == '.' && digit(q[1])) {
                ++q;
                while (q < e_ && digit(*q)) ++q;
                ok = true;
            }
            if (ok) {
                if (q < e_ && (*q == 'e' || *q == 'E')) {
                    ++q;
                    if (q < e_ && (*q == '+' || *q == '-')) ++q;
                    if (!(q < e_ && digit(*q))) {
                        p_ = q;
                        fail("expected exponent digits");  // nom cut(): hard failure
                    }
                    while (q < e_ && digit(*q)) ++q;
                }
                // Fast exact path: no exponent and at most 2^24 as an integer
                // d with k fraction digits -> d / 10^k in f32.  Both operands are
                // exact f32 values (d < 2^24, 10^k for k <= 10) and IEEE division
                // rounds correctly, so this is strtof's correctly rounded result.
                {
                    const char *r = p_;
                    const bool neg = *r == '-';
                    if (*r == '+' || *r == '-') ++r;
                    uint64_t d = 0;
                    int k = 0, nd = 0;
                    bool frac = false, fast = true;
                    for (; r < q; ++r) {
                        if (*r == '.') {
                            frac = true;
                            continue;
                        }
                        if (!digit(*r)) {
                            fast = false;  // exponent
                            break;
                        }
                        d = d * 10 + (uint64_t)(*r - '0');
                        if (d) ++nd;
                        if (frac) ++k;
                        if (nd > 9) {
                            fast = false;
                            break;
                        }
                    }
                    if (fast && d < (1u << 24) && k <= 10) {
                        static const float p10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f,
                                                      1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
                        float f = (float)d / p10[k];
                        if (neg) f = -f;
                        p_ = q;
                        if (newline()) {
                            v->t = VT::Float;
                            v->f = f;
                            return true;
                        }
                        p_ = save;
                        goto string_alt;
                    }
                }
                // strtof needs a terminated copy; short tokens stay on the stack
                const size_t tl = (size_t)(q - p_);
                char sbuf[64];
                std::string big;
                const char *tok = sbuf;
                if (tl < sizeof sbuf) {
                    std::memcpy(sbuf, p_, tl);
                    sbuf[tl] = 0;
                } else {
                    big.assign(p_, tl);
                    tok = big.c_str();
                }
                const float f = std::strtof(tok, nullptr);
                p_ = q;
                if (newline()) {
                    v->t = VT::Float;
                    v->f = f;
                    return true;
                }
                p_ = save;
            }
        }
    string_alt:
        if (p_ < e_ && *p_ == '"') {  // string: non-empty run of non-'"' bytes
            const char *b = p_ + 1, *q = b;
            while (q < e_ && *q != '"') ++q;
            if (q > b && q < e_) {
                p_ = q + 1;
                if (newline()) {
                    v->t = VT::Str;
                    v->s = std::string_view(b, (size_t)(q - b));
                    return true;
                }
            }
            p_ = save;
        }
        return false;
    }
    void block(std::vector<KV> *kvs) {
        sp0();
        if (!tag('[') || !newline()) fail("expected '[' and a newline");
        while (!tag(']')) {
            KV kv;
            if (!key(&kv.k)) fail("expected a key");
            if (!value(&kv.v)) fail("expected an int, float or string value");
            kvs->push_back(kv);
        }
        for (size_t i = 0; i < kvs->size(); ++i)
            for (size_t j = i + 1; j < kvs->size(); ++j)
                if ((*kvs)[i].k == (*kvs)[j].k) fail("Duplicate keys are not supported");
        if (!newline()) fail("expected a newline");
    }
    bool at_end() const { return p_ >= e_; }
    // a block whose '[' is at p_ and whose ']' is the last byte of the range:
    // the same grammar as block() without the leading sp0 and trailing newline
    bool block_body(std::vector<KV> *kvs) {
        if (!tag('[') || !newline()) return false;
        while (!tag(']')) {
            KV kv;
            if (!key(&kv.k) || !value(&kv.v)) return false;
            kvs->push_back(kv);
        }
        if (p_ != e_) return false;
        for (size_t i = 0; i < kvs->size(); ++i)
            for (size_t j = i + 1; j < kvs->size(); ++j)
                if ((*kvs)[i].k == (*kvs)[j].k) return false;
        return true;
    }

   private:
    const char *p_, *e_, *b_;
};

const Val *get(const std::vector<KV> &kvs, std::string_view k) {
    for (const KV &kv : kvs)
        if (kv.k == k) return &kv.v;
    return nullptr;
}

bool is_ws_byte_seq(std::string_view s, size_t i, size_t *len) {
    const unsigned char c = (unsigned char)s[i];
    if (c == ' ' || (c >= 0x09 && c <= 0x0d)) return *len = 1, true;
    if (c == 0xc2 && i + 1 < s.size() && ((unsigned char)s[i + 1] == 0x85 || (unsigned char)s[i + 1] == 0xa0))
        return *len = 2, true;
    if (i + 2 < s.size()) {
        const unsigned char c1 = (unsigned char)s[i + 1], c2 = (unsigned char)s[i + 2];
        if ((c == 0xe2 && c1 == 0x80 && ((c2 >= 0x80 && c2 <= 0x8a) || c2 == 0xa8 || c2 == 0xa9 || c2 == 0xaf)) ||
            (c == 0xe2 && c1 == 0x81 && c2 == 0x9f) || (c == 0xe3 && c1 == 0x80 && c2 == 0x80) ||
            (c == 0xe1 && c1 == 0x9a && c2 == 0x80))
            return *len = 3, true;
    }
    return false;
}

std::string_view trim_ws(std::string_view s) {
    size_t l;
    while (!s.empty() && is_ws_byte_seq(s, 0, &l)) s.remove_prefix(l);
    for (bool again = true; again && !s.empty();) {
        again = false;
        for (size_t k = 1; k <= 3 && k <= s.size(); ++k)
            if (is_ws_byte_seq(s, s.size() - k, &l) && l == k) {
                s.remove_suffix(k);
                again = true;
                break;
            }
    }
    return s;
}

// regex ^([+-]?[0-9\.]*)\s*(.*)$ then trim (units.rs:411-418)
bool split_unit(std::string_view s, std::string_view *val, std::string_view *unit) {
    size_t i = 0;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
    while (i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '.')) ++i;
    std::string_view v = s.substr(0, i);
    size_t l;
    while (i < s.size() && is_ws_byte_seq(s, i, &l)) i += l;
    std::string_view u = s.substr(i);
    if (u.find('\n') != std::string_view::npos) return false;
    *val = trim_ws(v);
    *unit = trim_ws(u);
    return true;
}

bool parse_u64(std::string_view s, uint64_t *out) {  // <u64 as FromStr>
    if (!s.empty() && s[0] == '+') s.remove_prefix(1);
    if (s.empty()) return false;
    uint64_t v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return false;
        const uint64_t d = (uint64_t)(c - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = v;
    return true;
}

// Time<TimePrefix>::from_str + convert(Nano); returns an error text or nullptr
const char *parse_time(std::string_view s, uint64_t *ns, uint64_t *value) {
    std::string_view v, u;
    if (!split_unit(s, &v, &u)) return "Unable to identify value and unit";
    static const std::pair<const char *, uint64_t> tab[] = {
        {"ns", 1ull}, {"nanosecond", 1ull}, {"nanoseconds", 1ull}, {"us", 1000ull}, {"\xce\xbcs", 1000ull},
        {"microsecond", 1000ull}, {"microseconds", 1000ull}, {"ms", 1000000ull}, {"millisecond", 1000000ull},
        {"milliseconds", 1000000ull}, {"s", 1000000000ull}, {"sec", 1000000000ull}, {"secs", 1000000000ull},
        {"second", 1000000000ull}, {"seconds", 1000000000ull}, {"m", 60000000000ull}, {"min", 60000000000ull},
        {"mins", 60000000000ull}, {"minute", 60000000000ull}, {"minutes", 60000000000ull},
        {"h", 3600000000000ull}, {"hr", 3600000000000ull}, {"hrs", 3600000000000ull},
        {"hour", 3600000000000ull}, {"hours", 3600000000000ull}};
    uint64_t mag = 0;
    if (u.empty()) mag = 1000000000ull;
    for (const auto &t : tab)
        if (u == t.first) {
            mag = t.second;  // the units are distinct: the first match is the only one
            break;
        }
    if (!mag) return "Unit was not one of (ns|nanosecond|...|h|hr|hrs|hour|hours)";
    uint64_t x;
    if (!parse_u64(v, &x)) return "invalid digit found in string";
    if (x > UINT64_MAX / mag) return "The resulting value is outside of the bounds";
    *ns = x * mag;
    *value = x;
    return nullptr;
}

bool bits_per_sec_ok(std::string_view s) {  // BitsPerSec<SiPrefixUpper>
    std::string_view v, u;
    if (!split_unit(s, &v, &u)) return false;
    if (u.size() >= 3 && u.substr(u.size() - 3) == "bit") u.remove_suffix(3);
    else if (u.size() >= 4 && u.substr(u.size() - 4) == "bits") u.remove_suffix(4);
    if (!u.empty()) {
        static const char *ok[] = {"K", "kilo", "Ki", "kibi", "M", "mega", "Mi", "mebi",
                                   "G", "giga", "Gi", "gibi", "T", "tera", "Ti", "tebi"};
        bool f = false;
        for (const char *o : ok) f |= (u == o);
        if (!f) return false;
    }
    uint64_t x;
    return parse_u64(v, &x);
}

// ---------------------------------------------------------------------------
// Parallel ingest.  A Shadow graph at config C3 scale is ~1.3e8 edge blocks
// (~12 GB of text), so parsing is split into segments that tile the text:
//   gap segments   -- top-level items between blocks, ending with the key
//                     ("node"/"edge") that opens the next block;
//   block segments -- "[" ... "]" of one node or edge.
// Block boundaries are the '[' / ']' bytes outside strings; string state at
// every byte comes from the parity of '"' before it (chunk-parallel count +
// prefix, then a chunk-parallel scan for structural bytes).  In valid GML a
// '"' only delimits string values and '[' ']' outside strings only delimit
// blocks, so every segment then parses with the exact sequential grammar of
// the Lexer; any input the segment parsers reject (including inputs whose
// stray quotes fool the parity) is re-parsed sequentially, which yields the
// reference-order error.  Syntax errors anywhere take precedence over
// node/edge validation (gml_parser::parse runs before NetworkGraph::parse),
// then nodes are validated in order, then edges (first failing edge wins).

struct EdgeRec {  // trivially constructible: check_edge fills every field
    int32_t s, t;
    uint64_t ns;
    float loss;
    uint8_t err;  // first failing ShadowEdge::try_from check (0 = ok)
    uint8_t sub;  // which Time error text
};

const char *time_err_text(uint8_t sub) {
    switch (sub) {
        case 1: return "Unable to identify value and unit";
        case 2: return "Unit was not one of (ns|nanosecond|...|h|hr|hrs|hour|hours)";
        case 3: return "invalid digit found in string";
        default: return "The resulting value is outside of the bounds";
    }
}
uint8_t time_err_code(const char *e) {
    if (!std::strcmp(e, time_err_text(1))) return 1;
    if (!std::strcmp(e, time_err_text(2))) return 2;
    if (!std::strcmp(e, time_err_text(3))) return 3;
    return 4;
}

// ShadowEdge::try_from (mod.rs:72-111) on one parsed block, minus the id
// lookups (done once every node is known)
EdgeRec check_edge(const std::vector<KV> &b) {
    EdgeRec r{0, 0, 0, 0.f, 0, 0};
    const Val *s = get(b, "source"), *t = get(b, "target");
    if (s && s->t != VT::Int) return r.err = 1, r;
    if (!s) return r.err = 2, r;
    if (t && t->t != VT::Int) return r.err = 3, r;
    if (!t) return r.err = 4, r;
    r.s = s->i;
    r.t = t->i;
    const Val *lat = get(b, "latency");
    if (!lat) return r.err = 5, r;
    if (lat->t != VT::Str) return r.err = 6, r;
    uint64_t v = 0;
    if (const char *e = parse_time(lat->s, &r.ns, &v)) return r.err = 7, r.sub = time_err_code(e), r;
    if (const Val *j = get(b, "jitter")) {
        if (j->t != VT::Str) return r.err = 8, r;
        uint64_t jn, jv;
        if (const char *e = parse_time(j->s, &jn, &jv)) return r.err = 9, r.sub = time_err_code(e), r;
    }
    if (const Val *pl = get(b, "packet_loss")) {
        if (pl->t != VT::Float) return r.err = 10, r;
        r.loss = pl->f;
    }
    if (r.loss < 0.f || r.loss > 1.f) return r.err = 11, r;
    if (v == 0) return r.err = 12, r;
    return r;
}

std::string edge_err_text(const EdgeRec &r) {
    switch (r.err) {
        case 1: return "Incorrect 'source' type";
        case 2: return "'source' doesn't exist";
        case 3: return "Incorrect 'target' type";
        case 4: return "'target' doesn't exist";
        case 5: return "Edge 'latency' was not provided";
        case 6: return "Edge 'latency' is not a string";
        case 7: return std::string("Edge 'latency' is not a valid unit: ") + time_err_text(r.sub);
        case 8: return "Edge 'jitter' is not a string";
        case 9: return std::string("Edge 'jitter' is not a valid unit: ") + time_err_text(r.sub);
        case 10: return "Edge 'packet_loss' is not a float";
        case 11: return "Edge 'packet_loss' is not in the range [0,1]";
        case 12: return "Edge 'latency' must not be 0";
        case 13: return "Edge source " + std::to_string((uint32_t)r.s) + " doesn't exist";
        default: return "Edge target " + std::to_string((uint32_t)r.t) + " doesn't exist";
    }
}

// ShadowNode::try_from (mod.rs:28-60)
void check_node(const std::vector<KV> &n, uint32_t *id_out) {
    const Val *id = get(n, "id");
    if (id && id->t != VT::Int) throw Fail{"Incorrect 'id' type"};
    if (!id) throw Fail{"Node 'id' was not provided"};
    for (const char *bw : {"host_bandwidth_down", "host_bandwidth_up"}) {
        const Val *x = get(n, bw);
        if (!x) continue;
        if (x->t != VT::Str) throw Fail{std::string("Node '") + bw + "' is not a string"};
        if (!bits_per_sec_ok(x->s)) throw Fail{std::string("Node '") + bw + "' is not a valid unit"};
    }
    *id_out = (uint32_t)id->i;
}

template <typename F>
void parallel_for(size_t n, unsigned T, F &&f);

// petgraph adjacency: outgoing (reverse insertion), then for undirected the
// incoming list (reverse insertion, self-loops skipped).  Edges are cut into T
// contiguous chunks; per-chunk row counts give every chunk its own write
// offsets (chunk T-1 first, since the order is reverse insertion), so the
// fill runs in parallel and lands exactly where the sequential fill would.
void build_csr(srt_gml *g, size_t V, const uvec<uint32_t> &es, const uvec<uint32_t> &ed, const uvec<uint64_t> &el,
               const uvec<float> &eo, unsigned T = 1) {
    const size_t m = es.size();
    if (m < 4 * (size_t)T || T < 2) T = 1;
    const bool und = !g->directed;
    std::vector<uint64_t> co((size_t)T * V, 0), ci(und ? (size_t)T * V : 0, 0);
    parallel_for(T, T, [&](size_t b, size_t e, unsigned) {
        for (size_t t = b; t < e; ++t)
            for (size_t i = m * t / T; i < m * (t + 1) / T; ++i) {
                co[t * V + es[i]]++;
                if (und && es[i] != ed[i]) ci[t * V + ed[i]]++;
            }
    });
    g->row_ptr.assign(V + 1, 0);
    std::vector<uint64_t> out_tot(V, 0);
    for (size_t v = 0; v < V; ++v) {
        uint64_t o = 0, in = 0;
        for (unsigned t = 0; t < T; ++t) o += co[t * V + v], in += und ? ci[t * V + v] : 0;
        out_tot[v] = o;
        g->row_ptr[v + 1] = g->row_ptr[v] + o + in;
    }
    // start offsets: outgoing of chunk t in row v after the chunks t' > t
    parallel_for(V, T, [&](size_t b, size_t e, unsigned) {
        for (size_t v = b; v < e; ++v) {
            uint64_t o = g->row_ptr[v], in = g->row_ptr[v] + out_tot[v];
            for (unsigned t = T; t-- > 0;) {
                const uint64_t c = co[t * V + v];
                co[t * V + v] = o;
                o += c;
                if (und) {
                    const uint64_t d = ci[t * V + v];
                    ci[t * V + v] = in;
                    in += d;
                }
            }
        }
    });
    const size_t A = g->row_ptr[V];
    g->col.resize(A);
    g->lat.resize(A);
    g->loss.resize(A);
    parallel_for(T, T, [&](size_t b, size_t e, unsigned) {
        for (size_t t = b; t < e; ++t) {
            for (size_t i = m * (t + 1) / T; i-- > m * t / T;) {
                const uint64_t k = co[t * V + es[i]]++;
                g->col[k] = ed[i];
                g->lat[k] = el[i];
                g->loss[k] = eo[i];
            }
            if (und)
                for (size_t i = m * (t + 1) / T; i-- > m * t / T;) {
                    if (es[i] == ed[i]) continue;
                    const uint64_t k = ci[t * V + ed[i]]++;
                    g->col[k] = es[i];
                    g->lat[k] = el[i];
                    g->loss[k] = eo[i];
                }
        }
    });
}

// Sequential reference path (small inputs, and the exact error for anything
// the parallel path rejects).
void parse_sequential(std::string_view text, srt_gml *g) {
    Lexer L(text);
    L.msp0();
    if (!L.tag(std::string_view("graph"))) L.fail("expected 'graph'");
    L.sp0();
    if (!L.tag('[') || !L.newline()) L.fail("expected '[' and a newline");
    std::vector<std::vector<KV>> nodes, edges;
    std::vector<KV> others;
    int ndirected = 0;
    while (!L.tag(']')) {
        std::string_view k;
        if (!L.key(&k)) L.fail("expected a key");
        if (k == "node") {
            nodes.emplace_back();
            L.block(&nodes.back());
        } else if (k == "edge") {
            edges.emplace_back();
            L.block(&edges.back());
        } else if (k == "directed") {
            Val v;
            if (!L.value(&v)) L.fail("expected a value for 'directed'");
            if (v.t != VT::Int) L.fail("Value was not an integer");
            if (v.i != 0 && v.i != 1) L.fail("Bool must be 0 or 1");
            g->directed = v.i == 1;
            ++ndirected;
        } else {
            KV kv{k, {}};
            if (!L.value(&kv.v)) L.fail("expected a value");
            others.push_back(kv);
        }
    }
    if (ndirected > 1) L.fail("The 'directed' key must only be specified once");
    for (size_t i = 0; i < others.size(); ++i)
        for (size_t j = i + 1; j < others.size(); ++j)
            if (others[i].k == others[j].k) L.fail("Duplicate keys are not supported");

    std::unordered_map<uint32_t, uint32_t> id_map;
    id_map.reserve(nodes.size() * 2);
    g->ids.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        check_node(nodes[i], &g->ids[i]);
        id_map[g->ids[i]] = (uint32_t)i;
    }
    const size_t m = edges.size();
    uvec<uint32_t> es(m), ed(m);
    uvec<uint64_t> el(m);
    uvec<float> eo(m);
    for (size_t i = 0; i < m; ++i) {
        EdgeRec r = check_edge(edges[i]);
        if (!r.err) {
            auto si = id_map.find((uint32_t)r.s), ti = id_map.find((uint32_t)r.t);
            if (si == id_map.end()) r.err = 13;
            else if (ti == id_map.end()) r.err = 14;
            else es[i] = si->second, ed[i] = ti->second;
        }
        if (r.err) throw Fail{edge_err_text(r)};
        el[i] = r.ns;
        eo[i] = r.loss;
    }
    build_csr(g, nodes.size(), es, ed, el, eo);
}

struct Bad {};  // the parallel path gives up: re-parse sequentially

template <typename F>
void parallel_for(size_t n, unsigned T, F &&f) {  // f(begin, end, thread)
    if (T <= 1 || n < 2 * T) {
        f((size_t)0, n, 0u);
        return;
    }
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> ex(T);
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            try {
                f(n * t / T, n * (t + 1) / T, t);
            } catch (...) {
                ex[t] = std::current_exception();
            }
        });
    for (auto &x : th) x.join();
    for (auto &e : ex)
        if (e) std::rethrow_exception(e);
}

void parse_parallel(std::string_view text, srt_gml *g, unsigned T) {
    const bool timing = std::getenv("SRT_GML_TIMING") != nullptr;  // phase times to stderr
    auto t_last = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[srt_gml] %-10s %8.3f s\n", what, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
    Lexer H(text);
    H.msp0();
    if (!H.tag(std::string_view("graph"))) throw Bad{};
    H.sp0();
    if (!H.tag('[') || !H.newline()) throw Bad{};
    const size_t h = H.pos(), N = text.size();
    const char *base = text.data();
    // 1. quote parity at chunk starts
    const size_t nch = std::max<size_t>(1, std::min<size_t>(T * 8, (N - h) / (1 << 20) + 1));
    std::vector<size_t> cb(nch + 1);
    for (size_t c = 0; c <= nch; ++c) cb[c] = h + (N - h) * c / nch;
    std::vector<uint64_t> quotes(nch);
    parallel_for(nch, T, [&](size_t b, size_t e, unsigned) {
        for (size_t c = b; c < e; ++c) quotes[c] = (uint64_t)std::count(base + cb[c], base + cb[c + 1], '"');
    });
    tick("quotes");
    // 2. structural bytes ('[' / ']' outside strings) per chunk
    std::vector<std::vector<uint64_t>> st(nch);
    parallel_for(nch, T, [&](size_t b, size_t e, unsigned) {
        for (size_t c = b; c < e; ++c) {
            uint64_t q = 0;
            for (size_t k = 0; k < c; ++k) q += quotes[k];
            bool in_str = q & 1;
            const char *p = base + cb[c], *end = base + cb[c + 1];
            std::vector<uint64_t> &out = st[c];
            out.reserve((size_t)(end - p) / 32 + 16);  // ~2 structural bytes per ~90-byte block
            // 8 bytes a step: a word with none of '"' '[' ']' is skipped whole
            // (SWAR zero-byte test on the XOR with each broadcast character)
            constexpr uint64_t ONES = 0x0101010101010101ull, HIGH = 0x8080808080808080ull;
            constexpr uint64_t QQ = ONES * '"', LB = ONES * '[', RB = ONES * ']';
            auto has0 = [](uint64_t x) { return (x - ONES) & ~x & HIGH; };
            while (p < end) {
                if (end - p >= 8) {
                    uint64_t w;
                    std::memcpy(&w, p, 8);
                    if (!(has0(w ^ QQ) | has0(w ^ LB) | has0(w ^ RB))) {
                        p += 8;
                        continue;
                    }
                }
                const char *stop = std::min(p + 8, end);
                for (; p < stop; ++p) {
                    const char x = *p;
                    if (x == '"') in_str = !in_str;
                    else if (!in_str && (x == '[' || x == ']')) out.push_back((uint64_t)(p - base));
                }
            }
        }
    });
    tick("structure");
    // 3. blocks.  In valid GML the structural bytes read "[ ] [ ] ... [ ] ]":
    // block j = entries (2j, 2j+1) of the concatenated list and the graph's
    // ']' is the first even entry that is a ']' (anything after it is trailing
    // text).  Concatenate the chunk lists by prefix offsets, find that entry,
    // check the alternation before it and pair the entries, chunk-parallel.
    std::vector<size_t> off(nch + 1, 0);
    for (size_t c = 0; c < nch; ++c) off[c + 1] = off[c] + st[c].size();
    uvec<uint64_t> E(off[nch]);
    parallel_for(nch, T, [&](size_t b, size_t e, unsigned) {
        for (size_t c = b; c < e; ++c) std::copy(st[c].begin(), st[c].end(), E.begin() + (ptrdiff_t)off[c]);
    });
    st.clear();
    st.shrink_to_fit();
    std::vector<size_t> first_close(T, SIZE_MAX);
    std::vector<uint8_t> alt_bad(T, 0);
    parallel_for(E.size(), T, [&](size_t b, size_t e, unsigned t) {
        for (size_t i = b; i < e; ++i) {
            const bool is_open = base[E[i]] == '[';
            if ((i & 1) == 0 && !is_open) {
                first_close[t] = i;
                return;
            }
            if ((i & 1) == 1 && is_open) alt_bad[t] = 1;  // only matters before the graph's ']'
        }
    });
    size_t gi = SIZE_MAX;
    unsigned tg = 0;
    for (unsigned t = 0; t < T; ++t)
        if (first_close[t] < gi) gi = first_close[t], tg = t;
    if (gi == SIZE_MAX) throw Bad{};
    // a nested '[' before the graph's ']' (threads past tg only saw trailing text)
    for (unsigned t = 0; t < tg; ++t)
        if (alt_bad[t]) throw Bad{};
    for (size_t i = E.size() * tg / T; i < gi; ++i)
        if ((i & 1) == 1 && base[E[i]] == '[') throw Bad{};
    const uint64_t gend = E[gi];
    const size_t nb = gi / 2;
    uvec<std::pair<uint64_t, uint64_t>> blocks(nb);
    parallel_for(nb, T, [&](size_t b, size_t e, unsigned) {
        for (size_t j = b; j < e; ++j) blocks[j] = {E[2 * j], E[2 * j + 1]};
    });
    E.clear();
    E.shrink_to_fit();
    tick("blocks");
    // 4. parse gaps (before block i: [prev_end+1, blocks[i].first); the last
    // gap ends at the graph's ']') and blocks, in parallel
    uvec<uint8_t> kind(nb);  // 1 node, 2 edge (every gap sets its block's)
    std::vector<std::vector<KV>> gap_others(T), nodes_kv;
    std::vector<int> gap_directed(T, 0);
    std::vector<int> directed_val(T, -1);
    uvec<EdgeRec> recs;
    // gaps first (they say which blocks are nodes), in order per thread
    auto parse_gap = [&](size_t i, unsigned t) {  // gap before block i (i == nb: the tail)
        const size_t b = i == 0 ? h : blocks[i - 1].second + 1;
        const size_t e = i == nb ? gend : blocks[i].first;
        Lexer L(text, b, e);
        if (i > 0 && !L.newline()) throw Bad{};
        for (;;) {
            if (L.at_end()) {
                if (i != nb) throw Bad{};
                return;
            }
            std::string_view k;
            if (!L.key(&k)) throw Bad{};
            if (k == "node" || k == "edge") {
                L.sp0();
                if (i == nb || !L.at_end()) throw Bad{};
                kind[i] = k == "node" ? 1 : 2;
                return;
            }
            if (k == "directed") {
                Val v;
                if (!L.value(&v) || v.t != VT::Int || (v.i != 0 && v.i != 1)) throw Bad{};
                gap_directed[t]++;
                directed_val[t] = v.i;
            } else {
                KV kv{k, {}};
                if (!L.value(&kv.v)) throw Bad{};
                gap_others[t].push_back(kv);
            }
        }
    };
    parallel_for(nb + 1, T, [&](size_t b, size_t e, unsigned t) {
        for (size_t i = b; i < e; ++i) parse_gap(i, t);
    });
    int ndirected = 0;
    std::vector<KV> others;
    for (unsigned t = 0; t < T; ++t) {
        ndirected += gap_directed[t];
        if (directed_val[t] >= 0) g->directed = directed_val[t] == 1;
        others.insert(others.end(), gap_others[t].begin(), gap_others[t].end());
    }
    if (ndirected > 1) throw Bad{};
    for (size_t i = 0; i < others.size(); ++i)
        for (size_t j = i + 1; j < others.size(); ++j)
            if (others[i].k == others[j].k) throw Bad{};
    tick("gaps");
    // node / edge numbering in file order
    uvec<uint32_t> idx(nb);
    uint32_t nn = 0, ne = 0;
    for (size_t i = 0; i < nb; ++i) idx[i] = kind[i] == 1 ? nn++ : ne++;
    nodes_kv.resize(nn);
    recs.resize(ne);
    parallel_for(nb, T, [&](size_t b, size_t e, unsigned) {
        std::vector<KV> kvs;
        for (size_t i = b; i < e; ++i) {
            Lexer L(text, blocks[i].first, blocks[i].second + 1);
            kvs.clear();
            if (!L.block_body(&kvs)) throw Bad{};
            if (kind[i] == 1) nodes_kv[idx[i]] = kvs;
            else recs[idx[i]] = check_edge(kvs);
        }
    });
    tick("parse");
    // 5. validation: nodes in order, then the first failing edge
    std::unordered_map<uint32_t, uint32_t> id_map;
    id_map.reserve((size_t)nn * 2);
    g->ids.resize(nn);
    for (uint32_t i = 0; i < nn; ++i) {
        check_node(nodes_kv[i], &g->ids[i]);
        id_map[g->ids[i]] = i;
    }
    nodes_kv.clear();
    uvec<uint32_t> es(ne), ed(ne);
    uvec<uint64_t> el(ne);
    uvec<float> eo(ne);
    std::vector<size_t> first_bad(T, SIZE_MAX);
    parallel_for(ne, T, [&](size_t b, size_t e, unsigned t) {
        for (size_t i = b; i < e; ++i) {
            EdgeRec &r = recs[i];
            if (!r.err) {
                auto si = id_map.find((uint32_t)r.s), ti = id_map.find((uint32_t)r.t);
                if (si == id_map.end()) r.err = 13;
                else if (ti == id_map.end()) r.err = 14;
                else es[i] = si->second, ed[i] = ti->second;
            }
            if (r.err) {
                first_bad[t] = std::min(first_bad[t], i);
                return;
            }
            el[i] = r.ns;
            eo[i] = r.loss;
        }
    });
    const size_t fb = *std::min_element(first_bad.begin(), first_bad.end());
    if (fb != SIZE_MAX) throw Fail{edge_err_text(recs[fb])};
    recs.clear();
    recs.shrink_to_fit();
    tick("validate");
    build_csr(g, nn, es, ed, el, eo, T);
    tick("csr");
}

void do_parse(std::string_view text, srt_gml *g) {
    unsigned T = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("SRT_GML_THREADS")) T = (unsigned)std::atoi(e);
    T = std::max(1u, std::min(T, 16u));
    size_t min_bytes = 16u << 20;  // below this the sequential parser is as fast
    if (const char *e = std::getenv("SRT_GML_PAR_BYTES")) min_bytes = (size_t)std::atoll(e);
    if (text.size() < min_bytes || T == 1) return parse_sequential(text, g);
    try {
        parse_parallel(text, g, T);
    } catch (const Bad &) {
        if (std::getenv("SRT_GML_STRICT_PARALLEL")) throw Fail{"parallel ingest rejected the input"};  // tests
        *g = srt_gml();
        parse_sequential(text, g);  // the exact reference-order error
    } catch (const Fail &) {
        *g = srt_gml();
        parse_sequential(text, g);  // same error text, found in reference order
    }
}

}  // namespace

extern "C" {

srt_status srt_gml_parse(const char *text, size_t len, srt_gml **out, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!text || !out) return SRT_ERR_INVALID;
    *out = nullptr;
    srt_gml *g = new (std::nothrow) srt_gml();
    if (!g) return SRT_ERR_OOM;
    try {
        do_parse(std::string_view(text, len), g);
    } catch (const Fail &f) {
        if (err) {
            err->code = SRT_ERR_INVALID;
            std::snprintf(err->msg, sizeof err->msg, "%s", f.msg.c_str());
        }
        delete g;
        return SRT_ERR_INVALID;
    } catch (...) {
        if (err) {
            err->code = SRT_ERR_OOM;
            std::snprintf(err->msg, sizeof err->msg, "out of memory while parsing GML");
        }
        delete g;
        return SRT_ERR_OOM;
    }
    *out = g;
    return SRT_OK;
}

srt_status srt_gml_csr(const srt_gml *g, srt_csr *c) {
    if (!g || !c) return SRT_ERR_INVALID;
    c->n_nodes = (uint32_t)g->ids.size();
    c->directed = g->directed;
    c->n_adj = g->col.size();
    c->row_ptr = g->row_ptr.data();
    c->col = g->col.data();
    c->lat_ns = g->lat.data();
    c->loss = g->loss.data();
    c->node_ids = g->ids.data();
    return SRT_OK;
}

void srt_gml_free(srt_gml *g) { delete g; }

}  // extern "C"
