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
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "srt_internal.h"

struct srt_gml {
    bool directed = false;
    std::vector<uint32_t> ids;
    std::vector<uint64_t> row_ptr;
    std::vector<uint32_t> col;
    std::vector<uint64_t> lat;
    std::vector<float> loss;
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
            if (!ovf && newline()) {
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
                std::string tok(p_, (size_t)(q - p_));
                const float f = std::strtof(tok.c_str(), nullptr);
                p_ = q;
                if (newline()) {
                    v->t = VT::Float;
                    v->f = f;
                    return true;
                }
                p_ = save;
            }
        }
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
        if (u == t.first) mag = t.second;
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

void do_parse(std::string_view text, srt_gml *g) {
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
        const Val *id = get(nodes[i], "id");
        if (id && id->t != VT::Int) throw Fail{"Incorrect 'id' type"};
        if (!id) throw Fail{"Node 'id' was not provided"};
        for (const char *bw : {"host_bandwidth_down", "host_bandwidth_up"}) {
            const Val *x = get(nodes[i], bw);
            if (!x) continue;
            if (x->t != VT::Str) throw Fail{std::string("Node '") + bw + "' is not a string"};
            if (!bits_per_sec_ok(x->s)) throw Fail{std::string("Node '") + bw + "' is not a valid unit"};
        }
        g->ids[i] = (uint32_t)id->i;
        id_map[(uint32_t)id->i] = (uint32_t)i;
    }
    const size_t m = edges.size();
    std::vector<uint32_t> es(m), ed(m);
    std::vector<uint64_t> el(m);
    std::vector<float> eo(m);
    for (size_t i = 0; i < m; ++i) {
        const auto &b = edges[i];
        const Val *s = get(b, "source"), *t = get(b, "target");
        if (s && s->t != VT::Int) throw Fail{"Incorrect 'source' type"};
        if (!s) throw Fail{"'source' doesn't exist"};
        if (t && t->t != VT::Int) throw Fail{"Incorrect 'target' type"};
        if (!t) throw Fail{"'target' doesn't exist"};
        const Val *lat = get(b, "latency");
        if (!lat) throw Fail{"Edge 'latency' was not provided"};
        if (lat->t != VT::Str) throw Fail{"Edge 'latency' is not a string"};
        uint64_t ns = 0, v = 0;
        if (const char *e = parse_time(lat->s, &ns, &v)) throw Fail{std::string("Edge 'latency' is not a valid unit: ") + e};
        if (const Val *j = get(b, "jitter")) {
            if (j->t != VT::Str) throw Fail{"Edge 'jitter' is not a string"};
            uint64_t jn, jv;
            if (const char *e = parse_time(j->s, &jn, &jv)) throw Fail{std::string("Edge 'jitter' is not a valid unit: ") + e};
        }
        float loss = 0.f;
        if (const Val *pl = get(b, "packet_loss")) {
            if (pl->t != VT::Float) throw Fail{"Edge 'packet_loss' is not a float"};
            loss = pl->f;
        }
        if (loss < 0.f || loss > 1.f) throw Fail{"Edge 'packet_loss' is not in the range [0,1]"};
        if (v == 0) throw Fail{"Edge 'latency' must not be 0"};
        auto si = id_map.find((uint32_t)s->i), ti = id_map.find((uint32_t)t->i);
        if (si == id_map.end()) throw Fail{"Edge source " + std::to_string((uint32_t)s->i) + " doesn't exist"};
        if (ti == id_map.end()) throw Fail{"Edge target " + std::to_string((uint32_t)t->i) + " doesn't exist"};
        es[i] = si->second;
        ed[i] = ti->second;
        el[i] = ns;
        eo[i] = loss;
    }
    // petgraph adjacency: outgoing (reverse insertion), then for undirected the
    // incoming list (reverse insertion, self-loops skipped)
    const size_t V = nodes.size();
    g->row_ptr.assign(V + 1, 0);
    for (size_t i = 0; i < m; ++i) {
        g->row_ptr[es[i] + 1]++;
        if (!g->directed && es[i] != ed[i]) g->row_ptr[ed[i] + 1]++;
    }
    for (size_t v = 0; v < V; ++v) g->row_ptr[v + 1] += g->row_ptr[v];
    const size_t A = g->row_ptr[V];
    g->col.resize(A);
    g->lat.resize(A);
    g->loss.resize(A);
    std::vector<uint64_t> fill(g->row_ptr.begin(), g->row_ptr.end() - 1);
    for (size_t i = m; i-- > 0;) {
        const uint64_t k = fill[es[i]]++;
        g->col[k] = ed[i];
        g->lat[k] = el[i];
        g->loss[k] = eo[i];
    }
    if (!g->directed)
        for (size_t i = m; i-- > 0;) {
            if (es[i] == ed[i]) continue;
            const uint64_t k = fill[ed[i]]++;
            g->col[k] = es[i];
            g->lat[k] = el[i];
            g->loss[k] = eo[i];
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
