/*
 * srt_oracle.c -- CPU restatement of Shadow's routing-table build and packet
 * drop decision.  TEST INFRASTRUCTURE ONLY (see srt_oracle.h): the product
 * never links this file; tests/, smoke() and bench.py's cpu_baseline leg use it
 * as the checker and as the timed "port" CPU baseline.
 *
 * Build: oracle/Makefile (gcc, -ffp-contract=off so f32 path-loss arithmetic
 * is rounded op by op exactly like Rust, which never contracts to FMA).
 */
#define _GNU_SOURCE
#include "srt_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ======================================================================== */
/* RNG                                                                      */
/* ======================================================================== */

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* rand_xoshiro 0.6.0 splitmix64.rs: SplitMix64::next_u64 */
uint64_t or_splitmix64_next(uint64_t *state) {
    *state += 0x9e3779b97f4a7c15ULL;
    uint64_t z = *state;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* rand_xoshiro 0.6.0 xoshiro256plusplus.rs: seed_from_u64 = SplitMix64(seed),
 * from_rng fills the 32-byte seed with four successive next_u64 (LE), so
 * s[i] = i-th splitmix output. */
void or_xoshiro_seed_from_u64(uint64_t seed, uint64_t s[4]) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) s[i] = or_splitmix64_next(&x);
}

/* rand_xoshiro 0.6.0 xoshiro256plusplus.rs: next_u64 */
uint64_t or_xoshiro_next(uint64_t s[4]) {
    const uint64_t result = rotl64(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return result;
}

/* rand 0.8.5 distributions/float.rs: Standard for f64 = (u64 >> 11) * 2^-53 */
double or_gen_f64(uint64_t s[4]) {
    const uint64_t v = or_xoshiro_next(s);
    return (double)(v >> 11) * (1.0 / (double)(1ULL << 53));
}

/* SipHash-c-d with keys (0,0); c=1,d=3 is std's DefaultHasher (SipHasher13).
 * c=2,d=4 is exposed for validating against the published SipHash-2-4 vector. */
#define SIPROUND                                                                      \
    do {                                                                              \
        v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);                \
        v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                                      \
        v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                                      \
        v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);                \
    } while (0)

uint64_t or_siphash_cd(const uint8_t *m, size_t len, uint64_t k0, uint64_t k1, int c, int d) {
    uint64_t v0 = k0 ^ 0x736f6d6570736575ULL, v1 = k1 ^ 0x646f72616e646f6dULL;
    uint64_t v2 = k0 ^ 0x6c7967656e657261ULL, v3 = k1 ^ 0x7465646279746573ULL;
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t w = 0;
        for (int b = 0; b < 8; b++) w |= (uint64_t)m[i + b] << (8 * b);
        v3 ^= w;
        for (int r = 0; r < c; r++) SIPROUND;
        v0 ^= w;
    }
    uint64_t b = (uint64_t)(len & 0xff) << 56;
    for (size_t j = 0; i + j < len; j++) b |= (uint64_t)m[i + j] << (8 * j);
    v3 ^= b;
    for (int r = 0; r < c; r++) SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    for (int r = 0; r < d; r++) SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

/* std 1.76: <str as Hash>::hash -> Hasher::write_str = write(bytes) + write_u8(0xff);
 * DefaultHasher::new() = SipHasher13 with keys (0, 0). */
uint64_t or_siphash13_str(const uint8_t *bytes, size_t len) {
    uint8_t stackbuf[256];
    uint8_t *buf = len + 1 <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(len + 1);
    memcpy(buf, bytes, len);
    buf[len] = 0xff;
    const uint64_t h = or_siphash_cd(buf, len + 1, 0, 0, 1, 3);
    if (buf != stackbuf) free(buf);
    return h;
}

/* sim_config.rs:49-53 (R = first u64 of seed_from_u64(general.seed)) and
 * sim_config.rs:222-227, 244 (seed = R ^ hash(hostname)). */
uint64_t or_host_seed(uint32_t general_seed, const char *hostname) {
    uint64_t s[4];
    or_xoshiro_seed_from_u64((uint64_t)general_seed, s);
    const uint64_t r = or_xoshiro_next(s);
    return r ^ or_siphash13_str((const uint8_t *)hostname, strlen(hostname));
}

/* ======================================================================== */
/* units.rs: Time<TimePrefix>::from_str + convert(Nano)                      */
/* ======================================================================== */

static void set_err(char *err, size_t errlen, const char *fmt, const char *a) {
    if (err && errlen) snprintf(err, errlen, fmt, a ? a : "");
}

/* Rust char::is_whitespace for the ASCII range plus the common Unicode spaces
 * that can appear in UTF-8 GML text. Returns the byte length of the whitespace
 * char at p (0 if none). */
static size_t ws_len(const unsigned char *p, const unsigned char *end) {
    if (p >= end) return 0;
    if (*p == ' ' || (*p >= 0x09 && *p <= 0x0d)) return 1;
    if (*p == 0xc2 && p + 1 < end && (p[1] == 0x85 || p[1] == 0xa0)) return 2;
    if (*p == 0xe3 && p + 2 < end && p[1] == 0x80 && p[2] == 0x80) return 3;
    if (*p == 0xe2 && p + 2 < end) {
        if (p[1] == 0x80 && ((p[2] >= 0x80 && p[2] <= 0x8a) || p[2] == 0xa8 || p[2] == 0xa9 ||
                             p[2] == 0xaf))
            return 3;
        if (p[1] == 0x81 && p[2] == 0x9f) return 3;
    }
    if (*p == 0xe1 && p + 2 < end && p[1] == 0x9a && p[2] == 0x80) return 3;
    return 0;
}

static void trim(const char **b, const char **e) {
    const unsigned char *p = (const unsigned char *)*b, *q = (const unsigned char *)*e;
    size_t k;
    while (p < q && (k = ws_len(p, q)) > 0) p += k;
    /* trailing: check the last 1..3 bytes */
    for (;;) {
        int found = 0;
        for (size_t l = 1; l <= 3 && l <= (size_t)(q - p); l++)
            if (ws_len(q - l, q) == l) { q -= l; found = 1; break; }
        if (!found) break;
    }
    *b = (const char *)p;
    *e = (const char *)q;
}

static int seq_eq(const char *b, const char *e, const char *lit) {
    size_t n = strlen(lit);
    return (size_t)(e - b) == n && memcmp(b, lit, n) == 0;
}

/* Rust <u64 as FromStr>: optional '+', then >=1 ASCII digits, no overflow. */
static int parse_u64_rust(const char *b, const char *e, uint64_t *out) {
    if (b < e && *b == '+') b++;
    if (b >= e) return -1;
    uint64_t v = 0;
    for (; b < e; b++) {
        if (*b < '0' || *b > '9') return -1;
        uint64_t d = (uint64_t)(*b - '0');
        if (v > (UINT64_MAX - d) / 10) return -1;
        v = v * 10 + d;
    }
    *out = v;
    return 0;
}

/* magnitude of a TimePrefix relative to ns (units.rs:264-280) */
static int time_prefix_ns(const char *b, const char *e, uint64_t *mag) {
    if (b == e) { *mag = 1000000000ULL; return 0; } /* default = Sec (units.rs:227-231) */
    static const struct { const char *s; uint64_t m; } tab[] = {
        {"ns", 1ULL}, {"nanosecond", 1ULL}, {"nanoseconds", 1ULL},
        {"us", 1000ULL}, {"\xce\xbcs", 1000ULL}, {"microsecond", 1000ULL}, {"microseconds", 1000ULL},
        {"ms", 1000000ULL}, {"millisecond", 1000000ULL}, {"milliseconds", 1000000ULL},
        {"s", 1000000000ULL}, {"sec", 1000000000ULL}, {"secs", 1000000000ULL},
        {"second", 1000000000ULL}, {"seconds", 1000000000ULL},
        {"m", 60000000000ULL}, {"min", 60000000000ULL}, {"mins", 60000000000ULL},
        {"minute", 60000000000ULL}, {"minutes", 60000000000ULL},
        {"h", 3600000000000ULL}, {"hr", 3600000000000ULL}, {"hrs", 3600000000000ULL},
        {"hour", 3600000000000ULL}, {"hours", 3600000000000ULL},
    };
    for (size_t i = 0; i < sizeof tab / sizeof tab[0]; i++)
        if (seq_eq(b, e, tab[i].s)) { *mag = tab[i].m; return 0; }
    return -1;
}

/* regex ^([+-]?[0-9\.]*)\s*(.*)$  then trim both groups (units.rs:411-418).
 * `.` does not match '\n' and `$` is end-of-text, so a '\n' left in group 2
 * means "Unable to identify value and unit". */
static int split_value_unit(const char *s, size_t len, const char **vb, const char **ve,
                            const char **ub, const char **ue) {
    const char *p = s, *end = s + len;
    const char *g1 = p;
    if (p < end && (*p == '+' || *p == '-')) p++;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.')) p++;
    const char *g1e = p;
    size_t k;
    while (p < end && (k = ws_len((const unsigned char *)p, (const unsigned char *)end)) > 0) p += k;
    for (const char *q = p; q < end; q++)
        if (*q == '\n') return -1;
    *vb = g1; *ve = g1e; *ub = p; *ue = end;
    trim(vb, ve);
    trim(ub, ue);
    return 0;
}

int or_parse_time_ns(const char *s, size_t len, uint64_t *ns_out, uint64_t *value_out, char *err,
                     size_t errlen) {
    const char *vb, *ve, *ub, *ue;
    if (split_value_unit(s, len, &vb, &ve, &ub, &ue) != 0) {
        set_err(err, errlen, "Unable to identify value and unit", NULL);
        return OR_ERR_PARSE;
    }
    uint64_t mag, v;
    if (time_prefix_ns(ub, ue, &mag) != 0) {
        set_err(err, errlen,
                "Unit was not one of (ns|nanosecond|nanoseconds|us|\xce\xbcs|microsecond|"
                "microseconds|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|mins|"
                "minute|minutes|h|hr|hrs|hour|hours)",
                NULL);
        return OR_ERR_PARSE;
    }
    if (parse_u64_rust(vb, ve, &v) != 0) {
        set_err(err, errlen, "invalid digit found in string", NULL);
        return OR_ERR_PARSE;
    }
    if (value_out) *value_out = v;
    /* convert(Nano): checked_mul (units.rs:377-388) */
    if (mag != 0 && v > UINT64_MAX / mag) {
        set_err(err, errlen, "The resulting value is outside of the bounds [0, 18446744073709551615]",
                NULL);
        return OR_ERR_PARSE;
    }
    if (ns_out) *ns_out = v * mag;
    return OR_OK;
}

/* BitsPerSec<SiPrefixUpper> validation (mod.rs:34-57; units.rs:143-176, 578) */
static int parse_bits_per_sec_ok(const char *s, size_t len) {
    const char *vb, *ve, *ub, *ue;
    if (split_value_unit(s, len, &vb, &ve, &ub, &ue) != 0) return -1;
    /* strip the first matching suffix of ["bit", "bits"] */
    size_t ul = (size_t)(ue - ub);
    if (ul >= 3 && memcmp(ue - 3, "bit", 3) == 0) ue -= 3;
    else if (ul >= 4 && memcmp(ue - 4, "bits", 4) == 0) ue -= 4;
    if (ub != ue) {
        static const char *ok[] = {"K", "kilo", "Ki", "kibi", "M", "mega", "Mi", "mebi",
                                   "G", "giga", "Gi", "gibi", "T", "tera", "Ti", "tebi"};
        int found = 0;
        for (size_t i = 0; i < sizeof ok / sizeof ok[0]; i++)
            if (seq_eq(ub, ue, ok[i])) found = 1;
        if (!found) return -1;
    }
    uint64_t v;
    return parse_u64_rust(vb, ve, &v);
}

/* ======================================================================== */
/* GML grammar (gml-parser/src/parser.rs)                                    */
/* ======================================================================== */

enum { V_INT = 0, V_FLOAT = 1, V_STR = 2 };
typedef struct {
    const char *kb, *ke; /* key */
    int type;
    int32_t i;
    float f;
    const char *sb, *se; /* string payload (no escapes are ever transformed, see below) */
} kv_t;

typedef struct {
    const char *p, *end;
    int failed;
    char msg[200];
} lexer;

static void lx_fail(lexer *L, const char *m) {
    if (!L->failed) {
        L->failed = 1;
        snprintf(L->msg, sizeof L->msg, "%s at byte %ld", m, (long)(L->end - L->p));
    }
}

static int is_sp(char c) { return c == ' ' || c == '\t'; }
static int is_msp(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

/* space0 */
static void sp0(lexer *L) { while (L->p < L->end && is_sp(*L->p)) L->p++; }
/* multispace0 */
static void msp0(lexer *L) { while (L->p < L->end && is_msp(*L->p)) L->p++; }
/* newline = space0 multispace1 space0 (parser.rs:252-254) */
static int newline(lexer *L) {
    sp0(L);
    if (L->p >= L->end || !is_msp(*L->p)) return -1;
    while (L->p < L->end && is_msp(*L->p)) L->p++;
    sp0(L);
    return 0;
}
static int tag(lexer *L, const char *t) {
    size_t n = strlen(t);
    if ((size_t)(L->end - L->p) < n || memcmp(L->p, t, n) != 0) return -1;
    L->p += n;
    return 0;
}
static int is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
static int is_digit(char c) { return c >= '0' && c <= '9'; }
/* key: [a-zA-Z_][a-zA-Z0-9_]* (parser.rs:45-51) */
static int key(lexer *L, const char **kb, const char **ke) {
    if (L->p >= L->end || !(is_alpha(*L->p) || *L->p == '_')) return -1;
    *kb = L->p++;
    while (L->p < L->end && (is_alpha(*L->p) || is_digit(*L->p) || *L->p == '_')) L->p++;
    *ke = L->p;
    return 0;
}

/* value = space0, alt((int newline), (float newline), (string newline)) (parser.rs:214-224)
 * returns 0 ok, -1 recoverable error, -2 hard failure (nom::Err::Failure from cut). */
static int value(lexer *L, kv_t *kv) {
    sp0(L);
    const char *save = L->p;
    /* int: digit1 -> i32 parse; overflow -> map_res error -> next alternative */
    if (L->p < L->end && is_digit(*L->p)) {
        const char *b = L->p;
        while (L->p < L->end && is_digit(*L->p)) L->p++;
        int64_t v = 0;
        int ovf = 0;
        for (const char *q = b; q < L->p; q++) {
            v = v * 10 + (*q - '0');
            if (v > INT32_MAX) { ovf = 1; break; }
        }
        if (!ovf && newline(L) == 0) {
            kv->type = V_INT;
            kv->i = (int32_t)v;
            return 0;
        }
        L->p = save;
    }
    /* float: nom recognize_float then <f32 as FromStr> */
    {
        const char *b = L->p, *q = L->p;
        if (q < L->end && (*q == '+' || *q == '-')) q++;
        int ok = 0;
        if (q < L->end && is_digit(*q)) {
            while (q < L->end && is_digit(*q)) q++;
            if (q < L->end && *q == '.') {
                q++;
                while (q < L->end && is_digit(*q)) q++;
            }
            ok = 1;
        } else if (q < L->end && *q == '.' && q + 1 < L->end && is_digit(q[1])) {
            q++;
            while (q < L->end && is_digit(*q)) q++;
            ok = 1;
        }
        if (ok) {
            if (q < L->end && (*q == 'e' || *q == 'E')) {
                q++;
                if (q < L->end && (*q == '+' || *q == '-')) q++;
                if (!(q < L->end && is_digit(*q))) { /* cut(digit1) */
                    lx_fail(L, "expected exponent digits");
                    return -2;
                }
                while (q < L->end && is_digit(*q)) q++;
            }
            char buf[128];
            size_t n = (size_t)(q - b);
            if (n < sizeof buf) {
                memcpy(buf, b, n);
                buf[n] = 0;
                errno = 0;
                float f = strtof(buf, NULL); /* glibc strtof is correctly rounded, like Rust */
                L->p = q;
                if (newline(L) == 0) {
                    kv->type = V_FLOAT;
                    kv->f = f;
                    return 0;
                }
            }
            L->p = save;
        }
    }
    /* string: '"' escaped_transform(is_not("\""), '\\', ...) '"'.  is_not("\"")
     * swallows backslashes itself, so the transform never fires; an empty
     * string fails (escaped_transform errors at index 0). */
    if (L->p < L->end && *L->p == '"') {
        const char *b = L->p + 1, *q = b;
        while (q < L->end && *q != '"') q++;
        if (q > b && q < L->end) {
            L->p = q + 1;
            if (newline(L) == 0) {
                kv->type = V_STR;
                kv->sb = b;
                kv->se = q;
                return 0;
            }
        }
        L->p = save;
    }
    return -1;
}

typedef struct {
    kv_t *v;
    size_t n, cap;
} kvvec;

static void kv_push(kvvec *a, kv_t x) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 8;
        a->v = (kv_t *)realloc(a->v, a->cap * sizeof(kv_t));
    }
    a->v[a->n++] = x;
}

static int kv_dup(const kvvec *a) {
    for (size_t i = 0; i < a->n; i++)
        for (size_t j = i + 1; j < a->n; j++)
            if (a->v[i].ke - a->v[i].kb == a->v[j].ke - a->v[j].kb &&
                memcmp(a->v[i].kb, a->v[j].kb, (size_t)(a->v[i].ke - a->v[i].kb)) == 0)
                return 1;
    return 0;
}

static const kv_t *kv_get(const kvvec *a, const char *k) {
    for (size_t i = 0; i < a->n; i++)
        if (seq_eq(a->v[i].kb, a->v[i].ke, k)) return &a->v[i];
    return NULL;
}

/* node/edge body: space0 '[' newline many_till((key value), ']') newline */
static int block(lexer *L, kvvec *kvs) {
    sp0(L);
    if (tag(L, "[") || newline(L)) return -1;
    for (;;) {
        if (tag(L, "]") == 0) break;
        kv_t kv;
        memset(&kv, 0, sizeof kv);
        if (key(L, &kv.kb, &kv.ke)) return -1;
        int r = value(L, &kv);
        if (r) return r;
        kv_push(kvs, kv);
    }
    if (kv_dup(kvs)) {
        lx_fail(L, "Duplicate keys are not supported");
        return -2;
    }
    if (newline(L)) return -1;
    return 0;
}

struct or_graph {
    int directed;
    uint32_t n_nodes, n_edges;
    uint32_t *ids;
    uint32_t *esrc, *edst;
    uint64_t *elat;
    float *eloss;
    /* id -> index (open addressing, last insert wins) */
    uint32_t hcap;
    uint32_t *hkey;
    int64_t *hval;
};

static uint32_t hmix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

int64_t or_graph_index_of(const or_graph *g, uint32_t id) {
    uint32_t m = g->hcap - 1, h = hmix(id) & m;
    while (g->hval[h] >= 0) {
        if (g->hkey[h] == id) return g->hval[h];
        h = (h + 1) & m;
    }
    return -1;
}

static void id_insert(or_graph *g, uint32_t id, int64_t idx) {
    uint32_t m = g->hcap - 1, h = hmix(id) & m;
    while (g->hval[h] >= 0 && g->hkey[h] != id) h = (h + 1) & m;
    g->hkey[h] = id;
    g->hval[h] = idx;
}

void or_graph_free(or_graph *g) {
    if (!g) return;
    free(g->ids); free(g->esrc); free(g->edst); free(g->elat); free(g->eloss);
    free(g->hkey); free(g->hval);
    free(g);
}

/* NetworkGraph::parse (mod.rs:134-181) on top of gml_parser::parse (parser.rs:68-150) */
or_graph *or_gml_parse(const char *text, size_t len, char *err, size_t errlen) {
    lexer L = {text, text + len, 0, {0}};
    kvvec nodes_kv = {0}, edges_kv = {0};
    size_t *node_off = NULL, *edge_off = NULL, nn = 0, ne = 0, ncap = 0, ecap = 0;
    int ndirected = 0, directed = 0;
    kvvec others = {0};
    or_graph *g = NULL;

    msp0(&L);
    if (tag(&L, "graph")) { lx_fail(&L, "expected 'graph'"); goto fail; }
    sp0(&L);
    if (tag(&L, "[") || newline(&L)) { lx_fail(&L, "expected '[' and newline"); goto fail; }
    for (;;) {
        if (tag(&L, "]") == 0) break;
        const char *kb, *ke;
        if (key(&L, &kb, &ke)) { lx_fail(&L, "expected key"); goto fail; }
        if (seq_eq(kb, ke, "node") || seq_eq(kb, ke, "edge")) {
            int is_node = kb[0] == 'n';
            kvvec *dst = is_node ? &nodes_kv : &edges_kv;
            size_t start = dst->n;
            kvvec tmp = {0};
            int r = block(&L, &tmp);
            if (r) { free(tmp.v); lx_fail(&L, "malformed node/edge"); goto fail; }
            for (size_t i = 0; i < tmp.n; i++) kv_push(dst, tmp.v[i]);
            free(tmp.v);
            if (is_node) {
                if (nn + 2 > ncap) { ncap = ncap ? ncap * 2 : 64; node_off = realloc(node_off, ncap * sizeof(size_t)); }
                node_off[nn] = start;
                node_off[++nn] = dst->n;
            } else {
                if (ne + 2 > ecap) { ecap = ecap ? ecap * 2 : 64; edge_off = realloc(edge_off, ecap * sizeof(size_t)); }
                edge_off[ne] = start;
                edge_off[++ne] = dst->n;
            }
        } else if (seq_eq(kb, ke, "directed")) {
            /* int_as_bool (parser.rs:264-273) */
            kv_t kv;
            memset(&kv, 0, sizeof kv);
            int r = value(&L, &kv);
            if (r) { lx_fail(&L, "bad 'directed' value"); goto fail; }
            if (kv.type != V_INT) { lx_fail(&L, "Value was not an integer"); goto fail; }
            if (kv.i != 0 && kv.i != 1) { lx_fail(&L, "Bool must be 0 or 1"); goto fail; }
            directed = kv.i;
            ndirected++;
        } else {
            kv_t kv;
            memset(&kv, 0, sizeof kv);
            kv.kb = kb; kv.ke = ke;
            if (value(&L, &kv)) { lx_fail(&L, "bad value"); goto fail; }
            kv_push(&others, kv);
        }
    }
    if (ndirected > 1) { lx_fail(&L, "The 'directed' key must only be specified once"); goto fail; }
    if (kv_dup(&others)) { lx_fail(&L, "Duplicate keys are not supported"); goto fail; }

    g = (or_graph *)calloc(1, sizeof *g);
    g->directed = directed;
    g->n_nodes = (uint32_t)nn;
    g->n_edges = (uint32_t)ne;
    g->ids = (uint32_t *)calloc(nn ? nn : 1, sizeof(uint32_t));
    g->hcap = 16;
    while (g->hcap < 2 * nn + 16) g->hcap <<= 1;
    g->hkey = (uint32_t *)calloc(g->hcap, sizeof(uint32_t));
    g->hval = (int64_t *)malloc(g->hcap * sizeof(int64_t));
    for (uint32_t i = 0; i < g->hcap; i++) g->hval[i] = -1;

    /* ShadowNode::try_from (mod.rs:28-60), in GML order */
    for (size_t i = 0; i < nn; i++) {
        kvvec b = {nodes_kv.v + node_off[i], node_off[i + 1] - node_off[i], 0};
        const kv_t *id = kv_get(&b, "id");
        if (id && id->type != V_INT) { set_err(err, errlen, "Incorrect 'id' type", NULL); goto fail_g; }
        if (!id) { set_err(err, errlen, "Node 'id' was not provided", NULL); goto fail_g; }
        const char *bw[2] = {"host_bandwidth_down", "host_bandwidth_up"};
        for (int k = 0; k < 2; k++) {
            const kv_t *x = kv_get(&b, bw[k]);
            if (!x) continue;
            if (x->type != V_STR) { set_err(err, errlen, "Node '%s' is not a string", bw[k]); goto fail_g; }
            if (parse_bits_per_sec_ok(x->sb, (size_t)(x->se - x->sb))) {
                set_err(err, errlen, "Node '%s' is not a valid unit", bw[k]);
                goto fail_g;
            }
        }
        g->ids[i] = (uint32_t)id->i;
        id_insert(g, (uint32_t)id->i, (int64_t)i);
    }

    g->esrc = (uint32_t *)malloc((ne ? ne : 1) * sizeof(uint32_t));
    g->edst = (uint32_t *)malloc((ne ? ne : 1) * sizeof(uint32_t));
    g->elat = (uint64_t *)malloc((ne ? ne : 1) * sizeof(uint64_t));
    g->eloss = (float *)malloc((ne ? ne : 1) * sizeof(float));
    /* ShadowEdge::try_from (mod.rs:72-111) then id lookup (mod.rs:164-175) */
    for (size_t i = 0; i < ne; i++) {
        kvvec b = {edges_kv.v + edge_off[i], edge_off[i + 1] - edge_off[i], 0};
        const kv_t *s = kv_get(&b, "source"), *t = kv_get(&b, "target");
        if (s && s->type != V_INT) { set_err(err, errlen, "Incorrect 'source' type", NULL); goto fail_g; }
        if (!s) { set_err(err, errlen, "'source' doesn't exist", NULL); goto fail_g; }
        if (t && t->type != V_INT) { set_err(err, errlen, "Incorrect 'target' type", NULL); goto fail_g; }
        if (!t) { set_err(err, errlen, "'target' doesn't exist", NULL); goto fail_g; }
        const kv_t *lat = kv_get(&b, "latency");
        if (!lat) { set_err(err, errlen, "Edge 'latency' was not provided", NULL); goto fail_g; }
        if (lat->type != V_STR) { set_err(err, errlen, "Edge 'latency' is not a string", NULL); goto fail_g; }
        uint64_t ns = 0, v = 0;
        char uerr[200];
        if (or_parse_time_ns(lat->sb, (size_t)(lat->se - lat->sb), &ns, &v, uerr, sizeof uerr)) {
            /* value() accepted in units but convert() overflow panics in the reference
             * (mod.rs:336 unwrap); parse errors are Err strings.  Both are errors here. */
            set_err(err, errlen, "Edge 'latency' is not a valid unit: %s", uerr);
            goto fail_g;
        }
        const kv_t *jit = kv_get(&b, "jitter");
        if (jit) {
            if (jit->type != V_STR) { set_err(err, errlen, "Edge 'jitter' is not a string", NULL); goto fail_g; }
            uint64_t jv;
            if (or_parse_time_ns(jit->sb, (size_t)(jit->se - jit->sb), NULL, &jv, uerr, sizeof uerr)) {
                set_err(err, errlen, "Edge 'jitter' is not a valid unit: %s", uerr);
                goto fail_g;
            }
        }
        float loss = 0.0f;
        const kv_t *pl = kv_get(&b, "packet_loss");
        if (pl) {
            if (pl->type != V_FLOAT) { set_err(err, errlen, "Edge 'packet_loss' is not a float", NULL); goto fail_g; }
            loss = pl->f;
        }
        if (loss < 0.0f || loss > 1.0f) {
            set_err(err, errlen, "Edge 'packet_loss' is not in the range [0,1]", NULL);
            goto fail_g;
        }
        if (v == 0) { set_err(err, errlen, "Edge 'latency' must not be 0", NULL); goto fail_g; }
        int64_t si = or_graph_index_of(g, (uint32_t)s->i), ti = or_graph_index_of(g, (uint32_t)t->i);
        char idbuf[32];
        if (si < 0) { snprintf(idbuf, sizeof idbuf, "%u", (uint32_t)s->i); set_err(err, errlen, "Edge source %s doesn't exist", idbuf); goto fail_g; }
        if (ti < 0) { snprintf(idbuf, sizeof idbuf, "%u", (uint32_t)t->i); set_err(err, errlen, "Edge target %s doesn't exist", idbuf); goto fail_g; }
        g->esrc[i] = (uint32_t)si;
        g->edst[i] = (uint32_t)ti;
        g->elat[i] = ns;
        g->eloss[i] = loss;
    }
    free(nodes_kv.v); free(edges_kv.v); free(others.v); free(node_off); free(edge_off);
    return g;

fail:
    set_err(err, errlen, "%s", L.failed ? L.msg : "GML syntax error");
fail_g:
    or_graph_free(g);
    free(nodes_kv.v); free(edges_kv.v); free(others.v); free(node_off); free(edge_off);
    return NULL;
}

int or_graph_directed(const or_graph *g) { return g->directed; }
uint32_t or_graph_num_nodes(const or_graph *g) { return g->n_nodes; }
uint32_t or_graph_num_edges(const or_graph *g) { return g->n_edges; }
void or_graph_node_ids(const or_graph *g, uint32_t *ids) { memcpy(ids, g->ids, g->n_nodes * sizeof(uint32_t)); }
void or_graph_edges(const or_graph *g, uint32_t *src, uint32_t *dst, uint64_t *lat, float *loss) {
    memcpy(src, g->esrc, g->n_edges * sizeof(uint32_t));
    memcpy(dst, g->edst, g->n_edges * sizeof(uint32_t));
    memcpy(lat, g->elat, g->n_edges * sizeof(uint64_t));
    memcpy(loss, g->eloss, g->n_edges * sizeof(float));
}

/* ======================================================================== */
/* PathProperties algebra (mod.rs:296-340)                                   */
/* ======================================================================== */

typedef struct {
    uint64_t lat;
    float loss;
} pp_t;

/* Add (mod.rs:322-331): u64 wrapping add (release build), f32 ops rounded one by one */
static inline pp_t pp_add(pp_t a, pp_t b) {
    pp_t r;
    r.lat = a.lat + b.lat;
    /* built with -ffp-contract=off: three separately rounded f32 ops, as in Rust */
    const float oa = 1.0f - a.loss;
    const float ob = 1.0f - b.loss;
    const float prod = oa * ob;
    r.loss = 1.0f - prod;
    return r;
}

/* PartialOrd (mod.rs:305-313): latency, then partial_cmp of loss */
static inline int pp_lt(pp_t a, pp_t b) {
    if (a.lat != b.lat) return a.lat < b.lat;
    return a.loss < b.loss;
}

void or_path_add(uint64_t la, float pa, uint64_t lb, float pb, uint64_t *lo, float *po) {
    pp_t a = {la, pa}, b = {lb, pb};
    pp_t r = pp_add(a, b);
    *lo = r.lat;
    *po = r.loss;
}

/* ======================================================================== */
/* adjacency in petgraph iteration order                                     */
/* ======================================================================== */

typedef struct {
    uint32_t n;
    uint32_t *ptr;  /* n+1 */
    uint32_t *nbr;  /* target of the EdgeReference as seen from the row node */
    uint32_t *eid;  /* GML edge index */
} adj_t;

/* petgraph Graph::edges(a): Directed -> outgoing list; Undirected -> outgoing
 * list then incoming list with self-loops skipped (petgraph 0.6.4 graph_impl
 * Edges::next).  add_edge prepends, so each list is in reverse insertion order. */
static void build_adj(const or_edge_list *g, adj_t *A) {
    uint32_t n = g->n_nodes;
    A->n = n;
    A->ptr = (uint32_t *)calloc((size_t)n + 1, sizeof(uint32_t));
    for (uint32_t e = 0; e < g->n_edges; e++) {
        A->ptr[g->src[e] + 1]++;
        if (!g->directed && g->src[e] != g->dst[e]) A->ptr[g->dst[e] + 1]++;
    }
    for (uint32_t i = 0; i < n; i++) A->ptr[i + 1] += A->ptr[i];
    size_t m = A->ptr[n];
    A->nbr = (uint32_t *)malloc((m ? m : 1) * sizeof(uint32_t));
    A->eid = (uint32_t *)malloc((m ? m : 1) * sizeof(uint32_t));
    uint32_t *fill = (uint32_t *)malloc(((size_t)n + 1) * sizeof(uint32_t));
    memcpy(fill, A->ptr, ((size_t)n + 1) * sizeof(uint32_t));
    /* outgoing, reverse insertion order */
    for (int64_t e = (int64_t)g->n_edges - 1; e >= 0; e--) {
        uint32_t s = g->src[e];
        A->nbr[fill[s]] = g->dst[e];
        A->eid[fill[s]++] = (uint32_t)e;
    }
    if (!g->directed) {
        for (int64_t e = (int64_t)g->n_edges - 1; e >= 0; e--) {
            uint32_t t = g->dst[e];
            if (g->src[e] == t) continue;
            A->nbr[fill[t]] = g->src[e];
            A->eid[fill[t]++] = (uint32_t)e;
        }
    }
    free(fill);
}

static void free_adj(adj_t *A) { free(A->ptr); free(A->nbr); free(A->eid); }

/* ======================================================================== */
/* petgraph 0.6.4 algo::dijkstra restated                                    */
/* ======================================================================== */
/*
 *   scores.insert(start, zero); visit_next.push(MinScored(zero, start));
 *   while let Some(MinScored(node_score, node)) = visit_next.pop() {
 *       if visited.is_visited(&node) { continue; }
 *       for edge in graph.edges(node) {
 *           let next = edge.target();
 *           if visited.is_visited(&next) { continue; }
 *           let next_score = node_score + edge_cost(edge);
 *           match scores.entry(next) {
 *               Occupied(ent) => if next_score < *ent.get() { *ent = next_score; push }
 *               Vacant(ent)   => { ent.insert(next_score); push }
 *           }
 *       }
 *       visited.visit(node);
 *   }
 */

typedef struct {
    uint64_t lat;
    float loss;
    uint32_t node;
} heap_item;

typedef struct {
    heap_item *a;
    size_t n, cap;
} heap_t;

/* MinScored ordering: smaller score pops first */
static inline int h_less(const heap_item *x, const heap_item *y) {
    pp_t a = {x->lat, x->loss}, b = {y->lat, y->loss};
    return pp_lt(a, b);
}

static void h_push(heap_t *h, heap_item it) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 64;
        h->a = (heap_item *)realloc(h->a, h->cap * sizeof(heap_item));
    }
    size_t i = h->n++;
    while (i > 0) {
        size_t p = (i - 1) / 2;
        if (!h_less(&it, &h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = it;
}

static heap_item h_pop(heap_t *h) {
    heap_item top = h->a[0];
    heap_item last = h->a[--h->n];
    size_t i = 0, n = h->n;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        const heap_item *best = &last;
        if (l < n && h_less(&h->a[l], best)) { m = l; best = &h->a[l]; }
        if (r < n && h_less(&h->a[r], best)) { m = r; best = &h->a[r]; }
        if (m == i) break;
        h->a[i] = h->a[m];
        i = m;
    }
    if (n) h->a[i] = last;
    return top;
}

/* open-addressing map u32 -> pp_t (stands in for the std HashMap of scores) */
typedef struct {
    uint32_t cap, n;
    uint32_t *key;
    pp_t *val;
    uint8_t *used;
} smap;

static void sm_init(smap *m, uint32_t cap) {
    m->cap = 16;
    while (m->cap < cap) m->cap <<= 1;
    m->n = 0;
    m->key = (uint32_t *)malloc(m->cap * sizeof(uint32_t));
    m->val = (pp_t *)malloc(m->cap * sizeof(pp_t));
    m->used = (uint8_t *)calloc(m->cap, 1);
}
static void sm_free(smap *m) { free(m->key); free(m->val); free(m->used); }
static pp_t *sm_find_or_insert(smap *m, uint32_t k, int *inserted);
static void sm_grow(smap *m) {
    smap o = *m;
    sm_init(m, o.cap * 2);
    for (uint32_t i = 0; i < o.cap; i++)
        if (o.used[i]) {
            int ins;
            *sm_find_or_insert(m, o.key[i], &ins) = o.val[i];
        }
    sm_free(&o);
}
static pp_t *sm_find_or_insert(smap *m, uint32_t k, int *inserted) {
    if (2 * (m->n + 1) > m->cap) sm_grow(m);
    uint32_t mask = m->cap - 1, h = hmix(k) & mask;
    while (m->used[h]) {
        if (m->key[h] == k) { *inserted = 0; return &m->val[h]; }
        h = (h + 1) & mask;
    }
    m->used[h] = 1;
    m->key[h] = k;
    m->n++;
    *inserted = 1;
    return &m->val[h];
}

/* ---- faithful (mode 0) per-source run: hash-map scores ---- */
typedef struct {
    /* per-source output map (dst node index -> pp) filtered by nodes.contains */
    uint32_t cnt;
    uint32_t *dst;
    pp_t *pp;
} src_result;

static void dijkstra_hashmap(const adj_t *A, const or_edge_list *g, uint32_t src, smap *scores,
                             uint8_t *visited, heap_t *heap) {
    memset(visited, 0, A->n);
    heap->n = 0;
    int ins;
    pp_t zero = {0, 0.0f};
    *sm_find_or_insert(scores, src, &ins) = zero;
    h_push(heap, (heap_item){0, 0.0f, src});
    while (heap->n) {
        heap_item it = h_pop(heap);
        uint32_t node = it.node;
        if (visited[node]) continue;
        pp_t ns = {it.lat, it.loss};
        for (uint32_t k = A->ptr[node]; k < A->ptr[node + 1]; k++) {
            uint32_t next = A->nbr[k];
            if (visited[next]) continue;
            uint32_t e = A->eid[k];
            pp_t ec = {g->lat_ns[e], g->loss[e]};
            pp_t sc = pp_add(ns, ec);
            pp_t *slot = sm_find_or_insert(scores, next, &ins);
            if (ins || pp_lt(sc, *slot)) {
                *slot = sc;
                h_push(heap, (heap_item){sc.lat, sc.loss, next});
            }
        }
        visited[node] = 1;
    }
}

/* ---- opt (mode 1): identical algorithm, array scores ---- */
static void dijkstra_array(const adj_t *A, const or_edge_list *g, uint32_t src, pp_t *score,
                           uint8_t *have, uint8_t *visited, heap_t *heap) {
    memset(visited, 0, A->n);
    memset(have, 0, A->n);
    heap->n = 0;
    score[src] = (pp_t){0, 0.0f};
    have[src] = 1;
    h_push(heap, (heap_item){0, 0.0f, src});
    while (heap->n) {
        heap_item it = h_pop(heap);
        uint32_t node = it.node;
        if (visited[node]) continue;
        pp_t ns = {it.lat, it.loss};
        for (uint32_t k = A->ptr[node]; k < A->ptr[node + 1]; k++) {
            uint32_t next = A->nbr[k];
            if (visited[next]) continue;
            uint32_t e = A->eid[k];
            pp_t ec = {g->lat_ns[e], g->loss[e]};
            pp_t sc = pp_add(ns, ec);
            if (!have[next] || pp_lt(sc, score[next])) {
                score[next] = sc;
                have[next] = 1;
                h_push(heap, (heap_item){sc.lat, sc.loss, next});
            }
        }
        visited[node] = 1;
    }
}

/* ---- thread pool (rayon global pool stand-in: all logical CPUs) ---- */
typedef struct {
    const or_edge_list *g;
    const adj_t *A;
    const uint32_t *nodes;
    uint32_t n, src_count;
    const int32_t *pos; /* node index -> column, -1 if not in use */
    int mode;
    _Atomic uint32_t next;
    src_result *res;   /* mode 0 */
    uint64_t *lat_out; /* mode 1 */
    float *loss_out;
    uint8_t *reached; /* mode 1: per (i,j) reached flag */
} sp_job;

static void *sp_worker(void *arg) {
    sp_job *J = (sp_job *)arg;
    uint32_t V = J->A->n;
    uint8_t *visited = (uint8_t *)malloc(V ? V : 1);
    heap_t heap = {0};
    if (J->mode == 0) {
        for (;;) {
            uint32_t i = atomic_fetch_add(&J->next, 1);
            if (i >= J->src_count) break;
            smap scores;
            sm_init(&scores, 64);
            dijkstra_hashmap(J->A, J->g, J->nodes[i], &scores, visited, &heap);
            /* .filter(|(dst, _)| nodes.contains(dst)).collect::<HashMap>() (mod.rs:201-206) */
            src_result *r = &J->res[i];
            r->dst = (uint32_t *)malloc((scores.n ? scores.n : 1) * sizeof(uint32_t));
            r->pp = (pp_t *)malloc((scores.n ? scores.n : 1) * sizeof(pp_t));
            r->cnt = 0;
            smap per_src;
            sm_init(&per_src, 64);
            for (uint32_t s = 0; s < scores.cap; s++) {
                if (!scores.used[s]) continue;
                uint32_t dst = scores.key[s];
                int contains = 0;
                for (uint32_t q = 0; q < J->n; q++) /* Vec::contains: linear scan */
                    if (J->nodes[q] == dst) { contains = 1; break; }
                if (!contains) continue;
                int ins;
                *sm_find_or_insert(&per_src, dst, &ins) = scores.val[s];
            }
            for (uint32_t s = 0; s < per_src.cap; s++) {
                if (!per_src.used[s]) continue;
                r->dst[r->cnt] = per_src.key[s];
                r->pp[r->cnt++] = per_src.val[s];
            }
            sm_free(&per_src);
            sm_free(&scores);
        }
    } else {
        pp_t *score = (pp_t *)malloc((V ? V : 1) * sizeof(pp_t));
        uint8_t *have = (uint8_t *)malloc(V ? V : 1);
        for (;;) {
            uint32_t i = atomic_fetch_add(&J->next, 1);
            if (i >= J->src_count) break;
            dijkstra_array(J->A, J->g, J->nodes[i], score, have, visited, &heap);
            for (uint32_t j = 0; j < J->n; j++) {
                uint32_t d = J->nodes[j];
                size_t o = (size_t)i * J->n + j;
                J->reached[o] = have[d];
                if (have[d]) {
                    J->lat_out[o] = score[d].lat;
                    J->loss_out[o] = score[d].loss;
                }
            }
        }
        free(score);
        free(have);
    }
    free(visited);
    free(heap.a);
    return NULL;
}

static int n_threads(int threads) {
    if (threads > 0) return threads;
    /* the job's CPU share when the box declares one (the GPU box: 16 of its
       many CPUs), else every online CPU (rayon's default pool) */
    const char *e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) return atoi(e);
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c > 0 ? (int)c : 1;
}

/* count edges connecting a -> b as petgraph's edges_connecting does (directed:
 * outgoing of a with target b; undirected: either orientation, self-loop once) */
static int edge_lookup(const adj_t *A, const or_edge_list *g, uint32_t a, uint32_t b, pp_t *out) {
    int cnt = 0;
    for (uint32_t k = A->ptr[a]; k < A->ptr[a + 1]; k++) {
        if (A->nbr[k] != b) continue;
        if (cnt == 0) {
            uint32_t e = A->eid[k];
            out->lat = g->lat_ns[e];
            out->loss = g->loss[e];
        }
        cnt++;
    }
    return cnt;
}

static int edge_err(or_err *err, int code, uint32_t a_id, uint32_t b_id) {
    if (err) {
        err->code = code;
        err->a_id = a_id;
        err->b_id = b_id;
        snprintf(err->msg, sizeof err->msg,
                 code == OR_ERR_NO_EDGE ? "No edge connecting node %u to %u"
                                        : "More than one edge connecting node %u to %u",
                 a_id, b_id);
    }
    return code;
}

int or_compute_shortest_paths(const or_edge_list *g, const uint32_t *ids, const uint32_t *nodes,
                              uint32_t n, uint32_t src_count, uint64_t *lat_out, float *loss_out,
                              int threads, int mode, or_err *err) {
    if (err) memset(err, 0, sizeof *err);
    if (src_count > n) src_count = n;
    for (uint32_t i = 0; i < n; i++)
        if (nodes[i] >= g->n_nodes) {
            if (err) { err->code = OR_ERR_ARG; snprintf(err->msg, sizeof err->msg, "node index out of range"); }
            return OR_ERR_ARG;
        }
    adj_t A;
    build_adj(g, &A);
    int32_t *pos = (int32_t *)malloc(((size_t)g->n_nodes + 1) * sizeof(int32_t));
    for (uint32_t v = 0; v < g->n_nodes; v++) pos[v] = -1;
    for (uint32_t i = 0; i < n; i++) pos[nodes[i]] = (int32_t)i;

    sp_job J;
    memset(&J, 0, sizeof J);
    J.g = g; J.A = &A; J.nodes = nodes; J.n = n; J.src_count = src_count; J.pos = pos; J.mode = mode;
    atomic_init(&J.next, 0);
    size_t nn = (size_t)n * n;
    uint8_t *reached = NULL;
    if (mode == 0) J.res = (src_result *)calloc(src_count ? src_count : 1, sizeof(src_result));
    else {
        reached = (uint8_t *)calloc(nn ? nn : 1, 1);
        J.reached = reached; J.lat_out = lat_out; J.loss_out = loss_out;
    }
    int T = n_threads(threads);
    if ((uint32_t)T > src_count) T = (int)src_count;
    if (T < 1) T = 1;
    pthread_t *th = (pthread_t *)malloc((size_t)T * sizeof(pthread_t));
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, sp_worker, &J);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    free(th);

    uint64_t total = 0;
    if (mode == 0) {
        /* flat_map(..).collect::<HashMap<(src,dst),_>>() : sequential merge into
         * one map keyed by the pair, then the dense copy-out */
        size_t cap = 16;
        size_t want = 0;
        for (uint32_t i = 0; i < src_count; i++) want += J.res[i].cnt;
        while (cap < 2 * want + 16) cap <<= 1;
        uint64_t *gk = (uint64_t *)malloc(cap * sizeof(uint64_t));
        pp_t *gv = (pp_t *)malloc(cap * sizeof(pp_t));
        uint8_t *gu = (uint8_t *)calloc(cap, 1);
        for (uint32_t i = 0; i < src_count; i++) {
            src_result *r = &J.res[i];
            for (uint32_t q = 0; q < r->cnt; q++) {
                uint64_t k = ((uint64_t)nodes[i] << 32) | r->dst[q];
                uint64_t h = (k * 0x9e3779b97f4a7c15ULL) >> 17;
                size_t s = (size_t)(h & (cap - 1));
                while (gu[s] && gk[s] != k) s = (s + 1) & (cap - 1);
                if (!gu[s]) total++;
                gu[s] = 1; gk[s] = k; gv[s] = r->pp[q];
            }
            free(r->dst); free(r->pp);
        }
        reached = (uint8_t *)calloc(nn ? nn : 1, 1);
        for (size_t s = 0; s < cap; s++) {
            if (!gu[s]) continue;
            uint32_t a = (uint32_t)(gk[s] >> 32), b = (uint32_t)gk[s];
            size_t o = (size_t)pos[a] * n + (size_t)pos[b];
            lat_out[o] = gv[s].lat;
            loss_out[o] = gv[s].loss;
            reached[o] = 1;
        }
        free(gk); free(gv); free(gu); free(J.res);
    } else {
        for (size_t o = 0; o < (size_t)src_count * n; o++) total += reached[o];
    }

    int rc = OR_OK;
    if (src_count == n) {
        /* diagonal override with the single self-loop (mod.rs:210-217) */
        for (uint32_t i = 0; i < n && rc == OR_OK; i++) {
            pp_t w;
            int c = edge_lookup(&A, g, nodes[i], nodes[i], &w);
            if (c == 0) rc = edge_err(err, OR_ERR_NO_EDGE, ids[nodes[i]], ids[nodes[i]]);
            else if (c > 1) rc = edge_err(err, OR_ERR_MULTI_EDGE, ids[nodes[i]], ids[nodes[i]]);
            else {
                size_t o = (size_t)i * n + i;
                lat_out[o] = w.lat;
                loss_out[o] = w.loss;
            }
        }
        /* assert_eq!(paths.len(), nodes.len().pow(2)) (mod.rs:219) */
        if (rc == OR_OK && total != (uint64_t)nn) {
            rc = OR_ERR_DISCONNECTED;
            if (err) {
                err->code = rc;
                snprintf(err->msg, sizeof err->msg,
                         "assertion `left == right` failed: %llu != %llu (graph not connected)",
                         (unsigned long long)total, (unsigned long long)nn);
            }
        }
    }
    free(reached);
    free(pos);
    free_adj(&A);
    return rc;
}

int or_get_direct_paths(const or_edge_list *g, const uint32_t *ids, const uint32_t *nodes,
                        uint32_t n, uint64_t *lat_out, float *loss_out, or_err *err) {
    if (err) memset(err, 0, sizeof *err);
    adj_t A;
    build_adj(g, &A);
    int rc = OR_OK;
    for (uint32_t i = 0; i < n && rc == OR_OK; i++)
        for (uint32_t j = 0; j < n && rc == OR_OK; j++) {
            pp_t w;
            int c = edge_lookup(&A, g, nodes[i], nodes[j], &w);
            if (c == 0) rc = edge_err(err, OR_ERR_NO_EDGE, ids[nodes[i]], ids[nodes[j]]);
            else if (c > 1) rc = edge_err(err, OR_ERR_MULTI_EDGE, ids[nodes[i]], ids[nodes[j]]);
            else {
                lat_out[(size_t)i * n + j] = w.lat;
                loss_out[(size_t)i * n + j] = w.loss;
            }
        }
    free_adj(&A);
    return rc;
}

/* ======================================================================== */
/* Worker::send_packet (worker.rs:326-410)                                    */
/* ======================================================================== */
void or_packet_batch(const uint64_t *lat_tab, const float *loss_tab, uint32_t n,
                     const or_pkt *pkts, uint64_t n_pkts, uint64_t *rng, uint64_t round_end_ns,
                     uint64_t bootstrap_end_ns, uint64_t sim_end_ns, uint32_t *flags_out,
                     uint64_t *deliver_out, uint64_t *counters, uint64_t *min_latency_out,
                     uint64_t *next_event_out) {
    uint64_t min_lat = UINT64_MAX, next_ev = UINT64_MAX;
    for (uint64_t p = 0; p < n_pkts; p++) {
        const or_pkt *k = &pkts[p];
        flags_out[p] = OR_PDS_NONE;
        deliver_out[p] = 0;
        const int is_completed = k->t_ns >= sim_end_ns;
        const int is_bootstrapping = k->t_ns < bootstrap_end_ns;
        if (is_completed) continue; /* return before the RNG draw (worker.rs:336-339) */
        size_t o = (size_t)k->src_row * n + k->dst_row;
        /* reliability: f32 = 1.0 - packet_loss, widened to f64 (worker.rs:359-361, 552) */
        const float rel32 = 1.0f - loss_tab[o];
        double reliability = (double)rel32;
        double chance = or_gen_f64(&rng[4 * (size_t)k->src_host]);
        if (!is_bootstrapping && chance >= reliability && k->payload_size > 0) {
            flags_out[p] = OR_PDS_INET_DROPPED;
            continue;
        }
        uint64_t delay = lat_tab[o];
        if (delay < min_lat) min_lat = delay; /* update_lowest_used_latency */
        if (counters && counters[o] != UINT64_MAX) counters[o]++; /* saturating_add (mod.rs:453) */
        flags_out[p] = OR_PDS_INET_SENT;
        uint64_t deliver = k->t_ns + delay;
        if (deliver < round_end_ns) deliver = round_end_ns;
        deliver_out[p] = deliver;
        if (deliver < next_ev) next_ev = deliver;
    }
    if (min_latency_out) *min_latency_out = min_lat;
    if (next_event_out) *next_event_out = next_ev;
}
