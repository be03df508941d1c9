/* gml_gen.c -- Shadow GML text of a complete n-node graph, written straight
 * into a caller buffer (the C1-C3 shape of tools/gml_bench.py: nodes with
 * host bandwidths, one edge block per pair i <= j with a latency string in ms
 * and a packet_loss float), for ingest throughput runs at config C3 scale
 * (16k nodes, ~12 GB of text) without Python string formatting.  Values come
 * from a splitmix64 stream (latency U{1..300} ms, loss U[0, 0.01] with 6
 * decimals): the same grammar and sizes as synth.gml_text, not its values.
 * Measurement tool, not part of the library or the oracle.
 *   gcc -O2 -shared -fPIC -o /tmp/libgmlgen.so tools/gml_gen.c
 */
#include <stdint.h>
#include <string.h>

static uint64_t sm(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static char *put_u(char *p, uint64_t v) {
    char t[24];
    int k = 0;
    do {
        t[k++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (k) *p++ = t[--k];
    return p;
}

static char *put_s(char *p, const char *s) {
    const size_t l = strlen(s);
    memcpy(p, s, l);
    return p + l;
}

/* returns the bytes written, 0 if cap is too small (upper bound: 110 B a node,
 * 100 B an edge) */
uint64_t gml_complete(uint32_t n, uint64_t seed, char *out, uint64_t cap) {
    const uint64_t need = 64 + (uint64_t)n * 110 + (uint64_t)n * (n + 1) / 2 * 100;
    if (cap < need) return 0;
    char *p = out;
    uint64_t s = seed;
    p = put_s(p, "graph [\n  directed 0\n");
    for (uint32_t i = 0; i < n; ++i) {
        p = put_s(p, "  node [\n    id ");
        p = put_u(p, i);
        p = put_s(p, "\n    host_bandwidth_up \"1 Gbit\"\n    host_bandwidth_down \"1 Gbit\"\n  ]\n");
    }
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = i; j < n; ++j) {
            const uint64_t r = sm(&s);
            const uint32_t lat = 1 + (uint32_t)(r % 300);
            const uint32_t loss = (uint32_t)((r >> 20) % 10001); /* millionths, 0 .. 0.010000 */
            p = put_s(p, "  edge [\n    source ");
            p = put_u(p, i);
            p = put_s(p, "\n    target ");
            p = put_u(p, j);
            p = put_s(p, "\n    latency \"");
            p = put_u(p, lat);
            p = put_s(p, " ms\"\n    packet_loss 0.");
            char d[6];
            uint32_t x = loss;
            for (int k = 5; k >= 0; --k) {
                d[k] = (char)('0' + x % 10);
                x /= 10;
            }
            memcpy(p, d, 6);
            p += 6;
            p = put_s(p, "\n  ]\n");
        }
    p = put_s(p, "]\n");
    return (uint64_t)(p - out);
}
