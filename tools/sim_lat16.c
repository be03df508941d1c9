/* sim_lat16.c -- CPU model of the two-phase sparse sweep: u16 latency-only
 * label-correcting sweeps (one 128-B line per (vertex, 64-source word)), then
 * the exact loss over the tight DAG by label-correcting sweeps on f32 loss.
 * Measurement tool, not part of the library or the oracle.
 *
 * Input (stdin): as tools/sim_sssp.c (u32 V, u64 E, E x {u, v, w}).
 * argv: [1] stride (0 = the first 64 vertices of a BFS from argv[2]).
 * Per sweep (Gauss-Seidel in vertex order) prints: active targets (some
 * in-neighbour word changed), lines gathered (in-edges whose source word
 * changed), and for the loss phase the same with only tight lanes counted.
 *   gcc -O2 -o /tmp/sim_lat16 tools/sim_lat16.c
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    const uint32_t STRIDE = argc > 1 ? (uint32_t)atoi(argv[1]) : 1;
    uint32_t V;
    uint64_t E;
    if (fread(&V, 4, 1, stdin) != 1 || fread(&E, 8, 1, stdin) != 1) return 1;
    uint32_t *eu = malloc(4 * E), *ev = malloc(4 * E), *ew = malloc(4 * E);
    for (uint64_t k = 0; k < E; ++k) {
        uint32_t rec[3];
        if (fread(rec, 4, 3, stdin) != 3) return 1;
        eu[k] = rec[0];
        ev[k] = rec[1];
        ew[k] = rec[2];
    }
    uint64_t *ptr = calloc(V + 1, 8);
    for (uint64_t k = 0; k < E; ++k) ptr[ev[k] + 1]++;
    for (uint32_t v = 0; v < V; ++v) ptr[v + 1] += ptr[v];
    uint32_t *iu = malloc(4 * E), *iw = malloc(4 * E);
    uint64_t *fill = malloc(8 * V);
    memcpy(fill, ptr, 8 * V);
    for (uint64_t k = 0; k < E; ++k) {
        const uint64_t p = fill[ev[k]]++;
        iu[p] = eu[k];
        iw[p] = ew[k];
    }
    uint32_t srcs[64];
    if (STRIDE == 0) {
        const uint32_t START = argc > 2 ? (uint32_t)atoi(argv[2]) : V / 2;
        uint32_t *q = malloc(4 * V);
        uint8_t *seen = calloc(V, 1);
        uint32_t h = 0, tl = 0;
        q[tl++] = START;
        seen[START] = 1;
        while (h < tl && tl < 64) {
            const uint32_t x = q[h++];
            for (uint64_t k = ptr[x]; k < ptr[x + 1] && tl < 64; ++k)
                if (!seen[iu[k]]) {
                    seen[iu[k]] = 1;
                    q[tl++] = iu[k];
                }
        }
        for (int s = 0; s < 64; ++s) srcs[s] = q[s % tl];
    } else {
        for (int s = 0; s < 64; ++s) srcs[s] = (uint32_t)((uint64_t)s * STRIDE % V);
    }
    uint32_t *L = malloc(4 * (uint64_t)V * 64);
    float *P = malloc(4 * (uint64_t)V * 64);
    uint8_t *chg = calloc(V, 1), *chg2 = calloc(V, 1);
    for (uint64_t i = 0; i < (uint64_t)V * 64; ++i) {
        L[i] = UINT32_MAX;
        P[i] = 2.0f;
    }
    for (int s = 0; s < 64; ++s) {
        L[(uint64_t)srcs[s] * 64 + s] = 0;
        P[(uint64_t)srcs[s] * 64 + s] = 0.0f;
        chg[srcs[s]] = 1;
    }
    /* symmetric seeding (argv[5] = percent F): a random F% of the vertices
       already hold their exact latency from every source (the columns of
       earlier launches' rows, L(s,v) = L(v,s) on undirected graphs), marked
       changed at the start like sources */
    const uint32_t FPCT = argc > 5 ? (uint32_t)atoi(argv[5]) : 0;
    if (FPCT) {
        /* exact distances by Bellman-Ford per source (model only) */
        uint32_t *ex = malloc(4 * (uint64_t)V * 64);
        for (uint64_t i = 0; i < (uint64_t)V * 64; ++i) ex[i] = UINT32_MAX;
        for (int s2 = 0; s2 < 64; ++s2) ex[(uint64_t)srcs[s2] * 64 + s2] = 0;
        for (int ch = 1; ch;) {
            ch = 0;
            for (uint32_t v = 0; v < V; ++v)
                for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k)
                    for (int s2 = 0; s2 < 64; ++s2) {
                        const uint32_t d = ex[(uint64_t)iu[k] * 64 + s2];
                        if (d != UINT32_MAX && d + iw[k] < ex[(uint64_t)v * 64 + s2]) {
                            ex[(uint64_t)v * 64 + s2] = d + iw[k];
                            ch = 1;
                        }
                    }
        }
        srand(7);
        uint32_t known = 0;
        for (uint32_t v = 0; v < V; ++v)
            if ((uint32_t)(rand() % 100) < FPCT) {
                for (int s2 = 0; s2 < 64; ++s2) L[(uint64_t)v * 64 + s2] = ex[(uint64_t)v * 64 + s2];
                chg[v] = 1;
                ++known;
            }
        printf("seeded %u vertices exact\n", known);
        free(ex);
    }
    /* word-level delta gating (argv[3] = DELTA > 0): a changed word moves on
       in sweep t only if its smallest changed latency is below theta_t; else it
       stays pending (chg kept) -- theta grows by DELTA a sweep, or jumps to the
       smallest pending latency + DELTA when a sweep moved nothing */
    const uint32_t DELTA = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    uint32_t *cmin = malloc(4 * V), *cmin2 = malloc(4 * V);
    uint8_t *go = calloc(V, 1);
    for (uint32_t v = 0; v < V; ++v) cmin[v] = UINT32_MAX;
    for (int s = 0; s < 64; ++s) cmin[srcs[s]] = 0;
    uint64_t theta = DELTA ? 2ull * DELTA : UINT64_MAX;
    /* ordered first pass (argv[4] = BW > 0): vertices bucketed by their
       distance from the word's first source c, bucket width BW units; the
       buckets run in order, each one Jacobi over the values left by the
       earlier buckets, every in-edge pulled.  Then the usual sweeps. */
    const uint32_t BW = argc > 4 ? (uint32_t)atoi(argv[4]) : 0;
    uint64_t pass_lines = 0;
    if (BW) {
        /* Dijkstra from c (binary heap-free: bucket queue on integer latencies) */
        uint32_t *dc = malloc(4 * V);
        for (uint32_t v = 0; v < V; ++v) dc[v] = UINT32_MAX;
        const uint32_t c = srcs[0];
        dc[c] = 0;
        uint8_t *done = calloc(V, 1);
        /* simple O(V^2)-free approach: repeated Bellman-Ford until stable (fine for a model) */
        for (int it = 0, ch = 1; ch && it < 100000; ++it) {
            ch = 0;
            for (uint32_t v = 0; v < V; ++v)
                for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k)
                    if (dc[iu[k]] != UINT32_MAX && dc[iu[k]] + iw[k] < dc[v]) {
                        dc[v] = dc[iu[k]] + iw[k];
                        ch = 1;
                    }
        }
        uint32_t maxd = 0;
        for (uint32_t v = 0; v < V; ++v)
            if (dc[v] != UINT32_MAX && dc[v] > maxd) maxd = dc[v];
        const uint32_t nbk = maxd / BW + 1;
        uint32_t *cnt = calloc(nbk + 1, 4), *ord = malloc(4 * V);
        for (uint32_t v = 0; v < V; ++v) cnt[(dc[v] == UINT32_MAX ? maxd : dc[v]) / BW + 1]++;
        for (uint32_t k = 0; k < nbk; ++k) cnt[k + 1] += cnt[k];
        uint32_t *pos = malloc(4 * (nbk + 1));
        memcpy(pos, cnt, 4 * (nbk + 1));
        for (uint32_t v = 0; v < V; ++v) ord[pos[(dc[v] == UINT32_MAX ? maxd : dc[v]) / BW]++] = v;
        uint32_t *nl = malloc(4 * 64 * (uint64_t)V);
        uint64_t improved_pass = 0;
        for (uint32_t bk = 0; bk < nbk; ++bk) {
            for (uint32_t i = cnt[bk]; i < cnt[bk + 1]; ++i) {
                const uint32_t v = ord[i];
                for (int s = 0; s < 64; ++s) nl[(uint64_t)i * 64 + s] = L[(uint64_t)v * 64 + s];
                for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                    ++pass_lines;
                    for (int s = 0; s < 64; ++s) {
                        const uint32_t d = L[(uint64_t)iu[k] * 64 + s];
                        if (d != UINT32_MAX && d + iw[k] < nl[(uint64_t)i * 64 + s]) nl[(uint64_t)i * 64 + s] = d + iw[k];
                    }
                }
            }
            for (uint32_t i = cnt[bk]; i < cnt[bk + 1]; ++i) {
                const uint32_t v = ord[i];
                int imp = 0;
                for (int s = 0; s < 64; ++s)
                    if (nl[(uint64_t)i * 64 + s] < L[(uint64_t)v * 64 + s]) {
                        L[(uint64_t)v * 64 + s] = nl[(uint64_t)i * 64 + s];
                        imp = 1;
                    }
                if (imp) {
                    chg[v] = 1;
                    cmin[v] = 0;
                    ++improved_pass;
                }
            }
        }
        printf("ordered pass: buckets %u lines %lu improved %lu\n", nbk, pass_lines, improved_pass);
    }
    uint64_t tot_lines = 0, tot_act = 0;
    uint32_t t = 0;
    printf("latency phase\n");
    for (;;) {
        uint64_t lines = 0, act = 0, impv = 0, moved = 0;
        uint32_t pmin = UINT32_MAX;
        for (uint32_t v = 0; v < V; ++v) {
            go[v] = chg[v] && cmin[v] < theta;
            moved += go[v];
            if (chg[v] && !go[v] && cmin[v] < pmin) pmin = cmin[v];
        }
        if (DELTA && !moved && pmin != UINT32_MAX) {
            theta = (uint64_t)pmin + DELTA;
            for (uint32_t v = 0; v < V; ++v) go[v] = chg[v] && cmin[v] < theta;
        }
        for (uint32_t v = 0; v < V; ++v) {
            int a = 0;
            uint32_t best[64];
            for (int s = 0; s < 64; ++s) best[s] = UINT32_MAX;
            for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                const uint32_t u = iu[k];
                if (!go[u]) continue;
                a = 1;
                ++lines;
                for (int s = 0; s < 64; ++s) {
                    const uint32_t d = L[(uint64_t)u * 64 + s];
                    if (d != UINT32_MAX && d + iw[k] < best[s]) best[s] = d + iw[k];
                }
            }
            act += a;
            int imp = 0;
            uint32_t mn = UINT32_MAX;
            for (int s = 0; s < 64; ++s)
                if (best[s] < L[(uint64_t)v * 64 + s]) {
                    L[(uint64_t)v * 64 + s] = best[s];
                    imp = 1;
                    if (best[s] < mn) mn = best[s];
                }
            /* pending words stay changed (with their smallest latency) */
            const int keep = chg[v] && !go[v];
            chg2[v] = imp || keep;
            cmin2[v] = imp ? (keep && cmin[v] < mn ? cmin[v] : mn) : (keep ? cmin[v] : UINT32_MAX);
            impv += imp || keep;
        }
        uint8_t *x = chg;
        chg = chg2;
        chg2 = x;
        uint32_t *y = cmin;
        cmin = cmin2;
        cmin2 = y;
        ++t;
        if (DELTA) theta += DELTA;
        tot_lines += lines;
        tot_act += act;
        printf("  sweep %2u: active %7lu lines %8lu improved %7lu\n", t, act, lines, impv);
        if (!impv) break;
    }
    uint32_t lmax = 0;
    for (uint64_t i = 0; i < (uint64_t)V * 64; ++i)
        if (L[i] != UINT32_MAX && L[i] > lmax) lmax = L[i];
    printf("latency: sweeps %u lines/word %lu (+pass %lu) active/sweep %.0f lmax %u\n", t, tot_lines, pass_lines, (double)tot_act / t, lmax);
    /* loss phase: tight in-edges only, f32 loss, 2 lines (32 lanes) per word */
    memset(chg, 0, V);
    for (int s = 0; s < 64; ++s) chg[srcs[s]] = 1;
    uint64_t tight = 0;
    for (uint32_t v = 0; v < V; ++v)
        for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k)
            for (int s = 0; s < 64; ++s) {
                const uint32_t d = L[(uint64_t)iu[k] * 64 + s];
                if (d != UINT32_MAX && d + iw[k] == L[(uint64_t)v * 64 + s]) ++tight;
            }
    printf("tight (edge, lane) pairs per (vertex, lane): %.3f\n", (double)tight / ((double)V * 64));
    /* loss-phase vertex order (argv[6]): 0 = vertex id, 1 = latency from the
       word's first source, 2 = hops from it */
    const int LORD = argc > 6 ? atoi(argv[6]) : 0;
    uint32_t *lord = malloc(4 * V);
    for (uint32_t v = 0; v < V; ++v) lord[v] = v;
    if (LORD) {
        uint64_t *key = malloc(8 * V);
        uint32_t *hop = malloc(4 * V), *qq = malloc(4 * V), h0 = 0, h1 = 0;
        for (uint32_t v = 0; v < V; ++v) hop[v] = UINT32_MAX;
        hop[srcs[0]] = 0;
        qq[h1++] = srcs[0];
        while (h0 < h1) {
            const uint32_t x = qq[h0++];
            for (uint64_t k = ptr[x]; k < ptr[x + 1]; ++k)
                if (hop[iu[k]] == UINT32_MAX) {
                    hop[iu[k]] = hop[x] + 1;
                    qq[h1++] = iu[k];
                }
        }
        for (uint32_t v = 0; v < V; ++v)
            key[v] = ((uint64_t)(LORD == 1 ? L[(uint64_t)v * 64] : hop[v]) << 32) | v;
        int cmp(const void *a, const void *b) {
            const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
            return x < y ? -1 : x > y;
        }
        qsort(key, V, 8, cmp);
        for (uint32_t i = 0; i < V; ++i) lord[i] = (uint32_t)key[i];
    }
    uint32_t tl = 0;
    uint64_t ltot = 0;
    for (;;) {
        uint64_t lines = 0, act = 0, impv = 0;
        for (uint32_t vi = 0; vi < V; ++vi) {
            const uint32_t v = lord[vi];
            int a = 0;
            float best[64];
            for (int s = 0; s < 64; ++s) best[s] = 2.0f;
            for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                const uint32_t u = iu[k];
                if (!chg[u]) continue;
                uint64_t tm = 0;
                for (int s = 0; s < 64; ++s) {
                    const uint32_t d = L[(uint64_t)u * 64 + s];
                    if (d != UINT32_MAX && d + iw[k] == L[(uint64_t)v * 64 + s]) tm |= 1ull << s;
                }
                if (!tm) continue;
                a = 1;
                lines += ((tm & 0xffffffffull) != 0) + ((tm >> 32) != 0);
                for (int s = 0; s < 64; ++s)
                    if (((tm >> s) & 1) && P[(uint64_t)u * 64 + s] <= 1.0f) {
                        const float c = 1.0f - (1.0f - P[(uint64_t)u * 64 + s]) * 0.995f;
                        if (c < best[s]) best[s] = c;
                    }
            }
            act += a;
            int imp = 0;
            for (int s = 0; s < 64; ++s)
                if (best[s] < P[(uint64_t)v * 64 + s]) {
                    P[(uint64_t)v * 64 + s] = best[s];
                    imp = 1;
                }
            chg2[v] = imp;
            impv += imp;
        }
        uint8_t *x = chg;
        chg = chg2;
        chg2 = x;
        ++tl;
        ltot += lines;
        printf("  loss sweep %2u: active %7lu lines %8lu improved %7lu\n", tl, act, lines, impv);
        if (!impv) break;
    }
    printf("loss: sweeps %u lines/word %lu\n", tl, ltot);
    return 0;
}
