/* sim_sssp.c -- CPU model of the batched sparse sweep (srt_sssp.hip), used to
 * choose the activation schedule before touching the kernel.  Measurement
 * tool, not part of the library or the oracle.
 *
 * Input (stdin, binary): u32 V, u64 E, then E x {u32 u, u32 v, u32 w} directed
 * in-edges u -> v (w = latency in units of g, self-loops already dropped).
 * One word of 64 sources (lanes) 0, stride, 2*stride, ...  For a threshold
 * step DELTA (0 = plain label-correcting), sweeps run the GPU's rule:
 *   a target v relaxes in-edge (u -> v) on lane s iff bit s of act[u] is set;
 *   pend(v) = (pend(v) & ~act(v)) | improved(v);
 *   act(v)  = pend(v) & { s : D[v][s] <= theta(t+1) },  theta(t) = t * DELTA
 * (after SWEEP_CAP sweeps theta = inf).  D is updated in place in vertex
 * order (Gauss-Seidel, as the GPU may); act/pend are double-buffered.
 * Reports sweeps, lane relaxations per (vertex, source), and the gather cost
 * in 128-B lines (16 lanes x 8 B) with at least one active lane, per source.
 *   gcc -O2 -o /tmp/sim_sssp tools/sim_sssp.c && python tools/sim_sssp.py
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    const uint32_t DELTA = argc > 1 ? (uint32_t)atoi(argv[1]) : 0;
    const uint32_t SWEEP_CAP = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
    const uint32_t STRIDE = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
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
    /* in-CSR by v */
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
    uint64_t *D = malloc(8 * (uint64_t)V * 64);
    uint64_t *act = calloc(V, 8), *act2 = calloc(V, 8), *pend = calloc(V, 8), *pend2 = calloc(V, 8);
    for (uint64_t i = 0; i < (uint64_t)V * 64; ++i) D[i] = UINT64_MAX;
    /* STRIDE > 0: sources s * STRIDE (unrelated); STRIDE == 0: the first 64
       vertices of a BFS from vertex START (neighbours of each other) */
    uint32_t bfs[64];
    if (STRIDE == 0) {
        const uint32_t START = argc > 4 ? (uint32_t)atoi(argv[4]) : V / 2;
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
        for (int s = 0; s < 64; ++s) bfs[s] = q[s % tl];
    }
    for (int s = 0; s < 64; ++s) {
        const uint32_t src = STRIDE ? (uint32_t)((uint64_t)s * STRIDE % V) : bfs[s];
        D[(uint64_t)src * 64 + s] = 0;
        act[src] |= 1ull << s;
        pend[src] |= 1ull << s;
    }
    uint64_t relax = 0, lines = 0, lines32 = 0, lines_loss = 0, scans = 0;
    uint32_t t = 0;
    for (;;) {
        int any_pend = 0;
        const uint64_t theta_next = (DELTA == 0 || t + 1 >= SWEEP_CAP) ? UINT64_MAX : (uint64_t)(t + 1) * DELTA;
        for (uint32_t v = 0; v < V; ++v) {
            uint64_t best[64];
            for (int s = 0; s < 64; ++s) best[s] = UINT64_MAX;
            for (uint64_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                const uint32_t u = iu[k];
                const uint64_t a = act[u];
                ++scans;
                if (!a) continue;
                for (int q = 0; q < 4; ++q)
                    if ((a >> (16 * q)) & 0xffffull) ++lines;
                for (int q = 0; q < 2; ++q)
                    if ((a >> (32 * q)) & 0xffffffffull) ++lines32;
                uint64_t need = 0;  /* split layout: lanes whose candidate latency can win */
                for (int s = 0; s < 64; ++s)
                    if ((a >> s) & 1) {
                        ++relax;
                        const uint64_t d = D[(uint64_t)u * 64 + s];
                        const uint64_t cur = best[s] < D[(uint64_t)v * 64 + s] ? best[s] : D[(uint64_t)v * 64 + s];
                        if (d != UINT64_MAX && d + iw[k] <= cur) need |= 1ull << s;
                        if (d != UINT64_MAX && d + iw[k] < best[s]) best[s] = d + iw[k];
                    }
                for (int q = 0; q < 2; ++q)
                    if ((need >> (32 * q)) & 0xffffffffull) ++lines_loss;
            }
            uint64_t imp = 0;
            for (int s = 0; s < 64; ++s)
                if (best[s] < D[(uint64_t)v * 64 + s]) {
                    D[(uint64_t)v * 64 + s] = best[s];
                    imp |= 1ull << s;
                }
            const uint64_t p = (pend[v] & ~act[v]) | imp;
            uint64_t a = 0;
            for (int s = 0; s < 64; ++s)
                if (((p >> s) & 1) && D[(uint64_t)v * 64 + s] <= theta_next) a |= 1ull << s;
            pend2[v] = p;
            act2[v] = a;
            any_pend |= p != 0;
        }
        uint64_t *x = act;
        act = act2;
        act2 = x;
        x = pend;
        pend = pend2;
        pend2 = x;
        ++t;
        if (!any_pend || t > 100000) break;
    }
    printf("{\"delta\": %u, \"cap\": %u, \"sweeps\": %u, \"relax_per_vs\": %.3f, \"lines_per_source\": %.1f, "
           "\"edge_scans_per_sweep\": %.0f, \"lines32_per_source\": %.1f, \"loss_lines32_per_source\": %.1f}\n",
           DELTA, SWEEP_CAP, t, (double)relax / ((double)V * 64), (double)lines / 64.0, (double)scans / t, (double)lines32 / 64.0, (double)lines_loss / 64.0);
    return 0;
}
