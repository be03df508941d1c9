"""Generate the committed golden fixtures in tests/golden/ (run in the build
container; the outputs are data, not code).

Sources of truth, in order of strength:
  1. the reference's own test vectors (src/main/network/graph/mod.rs:516-529,
     559-647; rand_xoshiro's published xoshiro256++ vector; the published
     SipHash-2-4 vectors) -- written verbatim;
  2. small graphs solved by the oracle (oracle/liboracle.so, mode 0 = faithful
     petgraph restatement) AND independently re-derived here with networkx
     (latency) and a pure-Python heapq Dijkstra over numpy.float32 (loss); the
     script refuses to write a fixture on any disagreement;
  3. packet rounds decided by the oracle's sequential send_packet restatement.

usage: python tools/make_golden.py
"""
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from shadow_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def py_dijkstra(n, src, dst, lat, loss, directed, s):
    adj = [[] for _ in range(n)]
    for a, b, l, p in zip(src.tolist(), dst.tolist(), lat.tolist(), loss.tolist()):
        adj[a].append((b, l, np.float32(p)))
        if not directed and a != b:
            adj[b].append((a, l, np.float32(p)))
    one = np.float32(1)
    scores = {s: (0, np.float32(0))}
    heap = [(0, np.float32(0), s)]
    done = set()
    while heap:
        l0, p0, u = heapq.heappop(heap)
        if u in done:
            continue
        for v, l, p in adj[u]:
            if v in done:
                continue
            cand = (l0 + l, one - (one - p0) * (one - p))
            if v not in scores or cand < scores[v]:
                scores[v] = cand
                heapq.heappush(heap, (cand[0], cand[1], v))
        done.add(u)
    return scores


def graph_fixture(name, n, seed, directed, **kw):
    import networkx as nx

    src, dst, lat, loss = synth.random_graph(n, seed, directed=directed, **kw)
    ids = (np.arange(n) * 7 + 3).astype(np.uint32)  # GML ids != NodeIndex
    g = O.Graph(directed, ids, src, dst, lat, loss)
    nodes = np.random.default_rng(seed + 1000).permutation(n).astype(np.uint32)
    L, P = O.compute_shortest_paths(g, nodes, mode=0, threads=4)
    G = nx.DiGraph() if directed else nx.Graph()
    G.add_nodes_from(range(n))
    for a, b, l in zip(src.tolist(), dst.tolist(), lat.tolist()):
        if a != b and not (G.has_edge(a, b) and G[a][b]["w"] <= l):
            G.add_edge(a, b, w=l)
    for i, a in enumerate(nodes.tolist()):
        d = nx.single_source_dijkstra_path_length(G, a, weight="w")
        sc = py_dijkstra(n, src, dst, lat, loss, directed, a)
        for j, b in enumerate(nodes.tolist()):
            if a == b:
                continue
            assert L[i, j] == d[b] == sc[b][0], (name, i, j)
            assert np.float32(sc[b][1]).view(np.uint32) == P[i, j].view(np.uint32), (name, i, j)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), n=n, directed=directed, ids=ids, src=src, dst=dst,
                        lat=lat, loss=loss, nodes=nodes, exp_lat=L, exp_loss=P)


def packet_fixture(name, n_nodes, n_hosts, n_pkts, seed, bootstrap_end, sim_end):
    src, dst, lat, loss = synth.complete_graph(n_nodes, seed, loss_max=0.25)
    g = O.Graph(False, np.arange(n_nodes), src, dst, lat, loss)
    nodes = np.arange(n_nodes, dtype=np.uint32)
    L, P = O.compute_shortest_paths(g, nodes, mode=0, threads=4)
    r0, r1 = 1_000_000_000, 1_000_000_000 + 5 * synth.MS
    pk, host_ptr, _ = synth.packet_round(n_hosts, n_nodes, n_pkts, seed, r0, r1)
    rng = np.zeros((n_hosts, 4), np.uint64)
    for h in range(n_hosts):
        rng[h] = O.xoshiro_seed(O.host_seed(1, f"host{h}"))
    rng_in = rng.copy()
    cnt = np.zeros((n_nodes, n_nodes), np.uint64)
    f, d, mn, ne = O.packet_batch(L, P, pk.view(O.PKT_DTYPE), rng, r1, bootstrap_end, sim_end, counters=cnt)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), table_lat=L, table_loss=P, pkts=pk.view(np.uint8),
                        host_ptr=host_ptr, rng_in=rng_in, rng_out=rng, round_end=r1, bootstrap_end=bootstrap_end,
                        sim_end=sim_end, flags=f, deliver=d, counters=cnt, min_latency=mn, next_event=ne)


def main():
    os.makedirs(OUT, exist_ok=True)
    ref = {
        "source": "reference tests, verbatim",
        "test_shortest_path": {"file": "src/main/network/graph/mod.rs:559-647",
                               "directed": [[3333, 3, 7], [5, 5555, 12], [16, 11, 7777]],
                               "undirected": [[3333, 3, 7], [3, 5555, 10], [7, 10, 7777]]},
        "test_path_add": {"file": "src/main/network/graph/mod.rs:516-529", "a": [23, 0.35], "b": [11, 0.85],
                          "latency_ns": 34, "loss_approx": 0.9025, "tol": 0.01},
        "xoshiro256pp_from_1234": {"source": "rand_xoshiro 0.6.0 xoshiro256plusplus.rs test vector",
                                   "values": [41943041, 58720359, 3588806011781223, 3591011842654386,
                                              9228616714210784205, 9973669472204895162, 14011001112246962877,
                                              12406186145184390807, 15849039046786891736, 10450023813501588000]},
        "splitmix64_state0_first": "0xe220a8397b1dcdaf",
        "siphash24_key_00_0f": {"empty": "0x726fdb47dd0e0e31", "00..0e": "0xa129ca6149be45e5"},
        "units": {"file": "src/main/utility/units.rs:585-620",
                  "ok": {"10": 10_000_000_000, "10 s": 10_000_000_000, "10s": 10_000_000_000,
                         "10   s": 10_000_000_000, "10sec": 10_000_000_000, "10  m": 600_000_000_000,
                         "10  min": 600_000_000_000, "10 ms": 10_000_000}},
    }
    json.dump(ref, open(os.path.join(OUT, "reference_vectors.json"), "w"), indent=1)
    graph_fixture("graph_undirected_ties", 48, 11, False, p_edge=0.15, lat_range_ns=(1, 4), loss_max=0.05)
    graph_fixture("graph_directed_ties", 48, 12, True, p_edge=0.12, lat_range_ns=(1, 4), loss_max=0.05)
    graph_fixture("graph_directed_highloss", 40, 13, True, p_edge=0.2, lat_range_ns=(1, 6), loss_max=0.9)
    graph_fixture("graph_undirected_wide", 130, 14, False, p_edge=0.04, lat_range_ns=(1, 1_000_000), loss_max=0.01)
    packet_fixture("packets_round", 40, 200, 20_000, 21, bootstrap_end=0, sim_end=2**62)
    packet_fixture("packets_sim_end", 24, 50, 5_000, 22, bootstrap_end=1_000_000_000 + 1 * synth.MS,
                   sim_end=1_000_000_000 + 4 * synth.MS)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
