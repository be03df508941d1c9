"""Seeded synthetic inputs for the BASELINE.json configs (no network, no
datasets): complete GML graphs (C1-C3), a Barabasi-Albert AS-like graph (C4)
and per-round packet batches (C5).

All generators are pure numpy with explicit seeds, so the same config is
bit-identical here and on the GPU box.
"""
from __future__ import annotations

import numpy as np

MS = 1_000_000  # ns per ms


def complete_graph(n: int, seed: int, lat_ms=(1, 300), loss_max=0.01, self_loops=True):
    """Undirected complete graph with self-loops, edges (i, j) for i <= j in GML
    order (row-major).  latency U{lat_ms} integer ms (ties are common), loss
    U[0, loss_max] rounded to 6 decimals (as printed in GML).
    Returns (src, dst, lat_ns, loss)."""
    rng = np.random.default_rng(seed)
    iu, ju = np.triu_indices(n, 0 if self_loops else 1)
    m = len(iu)
    lat = rng.integers(lat_ms[0], lat_ms[1] + 1, size=m, dtype=np.uint64) * np.uint64(MS)
    loss = np.round(rng.uniform(0.0, loss_max, size=m), 6).astype(np.float32)
    return iu.astype(np.uint32), ju.astype(np.uint32), lat, loss


def complete_graph_ns(n: int, seed: int, lat_ms=(1, 300), loss_max=0.01):
    """complete_graph(n, seed) with every latency given in ns plus a seeded
    sub-ms offset U{0..999_999} ns: the gcd of the latencies is 1 ns, so the
    closure carries ns units (u32 keys at 16k: the longest edge is < 3.01e8
    units) and the loss pass's tight weights exceed the level fold's classes
    (units.rs:377-388: Shadow reads latencies as any time unit down to ns)."""
    src, dst, lat, loss = complete_graph(n, seed, lat_ms, loss_max)
    off = np.random.default_rng(seed + 7).integers(0, MS, size=len(lat), dtype=np.uint64)
    return src, dst, lat + off, loss


def complete_csr(n: int, seed: int, lat_ms=(1, 300), loss_max=0.01, edges=None):
    """CSR (petgraph adjacency of the undirected complete graph) built directly,
    without the O(n^2) edge-list sort: row u lists all v (self-loop once).
    Values are identical to complete_graph(n, seed) traversed both ways
    (pass that edge list as `edges` to skip regenerating it)."""
    src, dst, lat, loss = complete_graph(n, seed, lat_ms, loss_max) if edges is None else edges
    L = np.zeros((n, n), np.uint64)
    P = np.zeros((n, n), np.float32)
    L[src, dst] = lat
    L[dst, src] = lat
    P[src, dst] = loss
    P[dst, src] = loss
    row_ptr = (np.arange(n + 1, dtype=np.uint64) * np.uint64(n))
    col = np.tile(np.arange(n, dtype=np.uint32), n)
    return row_ptr, col, L.reshape(-1), P.reshape(-1)


def dense_graph(n: int, seed: int, drop=0.3, lat_ms=(1, 300), loss_max=0.01):
    """The complete graph of complete_graph(n, seed) with a seeded fraction
    `drop` of its off-diagonal undirected edges removed (self-loops kept):
    a dense NON-complete graph, so the key-width proof cannot use the
    longest-edge bound and runs the eccentricity sweeps (fw_ecc_bound).
    Returns the kept edge list (i <= j)."""
    src, dst, lat, loss = complete_graph(n, seed, lat_ms, loss_max)
    keep = (src == dst) | (np.random.default_rng(seed + 1000).random(len(src)) >= drop)
    return src[keep], dst[keep], lat[keep], loss[keep]


def dense_csr(n: int, edges):
    """CSR of an undirected edge list without parallel edges (i <= j each
    once, self-loops once): row u lists its neighbours in increasing order,
    as the GML reader's adjacency of a graph written in node order."""
    src, dst, lat, loss = edges
    a = np.concatenate([src, dst[src != dst]]).astype(np.int64)
    b = np.concatenate([dst, src[src != dst]]).astype(np.int64)
    la = np.concatenate([lat, lat[src != dst]])
    lo = np.concatenate([loss, loss[src != dst]])
    order = np.lexsort((b, a))
    row_ptr = np.concatenate([[0], np.cumsum(np.bincount(a, minlength=n))]).astype(np.uint64)
    return (row_ptr, b[order].astype(np.uint32), la[order].astype(np.uint64),
            lo[order].astype(np.float32))


def gml_text(n_nodes: int, src, dst, lat_ns, loss, directed=False, bandwidth="1 Gbit") -> str:
    """Shadow GML (docs/network_graph_spec.md) for an edge list; latency is
    written in ms when exact, else ns; packet_loss as a 6-decimal float token."""
    out = ["graph [", f"  directed {1 if directed else 0}"]
    for i in range(n_nodes):
        out.append(f"  node [\n    id {i}\n    host_bandwidth_up \"{bandwidth}\"\n"
                   f"    host_bandwidth_down \"{bandwidth}\"\n  ]")
    for s, d, l, p in zip(np.asarray(src).tolist(), np.asarray(dst).tolist(), np.asarray(lat_ns).tolist(),
                          np.asarray(loss).tolist()):
        lat = f"{l // MS} ms" if l % MS == 0 else f"{l} ns"
        out.append(f"  edge [\n    source {s}\n    target {d}\n    latency \"{lat}\"\n"
                   f"    packet_loss {p:.6f}\n  ]")
    out.append("]")
    return "\n".join(out) + "\n"


def random_graph(n: int, seed: int, p_edge=0.3, directed=False, lat_range_ns=(1, 20), loss_max=0.05,
                 parallel=0.05):
    """Small random connected graph with self-loops, heavy latency ties (few
    distinct small latencies) and some parallel edges -- for parity tests."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    # a ring guarantees strong connectivity (both orientations when directed)
    for i in range(n):
        src.append(i)
        dst.append((i + 1) % n)
        if directed:
            src.append((i + 1) % n)
            dst.append(i)
    for i in range(n):
        for j in range(n):
            if i != j and (directed or i < j) and rng.random() < p_edge:
                src.append(i)
                dst.append(j)
                if rng.random() < parallel:
                    src.append(i)
                    dst.append(j)
    for i in range(n):  # exactly one self-loop each
        src.append(i)
        dst.append(i)
    m = len(src)
    lat = rng.integers(lat_range_ns[0], lat_range_ns[1] + 1, size=m).astype(np.uint64)
    loss = np.round(rng.uniform(0.0, loss_max, size=m), 6).astype(np.float32)
    perm = rng.permutation(m)
    return (np.array(src, np.uint32)[perm], np.array(dst, np.uint32)[perm], lat[perm], loss[perm])


def barabasi_albert(n: int, m: int, seed: int, lat_ms=(1, 300), loss_max=0.01):
    """Undirected BA graph (each new node attaches to m distinct existing nodes
    by degree) plus one self-loop per node.  Returns GML-order edge arrays."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    targets = list(range(m))
    repeated = []
    for v in range(m, n):
        for t in targets:
            src.append(v)
            dst.append(t)
        repeated.extend(targets)
        repeated.extend([v] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(len(repeated)))])
        targets = list(chosen)
    src.extend(range(n))
    dst.extend(range(n))
    k = len(src)
    lat = rng.integers(lat_ms[0], lat_ms[1] + 1, size=k, dtype=np.uint64) * np.uint64(MS)
    loss = np.round(rng.uniform(0.0, loss_max, size=k), 6).astype(np.float32)
    return np.array(src, np.uint32), np.array(dst, np.uint32), lat, loss


PKT_DTYPE = np.dtype([("src_host", "<u4"), ("src_row", "<u4"), ("dst_row", "<u4"), ("payload_size", "<u4"),
                      ("t_ns", "<u8")])
# srt_pkt_ip: the packet by address (IPv4 in network byte order)
PKT_IP_DTYPE = np.dtype([("src_host", "<u4"), ("src_ip", "<u4"), ("dst_ip", "<u4"), ("payload_size", "<u4"),
                         ("t_ns", "<u8")])


def packet_round(n_hosts: int, n_rows: int, n_pkts: int, seed: int, round_start: int, round_end: int):
    """One round of outgoing packets, grouped by source host in send order.
    Hosts sit round-robin on table rows; destinations uniform over other hosts;
    payload 0 with p=0.1 else U{1..1460}; send times uniform in the round.
    Returns (pkts structured array, host_ptr u32[n_hosts+1], host_row u32)."""
    rng = np.random.default_rng(seed)
    host_row = (np.arange(n_hosts) % n_rows).astype(np.uint32)
    src_host = np.sort(rng.integers(0, n_hosts, size=n_pkts)).astype(np.uint32)
    dst_host = rng.integers(0, n_hosts - 1, size=n_pkts).astype(np.uint32)
    dst_host = np.where(dst_host >= src_host, dst_host + 1, dst_host).astype(np.uint32)
    payload = rng.integers(1, 1461, size=n_pkts).astype(np.uint32)
    payload[rng.random(n_pkts) < 0.1] = 0
    t = rng.integers(round_start, round_end, size=n_pkts).astype(np.uint64)
    # send order within a host: non-decreasing time
    order = np.lexsort((t, src_host))
    pk = np.zeros(n_pkts, PKT_DTYPE)
    pk["src_host"] = src_host[order]
    pk["src_row"] = host_row[src_host[order]]
    pk["dst_row"] = host_row[dst_host[order]]
    pk["payload_size"] = payload[order]
    pk["t_ns"] = t[order]
    counts = np.bincount(src_host, minlength=n_hosts)
    host_ptr = np.zeros(n_hosts + 1, np.uint32)
    np.cumsum(counts, out=host_ptr[1:])
    return pk, host_ptr, host_row


def host_rng_states(n_hosts: int, general_seed: int = 1):
    """Per-host Xoshiro256PlusPlus::seed_from_u64(node_seed) as Shadow seeds it
    (sim_config.rs:49-53, 222-244; host.rs:233): node_seed = R ^ SipHash13(name)
    with R the first u64 of seed_from_u64(general.seed).  Hostnames host{i}."""
    def splitmix(x):
        x = (x + 0x9E3779B97F4A7C15) & M64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return x, z ^ (z >> 31)

    def seed_from_u64(seed):
        s, x = [], seed
        for _ in range(4):
            x, z = splitmix(x)
            s.append(z)
        return s

    def xnext(s):
        r = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return r

    R = xnext(seed_from_u64(general_seed))
    out = np.zeros((n_hosts, 4), np.uint64)
    for h in range(n_hosts):
        out[h] = seed_from_u64(R ^ siphash13_str(f"host{h}"))
    return out


M64 = (1 << 64) - 1


def _rotl(x, k):
    return ((x << k) | (x >> (64 - k))) & M64


def siphash13_str(s: str) -> int:
    """std DefaultHasher (SipHash-1-3, keys 0,0) of a &str: bytes then 0xff."""
    m = s.encode() + b"\xff"
    v0, v1, v2, v3 = 0x736F6D6570736575, 0x646F72616E646F6D, 0x6C7967656E657261, 0x7465646279746573

    def rnd(v0, v1, v2, v3):
        v0 = (v0 + v1) & M64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
        v2 = (v2 + v3) & M64; v3 = _rotl(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & M64; v3 = _rotl(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & M64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
        return v0, v1, v2, v3

    n = len(m)
    i = 0
    while i + 8 <= n:
        w = int.from_bytes(m[i:i + 8], "little")
        v3 ^= w
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= w
        i += 8
    b = ((n & 0xFF) << 56) | int.from_bytes(m[i:], "little")
    v3 ^= b
    v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(3):
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
    return v0 ^ v1 ^ v2 ^ v3
