"""Every BASELINE.json config at its real size on one MI355X, through the C ABI
(configs_untested).  Bars as everywhere else: latency and loss
bit-exact vs the oracle (the petgraph-faithful restatement), diagonal = the raw
self-loop, min latency exact, packet decisions bit-exact.  Where the oracle
cannot produce the whole table in seconds (C3: 2.7e8 pairs, C4: 1e10 pairs)
it checks seeded sample rows, and size-independent properties cover the rest
on the device (latency symmetry of undirected graphs, every pair reachable).

  C1  1,000-node complete graph through its GML text: the full table
  C1  also against tests/golden/c1_table.json: the SHA-256 of the oracle's table
  C3  16,384-node complete graph: 128 oracle rows (every 8-rank shard's first
      and last) + symmetry
  C4  100,000-node Barabasi-Albert graph, ALL nodes in use (the sparse sweep's
      256 groups in flight): 32 seeded oracle rows, symmetric blocks, no
      unreachable pair; the 120 GB table never leaves the device
  C5  1M packets / 10k hosts on the C1 nodes (loss U[0,0.25]), decided on the
      GPU's table and by the oracle on ITS OWN table
"""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _device_table(plan):
    import torch

    from shadow_amd.dist import _CudaBuf
    lat_p, loss_p, n = plan.table_ptrs()
    dev = torch.device("cuda", 0)
    L = torch.as_tensor(_CudaBuf(lat_p, n * n * 8), device=dev).view(torch.int64).view(n, n)
    P = torch.as_tensor(_CudaBuf(loss_p, n * n * 4), device=dev).view(torch.int32).view(n, n)
    return L, P


def _check_rows(L, P, rows, nodes_dev_order, elat, eloss, sl_lat, sl_loss):
    """rows: table rows sampled; elat/eloss: the oracle's rows over the same
    column order; the diagonal comes from the self-loop."""
    for i, r in enumerate(rows):
        got_l = L[r].cpu().numpy().view(np.uint64)
        got_p = P[r].cpu().numpy().view(np.uint32)
        exp_l = elat[i].copy()
        exp_p = eloss[i].copy().view(np.uint32)
        exp_l[r] = sl_lat[r]
        exp_p[r] = np.float32(sl_loss[r]).view(np.uint32)
        assert np.array_equal(got_l, exp_l), f"row {r}: latency"
        assert np.array_equal(got_p, exp_p), f"row {r}: loss bits"


def test_c1_full_table_through_gml():
    n = 1000
    src, dst, lat, loss = synth.complete_graph(n, 1)
    text = synth.gml_text(n, src, dst, lat, loss)
    g = NetworkGraph.parse(text)
    nodes = np.random.default_rng(1).permutation(n).astype(np.uint32)  # HashSet order: arbitrary
    t = g.compute_shortest_paths(nodes)
    elat, eloss = O.compute_shortest_paths(O.gml_parse(text), nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))
    assert t.min_latency_ns == int(elat.min())


def test_c1_table_matches_pinned_fixture():
    """C1 pinned without a live oracle run: the GPU table (GML text ->
    srt_compute_shortest_paths, nodes in GML order) hashes to the SHA-256 of
    the oracle's table committed in tests/golden/c1_table.json
    (tools/make_c1_fixture.py), and the 1,000 sampled pairs match."""
    import hashlib
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1_table.json")))
    n = fx["nodes"]
    src, dst, lat, loss = synth.complete_graph(n, fx["seed"])
    text = synth.gml_text(n, src, dst, lat, loss)
    assert hashlib.sha256(text.encode()).hexdigest() == fx["gml_sha256"]
    t = NetworkGraph.parse(text).compute_shortest_paths(np.arange(n, dtype=np.uint32))
    h = hashlib.sha256(np.ascontiguousarray(t.latency_ns, np.uint64).tobytes() +
                       np.ascontiguousarray(t.packet_loss, np.float32).tobytes()).hexdigest()
    assert h == fx["table_sha256"]
    for i, j, l, p in fx["samples"]:
        assert int(t.latency_ns[i, j]) == l and int(t.packet_loss[i, j:j + 1].view(np.uint32)[0]) == p
    assert t.min_latency_ns == fx["min_latency_ns"]


def test_c3_16k_rows_vs_oracle_and_symmetry():
    """C3 as the drop-in runs it (AUTO: the level solve -- B from the probe)
    and forced onto the Floyd-Warshall family: 128 oracle rows bit-exact (the
    first and last row of every shard of an 8-rank build plus 112 seeded
    ones), latency symmetry on the device, and the two families' tables equal
    bit for bit."""
    import torch

    n = 16384
    edges = synth.complete_graph(n, 3)
    row_ptr, col, lat, loss = synth.complete_csr(n, 3, edges=edges)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes).run()
    assert plan.describe().startswith("level:u16"), plan.describe()  # AUTO: the level solve is priced cheapest
    assert "rows=sym lat16" in plan.describe(), plan.describe()  # the class out-rows from the u16-unit copy
    plan.fetch(table=False)  # every pair reachable (else DISCONNECTED), min latency
    L, P = _device_table(plan)
    assert torch.equal(L, L.t()), "undirected latency table must be symmetric"
    edges8 = np.array([b for r in range(8) for b in (r * n // 8, (r + 1) * n // 8 - 1)])
    rest = np.setdiff1d(np.arange(n), edges8)
    rows = np.concatenate([edges8, np.random.default_rng(3).choice(rest, 112, replace=False)])
    k = len(rows)
    order = np.concatenate([rows, np.setdiff1d(nodes, rows)]).astype(np.uint32)
    og = O.Graph(False, nodes, *edges)
    del row_ptr, col
    elat, eloss = O.compute_shortest_paths(og, order, src_count=k, mode=1)
    # oracle columns are in `order`; put them back in node order
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    sl_l = lat.reshape(n, n).diagonal().copy()
    sl_p = loss.reshape(n, n).diagonal().copy()
    _check_rows(L, P, rows, nodes, elat[:k][:, inv], eloss[:k][:, inv], sl_l, sl_p)
    # get_smallest_latency_ns over the whole device table == the smallest edge
    assert plan.min_latency_ns == L.min().item() == int(lat.min())
    fw = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW).run()
    try:
        assert fw.describe().startswith("fw:f16key")  # complete graph: lmax = the longest edge (300 units < 1024)
        assert fw.timing()["loss_fold"] == 1  # tight weights <= 15 units, latencies < 2048: the level fold
        fw.fetch(table=False)
        L2, P2 = _device_table(fw)
        assert torch.equal(L, L2) and torch.equal(P, P2), "level solve != Floyd-Warshall tables"
    finally:
        fw.close()
        plan.close()


def test_c3ns_16k_u32_keys_rows_vs_oracle():
    """C3 with ns latencies (bench --config c3ns): g = 1 ns, so no bound fits
    31 units and AUTO takes the quantized level solve (buckets as wide as the
    shortest edge, ~1 ms); its device table equals the Floyd-Warshall family's
    (u32 keys, quantized level fold) bit for bit, 16 seeded rows bit-exact
    against the oracle, symmetry over the device table."""
    import torch

    n = 16384
    edges = synth.complete_graph_ns(n, 3)
    row_ptr, col, lat, loss = synth.complete_csr(n, 3, edges=edges)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes).run()
    d = plan.describe()
    assert d.startswith("level:u32 ") and " g=1 " in d and " q=" in d, d
    plan.fetch(table=False)
    L, P = _device_table(plan)
    assert torch.equal(L, L.t())
    fw = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW).run()
    try:
        assert fw.describe().startswith("fw:u32key ") and fw.timing()["loss_fold"] == 1
        fw.fetch(table=False)
        assert fw.min_latency_ns == plan.min_latency_ns
        L2, P2 = _device_table(fw)
        assert torch.equal(L, L2) and torch.equal(P, P2), "quantized level solve != Floyd-Warshall tables"
        del L2, P2
    finally:
        fw.close()
    rows = np.random.default_rng(33).choice(n, 16, replace=False)
    order = np.concatenate([rows, np.setdiff1d(nodes, rows)]).astype(np.uint32)
    og = O.Graph(False, nodes, *edges)
    del row_ptr, col
    elat, eloss = O.compute_shortest_paths(og, order, src_count=16, mode=1)
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    sl_l = lat.reshape(n, n).diagonal().copy()
    sl_p = loss.reshape(n, n).diagonal().copy()
    _check_rows(L, P, rows, nodes, elat[:16][:, inv], eloss[:16][:, inv], sl_l, sl_p)
    plan.close()


def test_c4_100k_all_in_use():
    import torch

    n = 100_000
    src, dst, lat, loss = synth.barabasi_albert(n, 4, 4)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes).run()
    assert plan.describe().startswith("sssp")
    plan.fetch(table=False)  # no unreachable pair among the 1e10
    L, P = _device_table(plan)
    rng = np.random.default_rng(4)
    for _ in range(16):  # symmetric 2048 x 2048 blocks
        a, b = rng.integers(0, n - 2048, size=2)
        assert torch.equal(L[a:a + 2048, b:b + 2048], L[b:b + 2048, a:a + 2048].t())
    rows = np.sort(rng.choice(n, 32, replace=False))
    order = np.concatenate([rows, np.setdiff1d(nodes, rows)]).astype(np.uint32)
    og = O.Graph(False, nodes, src, dst, lat, loss)
    elat, eloss = O.compute_shortest_paths(og, order, src_count=32, mode=1)
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    sl = src == dst
    sl_l = np.empty(n, np.uint64)
    sl_p = np.empty(n, np.float32)
    sl_l[src[sl]] = lat[sl]
    sl_p[src[sl]] = loss[sl]
    _check_rows(L, P, rows, nodes, elat[:32][:, inv], eloss[:32][:, inv], sl_l, sl_p)
    plan.close()


def test_c5_1m_packets_on_the_oracles_own_table():
    import torch

    n_nodes, n_hosts, n_pkts = 1000, 10_000, 1_000_000
    src, dst, lat, loss = synth.complete_graph(n_nodes, 5, loss_max=0.25)
    g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss)
    nodes = np.arange(n_nodes, dtype=np.uint32)
    plan = RoutingPlan(g, nodes).run()
    table = plan.fetch()
    o_lat, o_loss = O.compute_shortest_paths(O.Graph(False, nodes, src, dst, lat, loss), nodes)
    assert np.array_equal(table.latency_ns, o_lat)
    assert np.array_equal(table.packet_loss.view(np.uint32), o_loss.view(np.uint32))
    r0, r1 = 1_000_000_000, 1_000_000_000 + 5 * synth.MS
    pk, host_ptr, _ = synth.packet_round(n_hosts, n_nodes, n_pkts, 5, r0, r1)
    rng = synth.host_rng_states(n_hosts, general_seed=1)
    for boot_end in (0, r0 + 2 * synth.MS):  # drops on / suppressed for part of the round
        rng_o = rng.copy()
        cnt_o = np.zeros((n_nodes, n_nodes), np.uint64)
        f_o, d_o, mn_o, ne_o = O.packet_batch(o_lat, o_loss, pk.view(O.PKT_DTYPE), rng_o, r1, boot_end, 2**62,
                                              counters=cnt_o)
        dev = torch.device("cuda:0")
        t_pk = torch.from_numpy(pk.view(np.uint8).copy()).to(dev)
        t_hp = torch.from_numpy(host_ptr.view(np.int32).copy()).to(dev)
        t_rng = torch.from_numpy(rng.view(np.int64).copy()).to(dev)
        t_f = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
        t_d = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
        t_c = torch.zeros(n_nodes * n_nodes, dtype=torch.int64, device=dev)
        t_s = torch.full((2,), -1, dtype=torch.int64, device=dev)
        plan.packet_batch(t_pk, t_hp, t_rng, r1, boot_end, 2**62, t_f, t_d, t_c, t_s)
        f = t_f.cpu().numpy().view(np.uint32)
        assert np.array_equal(f, f_o)
        assert np.array_equal(t_d.cpu().numpy().view(np.uint64), d_o)
        assert np.array_equal(t_rng.cpu().numpy().view(np.uint64), rng_o)
        assert np.array_equal(t_c.cpu().numpy().view(np.uint64).reshape(n_nodes, n_nodes), cnt_o)
        s = t_s.cpu().numpy().view(np.uint64)
        assert int(s[0]) == mn_o and int(s[1]) == ne_o
        if boot_end == 0:
            assert (f == O.PDS_INET_DROPPED).sum() > 10_000
    plan.close()
