"""GPU parity of the routing build (libsrt.so on gfx950) against the oracle.

Bar: latency AND packet_loss bit-exact for both kernel families (the dense
closure's loss is folded over the tight shortest-path DAG, srt_loss.hip; the
north_star's 1e-6 tolerance is not needed), min latency exact, error
codes/texts as the reference.  All calls go through the C ABI
(shadow_amd.graph -> libsrt.so).
"""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, RoutingInfo, _lib, synth

pytestmark = pytest.mark.gpu


GOLDEN_DIRECTED = [[3333, 3, 7], [5, 5555, 12], [16, 11, 7777]]
GOLDEN_UNDIRECTED = [[3333, 3, 7], [3, 5555, 10], [7, 10, 7777]]


def _three(directed):
    from tests.test_oracle import THREE_NODE
    return THREE_NODE.format(d=directed)


def _check(graph_edges, nodes, directed, n_nodes, node_ids=None, algo=_lib.SRT_ALGO_AUTO):
    src, dst, lat, loss = graph_edges
    ids = np.arange(n_nodes) if node_ids is None else node_ids
    og = O.Graph(directed, ids, src, dst, lat, loss)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss, directed=directed, node_ids=ids)
    t = g.compute_shortest_paths(nodes, algo=algo)
    assert np.array_equal(t.latency_ns, elat), "latency must be bit-exact"
    bad = t.packet_loss.view(np.uint32) != eloss.view(np.uint32)
    assert not bad.any(), f"{int(bad.sum())} loss entries differ in bits"
    assert t.min_latency_ns == int(elat.min())
    return t


@pytest.mark.parametrize("directed", [1, 0])
def test_reference_golden_three_node(directed):
    g = NetworkGraph.parse(_three(directed))
    nodes = [g.node_id_to_index(0), g.node_id_to_index(1), g.node_id_to_index(2)]
    t = g.compute_shortest_paths(nodes)
    assert t.latency_ns.tolist() == (GOLDEN_DIRECTED if directed else GOLDEN_UNDIRECTED)
    assert t.min_latency_ns == 3
    assert t[(nodes[2], nodes[0])].latency_ns == (16 if directed else 7)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("directed", [False, True])
def test_random_tie_heavy(seed, directed):
    n = 70 + 13 * seed  # crosses the 64-node block boundary, ragged padding
    e = synth.random_graph(n, seed, p_edge=0.15, directed=directed, lat_range_ns=(1, 4), loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    _check(e, nodes, directed, n)


@pytest.mark.parametrize("seed", range(3))
def test_subset_in_use(seed):
    # intermediates may be any graph node; sources/destinations only in-use nodes (mod.rs:203)
    n = 150
    e = synth.random_graph(n, 100 + seed, p_edge=0.05, directed=True, lat_range_ns=(1, 30))
    nodes = np.random.default_rng(seed).choice(n, 37, replace=False).astype(np.uint32)
    _check(e, nodes, True, n)


def test_complete_c1_slice_through_gml():
    n = 256
    src, dst, lat, loss = synth.complete_graph(n, 1)
    text = synth.gml_text(n, src, dst, lat, loss)
    g = NetworkGraph.parse(text)
    og = O.gml_parse(text)
    nodes = np.arange(n, dtype=np.uint32)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    t = g.compute_shortest_paths(nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))


def test_loss_free_graph_exact_zero_loss():
    n = 90
    src, dst, lat, loss = synth.random_graph(n, 5, p_edge=0.1, loss_max=0.0)
    t = _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n)
    assert not t.packet_loss.any()


def test_single_node():
    g = NetworkGraph.from_edges(1, [0], [0], [42], [0.25], directed=False, node_ids=[9])
    t = g.compute_shortest_paths([0])
    assert t.latency_ns.tolist() == [[42]] and t.packet_loss[0, 0] == np.float32(0.25)


def test_high_loss_and_loss_one_edges():
    n = 40
    src, dst, lat, loss = synth.random_graph(n, 11, p_edge=0.2, lat_range_ns=(1, 3), loss_max=0.9)
    loss[::7] = 1.0
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n)


def test_disconnected_raises():
    g = NetworkGraph.from_edges(3, [0, 1, 2, 0], [0, 1, 2, 1], [5, 5, 5, 3], directed=True)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1, 2])
    assert e.value.code == _lib.SRT_ERR_DISCONNECTED
    # Rust's assert_eq! panic text for paths.len() == nodes.len().pow(2) (mod.rs:219):
    # sources 0 / 1 / 2 reach {0, 1} / {1} / {2}
    assert str(e.value) == "assertion `left == right` failed\n  left: 4\n right: 9"


def test_missing_selfloop_error_text():
    g = NetworkGraph.from_edges(2, [0, 0], [0, 1], [5, 5], directed=False, node_ids=[4, 8])
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1])
    assert e.value.code == _lib.SRT_ERR_NO_EDGE and str(e.value) == "No edge connecting node 8 to 8"


def test_direct_paths_parity():
    n = 33
    src, dst, lat, loss = synth.complete_graph(n, 9)
    og = O.Graph(False, np.arange(n) + 1000, src, dst, lat, loss)
    nodes = np.random.default_rng(1).permutation(n).astype(np.uint32)
    elat, eloss = O.get_direct_paths(og, nodes)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=False, node_ids=np.arange(n) + 1000)
    t = g.get_direct_paths(nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))  # verbatim edge values
    assert t.min_latency_ns == int(elat.min())


def test_direct_paths_errors_in_reference_order():
    n = 6
    src, dst, lat, loss = synth.complete_graph(n, 2)
    keep = ~((src == 2) & (dst == 4))
    g = NetworkGraph.from_edges(n, src[keep], dst[keep], lat[keep], loss[keep], node_ids=np.arange(n) + 50)
    with pytest.raises(_lib.SrtError) as e:
        g.get_direct_paths([0, 4, 2, 1])
    assert str(e.value) == "No edge connecting node 54 to 52"
    src2 = np.concatenate([src, [1]]).astype(np.uint32)
    dst2 = np.concatenate([dst, [3]]).astype(np.uint32)
    g2 = NetworkGraph.from_edges(n, src2, dst2, np.concatenate([lat, [lat[0]]]), np.concatenate([loss, [0]]),
                                 node_ids=np.arange(n) + 50)
    with pytest.raises(_lib.SrtError) as e:
        g2.get_direct_paths([3, 1])
    assert str(e.value) == "More than one edge connecting node 53 to 51"


def test_c2_scale_row_sample():
    """4096-node complete graph (config C2): full GPU table vs oracle rows for a
    seeded sample of sources, plus size-independent properties."""
    n = 4096
    src, dst, lat, loss = synth.complete_graph(n, 2)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    t = g.compute_shortest_paths(np.arange(n, dtype=np.uint32))
    L = t.latency_ns
    # symmetric for an undirected graph, and <= the direct edge
    assert np.array_equal(L, L.T)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    rows = np.random.default_rng(0).choice(n, 16, replace=False)
    nodes = np.concatenate([rows, np.setdiff1d(np.arange(n), rows)]).astype(np.uint32)
    elat, eloss = O.compute_shortest_paths(og, nodes, src_count=16)
    for i, r in enumerate(rows):
        exp_lat = np.empty(n, np.uint64)
        exp_lat[nodes] = elat[i]
        exp_loss = np.empty(n, np.float32)
        exp_loss[nodes] = eloss[i]
        exp_lat[r] = L[r, r]
        exp_loss[r] = t.packet_loss[r, r]
        assert np.array_equal(L[r], exp_lat)
        assert np.array_equal(t.packet_loss[r].view(np.uint32), exp_loss.view(np.uint32))


def test_u64_key_path_large_latencies(monkeypatch):
    """Latencies up to 2^51 ns with no common unit on a 20-node sparse graph:
    with the (V-1) x max edge proof (SRT_FW_NO_ECC: the eccentricity bound
    would allow f64) 2 * Lmax does not fit 53 bits, so the closure runs on u64
    keys (the LDS-DMA tile kernel's integer branch) and the loss pass on u64
    latencies (rows in global memory); latency and loss stay bit-exact."""
    monkeypatch.setenv("SRT_FW_NO_ECC", "1")
    n = 20
    src, dst, lat, loss = synth.random_graph(n, 31, p_edge=0.3, lat_range_ns=(1, 2**31), loss_max=0.01)
    lat = (lat.astype(np.uint64) << np.uint64(20)) + np.uint64(1)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    from shadow_amd.plan import RoutingPlan
    plan = RoutingPlan(g, np.arange(n, dtype=np.uint32), algo=_lib.SRT_ALGO_FW)
    assert "u64key" in plan.describe() and "loss=tight-dag/u64" in plan.describe()
    plan.close()
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_FW)


def test_f64_key_wide_latency_range_buckets():
    """ns latencies with no common unit (up to 2^31): the loss pass's latency
    buckets are wider than one value (shift > 0) and repeat until stable."""
    n = 60
    src, dst, lat, loss = synth.random_graph(n, 32, p_edge=0.2, lat_range_ns=(1, 2**31), loss_max=0.05)
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_FW)
    src, dst, lat, loss = synth.random_graph(n, 33, p_edge=0.2, directed=True, lat_range_ns=(1000, 1900),
                                             loss_max=0.05)
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), True, n, algo=_lib.SRT_ALGO_FW)


def test_zero_latency_rejected():
    # ShadowEdge::try_from: "Edge 'latency' must not be 0" (mod.rs:104-106)
    g = NetworkGraph.from_edges(2, [0, 1, 0], [0, 1, 1], [5, 5, 0], directed=False)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1])
    assert e.value.code == _lib.SRT_ERR_INVALID and "must not be 0" in str(e.value)


@pytest.mark.parametrize("algo", [_lib.SRT_ALGO_FW, _lib.SRT_ALGO_SSSP])
def test_empty_in_use_set(algo):
    # compute_shortest_paths(&[]) -> empty map, no panic (mod.rs:219: 0 == 0)
    src, dst, lat, loss = synth.random_graph(20, 3)
    g = NetworkGraph.from_edges(20, src, dst, lat, loss)
    t = g.compute_shortest_paths(np.zeros(0, np.uint32), algo=algo)
    assert t.latency_ns.shape == (0, 0) and len(t) == 0


def test_isolated_unused_nodes_are_fine():
    # nodes outside the in-use set may be unreachable: only in-use pairs must connect
    n = 80
    src, dst, lat, loss = synth.random_graph(n, 8, p_edge=0.1)
    keep = (src < 70) & (dst < 70)  # nodes 70..79 keep only their self-loops
    sl = (src == dst) & (src >= 70)
    m = keep | sl
    nodes = np.arange(70, dtype=np.uint32)
    for algo in (_lib.SRT_ALGO_FW, _lib.SRT_ALGO_SSSP):
        _check((src[m], dst[m], lat[m], loss[m]), nodes, False, n, algo=algo)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("directed", [False, True])
def test_loss_pass_unpacked_form(monkeypatch, seed, directed):
    """The loss pass's unpacked tight-edge form (separate u / w arrays, rows not
    sorted by w: the fallback when vertex index and tight latency do not share
    32 bits) gives the same bits as the oracle."""
    monkeypatch.setenv("SRT_LOSS_UNPACKED", "1")
    n = 90 + 17 * seed
    e = synth.random_graph(n, 200 + seed, p_edge=0.12, directed=directed, lat_range_ns=(1, 5), loss_max=0.05)
    _check(e, np.random.default_rng(seed).permutation(n).astype(np.uint32), directed, n, algo=_lib.SRT_ALGO_FW)


def test_end_to_end_compact_download_matches_device_table(monkeypatch):
    """srt_compute_shortest_paths on a dense graph downloads the table as
    5-byte records (every finite latency <= 510 units: the units' low 8 bits,
    the loss bits with the 9th unit bit in the sign) in pieces behind the
    chunked fold, expanded on host threads; 9,000 nodes = 2 fold chunks, 10
    pieces.  The host table must equal, bit for bit, the device table of the
    same build, the 6-byte records (SRT_FETCH6=1), the 8-byte records
    (SRT_FETCH8=1) and the 16-byte download (SRT_FETCH16=1)."""
    import torch

    from shadow_amd.dist import _CudaBuf
    from shadow_amd.plan import RoutingPlan
    n = 9000
    row_ptr, col, lat, loss = synth.complete_csr(n, 21)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    t = g.compute_shortest_paths(nodes)
    plan = RoutingPlan(g, nodes).run()
    lat_p, loss_p, m = plan.table_ptrs()
    dev = torch.device("cuda", 0)
    L = torch.as_tensor(_CudaBuf(lat_p, m * m * 8), device=dev).view(torch.int64).cpu().numpy().view(np.uint64)
    P = torch.as_tensor(_CudaBuf(loss_p, m * m * 4), device=dev).view(torch.int32).cpu().numpy().view(np.uint32)
    plan.close()
    assert np.array_equal(t.latency_ns.reshape(-1), L)
    assert np.array_equal(t.packet_loss.reshape(-1).view(np.uint32), P)
    for knob in ("SRT_FETCH6", "SRT_FETCH8", "SRT_FETCH16"):  # 6- and 8-byte records; the 16-byte download
        monkeypatch.setenv(knob, "1")
        t2 = g.compute_shortest_paths(nodes)
        monkeypatch.delenv(knob)
        assert np.array_equal(t2.latency_ns, t.latency_ns), knob
        assert np.array_equal(t2.packet_loss.view(np.uint32), t.packet_loss.view(np.uint32)), knob


@pytest.fixture
def small_upload_pieces(monkeypatch):
    """Force the piece-pipelined CSR scan + upload on small graphs: pieces of
    2^6 adjacency entries (many pieces, 3 in flight)."""
    monkeypatch.setenv("SRT_UPLOAD_PIECE", "6")
    yield
    monkeypatch.delenv("SRT_UPLOAD_PIECE")


@pytest.mark.parametrize("seed", range(3))
def test_piece_upload_irregular_rows(small_upload_pieces, seed):
    """Sparse rows (col uploaded per piece) and u32 latencies, both families."""
    n = 120
    edges = synth.random_graph(n, 40 + seed, p_edge=0.08, lat_range_ns=(1, 50), loss_max=0.05)
    _check(edges, np.arange(n, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_FW)
    _check(edges, np.arange(0, n, 3, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_SSSP)


def test_piece_upload_identity_rows(small_upload_pieces):
    """A complete graph with self-loops, rows in node order: every piece's
    col is written on the device, nothing uploaded."""
    n = 70
    row_ptr, col, lat, loss = synth.complete_csr(n, 44)
    src = np.repeat(np.arange(n), n)
    # the same graph as a directed edge list (both orientations): checked vs the oracle
    t1 = _check((src, col, lat, loss), np.arange(n, dtype=np.uint32), True, n, algo=_lib.SRT_ALGO_FW)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    t = g.compute_shortest_paths(np.arange(n, dtype=np.uint32))
    assert np.array_equal(t.latency_ns, t1.latency_ns)
    assert np.array_equal(t.packet_loss.view(np.uint32), t1.packet_loss.view(np.uint32))


def test_piece_upload_wide_latencies(small_upload_pieces):
    """Latencies past 2^32 ns: those pieces send the caller's u64 array."""
    n = 20
    src, dst, lat, loss = synth.random_graph(n, 31, p_edge=0.3, lat_range_ns=(1, 2**31), loss_max=0.01)
    lat = (lat.astype(np.uint64) << np.uint64(20)) + np.uint64(1)
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_FW)


def test_piece_upload_errors_in_reference_order(small_upload_pieces):
    """The scan's checks are the same under the pipeline: a zero latency, a
    missing self-loop."""
    g = NetworkGraph.from_edges(2, [0, 1, 0], [0, 1, 1], [5, 5, 0], directed=False)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1])
    assert e.value.code == _lib.SRT_ERR_INVALID and "must not be 0" in str(e.value)
    n = 40
    src, dst, lat, loss = synth.random_graph(n, 3, p_edge=0.3)
    keep = ~((src == 8) & (dst == 8))
    g = NetworkGraph.from_edges(n, src[keep], dst[keep], lat[keep], loss[keep])
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths(np.arange(n, dtype=np.uint32))
    assert e.value.code == _lib.SRT_ERR_NO_EDGE and str(e.value) == "No edge connecting node 8 to 8"


def _plan_table(g, nodes, algo=_lib.SRT_ALGO_FW):
    from shadow_amd.plan import RoutingPlan
    plan = RoutingPlan(g, nodes, algo=algo).run()
    return plan, plan.fetch()


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("directed", [False, True])
def test_level_fold_equals_scan_fold(monkeypatch, seed, directed):
    """The level fold (tight edges grouped by exact weight class, each class
    walked from the smaller of its two latency levels: push from N_{l-w} or
    pull into N_l, srt_loss.hip level_loss_kernel) and the single-direction
    push scan (SRT_LOSS_LEVEL=0) both give the oracle's bits, on tie-heavy
    graphs (latencies 1..6 units) both directed and undirected; the plan
    reports which fold ran."""
    n = 100 + 29 * seed
    src, dst, lat, loss = synth.random_graph(n, 300 + seed, p_edge=0.2, directed=directed, lat_range_ns=(1, 6),
                                             loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    elat, eloss = O.compute_shortest_paths(O.Graph(directed, np.arange(n), src, dst, lat, loss), nodes)
    for level in (1, 0):
        monkeypatch.setenv("SRT_LOSS_LEVEL", str(level))
        g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=directed)
        plan, t = _plan_table(g, nodes)
        assert plan.timing()["loss_fold"] == level
        assert np.array_equal(t.latency_ns, elat)
        assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32)), f"level={level}"


@pytest.mark.parametrize("lat_hi,level", [(31, 1), (40, 0)])
def test_level_fold_weight_class_limit(lat_hi, level):
    """Tight edges heavier than the 31 weight classes (and a smallest tight
    weight of 1 unit: no quantized levels) send the build to the scan fold; at
    the limit it stays on the level fold; bits as the oracle."""
    n = 140
    src, dst, lat, loss = synth.random_graph(n, 77, p_edge=0.08, directed=False, lat_range_ns=(1, lat_hi),
                                             loss_max=0.05)
    # make sure a tight edge of the top weight exists: a pendant vertex
    src = np.append(src, np.uint32(n - 1)).astype(np.uint32)
    dst = np.append(dst, np.uint32(0)).astype(np.uint32)
    keep = ~(((src == n - 1) | (dst == n - 1)) & (src != dst))
    keep[-1] = True
    src, dst = src[keep], dst[keep]
    lat = np.append(lat, np.uint64(lat_hi))[keep]
    loss = np.append(loss, np.float32(0.01))[keep]
    nodes = np.arange(n, dtype=np.uint32)
    elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=False)
    plan, t = _plan_table(g, nodes)
    assert plan.timing()["loss_fold"] == level
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))


@pytest.mark.parametrize("bad", [1.5, -0.5, float("nan")])
def test_loss_out_of_range_rejected(bad):
    """ShadowEdge::try_from's loss range (mod.rs:72-111): the one-call entry
    points check it on the device as the losses upload (the host scan skips
    them), srt_plan_create on the host, the sparse family on the host; all
    report the reference's text.  -0.0 is in range (IEEE -0.0 >= 0)."""
    from shadow_amd.plan import RoutingPlan
    g = NetworkGraph.from_edges(3, [0, 1, 2, 0, 1], [0, 1, 2, 1, 2], [5, 5, 5, 7, 9], [0.0, 0.0, 0.0, 0.1, bad],
                                directed=False)
    for algo in (_lib.SRT_ALGO_FW, _lib.SRT_ALGO_SSSP):
        with pytest.raises(_lib.SrtError) as e:
            g.compute_shortest_paths([0, 1, 2], algo=algo)
        assert e.value.code == _lib.SRT_ERR_INVALID and str(e.value) == "Edge 'packet_loss' is not in the range [0,1]"
        with pytest.raises(_lib.SrtError) as e:
            RoutingPlan(g, np.arange(3, dtype=np.uint32), algo=algo, device=0)
        assert e.value.code == _lib.SRT_ERR_INVALID and "packet_loss" in str(e.value)
    with pytest.raises(_lib.SrtError) as e:
        RoutingInfo.build(g, [0, 1, 2])
    assert "packet_loss" in str(e.value)
    ok = NetworkGraph.from_edges(3, [0, 1, 2, 0, 1], [0, 1, 2, 1, 2], [5, 5, 5, 7, 9], [0.0, 0.0, 0.0, 0.1, -0.0],
                                 directed=False)
    t = ok.compute_shortest_paths([0, 1, 2])
    assert t.latency_ns[0, 2] == 16


def test_loss_error_precedes_self_loop_error():
    """A bad loss and a missing self-loop: the parse-time loss error wins
    (mod.rs:72-111 before 210-217), although the end-to-end scan left the
    losses to the device."""
    g = NetworkGraph.from_edges(3, [0, 1, 0, 1], [0, 1, 1, 2], [5, 5, 7, 9], [0.0, 0.0, 2.0, 0.0], directed=False)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1, 2])
    assert str(e.value) == "Edge 'packet_loss' is not in the range [0,1]"
    g2 = NetworkGraph.from_edges(3, [0, 1, 0, 1], [0, 1, 1, 2], [5, 5, 7, 9], [0.0, 0.0, 0.5, 0.0], directed=False)
    with pytest.raises(_lib.SrtError) as e:
        g2.compute_shortest_paths([0, 1, 2])
    assert str(e.value) == "No edge connecting node 2 to 2"


def test_loss_checked_on_device_in_pieces():
    """4,200-node complete graph (17.6 Mi entries: two 16 Mi upload pieces):
    a bad loss in the second piece's last row is found by the device check;
    the clean graph then builds."""
    n = 4200
    row_ptr, col, lat, loss = synth.complete_csr(n, 23)
    loss = loss.copy()
    k = len(loss) - 3
    keep = loss[k]
    loss[k] = np.float32(1.25)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    with pytest.raises(_lib.SrtError) as e:
        RoutingInfo.build(g, np.arange(n, dtype=np.uint32))
    assert str(e.value) == "Edge 'packet_loss' is not in the range [0,1]"
    loss[k] = keep
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(0, n, 7, dtype=np.uint32)
    t = g.compute_shortest_paths(nodes)
    assert t.latency_ns.shape == (len(nodes), len(nodes)) and (t.latency_ns > 0).all()


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("lat_range", [(100, 1400), (1000, 1003)])
def test_quantized_level_fold(monkeypatch, seed, directed, lat_range):
    """Tight weights above the 15 exact classes but within 15x of the smallest
    one (ns-resolution latencies: C3ns): the level fold on quantized levels
    floor(L / minw) with the exact test L(s,u) + w == L(s,v) (level_q), bit for
    bit the oracle and the scan fold (SRT_LOSS_NOQ=1); (1000, 1003): heavy
    ties at one quantized level."""
    n = 120 + 31 * seed
    src, dst, lat, loss = synth.random_graph(n, 500 + seed, p_edge=0.15, directed=directed, lat_range_ns=lat_range,
                                             loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    elat, eloss = O.compute_shortest_paths(O.Graph(directed, np.arange(n), src, dst, lat, loss), nodes)
    for noq in ("0", "1"):
        if noq == "1":
            monkeypatch.setenv("SRT_LOSS_NOQ", "1")
        g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=directed)
        plan, t = _plan_table(g, nodes)
        assert plan.timing()["loss_fold"] == (1 if noq == "0" else 0), noq
        assert np.array_equal(t.latency_ns, elat)
        assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32)), f"noq={noq}"


@pytest.mark.parametrize("mixed", [False, True])
def test_piece_upload_whole_ms(small_upload_pieces, mixed):
    """The piece upload on whole-millisecond latencies (u32 ns pieces), and
    with one latency off the millisecond grid (g = 1 ns); both families,
    oracle bits (the one-call build takes the piece upload once the staging is
    pinned: srt_init first).  (A u16-millisecond upload copy halved the PCIe
    bytes but slowed the host scan that feeds it 1.8x: not kept.)"""
    err = _lib.SrtErr()
    assert _lib.lib().srt_init(0, err) == 0
    n = 150
    src, dst, lat, loss = synth.random_graph(n, 77 + mixed, p_edge=0.1, lat_range_ns=(1, 50), loss_max=0.05)
    lat = np.asarray(lat, np.uint64) * np.uint64(synth.MS)
    if mixed:
        lat[len(lat) // 2] += np.uint64(1)  # one latency off the millisecond grid
    edges = (src, dst, lat, loss)
    _check(edges, np.arange(n, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_FW)
    if not mixed:  # (g = 1 ns: the packed sparse key has no room for V x 50 ms)
        _check(edges, np.arange(0, n, 3, dtype=np.uint32), False, n, algo=_lib.SRT_ALGO_SSSP)
    _check(edges, np.arange(n, dtype=np.uint32), False, n)
