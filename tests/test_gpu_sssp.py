"""GPU parity of the sparse routing build (srt_frontier.hip / srt_sssp.hip, SRT_ALGO_SSSP) against
the oracle's restatement of petgraph's Dijkstra.

Bar: latency bit-exact AND packet_loss bit-exact -- the sweep folds loss with
the reference's own f32 Add (mod.rs:322-331), so unlike the dense closure no
tolerance is needed; diagonal = raw self-loop; min latency exact; reference
error codes.  All calls go through the C ABI (shadow_amd.graph -> libsrt.so).
"""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu
SSSP = _lib.SRT_ALGO_SSSP


@pytest.fixture(autouse=True, params=["frontier", "frontier-small", "frontier-first", "frontier-nosym", "packed",
                                      "packed-delta", "packed-fine"])
def sweep_mode(request, monkeypatch):
    """Every test runs the sparse build five ways, all of which must give the
    same bits: the latency-first frontier sweeps (srt_frontier.hip, the default
    when every distance fits u16 units), the same with one 512-source block a
    launch, a 3-workgroup sweep grid and sources in table order (several
    launches share the sweep stamps; waves loop over many chunks; undirected
    graphs seed each launch from the earlier rows' columns), launches of two
    blocks after a first launch of one, with the dense sweeps off (unequal
    launches, buffers larger than a launch; every sweep on its marks), the
    same without that symmetric seeding, and the
    packed-key sweep (srt_sssp.hip, SRT_SSSP_KEY=64) ungated, with
    delta-stepping at a quarter of the mean in-edge latency and with very narrow
    buckets (factor 0.01: most keys wait in the pending masks)."""
    for k in ("SRT_SSSP_DELTA", "SRT_SSSP_ORDER", "SRT_SSSP_KEY", "SRT_SSSP_FR_NB", "SRT_SSSP_FR_GRID",
              "SRT_SSSP_SYM", "SRT_FR_FIRST", "SRT_FR_DENSE"):
        monkeypatch.delenv(k, raising=False)
    if request.param == "frontier-nosym":
        monkeypatch.setenv("SRT_SSSP_FR_NB", "1")
        monkeypatch.setenv("SRT_SSSP_SYM", "0")
    if request.param == "frontier-first":
        monkeypatch.setenv("SRT_SSSP_FR_NB", "2")
        monkeypatch.setenv("SRT_FR_FIRST", "1")
        monkeypatch.setenv("SRT_FR_DENSE", "0")
    if request.param == "frontier-small":
        monkeypatch.setenv("SRT_SSSP_FR_NB", "1")
        monkeypatch.setenv("SRT_SSSP_FR_GRID", "3")
        monkeypatch.setenv("SRT_SSSP_ORDER", "0")
    elif request.param.startswith("packed"):
        monkeypatch.setenv("SRT_SSSP_KEY", "64")
    if request.param == "packed-delta":
        monkeypatch.setenv("SRT_SSSP_DELTA", "0.25")
        monkeypatch.setenv("SRT_SSSP_ORDER", "0")  # sources in table order (default: BFS order)
    elif request.param == "packed-fine":
        monkeypatch.setenv("SRT_SSSP_DELTA", "0.01")
    return request.param


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check(edges, nodes, directed, n_nodes, node_ids=None):
    src, dst, lat, loss = edges
    ids = np.arange(n_nodes) if node_ids is None else node_ids
    elat, eloss = O.compute_shortest_paths(O.Graph(directed, ids, src, dst, lat, loss), nodes)
    g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss, directed=directed, node_ids=ids)
    t = g.compute_shortest_paths(nodes, algo=SSSP)
    assert np.array_equal(t.latency_ns, elat), "latency must be bit-exact"
    assert np.array_equal(_bits(t.packet_loss), _bits(eloss)), "loss must be bit-exact (reference f32 fold)"
    assert t.min_latency_ns == int(elat.min())
    return t


@pytest.mark.parametrize("directed", [1, 0])
def test_reference_golden_three_node(directed):
    from tests.test_gpu_apsp import GOLDEN_DIRECTED, GOLDEN_UNDIRECTED, _three
    g = NetworkGraph.parse(_three(directed))
    nodes = [g.node_id_to_index(0), g.node_id_to_index(1), g.node_id_to_index(2)]
    t = g.compute_shortest_paths(nodes, algo=SSSP)
    assert t.latency_ns.tolist() == (GOLDEN_DIRECTED if directed else GOLDEN_UNDIRECTED)
    assert t.min_latency_ns == 3


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("directed", [False, True])
def test_random_tie_heavy(seed, directed):
    # few distinct latencies -> many equal-latency paths: the loss tie-break decides
    n = 60 + 37 * seed  # ragged batches of 64 sources
    e = synth.random_graph(n, 20 + seed, p_edge=0.08, directed=directed, lat_range_ns=(1, 4), loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    _check(e, nodes, directed, n)


@pytest.mark.parametrize("seed", range(3))
def test_subset_in_use_intermediates(seed):
    # sources/destinations only in-use nodes; any node is an intermediate (mod.rs:203)
    n = 400
    e = synth.random_graph(n, 200 + seed, p_edge=0.01, directed=True, lat_range_ns=(1, 30))
    nodes = np.random.default_rng(seed).choice(n, 97, replace=False).astype(np.uint32)
    _check(e, nodes, True, n)


def test_high_loss_and_loss_one_edges():
    n = 90
    src, dst, lat, loss = synth.random_graph(n, 11, p_edge=0.05, lat_range_ns=(1, 3), loss_max=0.9)
    loss[::7] = 1.0
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n)


def test_ms_latencies_gcd_unit():
    # latencies in whole ms: the key carries latency / gcd (1 ms) and must scale back exactly
    n = 150
    src, dst, lat, loss = synth.random_graph(n, 12, p_edge=0.04, lat_range_ns=(1, 300))
    lat = lat * np.uint64(synth.MS)
    _check((src, dst, lat, loss), np.arange(n, dtype=np.uint32), False, n)


def test_single_node():
    g = NetworkGraph.from_edges(1, [0], [0], [42], [0.25], directed=False, node_ids=[9])
    t = g.compute_shortest_paths([0], algo=SSSP)
    assert t.latency_ns.tolist() == [[42]] and t.packet_loss[0, 0] == np.float32(0.25)


def test_disconnected_raises():
    g = NetworkGraph.from_edges(3, [0, 1, 2, 0], [0, 1, 2, 1], [5, 5, 5, 3], directed=True)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1, 2], algo=SSSP)
    assert e.value.code == _lib.SRT_ERR_DISCONNECTED


def test_missing_selfloop_error_text():
    g = NetworkGraph.from_edges(2, [0, 0], [0, 1], [5, 5], directed=False, node_ids=[4, 8])
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1], algo=SSSP)
    assert e.value.code == _lib.SRT_ERR_NO_EDGE and str(e.value) == "No edge connecting node 8 to 8"


def test_latency_field_overflow_is_refused():
    # V * max latency must fit the 32-bit latency field; otherwise SSSP is unsupported
    n = 4
    src = np.array([0, 1, 2, 3, 0, 1, 2], np.uint32)
    dst = np.array([0, 1, 2, 3, 1, 2, 3], np.uint32)
    lat = np.array([1, 1, 1, 1, 1, 1, 2**31], np.uint64)
    g = NetworkGraph.from_edges(n, src, dst, lat, directed=False)
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths(np.arange(n), algo=SSSP)
    assert e.value.code == _lib.SRT_ERR_UNSUPPORTED


def test_auto_picks_sssp_for_sparse():
    src, dst, lat, loss = synth.barabasi_albert(3000, 4, 4)
    g = NetworkGraph.from_edges(3000, src, dst, lat, loss)
    plan = RoutingPlan(g, np.arange(64, dtype=np.uint32))
    assert plan.describe().startswith("sssp")
    plan.close()


def test_c4_graph_row_sample():
    """Config C4's graph (100k-node Barabasi-Albert, m=4, seed 4): 2,048 in-use
    nodes spread over the graph (every other node is an intermediate), several
    source groups; oracle rows for a seeded sample, plus symmetry."""
    V = 100_000
    src, dst, lat, loss = synth.barabasi_albert(V, 4, 4)
    g = NetworkGraph.from_edges(V, src, dst, lat, loss)
    rng = np.random.default_rng(4)
    nodes = rng.choice(V, 2048, replace=False).astype(np.uint32)
    t = g.compute_shortest_paths(nodes)  # AUTO must pick the sparse path here
    L = t.latency_ns
    assert np.array_equal(L, L.T)  # undirected
    og = O.Graph(False, np.arange(V), src, dst, lat, loss)
    k = 12
    rows = rng.choice(len(nodes), k, replace=False)
    order = np.concatenate([rows, np.setdiff1d(np.arange(len(nodes)), rows)])
    elat, eloss = O.compute_shortest_paths(og, nodes[order], src_count=k)
    inv = np.argsort(order)
    for i, r in enumerate(rows):
        el, ep = elat[i][inv], eloss[i][inv]
        el[r], ep[r] = L[r, r], t.packet_loss[r, r]  # diagonal: raw self-loop
        assert np.array_equal(L[r], el)
        assert np.array_equal(_bits(t.packet_loss[r]), _bits(ep))


@pytest.mark.parametrize("seed", [31, 32])
def test_loss_sweeps_over_reused_rows(monkeypatch, sweep_mode, seed):
    """The frontier loss sweeps' same-sweep reads: a reader can see a parent's
    change bit before that parent's P store lands (or a stale line in its own
    L1).  Correct because every P value a reader can see for (s, v) within a
    launch is >= the final one -- the tight pass stores 2.0 ("not reached"),
    then only improvements follow -- so a stale read delays a fold to the next
    sweep and never corrupts it.  Here one 512-source block a launch, so every
    launch reuses the P rows the previous launch left (without the 2.0 start a
    stale read returns another source's loss: the r05 failure that
    test_c4_graph_row_sample caught at C4 scale), over tie-heavy latencies
    (many tight in-edges, many loss sweeps); every row against the oracle."""
    if sweep_mode.startswith("frontier"):
        monkeypatch.setenv("SRT_SSSP_FR_NB", "1")
    n = 2500
    e = synth.barabasi_albert(n, 4, seed, lat_ms=(1, 6), loss_max=0.05)
    _check(e, np.arange(n, dtype=np.uint32), False, n)


def test_fw_and_sssp_agree_on_latency():
    # the dense closure + exact-loss pass and the sparse sweep on one graph: same bits
    n = 300
    e = synth.random_graph(n, 77, p_edge=0.03, lat_range_ns=(1, 6), loss_max=0.02)
    g = NetworkGraph.from_edges(n, *e)
    nodes = np.arange(n, dtype=np.uint32)
    a = g.compute_shortest_paths(nodes, algo=_lib.SRT_ALGO_FW)
    b = g.compute_shortest_paths(nodes, algo=SSSP)
    assert np.array_equal(a.latency_ns, b.latency_ns)
    assert np.array_equal(a.packet_loss.view(np.uint32), b.packet_loss.view(np.uint32))


@pytest.mark.parametrize("act", ["2", "3", "0"])
@pytest.mark.parametrize("directed", [False, True])
def test_target_activation_bit_exact(monkeypatch, act, directed):
    """Tail-sweep target activation (srt_sssp.hip ACT_SET/ACT_USE): forced on
    from an early sweep (SRT_SSSP_ACT=k) or off, the sweep must return the same
    bits as the oracle -- a target is skipped only when no in-neighbour changed.
    Directed graphs take the out-neighbour marks from the outgoing CSR rows."""
    monkeypatch.setenv("SRT_SSSP_ACT", act)
    n = 700
    if directed:
        edges = synth.random_graph(n, 11, p_edge=0.012, directed=True, lat_range_ns=(1, 40), loss_max=0.05)
    else:
        edges = synth.barabasi_albert(n, 3, 12)
    nodes = np.arange(0, n, 2, dtype=np.uint32)
    _check(edges, nodes, directed, n)


def test_long_ring(sweep_mode):
    """A 90-node ring of 1,000-2,000 ns edges (gcd 1: the far side is ~67k
    latency units away, thousands of narrow buckets deep), bit-exact."""
    n = 90
    rng = np.random.default_rng(5)
    src = np.concatenate([np.arange(n), np.arange(n)]).astype(np.uint32)
    dst = np.concatenate([np.arange(n), (np.arange(n) + 1) % n]).astype(np.uint32)
    lat = rng.integers(1000, 2000, 2 * n).astype(np.uint64) | np.uint64(1)
    loss = rng.uniform(0, 0.05, 2 * n).astype(np.float32)
    nodes = np.arange(n, dtype=np.uint32)
    _check((src, dst, lat, loss), nodes, False, n)


def test_sweep_family_is_reported(sweep_mode):
    """The plan names its sweep: the frontier sweeps (u16 latencies) unless the
    packed-key sweep is forced, which names its bucket width (0 = ungated)."""
    src, dst, lat, loss = synth.barabasi_albert(500, 3, 9)
    g = NetworkGraph.from_edges(500, src, dst, lat, loss)
    plan = RoutingPlan(g, np.arange(100, dtype=np.uint32), algo=SSSP)
    d = plan.describe()
    if sweep_mode.startswith("frontier"):
        assert d.startswith("sssp:frontier u16") and "(ecc)" in d, d
        # source order: launches breadth-first, rows within them in
        # shortest-latency-tree level order (table order when forced)
        assert (" order=table " in d) if sweep_mode == "frontier-small" else (" order=bfs+tree " in d), d
    else:
        delta = int(d.split(" delta=")[1].split()[0])
        assert (delta == 0) == (sweep_mode == "packed"), d
    plan.close()


def test_wide_latencies_fall_back_to_packed_keys(sweep_mode):
    """A 90-node ring at ns resolution (gcd 1): the far side is ~67k units away,
    past the frontier's u16 latencies, so the plan keeps the packed u64 keys."""
    n = 90
    rng = np.random.default_rng(5)
    src = np.concatenate([np.arange(n), np.arange(n)]).astype(np.uint32)
    dst = np.concatenate([np.arange(n), (np.arange(n) + 1) % n]).astype(np.uint32)
    lat = rng.integers(1000, 2000, 2 * n).astype(np.uint64) | np.uint64(1)
    g = NetworkGraph.from_edges(n, src, dst, lat, np.zeros(2 * n, np.float32))
    plan = RoutingPlan(g, np.arange(n, dtype=np.uint32), algo=SSSP)
    assert plan.describe().startswith("sssp:lat32"), plan.describe()
    plan.close()


def test_repeated_runs_same_bits(sweep_mode):
    """Sweep stamps grow across launches and runs and are never cleared: a plan
    run three times returns the same table (several launches per run in the
    small-block mode)."""
    n = 1300
    src, dst, lat, loss = synth.barabasi_albert(n, 3, 21)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(0, n, 1, dtype=np.uint32)
    plan = RoutingPlan(g, nodes, algo=SSSP)
    if sweep_mode == "frontier-small":
        assert "seed=sym" in plan.describe(), plan.describe()
    if sweep_mode == "frontier-first":
        assert "seed=sym" in plan.describe() and " first=1 " in plan.describe(), plan.describe()
    ref = None
    for _ in range(3):
        plan.run()
        t = plan.fetch()
        if ref is None:
            ref = t
            elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
            assert np.array_equal(t.latency_ns, elat)
            assert np.array_equal(_bits(t.packet_loss), _bits(eloss))
        else:
            assert np.array_equal(t.latency_ns, ref.latency_ns)
            assert np.array_equal(_bits(t.packet_loss), _bits(ref.packet_loss))
    plan.close()
