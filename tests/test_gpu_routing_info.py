"""Dense RoutingInfo behind the C ABI (srt_routing_info_*, include/srt.h) vs
the reference's generate_routing_info + RoutingInfo (sim_config.rs:424-461,
graph/mod.rs:428-477) restated over the oracle's table: path() keyed by GML
ids (None for ids that are not in use), get_smallest_latency_ns, packet
counters with saturating add, and the direct-path mode."""
import os
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, RoutingInfo, generate_routing_info, synth
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _graph(n, seed, directed=False):
    src, dst, lat, loss = synth.random_graph(n, seed, p_edge=0.1, directed=directed, lat_range_ns=(1, 7),
                                             loss_max=0.05)
    ids = (np.random.default_rng(seed).permutation(n) * 7 + 1000).astype(np.uint32)  # sparse GML ids
    return NetworkGraph.from_edges(n, src, dst, lat, loss, directed=directed, node_ids=ids), (src, dst, lat, loss), ids


@pytest.mark.parametrize("directed", [False, True])
def test_generate_routing_info_matches_reference_keying(directed):
    n = 150
    g, e, ids = _graph(n, 21, directed)
    in_use = set(int(x) for x in ids[np.random.default_rng(2).choice(n, 60, replace=False)])
    ri = generate_routing_info(g, in_use)
    assert len(ri) == 60
    # the reference: shortest paths between the in-use NodeIndexes, re-keyed by GML id
    nodes = np.array([g.node_id_to_index(x) for x in in_use], np.uint32)
    elat, eloss = O.compute_shortest_paths(O.Graph(directed, ids, *e), nodes)
    gid = [int(ids[v]) for v in nodes]
    for i, a in enumerate(gid):
        for j, b in enumerate(gid):
            p = ri.path(a, b)
            assert p.latency_ns == int(elat[i, j])
            assert np.float32(p.packet_loss).view(np.uint32) == eloss[i, j].view(np.uint32)
    assert ri.path(gid[0], 999_999) is None and ri.path(5, gid[0]) is None  # not in use -> None
    not_in_use = int(next(x for x in ids if int(x) not in in_use))
    assert ri.path(not_in_use, gid[0]) is None and ri.row_of(not_in_use) is None
    assert ri.get_smallest_latency_ns() == int(elat.min())
    ri.close()


def test_packet_counters_saturate_and_merge_device_counts():
    n = 40
    g, _, ids = _graph(n, 22)
    ri = generate_routing_info(g, set(int(x) for x in ids))
    a, b = int(ids[3]), int(ids[7])
    for _ in range(5):
        ri.increment_packet_count(a, b)
    assert ri.packet_count(a, b) == 5 and ri.packet_count(b, a) == 0
    counts = np.zeros((n, n), np.uint64)
    i, j = ri.row_of(a), ri.row_of(b)
    counts[i, j] = np.uint64(2**64 - 3)
    counts[j, i] = np.uint64(11)
    ri.add_packet_counts(counts)
    assert ri.packet_count(a, b) == 2**64 - 1  # saturating_add (mod.rs:453)
    ri.increment_packet_count(a, b)
    assert ri.packet_count(a, b) == 2**64 - 1
    assert ri.packet_count(b, a) == 11
    ri.increment_packet_count(12345678, b)  # not in use: ignored
    ri.close()


def test_direct_paths_mode_and_from_plan():
    n = 30
    src, dst, lat, loss = synth.complete_graph(n, 23)
    ids = (np.arange(n) + 50).astype(np.uint32)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, node_ids=ids)
    ri = generate_routing_info(g, set(int(x) for x in ids), use_shortest_paths=False)
    og = O.Graph(False, ids, src, dst, lat, loss)
    nodes = np.array([g.node_id_to_index(int(x)) for x in ids], np.uint32)
    dl, dp = O.get_direct_paths(og, nodes)
    for i, v in enumerate(nodes):
        for j, w in enumerate(nodes):
            p = ri.path(int(ids[v]), int(ids[w]))
            assert p.latency_ns == int(dl[i, j]) and np.float32(p.packet_loss) == dp[i, j]
    ri.close()
    # from a plan that has run: same table as the one-shot build
    nodes = np.random.default_rng(3).permutation(n).astype(np.uint32)
    plan = RoutingPlan(g, nodes).run()
    r2 = RoutingInfo.from_plan(plan)
    r3 = RoutingInfo.build(g, nodes)
    l2, p2 = r2.table()
    l3, p3 = r3.table()
    assert np.array_equal(l2, l3) and np.array_equal(p2.view(np.uint32), p3.view(np.uint32))
    assert r2.get_smallest_latency_ns() == r3.get_smallest_latency_ns()
    plan.close()
    r2.close()
    r3.close()


def test_empty_in_use_set():
    g, _, _ = _graph(10, 24)
    ri = generate_routing_info(g, set())
    assert len(ri) == 0 and ri.get_smallest_latency_ns() is None
    ri.close()


@pytest.mark.parametrize("key,rec", [(None, 6), ("u32", 8)])
def test_compact_storage_matches_oracle(monkeypatch, key, rec):
    """srt_routing_info_build keeps the dense build's table as downloaded --
    6-byte records (u16 latency units + f32 loss) for u16/f16-key closures, 8
    bytes (u32 units + loss) for u32 keys -- and path() decodes them: every
    pair equals the oracle's bits, the diagonal is the raw self-loop."""
    from shadow_amd import _lib
    if key:
        monkeypatch.setenv("SRT_FW_KEY", key)
    n = 600
    src, dst, lat, loss = synth.complete_graph(n, 25)
    ids = (np.arange(n) * 3 + 7).astype(np.uint32)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, node_ids=ids)
    nodes = np.arange(n, dtype=np.uint32)
    ri = RoutingInfo.build(g, nodes, algo=_lib.SRT_ALGO_FW)
    assert ri.record_bytes() == rec
    L, P = ri.table()
    elat, eloss = O.compute_shortest_paths(O.Graph(False, ids, src, dst, lat, loss), nodes)
    assert np.array_equal(L, elat)
    assert np.array_equal(P.view(np.uint32), eloss.view(np.uint32))
    p = ri.path(int(ids[5]), int(ids[5]))
    assert p.latency_ns == int(elat[5, 5])
    ri.close()


def test_self_loop_beyond_the_record_field():
    """A non-complete graph whose key width comes from the eccentricity proof
    (path latencies < 1024 units: f16 keys, 6-byte records) but with one
    self-loop of 200 s (200,000 units, past the u16 field): the diagonal is the
    raw self-loop in both the end-to-end srt_path table and the compact
    RoutingInfo -- it travels beside the records, not in them."""
    from shadow_amd import _lib
    n = 300
    src, dst, lat, loss = synth.dense_graph(n, 26, drop=0.4)
    lat = lat.copy()
    big = np.nonzero((src == dst) & (src == 17))[0][0]
    lat[big] = np.uint64(200_000) * np.uint64(synth.MS)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
    t = g.compute_shortest_paths(nodes, algo=_lib.SRT_ALGO_FW)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))
    ri = RoutingInfo.build(g, nodes, algo=_lib.SRT_ALGO_FW)
    assert ri.record_bytes() == 6
    assert ri.path(17, 17).latency_ns == 200_000 * synth.MS
    L, P = ri.table()
    assert np.array_equal(L, elat) and np.array_equal(P.view(np.uint32), eloss.view(np.uint32))
    ri.close()


def test_init_then_build():
    """srt_init (HIP runtime, kernel code objects, pinned staging) and
    srt_init_async ahead of a build: idempotent, and the build that follows
    waits for a pending init and matches the oracle."""
    import shadow_amd
    shadow_amd.init_async(0)
    shadow_amd.init(0)
    shadow_amd.init(0)
    shadow_amd.init_async(0)
    n = 120
    src, dst, lat, loss = synth.complete_graph(n, 27)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    ri = RoutingInfo.build(g, nodes)
    L, P = ri.table()
    elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
    assert np.array_equal(L, elat) and np.array_equal(P.view(np.uint32), eloss.view(np.uint32))
    ri.close()


@pytest.mark.gpu
def test_init_async_then_exit_without_building():
    """srt_init_async, then the process exits at once: the library joins its
    init thread before the HIP runtime goes away (no std::terminate, no abort),
    and a plan created right after the call waits for the init first."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import shadow_amd; shadow_amd.init_async(0)"
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    # straight through ctypes, without the package's atexit wait: the
    # library's own exit-time join (a thread_local guard) must suffice
    code = "from shadow_amd import _lib; _lib.lib().srt_init_async(0)"
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    code = ("import numpy as np, shadow_amd; from shadow_amd import synth, NetworkGraph; "
            "from shadow_amd.plan import RoutingPlan; shadow_amd.init_async(0); "
            "s, d, l, p = synth.complete_graph(8, 1); "
            "pl = RoutingPlan(NetworkGraph.from_edges(8, s, d, l, p), np.arange(8, dtype=np.uint32)).run(); "
            "print(pl.fetch().latency_ns[0, 1])")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip(), r.stderr[-2000:]
