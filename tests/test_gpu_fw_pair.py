"""Grouped-round Floyd-Warshall schedule (srt_fw.hip fw_rounds_group_t) on gfx950.

One GPU at rest-bound sizes fuses FW rounds in groups: g = 4 when the block
count is a multiple of 4 and >= 96 (12k nodes), else 2 (srt_fw.hip
fw_rounds_t); an odd block count, or fewer than 2 g blocks, keeps the
single-round schedule.  SRT_FW_PAIR forces the grouped schedule at small
sizes, SRT_FW_GROUP picks g, SRT_FW_NO_PAIR turns it off and SRT_FW_BAND=1
turns on the banded tile order of grouped launches, so the same graph is
closed every way.  Bar: latency bit-exact vs the
oracle (reference Dijkstra restatement), loss bit-exact (the exact-loss pass
after the closure), and the grouped table bit-identical to the single-round
one (both compute the unique minimum latencies).
"""
import numpy as np
import pytest

from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd.plan import RoutingPlan
from tests.test_gpu_apsp import _check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("band", ["1", "0"])
@pytest.mark.parametrize("group", ["2", "4"])
@pytest.mark.parametrize("n,seed,directed", [(400, 0, False), (500, 1, True), (777, 2, False),
                                             (1000, 3, True), (1500, 5, False), (300, 4, False)])
def test_forced_groups_vs_oracle(monkeypatch, band, group, n, seed, directed):
    # 400/500 -> 4 blocks, 777/1000 -> 8, 1500 -> 12 (g=4: 3 groups); 300 -> 3
    # blocks (odd: single-round fallback); g=4 needs >= 8 blocks
    monkeypatch.setenv("SRT_FW_PAIR", "1")
    monkeypatch.setenv("SRT_FW_GROUP", group)
    monkeypatch.setenv("SRT_FW_BAND", band)
    e = synth.random_graph(n, 40 + seed, p_edge=8.0 / n, directed=directed, lat_range_ns=(1, 6), loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    _check(e, nodes, directed, n, algo=_lib.SRT_ALGO_FW)


def _table(monkeypatch, g, nodes, group):
    for k in ("SRT_FW_PAIR", "SRT_FW_NO_PAIR", "SRT_FW_GROUP"):
        monkeypatch.delenv(k, raising=False)
    if group > 1:
        monkeypatch.setenv("SRT_FW_PAIR", "1")
        monkeypatch.setenv("SRT_FW_GROUP", str(group))
    else:
        monkeypatch.setenv("SRT_FW_NO_PAIR", "1")
    plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
    try:
        plan.run()
        a, launches, work, _ = plan.kernel_stats()
        tiles = plan.kernel_tiles()
        t = plan.fetch()
    finally:
        plan.close()
    return t, launches, work / max(tiles * 128 ** 3, 1)


@pytest.mark.parametrize("n", [2048, 8192])
def test_groups_equal_single_round(monkeypatch, n):
    if n <= 2048:
        src, dst, lat, loss = synth.complete_graph(n, 7)
        g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    else:
        row_ptr, col, lat, loss = synth.complete_csr(n, 7)
        g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    nblk = n // 128
    ts, ls, rs = _table(monkeypatch, g, nodes, 1)
    assert ls == nblk and rs == 1.0
    for grp in (2, 4):
        tp, lp, rp = _table(monkeypatch, g, nodes, grp)
        assert lp == nblk // grp  # one rest launch per group of rounds
        assert 0.7 * grp < rp <= grp
        assert np.array_equal(tp.latency_ns, ts.latency_ns)
        assert np.array_equal(tp.packet_loss.view(np.uint32), ts.packet_loss.view(np.uint32))
        assert tp.min_latency_ns == ts.min_latency_ns
    L = ts.latency_ns
    assert np.array_equal(L, L.T)


@pytest.mark.parametrize("n,seed,directed", [(1000, 11, False), (1300, 12, True)])
def test_key_types_agree(monkeypatch, n, seed, directed):
    """The closure's five key representations (f16 by default here: the
    eccentricity proof; u16, u32, f64 and u64 forced by SRT_FW_KEY) produce
    the same table bits, single-round and grouped by 2 and 4."""
    e = synth.random_graph(n, seed, p_edge=6.0 / n, directed=directed, lat_range_ns=(1, 9), loss_max=0.05)
    g = NetworkGraph.from_edges(n, *e, directed=directed)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    tabs = {}
    # default: f16 keys (the eccentricity proof bounds every distance far below
    # 1024 units: a random graph of 9-unit edges); the rest forced
    for key in ("f16", "u16", "u32", "f64", "u64"):
        if key == "f16":
            monkeypatch.delenv("SRT_FW_KEY", raising=False)
        else:
            monkeypatch.setenv("SRT_FW_KEY", key)
        for grp in ("1", "2", "4"):
            monkeypatch.setenv("SRT_FW_PAIR", "1")
            monkeypatch.setenv("SRT_FW_GROUP", grp)
            plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
            assert f"{key}key" in plan.describe()
            tabs[(key, grp)] = plan.run().fetch()
            plan.close()
    ref = tabs[("u32", "1")]
    for k, t in tabs.items():
        assert np.array_equal(t.latency_ns, ref.latency_ns), k
        assert np.array_equal(t.packet_loss.view(np.uint32), ref.packet_loss.view(np.uint32)), k


@pytest.mark.parametrize("n,sym,group", [(1000, "1", None), (2048, "1", "2"), (2048, "1", "4"), (2048, "0", "4"),
                                         (4096, "1", None), (4096, "0", None), (8192, "1", None)])
def test_f16_keys_equal_u16(monkeypatch, n, sym, group):
    """Complete graphs (lmax = the longest edge, 300 units < 1024) close on
    f16 integer keys by default (v_pk_add_f16 + v_pk_minimum3_f16); the table
    must be bit-identical to the u16-integer closure (SRT_FW_KEY=u16) -- and,
    at 1000 nodes, to the oracle.  Covers the single-round schedule with the
    quarter-tile chain (1000, 4096: C2), forced groups, the grouped triangle
    (8192) and the square (SRT_FW_SYM=0)."""
    monkeypatch.setenv("SRT_FW_SYM", sym)
    if group:
        monkeypatch.setenv("SRT_FW_PAIR", "1")
        monkeypatch.setenv("SRT_FW_GROUP", group)
    if n <= 2048:
        src, dst, lat, loss = synth.complete_graph(n, 20 + n % 7)
        g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    else:
        row_ptr, col, lat, loss = synth.complete_csr(n, 21)
        g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    tabs = {}
    for key in ("f16", "u16"):
        if key == "u16":
            monkeypatch.setenv("SRT_FW_KEY", "u16")
        else:
            monkeypatch.delenv("SRT_FW_KEY", raising=False)
        plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
        try:
            assert plan.describe().startswith(f"fw:{key}key"), plan.describe()
            tabs[key] = plan.run().fetch()
            assert ("sym=triangle" in plan.describe()) == (sym == "1")
        finally:
            plan.close()
    assert np.array_equal(tabs["f16"].latency_ns, tabs["u16"].latency_ns)
    assert np.array_equal(tabs["f16"].packet_loss.view(np.uint32), tabs["u16"].packet_loss.view(np.uint32))
    assert tabs["f16"].min_latency_ns == tabs["u16"].min_latency_ns
    if n == 1000:
        from oracle import oracle as O
        elat, eloss = O.compute_shortest_paths(O.Graph(False, nodes, src, dst, lat, loss), nodes)
        assert np.array_equal(tabs["f16"].latency_ns, elat)
        assert np.array_equal(tabs["f16"].packet_loss.view(np.uint32), eloss.view(np.uint32))


@pytest.mark.parametrize("n,complete", [(8192, True), (1500, False)])
def test_symmetric_triangle_equals_full(monkeypatch, n, complete):
    """Undirected graph, u16 keys, grouped schedule: the rest launches run only
    the tiles on or above the diagonal and store each result twice
    (minplus_u16_kernel<0, true>); the table must be bit-identical to the
    full-square schedule (SRT_FW_SYM=0), and the plan must report the
    triangle.  8192 = 64 blocks (g = 2, no quarter-tile chain); 1500 forced
    to g = 4."""
    if complete:
        row_ptr, col, lat, loss = synth.complete_csr(n, 8)
        g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    else:
        monkeypatch.setenv("SRT_FW_PAIR", "1")
        monkeypatch.setenv("SRT_FW_GROUP", "4")
        e = synth.random_graph(n, 77, p_edge=8.0 / n, lat_range_ns=(1, 6), loss_max=0.05)
        g = NetworkGraph.from_edges(n, *e, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    tabs = []
    for sym in ("1", "0"):
        monkeypatch.setenv("SRT_FW_SYM", sym)
        plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
        try:
            plan.run()
            desc = plan.describe()
            tabs.append(plan.fetch())
        finally:
            plan.close()
        assert ("sym=triangle" in desc) == (sym == "1"), desc
    assert np.array_equal(tabs[0].latency_ns, tabs[1].latency_ns)
    assert np.array_equal(tabs[0].packet_loss.view(np.uint32), tabs[1].packet_loss.view(np.uint32))


def test_directed_graph_keeps_the_full_square():
    n = 1000
    e = synth.random_graph(n, 78, p_edge=8.0 / n, directed=True, lat_range_ns=(1, 6), loss_max=0.05)
    g = NetworkGraph.from_edges(n, *e, directed=True)
    plan = RoutingPlan(g, np.arange(n, dtype=np.uint32), algo=_lib.SRT_ALGO_FW)
    try:
        plan.run()
        assert "sym=triangle" not in plan.describe()
    finally:
        plan.close()


def _dense_nc(n, seed, drop=0.3):
    e = synth.dense_graph(n, seed, drop=drop)
    row_ptr, col, lat, loss = synth.dense_csr(n, e)
    return e, NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)


@pytest.mark.parametrize("n,rows", [(1024, None), (4096, 16)])
def test_eccentricity_proof_dense_noncomplete(n, rows):
    """A dense NON-complete graph (30% of the complete graph's edges dropped):
    the longest-edge bound does not apply and (V-1) x 300 units would force
    u32 keys; the eccentricity sweeps bound every distance by d(u,s) + d(s,v)
    and the plan closes on f16 keys.  Table vs the oracle: in full at 1024,
    16 seeded rows at 4096 (C2-sized)."""
    from oracle import oracle as O
    e, g = _dense_nc(n, 30 + n % 5)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
    try:
        d = plan.describe()
        assert d.startswith("fw:f16key") and "(ecc)" in d, d
        t = plan.run().fetch()
    finally:
        plan.close()
    og = O.Graph(False, nodes, *e)
    if rows is None:
        elat, eloss = O.compute_shortest_paths(og, nodes)
        assert np.array_equal(t.latency_ns, elat)
        assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))
        return
    pick = np.random.default_rng(n).choice(n, rows, replace=False)
    order = np.concatenate([pick, np.setdiff1d(nodes, pick)]).astype(np.uint32)
    elat, eloss = O.compute_shortest_paths(og, order, src_count=rows, mode=1)
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    for i, r in enumerate(pick):
        exp_l, exp_p = elat[i][inv], eloss[i][inv].view(np.uint32)
        exp_l[r], exp_p[r] = t.latency_ns[r, r], t.packet_loss[r, r].view(np.uint32)  # raw self-loop
        assert np.array_equal(t.latency_ns[r], exp_l), r
        assert np.array_equal(t.packet_loss[r].view(np.uint32), exp_p), r


def test_eccentricity_proof_saturates_long_edges():
    """Edges far longer than the graph's diameter (50,000 units, > the u16
    and f16 key ranges) cannot lie on a shortest path: the init stores them
    as INF and the narrow key stays exact -- vs the oracle in full."""
    from oracle import oracle as O
    n = 600
    src, dst, lat, loss = synth.random_graph(n, 91, p_edge=0.05, lat_range_ns=(1, 9), loss_max=0.05)
    lat = lat.copy()
    long_ = np.random.default_rng(91).random(len(lat)) < 0.02
    lat[long_ & (src != dst)] = 50_000
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
    try:
        assert plan.describe().startswith("fw:f16key") and "(ecc)" in plan.describe(), plan.describe()
        t = plan.run().fetch()
    finally:
        plan.close()
    elat, eloss = O.compute_shortest_paths(O.Graph(False, nodes, src, dst, lat, loss), nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))


def test_eccentricity_proof_needs_strong_connectivity():
    """A directed graph with a node nobody reaches: the sweeps from node 0 miss
    it, so no diameter bound is claimed and the (V-1) x max edge proof picks
    the key (u16 here: 2 x 299 x 9 < 2^15)."""
    n = 300
    src, dst, lat, loss = synth.random_graph(n, 92, p_edge=0.05, directed=True, lat_range_ns=(1, 9))
    keep = dst != 7  # no edge into node 7 (its self-loop is dropped too ...)
    src, dst, lat, loss = src[keep], dst[keep], lat[keep], loss[keep]
    src, dst = np.append(src, 7).astype(np.uint32), np.append(dst, 7).astype(np.uint32)  # ... and restored
    lat, loss = np.append(lat, 3).astype(np.uint64), np.append(loss, 0.0).astype(np.float32)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=True)
    plan = RoutingPlan(g, np.array([0, 1, 2], np.uint32), algo=_lib.SRT_ALGO_FW)
    try:
        assert plan.describe().startswith("fw:u16key") and "(V-1)" in plan.describe(), plan.describe()
    finally:
        plan.close()


@pytest.mark.parametrize("key", ["f16", "u16"])
@pytest.mark.parametrize("rows", ["2", "4", "8"])
def test_phase1_two_steps_per_barrier(monkeypatch, key, rows):
    """Phase 1 at two FW steps per barrier (fw_phase1_pk2_kernel: rows and
    columns k, k+1 published together, column/row k+1 advanced by step k in
    registers) gives the one-step kernel's bits and the oracle's, for f16 and
    u16 keys and every rows-per-thread layout."""
    monkeypatch.setenv("SRT_FW_P1_ROWS", rows)
    if key == "u16":
        monkeypatch.setenv("SRT_FW_KEY", "u16")
    n = 700
    src, dst, lat, loss = synth.complete_graph(n, 40 + int(rows))
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    tabs = {}
    for two in ("1", "0"):
        monkeypatch.setenv("SRT_FW_P1", two)
        plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
        try:
            assert plan.describe().startswith(f"fw:{key}key"), plan.describe()
            tabs[two] = plan.run().fetch()
        finally:
            plan.close()
    from oracle import oracle as O
    elat, eloss = O.compute_shortest_paths(O.Graph(False, nodes, src, dst, lat, loss), nodes)
    for two, t in tabs.items():
        assert np.array_equal(t.latency_ns, elat), two
        assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32)), two


@pytest.mark.parametrize("key", ["f16", "u16"])
@pytest.mark.parametrize("directed", [False, True])
def test_phase1_long_paths(monkeypatch, key, directed):
    """Pivot blocks whose shortest paths run through ~127 hops inside the block
    (a path graph over consecutive ids, plus a few chords): both phase-1 forms
    equal the oracle."""
    if key == "u16":
        monkeypatch.setenv("SRT_FW_KEY", "u16")
    n = 390
    rng = np.random.default_rng(7)
    ids = np.arange(n - 1, dtype=np.uint32)
    pairs = {(min(a, b), max(a, b)) for a, b in rng.integers(0, n, size=(24, 2)) if abs(int(a) - int(b)) > 1}
    ch = np.array(sorted(pairs), np.uint32)[:12]
    if directed:  # the path both ways (own weights), chords one way
        src = np.concatenate([ids, ids + 1, ch[:, 0], np.arange(n, dtype=np.uint32)])
        dst = np.concatenate([ids + 1, ids, ch[:, 1], np.arange(n, dtype=np.uint32)])
        npath = 2 * (n - 1)
    else:
        src = np.concatenate([ids, ch[:, 0], np.arange(n, dtype=np.uint32)])
        dst = np.concatenate([ids + 1, ch[:, 1], np.arange(n, dtype=np.uint32)])
        npath = n - 1
    m = len(src)
    lat = (rng.choice([1, 2], size=m, p=[0.85, 0.15]) * 1_000_000).astype(np.uint64)
    lat[npath:npath + len(ch)] = 900_000_000  # long chords: the path stays the shortest way
    lat[m - n:] = 1_000_000  # self-loops
    loss = np.round(rng.uniform(0.0, 0.01, size=m), 6).astype(np.float32)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=directed)
    nodes = np.arange(n, dtype=np.uint32)
    tabs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SRT_FW_P1", mode)
        plan = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW)
        try:
            assert plan.describe().startswith(f"fw:{key}key"), plan.describe()
            tabs[mode] = plan.run().fetch()
        finally:
            plan.close()
    from oracle import oracle as O
    elat, eloss = O.compute_shortest_paths(O.Graph(directed, nodes, src, dst, lat, loss), nodes)
    for mode, t in tabs.items():
        assert np.array_equal(t.latency_ns, elat), mode
        assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32)), mode
