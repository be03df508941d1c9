"""GPU parity of the level solve (SRT_ALGO_LEVEL, srt_loss.hip
level_solve_kernel): per-source bucket Dijkstra over the edges of at most B
latency units, B the create-time probe's bound on every in-use shortest path.

Bar: latency and loss bit-exact against the oracle (the petgraph-faithful
restatement of mod.rs:183-228), diagonal = the raw self-loop, min latency
exact; the level tables equal the Floyd-Warshall family's bit for bit; graphs
the probe cannot bound are refused when LEVEL is forced, and AUTO then takes
another family with the same result."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, RoutingInfo, _lib, synth
from shadow_amd import dist as sdist
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _random(n, seed, directed, lat=(1, 9), p_edge=0.08, subset=None):
    src, dst, l, loss = synth.random_graph(n, seed, p_edge=p_edge, directed=directed, lat_range_ns=lat, loss_max=0.05)
    g = NetworkGraph.from_edges(n, src, dst, l, loss, directed=directed)
    rng = np.random.default_rng(seed)
    nodes = rng.permutation(n).astype(np.uint32)
    if subset:
        nodes = nodes[:subset]
    return g, nodes, O.Graph(directed, np.arange(n), src, dst, l, loss)


def _check(t, og, nodes):
    elat, eloss = O.compute_shortest_paths(og, nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(_bits(t.packet_loss), _bits(eloss))
    assert t.min_latency_ns == int(elat.min())


@pytest.mark.parametrize("n,seed,directed,lat,p_edge,subset", [
    (40, 1, False, (1, 9), 0.2, None), (300, 2, False, (1, 9), 0.08, None), (300, 3, True, (1, 9), 0.08, None),
    (1000, 4, False, (1, 20), 0.05, 700), (1000, 5, True, (1, 5), 0.05, None), (2000, 6, False, (1, 31), 0.3, 1500),
    (777, 7, True, (2, 12), 0.05, 300)])
def test_level_matches_oracle(n, seed, directed, lat, p_edge, subset):
    g, nodes, og = _random(n, seed, directed, lat, p_edge, subset)
    p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    try:
        assert p.describe().startswith("level:"), p.describe()
        _check(p.fetch(), og, nodes)
    finally:
        p.close()


def test_level_c1_complete_graph_auto():
    """C1's 1,000-node complete graph (1-300 ms): AUTO takes the level solve
    (B from the probe, a few ms) and matches the oracle."""
    n = 1000
    src, dst, lat, loss = synth.complete_graph(n, 1)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.random.default_rng(1).permutation(n).astype(np.uint32)
    p = RoutingPlan(g, nodes, device=0).run()
    try:
        d = p.describe()
        assert d.startswith("level:") and "auto-price=" in d, d
        _check(p.fetch(), O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
    finally:
        p.close()


@pytest.mark.parametrize("n,drop", [(4096, 0.0), (3000, 0.3)])
def test_level_equals_fw(n, drop):
    """C2's 4k complete graph (and a 30%-dropped dense one): the level tables
    equal the Floyd-Warshall family's bit for bit, on the device."""
    import torch

    edges = synth.complete_graph(n, 2) if drop == 0.0 else synth.dense_graph(n, 2, drop=drop)
    g = NetworkGraph.from_edges(n, *edges)
    nodes = np.arange(n, dtype=np.uint32)
    a = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    b = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW, device=0).run()
    try:
        a.fetch(table=False)
        b.fetch(table=False)
        assert a.min_latency_ns == b.min_latency_ns
        la, pa, _ = a.table_ptrs()
        lb, pb, _ = b.table_ptrs()
        dev = torch.device("cuda", 0)
        t = lambda ptr, nb: torch.as_tensor(sdist._CudaBuf(ptr, nb), device=dev)
        assert torch.equal(t(la, n * n * 8), t(lb, n * n * 8)), "latency"
        assert torch.equal(t(pa, n * n * 4), t(pb, n * n * 4)), "loss bits"
        rows = np.random.default_rng(n).choice(n, 6, replace=False)
        order = np.concatenate([rows, np.setdiff1d(nodes, rows)]).astype(np.uint32)
        elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), *edges), order, src_count=6)
        inv = np.empty(n, np.int64)
        inv[order] = np.arange(n)
        L = t(la, n * n * 8).view(torch.int64).view(n, n)
        P = t(pa, n * n * 4).view(torch.int32).view(n, n)
        for k, r in enumerate(rows):
            got_l = L[r].cpu().numpy().view(np.uint64)
            got_p = P[r].cpu().numpy().view(np.uint32)
            exp_l, exp_p = elat[k][inv], _bits(eloss[k][inv])
            m = np.arange(n) != r  # the diagonal: the raw self-loop (checked by the oracle tests)
            assert np.array_equal(got_l[m], exp_l[m]) and np.array_equal(got_p[m], exp_p[m]), f"row {r}"
    finally:
        a.close()
        b.close()


def test_level_refused_when_unbounded_auto_falls_back():
    """A ring of 100 unit edges: shortest paths up to 50 units, beyond the
    probe's 31 levels -- forced LEVEL is refused (SRT_ERR_UNSUPPORTED), AUTO
    builds with another family and matches the oracle."""
    n = 100
    src = np.concatenate([np.arange(n), np.arange(n)]).astype(np.uint32)
    dst = np.concatenate([(np.arange(n) + 1) % n, np.arange(n)]).astype(np.uint32)
    lat = np.ones(len(src), np.uint64) * np.uint64(synth.MS)
    loss = np.full(len(src), 0.001, np.float32)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    with pytest.raises(_lib.SrtError) as e:
        RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0)
    assert e.value.code == _lib.SRT_ERR_UNSUPPORTED
    p = RoutingPlan(g, nodes, device=0).run()
    try:
        assert not p.describe().startswith("level:")
        _check(p.fetch(), O.Graph(False, np.arange(n), src, dst, lat, loss), nodes)
    finally:
        p.close()


def test_level_disconnected_in_use_node():
    """An in-use node no edge reaches: the probe finds no bound (LEVEL is
    refused), and AUTO's build reports the reference's assert_eq! panic."""
    n = 50
    g0, nodes, og = _random(n, 11, False, (1, 9), 0.3)
    src, dst, lat, loss = og.src, og.dst, og.lat, og.loss
    keep = (src != 7) & (dst != 7) | ((src == 7) & (dst == 7))
    g = NetworkGraph.from_edges(n, src[keep], dst[keep], lat[keep], loss[keep])
    with pytest.raises(_lib.SrtError) as e:
        RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0)
    assert e.value.code == _lib.SRT_ERR_UNSUPPORTED
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths(nodes)
    assert e.value.code == _lib.SRT_ERR_DISCONNECTED


@pytest.mark.parametrize("n", [1000, 2500])
def test_level_one_call_and_routing_info(n):
    """The one-call builds (srt_compute_shortest_paths into srt_path,
    srt_routing_info_build into download records) over the level solve."""
    src, dst, lat, loss = synth.complete_graph(n, 21)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.random.default_rng(n).permutation(n).astype(np.uint32)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    t = g.compute_shortest_paths(nodes, algo=_lib.SRT_ALGO_LEVEL)
    _check(t, og, nodes)
    ri = RoutingInfo.build(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0)
    try:
        elat, eloss = O.compute_shortest_paths(og, nodes)
        rng = np.random.default_rng(3)
        for _ in range(300):
            a, b = (int(x) for x in rng.integers(0, n, 2))
            p = ri.path(int(nodes[a]), int(nodes[b]))
            if a == b:
                continue
            assert p.latency_ns == int(elat[a, b]) and np.float32(p.packet_loss).view(np.uint32) == _bits(eloss[a, b])
        assert ri.get_smallest_latency_ns() == int(elat.min())
    finally:
        ri.close()


@pytest.mark.parametrize("world,directed", [(2, False), (3, True), (8, False)])
def test_level_sharded_rows(world, directed):
    """Rows sharded over in-process ranks (every rank on device 0): each rank
    solves its own rows, the rows are all-gathered, rank 0's table is the
    oracle's."""
    g, nodes, og = _random(900, 30 + world, directed, (1, 9), 0.05)
    t, descs, _ = sdist.local_build(g, nodes, [0] * world, algo=_lib.SRT_ALGO_LEVEL)
    for d in descs:
        assert d.startswith("level:") and f"ranks={world}" in d, d
    _check(t, og, nodes)


def _random_ns(n, seed, directed, p_edge=0.08, lat_ms=(1, 9), subset=None):
    """A random graph in ns: integer-ms latencies plus a seeded sub-ms offset
    (g = 1 ns, like bench --config c3ns), so no bound fits 31 units and the
    quantized solve (buckets of 2^19 ns) takes it."""
    src, dst, l, loss = synth.random_graph(n, seed, p_edge=p_edge, directed=directed, lat_range_ns=lat_ms,
                                           loss_max=0.05)
    off = np.random.default_rng(seed + 7).integers(0, synth.MS, size=len(l), dtype=np.uint64)
    l = np.asarray(l, np.uint64) * np.uint64(synth.MS) + off
    g = NetworkGraph.from_edges(n, src, dst, l, loss, directed=directed)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    if subset:
        nodes = nodes[:subset]
    return g, nodes, O.Graph(directed, np.arange(n), src, dst, l, loss)


@pytest.mark.parametrize("n,seed,directed,p_edge,lat_ms,subset", [
    (60, 1, False, 0.3, (1, 9), None), (400, 2, False, 0.08, (1, 9), None), (400, 3, True, 0.08, (1, 9), 250),
    (1200, 4, False, 0.3, (1, 40), None), (900, 5, True, 0.05, (2, 6), None)])
def test_level_quantized_matches_oracle(n, seed, directed, p_edge, lat_ms, subset):
    """ns latencies: the quantized level solve (level:u32, buckets as wide as the
    shortest edge) is bit-exact against the oracle."""
    g, nodes, og = _random_ns(n, seed, directed, p_edge, lat_ms, subset)
    p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    try:
        d = p.describe()
        assert d.startswith("level:u32 ") and " g=1 " in d and " q=" in d, d
        _check(p.fetch(), og, nodes)
    finally:
        p.close()


def test_level_quantized_integer_units():
    """Integer-ms latencies 2-9 ms over a sparse ring-heavy graph whose probe
    bound (72 units) exceeds the 63 unit levels: the integer probes fail, the
    quantized one (64 buckets of 2 ms, the shortest edge) bounds it; AUTO ==
    oracle."""
    n = 300
    src, dst, lat, loss = synth.random_graph(n, 8, p_edge=0.006, directed=False, lat_range_ns=(2, 9), loss_max=0.05)
    lat = np.asarray(lat, np.uint64) * np.uint64(synth.MS)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    try:
        d = p.describe()
        assert d.startswith("level:u32 ") and " q=2 " in d, d
        _check(p.fetch(), og, nodes)
    finally:
        p.close()


def test_level_63_unit_levels():
    """Shortest paths past 31 units (probe bound 38): the 31-class probe fails,
    the 63-class one bounds it (64 class offsets a vertex); level == oracle."""
    n = 300
    src, dst, lat, loss = synth.random_graph(n, 8, p_edge=0.012, directed=False, lat_range_ns=(1, 9), loss_max=0.05)
    lat = np.asarray(lat, np.uint64) * np.uint64(synth.MS)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    try:
        d = p.describe()
        lmax = int(d.split(" lmax=")[1].split("(")[0])
        assert d.startswith("level:u16 ") and 31 < lmax <= 63, d
        _check(p.fetch(), og, nodes)
    finally:
        p.close()


def test_level_quantized_equals_fw_dense():
    """A 3,000-node complete ns graph (C3ns's shape at 3k): the quantized
    level tables equal the Floyd-Warshall family's (u32 keys) bit for bit on
    the device, and AUTO takes the level solve."""
    import torch

    n = 3000
    edges = synth.complete_graph_ns(n, 5)
    g = NetworkGraph.from_edges(n, *edges)
    nodes = np.arange(n, dtype=np.uint32)
    a = RoutingPlan(g, nodes, device=0).run()
    b = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW, device=0).run()
    try:
        assert a.describe().startswith("level:u32 "), a.describe()
        assert b.describe().startswith("fw:u32key "), b.describe()
        a.fetch(table=False)
        b.fetch(table=False)
        assert a.min_latency_ns == b.min_latency_ns
        la, pa, _ = a.table_ptrs()
        lb, pb, _ = b.table_ptrs()
        dev = torch.device("cuda", 0)
        t = lambda ptr, nb: torch.as_tensor(sdist._CudaBuf(ptr, nb), device=dev)
        assert torch.equal(t(la, n * n * 8), t(lb, n * n * 8)), "latency"
        assert torch.equal(t(pa, n * n * 4), t(pb, n * n * 4)), "loss bits"
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("n_gpus", [1, 3])
def test_level_quantized_routing_info(n_gpus):
    """RoutingInfo over a quantized plan: 8-byte records (u32 units), one GPU
    and 3 in-process ranks (every rank's records downloaded straight into the
    caller's array); paths and the min latency against the oracle."""
    n = 1500
    src, dst, lat, loss = synth.complete_graph_ns(n, 9)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.random.default_rng(n).permutation(n).astype(np.uint32)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    ri = RoutingInfo.build(g, nodes, device=0, n_gpus=n_gpus, same_device=n_gpus > 1)
    try:
        assert ri.record_bytes() == 8
        elat, eloss = O.compute_shortest_paths(og, nodes)
        ml, mp = ri.table()
        off = ~np.eye(n, dtype=bool)
        assert np.array_equal(ml[off], elat[off]) and np.array_equal(_bits(mp[off]), _bits(eloss[off]))
        assert ri.get_smallest_latency_ns() == int(elat.min())
    finally:
        ri.close()
    t = g.compute_shortest_paths(nodes, n_gpus=n_gpus, same_device=n_gpus > 1)
    _check(t, og, nodes)


@pytest.mark.parametrize("world,directed", [(2, False), (3, True)])
def test_level_quantized_sharded_rows(world, directed):
    """Quantized rows sharded over in-process communicator ranks: u32 staging
    all-gathered chunk by chunk; rank 0's table is the oracle's."""
    g, nodes, og = _random_ns(700, 40 + world, directed, 0.05)
    t, descs, _ = sdist.local_build(g, nodes, [0] * world, algo=_lib.SRT_ALGO_LEVEL)
    for d in descs:
        assert d.startswith("level:u32 ") and f"ranks={world}" in d, d
    _check(t, og, nodes)


@pytest.mark.parametrize("quant", [False, True])
def test_level_shard_rows_no_exchange(quant):
    """srt_plan_shard_rows (the multi-process form, no collective): 3 plans,
    each building only its third of the rows into its own table; together the
    rows are the oracle's table.  fetch(out) is refused on a sharded plan, and
    Floyd-Warshall plans refuse the sharding."""
    import torch

    if quant:
        g, nodes, og = _random_ns(500, 61, False, 0.08)
    else:
        g, nodes, og = _random(500, 61, False, (1, 9), 0.08)
    n = len(nodes)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    dev = torch.device("cuda", 0)
    mins = []
    for r in range(3):
        p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).shard_rows(3, r)
        try:
            assert f"shard={r}/3" in p.describe()
            p.run()
            p.fetch(table=False)
            mins.append(p.min_latency_ns)
            with pytest.raises(_lib.SrtError) as e:
                p.fetch()
            assert e.value.code == _lib.SRT_ERR_INVALID
            la, pa, _ = p.table_ptrs()
            L = torch.as_tensor(sdist._CudaBuf(la, n * n * 8), device=dev).view(torch.int64).view(n, n)
            P = torch.as_tensor(sdist._CudaBuf(pa, n * n * 4), device=dev).view(torch.int32).view(n, n)
            r0, r1 = n * r // 3, n * (r + 1) // 3
            assert np.array_equal(L[r0:r1].cpu().numpy().view(np.uint64), elat[r0:r1])
            assert np.array_equal(P[r0:r1].cpu().numpy().view(np.uint32), _bits(eloss[r0:r1]))
        finally:
            p.close()
    assert min(mins) == int(elat.min())
    fw = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW, device=0)
    try:
        with pytest.raises(_lib.SrtError) as e:
            fw.shard_rows(2, 0)
        assert e.value.code == _lib.SRT_ERR_UNSUPPORTED
    finally:
        fw.close()


def test_level_one_call_uploads_needed_losses(monkeypatch):
    """One-call builds of a level plan upload only the losses the class CSRs
    read (indices listed on the device, gathered on the host) and range-check
    every loss on host threads: a bad loss on an edge the solve never reads is
    still the reference's parse-time error; the tables equal the full-upload
    path's (SRT_LOSS_FULL=1) and the oracle's rows."""
    err = _lib.SrtErr()
    assert _lib.lib().srt_init(0, err) == 0  # pins the staging the upload uses
    n = 4200
    row_ptr, col, lat, loss = synth.complete_csr(n, 31)
    loss = loss.copy()
    far = int(np.argmax(lat[: n]))  # row 0's longest edge: never on a shortest path
    assert lat[far] > 100 * synth.MS
    keep = loss[far]
    loss[far] = np.float32(1.5)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    with pytest.raises(_lib.SrtError) as e:
        RoutingInfo.build(g, np.arange(n, dtype=np.uint32))
    assert str(e.value) == "Edge 'packet_loss' is not in the range [0,1]"
    loss[far] = keep
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.random.default_rng(31).permutation(n).astype(np.uint32)
    a = RoutingInfo.build(g, nodes, device=0)
    monkeypatch.setenv("SRT_LOSS_FULL", "1")
    b = RoutingInfo.build(g, nodes, device=0)
    try:
        la, pa = a.table()
        lb, pb = b.table()
        assert np.array_equal(la, lb) and np.array_equal(_bits(pa), _bits(pb))
        src, dst, l2, p2 = synth.complete_graph(n, 31)
        rows = np.arange(5)
        order = np.concatenate([nodes[rows], np.setdiff1d(nodes, nodes[rows])]).astype(np.uint32)
        elat, eloss = O.compute_shortest_paths(O.Graph(False, np.arange(n), src, dst, l2, p2), order, src_count=5)
        pos = {int(v): i for i, v in enumerate(order)}
        inv = np.array([pos[int(v)] for v in nodes])
        for r in rows:
            m = np.arange(n) != r
            assert np.array_equal(la[r][m], elat[r][inv][m]) and np.array_equal(_bits(pa[r][m]), _bits(eloss[r][inv][m]))
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("ns", [False, True])
def test_level_symmetric_rows(monkeypatch, ns):
    """Complete graphs in identity rows whose pairs mirror exactly build only
    the class out-rows (the in-rows are the same entries: 'rows=sym'); the
    tables equal the two-CSR build's (SRT_LVL_SYM=0) bit for bit, and a
    directed complete graph (different latency each way) keeps both CSRs."""
    import torch

    n = 2000
    edges = synth.complete_graph_ns(n, 41) if ns else synth.complete_graph(n, 41)
    row_ptr, col, lat, loss = synth.complete_csr(n, 41, edges=edges)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.random.default_rng(41).permutation(n).astype(np.uint32)
    a = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    monkeypatch.setenv("SRT_LVL_SYM", "0")
    b = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    monkeypatch.delenv("SRT_LVL_SYM")
    try:
        assert "rows=sym" in a.describe() and "rows=sym" not in b.describe(), (a.describe(), b.describe())
        dev = torch.device("cuda", 0)
        t = lambda ptr, nb: torch.as_tensor(sdist._CudaBuf(ptr, nb), device=dev)
        la, pa, _ = a.table_ptrs()
        lb, pb, _ = b.table_ptrs()
        assert torch.equal(t(la, n * n * 8), t(lb, n * n * 8)) and torch.equal(t(pa, n * n * 4), t(pb, n * n * 4))
        _check(a.fetch(), O.Graph(False, np.arange(n), *edges), nodes)
        # the class out-rows streamed from the u16-unit adjacency copy (on by
        # default from 8,192 vertices; forced here): the same tables bit for bit
        monkeypatch.setenv("SRT_LAT16", "1")
        c16 = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
        monkeypatch.delenv("SRT_LAT16")
        try:
            assert ("lat16" in c16.describe()) == (not ns) and "lat16" not in a.describe(), (c16.describe(), a.describe())
            lc, pc, _ = c16.table_ptrs()
            assert torch.equal(t(la, n * n * 8), t(lc, n * n * 8)) and torch.equal(t(pa, n * n * 4), t(pc, n * n * 4))
        finally:
            c16.close()
    finally:
        a.close()
        b.close()
    # directed complete graph: row u's latencies differ from column u's
    rng = np.random.default_rng(42)
    lat2 = lat.copy().reshape(n, n)
    lat2 += (rng.integers(0, 3, size=(n, n)).astype(np.uint64) * np.uint64(synth.MS))
    np.fill_diagonal(lat2, lat.reshape(n, n).diagonal())
    lat2 = lat2.reshape(-1)
    g2 = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat2, loss, directed=True)
    c = RoutingPlan(g2, nodes, device=0).run()
    try:
        assert c.describe().startswith("level:") and "rows=sym" not in c.describe(), c.describe()
        src = np.repeat(np.arange(n, dtype=np.uint32), n)
        dst = np.tile(np.arange(n, dtype=np.uint32), n)
        _check(c.fetch(), O.Graph(True, np.arange(n), src, dst, lat2, loss), nodes)
    finally:
        c.close()
    # mirrored latencies, one short edge's loss differing from its mirror's:
    # the symmetry check compares the losses beside short latencies too
    loss3 = loss.copy().reshape(n, n)
    row = lat.reshape(n, n)[7].copy()
    row[7] = np.iinfo(np.uint64).max
    v = int(np.argmin(row))
    loss3[7, v] = np.float32(0.5) if loss3[7, v] != np.float32(0.5) else np.float32(0.25)
    loss3 = loss3.reshape(-1)
    g3 = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss3, directed=True)
    d = RoutingPlan(g3, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).run()
    try:
        assert "rows=sym" not in d.describe(), d.describe()
        src = np.repeat(np.arange(n, dtype=np.uint32), n)
        dst = np.tile(np.arange(n, dtype=np.uint32), n)
        _check(d.fetch(), O.Graph(True, np.arange(n), src, dst, lat, loss3), nodes)
    finally:
        d.close()


def _complete_identity(n, seed):
    """A complete undirected graph in identity rows (row u = columns 0 .. n-1,
    as bench.py's C3 CSR): the symmetric level plans' shape (rows=sym)."""
    edges = synth.complete_graph(n, seed, lat_ms=(1, 40))
    row_ptr, col, lat, loss = synth.complete_csr(n, seed, edges=edges)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    return g, np.arange(n, dtype=np.uint32), O.Graph(False, np.arange(n), *edges)


@pytest.mark.parametrize("world", [3, 8])
def test_level_sharded_class_csr(world):
    """Communicator-bound symmetric level plans build the class CSR sharded
    (each rank its vertex slice into its own slot, the slots all-gathered) and
    then their rows: rank 0's whole table is the oracle's, at 3 ranks (slices
    of unequal fill) and 8."""
    g, nodes, og = _complete_identity(1200, 70 + world)
    t, descs, _ = sdist.local_build(g, nodes, [0] * world, algo=_lib.SRT_ALGO_LEVEL)
    for d in descs:
        assert d.startswith("level:u16 ") and " rows=sym" in d and f"ranks={world}" in d, d
    _check(t, og, nodes)


def test_level_rank_share_emulated(monkeypatch):
    """bench.py --rank-share's measured form (SRT_LVL_SHARD_EMU=1): a
    row-sharded plan's class CSR built as N slices (all at the first run, the
    own slice after it); the rank's rows stay the oracle's over three runs."""
    import torch

    monkeypatch.setenv("SRT_LVL_SHARD_EMU", "1")
    g, nodes, og = _complete_identity(1000, 91)
    n = len(nodes)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    dev = torch.device("cuda", 0)
    for r in (0, 5):
        p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_LEVEL, device=0).shard_rows(8, r)
        try:
            assert " rows=sym" in p.describe(), p.describe()
            for _ in range(3):
                p.run()
                la, pa, _ = p.table_ptrs()
                L = torch.as_tensor(sdist._CudaBuf(la, n * n * 8), device=dev).view(torch.int64).view(n, n)
                P = torch.as_tensor(sdist._CudaBuf(pa, n * n * 4), device=dev).view(torch.int32).view(n, n)
                r0, r1 = n * r // 8, n * (r + 1) // 8
                exp_l, exp_p = elat[r0:r1].copy(), _bits(eloss[r0:r1]).copy()
                got_l, got_p = L[r0:r1].cpu().numpy().view(np.uint64), P[r0:r1].cpu().numpy().view(np.uint32)
                assert np.array_equal(got_l, exp_l) and np.array_equal(got_p, exp_p)
        finally:
            p.close()
