"""The in-process multi-GPU build at the BASELINE configs' own sizes
(VERDICT r4 item 1): the default drop-in passes srt_opts.n_gpus =
srt_device_count(), so the sharded schedules must build C3's 16k graph and a
100k sparse graph, not only the <= 1,500-node graphs of test_gpu_local.py.

On the one-GPU box every rank shares device 0 (SRT_OPT_SAME_DEVICE: the same
schedules, the same exchange code).  Bars: rank 0's device table equals the
one-GPU plan's device table bit for bit (torch.equal on latency and loss), and
16 (C3) / 8 (C4) seeded rows equal the oracle's, diagonal = the raw self-loop.
Reference: rayon fans the sources out over every core
(src/main/network/graph/mod.rs:190-208)."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd import dist as sdist
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _device_table(plan):
    import torch

    lat_p, loss_p, n = plan.table_ptrs()
    dev = torch.device("cuda", 0)
    L = torch.as_tensor(sdist._CudaBuf(lat_p, n * n * 8), device=dev).view(torch.int64).view(n, n)
    P = torch.as_tensor(sdist._CudaBuf(loss_p, n * n * 4), device=dev).view(torch.int32).view(n, n)
    return L, P


def _oracle_rows(og, nodes, rows):
    """The oracle's rows `rows` (indices into nodes) over the columns in node order."""
    n = len(nodes)
    order = np.concatenate([nodes[rows], np.setdiff1d(nodes, nodes[rows])]).astype(np.uint32)
    elat, eloss = O.compute_shortest_paths(og, order, src_count=len(rows), mode=1)
    pos = {int(v): i for i, v in enumerate(order)}
    inv = np.array([pos[int(v)] for v in nodes], np.int64)
    assert len(inv) == n
    return elat[:len(rows)][:, inv], eloss[:len(rows)][:, inv]


def _check_rows(L, P, rows, elat, eloss, sl_lat, sl_loss):
    for i, r in enumerate(rows):
        got_l = L[r].cpu().numpy().view(np.uint64)
        got_p = P[r].cpu().numpy().view(np.uint32)
        exp_l = elat[i].copy()
        exp_p = eloss[i].copy().view(np.uint32)
        exp_l[r] = sl_lat[r]
        exp_p[r] = np.float32(sl_loss[r]).view(np.uint32)
        assert np.array_equal(got_l, exp_l), f"row {r}: latency"
        assert np.array_equal(got_p, exp_p), f"row {r}: loss bits"


@pytest.fixture(scope="module")
def c3():
    """C3: the 16,384-node complete graph, its one-GPU plan (table kept on the
    device) and 16 oracle rows."""
    n = 16384
    edges = synth.complete_graph(n, 3)
    row_ptr, col, lat, loss = synth.complete_csr(n, 3, edges=edges)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    one = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_FW, device=0).run()
    one.fetch(table=False)
    rows = np.random.default_rng(5).choice(n, 16, replace=False)
    elat, eloss = _oracle_rows(O.Graph(False, nodes, *edges), nodes, rows)
    sl_l = lat.reshape(n, n).diagonal().copy()
    sl_p = loss.reshape(n, n).diagonal().copy()
    del edges, row_ptr, col
    yield g, nodes, one, rows, elat, eloss, sl_l, sl_p
    one.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c3_16k_sharded_equals_one_gpu(c3, world):
    """C3 over `world` in-process ranks: every rank ran the symmetric triangle
    schedule and the sharded loss tail; rank 0's table is the one-GPU table."""
    import torch

    g, nodes, one, rows, elat, eloss, sl_l, sl_p = c3
    kept = sdist.local_build(g, nodes, [0] * world, algo=_lib.SRT_ALGO_FW, keep=True)
    try:
        for r, p in enumerate(kept.plans):
            d = p.describe()
            assert f"ranks={world}" in d and "sym=triangle" in d and d.startswith("fw:f16key"), d
            assert p.timing()["sharded_tail"] == 1, (r, d)
        p0 = kept.plans[0]
        p0.fetch(table=False)  # connectivity + min latency over rank 0's table
        assert p0.min_latency_ns == one.min_latency_ns
        L1, P1 = _device_table(one)
        L, P = _device_table(p0)
        assert torch.equal(L, L1), "rank 0 latency table != one-GPU table"
        assert torch.equal(P, P1), "rank 0 loss bits != one-GPU table"
        _check_rows(L, P, rows, elat, eloss, sl_l, sl_p)
    finally:
        kept.close()


def test_c4_100k_sparse_two_ranks():
    """C4's 100k Barabasi-Albert graph, 20,000 nodes in use, source rows
    sharded over 2 in-process ranks: rank 0's table equals the one-GPU table
    bit for bit, 8 oracle rows."""
    import torch

    n = 100_000
    src, dst, lat, loss = synth.barabasi_albert(n, 4, 4)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=False)
    nodes = np.sort(np.random.default_rng(44).choice(n, 20_000, replace=False)).astype(np.uint32)
    one = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_SSSP, device=0).run()
    try:
        one.fetch(table=False)
        kept = sdist.local_build(g, nodes, [0, 0], algo=_lib.SRT_ALGO_SSSP, keep=True)
        try:
            for p in kept.plans:
                d = p.describe()
                assert d.startswith("sssp") and "ranks=2" in d, d
            p0 = kept.plans[0]
            p0.fetch(table=False)
            assert p0.min_latency_ns == one.min_latency_ns
            L1, P1 = _device_table(one)
            L, P = _device_table(p0)
            assert torch.equal(L, L1) and torch.equal(P, P1), "rank 0 table != one-GPU table"
            rows = np.sort(np.random.default_rng(4).choice(len(nodes), 8, replace=False))
            elat, eloss = _oracle_rows(O.Graph(False, np.arange(n), src, dst, lat, loss), nodes, rows)
            sl = src == dst
            sl_lat = np.zeros(n, np.uint64)
            sl_loss = np.zeros(n, np.float32)
            sl_lat[src[sl]] = lat[sl]
            sl_loss[src[sl]] = loss[sl]
            _check_rows(L, P, rows, elat, eloss, sl_lat[nodes], sl_loss[nodes])
        finally:
            kept.close()
    finally:
        one.close()


@pytest.mark.parametrize("world", [2, 8])
def test_c3_16k_routing_info_in_process_ranks(c3, world):
    """generate_routing_info over `world` in-process ranks (the drop-in's
    srt_opts.n_gpus; here every rank on device 0): rank 0's plan scans the CSR
    once, every rank solves its rows and downloads them into the RoutingInfo
    records -- the table equals the one-GPU RoutingInfo's bit for bit, and the
    16 oracle rows."""
    from shadow_amd import RoutingInfo

    g, nodes, one, rows, elat, eloss, sl_l, sl_p = c3
    multi = RoutingInfo.build(g, nodes, device=0, n_gpus=world, same_device=True)
    single = RoutingInfo.build(g, nodes, device=0)
    try:
        assert multi.record_bytes() == single.record_bytes() == 6
        assert multi.get_smallest_latency_ns() == single.get_smallest_latency_ns() == one.min_latency_ns
        ml, mp = multi.table()
        sl, sp = single.table()
        assert np.array_equal(ml, sl) and np.array_equal(mp.view(np.uint32), sp.view(np.uint32))
        del sl, sp
        for k, r in enumerate(rows):
            exp_l, exp_p = elat[k].copy(), eloss[k].copy()
            exp_l[r], exp_p[r] = sl_l[r], sl_p[r]
            assert np.array_equal(ml[r], exp_l) and np.array_equal(mp[r].view(np.uint32), exp_p.view(np.uint32)), r
    finally:
        multi.close()
        single.close()


def test_level_two_distinct_devices():
    """The in-process level build across two physical devices (peer copies of
    the class CSRs over xGMI, one solve and one PCIe download per device):
    equal to the one-GPU RoutingInfo.  Skipped on a one-GPU box -- the
    cross-device path is unverified until a multi-GPU lease runs it."""
    from shadow_amd import RoutingInfo

    if _lib.lib().srt_device_count() < 2:
        pytest.skip("needs two visible devices")
    n = 3000
    src, dst, lat, loss = synth.complete_graph(n, 12)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.random.default_rng(12).permutation(n).astype(np.uint32)
    multi = RoutingInfo.build(g, nodes, device=0, n_gpus=2)
    single = RoutingInfo.build(g, nodes, device=0)
    try:
        ml, mp = multi.table()
        sl, sp = single.table()
        assert np.array_equal(ml, sl) and np.array_equal(mp.view(np.uint32), sp.view(np.uint32))
        assert multi.get_smallest_latency_ns() == single.get_smallest_latency_ns()
    finally:
        multi.close()
        single.close()
