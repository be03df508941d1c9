"""Paired-round Floyd-Warshall schedule (srt_fw.hip fw_rounds_pair_t) on gfx950.

One GPU at rest-bound sizes (>= 64 blocks of 128) fuses FW rounds in pairs;
SRT_FW_PAIR forces the paired schedule at small sizes and SRT_FW_NO_PAIR
turns it off, so the same graph is closed both ways.  Bar: latency bit-exact
vs the oracle (reference Dijkstra restatement), loss within 1e-6, and the
paired table bit-identical to the single-round one (both compute the unique
lexicographic minimum over paths of the exact integer keys).
"""
import numpy as np
import pytest

from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd.plan import RoutingPlan
from tests.test_gpu_apsp import _check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,seed,directed", [(400, 0, False), (500, 1, True), (777, 2, False),
                                             (1000, 3, True), (300, 4, False)])
def test_forced_pair_vs_oracle(monkeypatch, n, seed, directed):
    # 400/500 -> 4 blocks, 777/1000 -> 8 blocks (paired); 300 -> 3 blocks (odd:
    # single-round fallback)
    monkeypatch.setenv("SRT_FW_PAIR", "1")
    e = synth.random_graph(n, 40 + seed, p_edge=8.0 / n, directed=directed, lat_range_ns=(1, 6), loss_max=0.05)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    _check(e, nodes, directed, n, algo=_lib.SRT_ALGO_FW)


def _table(monkeypatch, g, nodes, pair):
    monkeypatch.delenv("SRT_FW_PAIR", raising=False)
    monkeypatch.delenv("SRT_FW_NO_PAIR", raising=False)
    monkeypatch.setenv("SRT_FW_PAIR" if pair else "SRT_FW_NO_PAIR", "1")
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
def test_pair_equals_single_round(monkeypatch, n):
    src, dst, lat, loss = synth.complete_graph(n, 7) if n <= 2048 else (None,) * 4
    if n <= 2048:
        g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    else:
        row_ptr, col, lat, loss = synth.complete_csr(n, 7)
        g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    tp, lp, rp = _table(monkeypatch, g, nodes, True)
    ts, ls, rs = _table(monkeypatch, g, nodes, False)
    nblk = n // 128
    assert lp == nblk // 2 and ls == nblk  # one rest launch per pair vs per round
    assert 1.8 < rp <= 2.0 and rs == 1.0
    assert np.array_equal(tp.latency_ns, ts.latency_ns)
    assert np.array_equal(tp.packet_loss.view(np.uint32), ts.packet_loss.view(np.uint32))
    assert tp.min_latency_ns == ts.min_latency_ns
    L = tp.latency_ns
    assert np.array_equal(L, L.T)
