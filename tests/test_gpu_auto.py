"""GPU test of the AUTO family chooser (srt_api.cpp price_fw / price_sparse):
priced from the measured rates per key type and symmetry, it must pick the
faster family on a mid-density graph the old flat pricing (Vp^3 / 1.2e13
against 64 B per source-edge at 3e12 B/s) sent to the sparse sweeps."""
import numpy as np
import pytest

from shadow_amd import NetworkGraph, _lib, synth
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _device_ms(g, nodes, algo):
    p = RoutingPlan(g, nodes, algo=algo, device=0)
    try:
        best = float("inf")
        for _ in range(2):
            p.run()
            best = min(best, p.kernel_stats()[3])
        return best, p.describe()
    finally:
        p.close()


def test_auto_picks_faster_family_mid_density():
    # 16k-node BA graph, m = 16 (mean degree 32): old prices fw 366 ms vs
    # sparse 189 ms (picked sparse); measured-rate prices fw ~58 vs ~105 ms
    n = 16384
    src, dst, lat, loss = synth.barabasi_albert(n, 16, 5)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    t = {}
    for algo in (_lib.SRT_ALGO_FW, _lib.SRT_ALGO_SSSP):
        t[algo], _ = _device_ms(g, nodes, algo)
    p = RoutingPlan(g, nodes, algo=_lib.SRT_ALGO_AUTO, device=0)
    desc = p.describe()
    p.close()
    assert "auto-price=" in desc, desc
    picked = _lib.SRT_ALGO_FW if desc.startswith("fw") else _lib.SRT_ALGO_SSSP
    assert t[picked] <= 1.15 * min(t.values()), (desc, t)
