"""Measurement only: time the u32 rest kernel of the C3 build under the
SRT_FW_ABLATE variants (1 no C load, 2 no C store, 4 no chunk staging after
the first, 8 no per-chunk wait + barrier; the closure is wrong with any of
them, so nothing is checked).  Prints ms per rest launch for each variant.
usage: python tools/fw_ablate.py [nodes] [variants...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(nodes):
    sys.path.insert(0, ROOT)
    import numpy as np

    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan
    row_ptr, col, lat, loss = synth.complete_csr(nodes, 3)
    g = NetworkGraph(nodes, np.arange(nodes, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    plan = RoutingPlan(g, np.arange(nodes, dtype=np.uint32), device=0)
    best = None
    for _ in range(3):
        plan.run()
        t = plan.timing()
        per = t["dominant_ms"] / max(t["dominant_launches"], 1)
        best = per if best is None else min(best, per)
    print(f"ABL {os.environ.get('SRT_FW_ABLATE', '0')} rest_ms_per_launch {best:.3f} "
          f"launches {t['dominant_launches']} build_ms {t['total_ms']:.1f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]))
        sys.exit(0)
    nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    for v in (sys.argv[2:] or ["0", "1", "2", "3", "4", "8", "12", "15"]):
        env = dict(os.environ, SRT_FW_ABLATE=v)
        r = subprocess.run([sys.executable, __file__, "--child", str(nodes)], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
