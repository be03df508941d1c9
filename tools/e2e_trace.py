"""C3 end-to-end build (srt_compute_shortest_paths: host CSR in, srt_path
table out) with SRT_TRACE=1 host phase marks on stderr, for a list of knob
sets, plus the device-only build time of the same graph for the ratio.
Measurement tool.
usage: python tools/e2e_trace.py [n_nodes] ["K=V,K=V" ...]   ("" = defaults)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SRT_TRACE"] = "1"

import numpy as np  # noqa: E402

import bench  # noqa: E402
from shadow_amd import NetworkGraph, synth  # noqa: E402
from shadow_amd.plan import RoutingPlan  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    variants = sys.argv[2:] or ["", "SRT_FETCH16=1", ""]
    row_ptr, col, lat, loss = synth.complete_csr(n, 3)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    knobs = set()
    for v in variants:
        for kv in filter(None, v.split(",")):
            knobs.add(kv.split("=")[0])
    for v in variants:
        for k in knobs:
            os.environ.pop(k, None)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=")
            os.environ[k] = val
        r = bench.e2e_build(g, nodes, reps=4)
        print(f"e2e best ms [{v}]", round(r["ms"], 1), flush=True)
    plan = RoutingPlan(g, nodes)
    for _ in range(3):
        plan.run()
    plan.sync()
    print("device build ms", round(plan.timing()["total_ms"], 1), flush=True)
    plan.close()


if __name__ == "__main__":
    main()
