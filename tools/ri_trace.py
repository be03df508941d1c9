"""srt_routing_info_build (generate_routing_info) on the C3 graph with
SRT_TRACE=1 host phase marks on stderr: a cold first call in this fresh
process (optionally after srt_init_async at start, overlapped with the graph
build), then warm calls.  Measurement tool.
usage: python tools/ri_trace.py [n_nodes] [init|plain]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SRT_TRACE"] = "1"

import shadow_amd  # noqa: E402

mode = sys.argv[2] if len(sys.argv) > 2 else "init"
if mode == "init":
    shadow_amd.init_async(0)

import numpy as np  # noqa: E402

from shadow_amd import NetworkGraph, RoutingInfo, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    row_ptr, col, lat, loss = synth.complete_csr(n, 3)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    for i in range(4):
        print(f"--- call {i} ({'cold' if i == 0 else 'warm'}, {mode})", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        ri = RoutingInfo.build(g, nodes)
        dt = (time.perf_counter() - t0) * 1e3
        print(f"call {i}: {dt:.1f} ms, {ri.record_bytes()}-byte records", flush=True)
        ri.close()


if __name__ == "__main__":
    main()
