"""GML ingest throughput: a complete n-node Shadow GML graph
(the C1-C3 shape) parsed by srt_gml_parse sequentially and chunk-parallel.

usage: python tools/gml_bench.py [n_nodes] [threads]
Prints one JSON line (text MB, seconds and MB/s per mode, edges/s)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import synth  # noqa: E402
from shadow_amd.graph import NetworkGraph  # noqa: E402


def complete_gml(n, seed=1):
    src, dst, lat, loss = synth.complete_graph(n, seed)
    head = ["graph [", "  directed 0"]
    head += [f"  node [\n    id {i}\n    host_bandwidth_up \"1 Gbit\"\n    host_bandwidth_down \"1 Gbit\"\n  ]"
             for i in range(n)]
    parts = ["\n".join(head)]
    ms = (lat // np.uint64(synth.MS)).astype(np.int64)
    step = 1 << 20
    for b in range(0, len(src), step):
        s, d, l, p = src[b:b + step], dst[b:b + step], ms[b:b + step], loss[b:b + step]
        parts.append("\n".join(f"  edge [\n    source {a}\n    target {c}\n    latency \"{x} ms\"\n"
                               f"    packet_loss {y:.6f}\n  ]"
                               for a, c, x, y in zip(s.tolist(), d.tolist(), l.tolist(), p.tolist())))
    parts.append("]\n")
    return "\n".join(parts), len(src)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    t0 = time.perf_counter()
    text, m = complete_gml(n)
    gen_s = time.perf_counter() - t0
    mb = len(text) / 1e6
    out = {"nodes": n, "edges": m, "text_MB": round(mb, 1), "gen_s": round(gen_s, 1)}
    for mode, env in (("sequential", {"SRT_GML_PAR_BYTES": str(1 << 50)}),
                      ("parallel", {"SRT_GML_PAR_BYTES": "0", "SRT_GML_THREADS": str(threads)})):
        os.environ.update(env)
        t0 = time.perf_counter()
        g = NetworkGraph.parse(text)
        dt = time.perf_counter() - t0
        assert len(g.col) == 2 * m - n
        out[mode] = {"s": round(dt, 3), "MB_per_s": round(mb / dt, 1), "edges_per_s": round(m / dt)}
    out["threads"] = threads
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
