"""The in-process multi-GPU level build of C3 (srt_opts.n_gpus = N), rank 0's
share measured alone on one GPU (SRT_MULTI_EMULATE=1: rank 0's rows solved and
downloaded into the RoutingInfo's records; the other ranks skipped -- on a
node they run the same work on their own device and PCIe link, no exchange).
Prints one JSON line per N: wall ms of srt_routing_info_build (min of reps).

usage: python tools/multi_emulate.py [N ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from shadow_amd import NetworkGraph, RoutingInfo, _lib, synth

    ns = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    n = 16384
    row_ptr, col, lat, loss = synth.complete_csr(n, 3)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    err = _lib.SrtErr()
    _lib.lib().srt_init(0, err)
    for N in ns:
        if N > 1:
            os.environ["SRT_MULTI_EMULATE"] = "1"
        else:
            os.environ.pop("SRT_MULTI_EMULATE", None)
        ms = []
        for _ in range(4):
            t0 = time.perf_counter()
            ri = RoutingInfo.build(g, nodes, device=0, n_gpus=N, same_device=N > 1)
            ms.append((time.perf_counter() - t0) * 1e3)
            ri.close()
        print(json.dumps({"n_gpus": N, "emulated": N > 1, "routing_info_ms": min(ms[1:]),
                          "reps_ms": [round(x, 2) for x in ms],
                          "what": "srt_routing_info_build of C3 (16k complete, host CSR in, RoutingInfo out); "
                                  "N > 1: rank 0's share alone (its rows solved and downloaded), the other "
                                  "ranks' identical shares run on their own devices and links"}), flush=True)


if __name__ == "__main__":
    main()
