"""Drive tools/sim_sssp.c on the C4 graph (100k BA, m=4, seed 4) for a few
threshold steps DELTA (units of g = 1 ms).  Measurement tool.
usage: gcc -O2 -o /tmp/sim_sssp tools/sim_sssp.c && python tools/sim_sssp.py [deltas...]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import synth  # noqa: E402


def main():
    n = int(os.environ.get("SIM_N", "100000"))
    src, dst, lat, _ = synth.barabasi_albert(n, 4, 4)
    keep = src != dst
    s, d, w = src[keep], dst[keep], (lat[keep] // synth.MS).astype(np.uint32)
    # undirected: both directions
    u = np.concatenate([s, d]).astype(np.uint32)
    v = np.concatenate([d, s]).astype(np.uint32)
    ww = np.concatenate([w, w]).astype(np.uint32)
    blob = np.uint32(n).tobytes() + np.uint64(len(u)).tobytes() + np.stack([u, v, ww], 1).astype(np.uint32).tobytes()
    for arg in (sys.argv[1:] or ["0", "25", "50", "100", "200"]):
        delta, _, cap = arg.partition(":")
        stride = os.environ.get("SIM_STRIDE", str(n // 64))
        out = subprocess.run(["/tmp/sim_sssp", delta, cap or "1000", stride, os.environ.get("SIM_START", str(n // 2))], input=blob, capture_output=True)
        print(out.stdout.decode().strip(), flush=True)


if __name__ == "__main__":
    main()
