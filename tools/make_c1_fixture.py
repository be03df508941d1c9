"""Pins config C1 (1,000-node complete graph, seed 1, through its GML text)
without a live oracle run: tests/golden/c1_table.json holds the SHA-256 of the
oracle's whole table (latency u64 bytes then loss f32 bytes, row-major over
the nodes in GML order) and 1,000 seeded sample pairs with their values.
tests/test_golden.py checks the oracle's sampled rows against it on the CPU;
tests/test_gpu_configs.py hashes the GPU's table against it.

usage: python tools/make_c1_fixture.py   (about a minute on 8 threads)
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from shadow_amd import synth  # noqa: E402


def main():
    n, seed = 1000, 1
    src, dst, lat, loss = synth.complete_graph(n, seed)
    text = synth.gml_text(n, src, dst, lat, loss)
    og = O.gml_parse(text)
    nodes = np.arange(n, dtype=np.uint32)
    elat, eloss = O.compute_shortest_paths(og, nodes, mode=1)
    h = hashlib.sha256(np.ascontiguousarray(elat, np.uint64).tobytes() +
                       np.ascontiguousarray(eloss, np.float32).tobytes()).hexdigest()
    rng = np.random.default_rng(2026)
    ii = rng.integers(0, n, 1000)
    jj = rng.integers(0, n, 1000)
    out = {"config": "C1: synth.complete_graph(1000, seed=1) -> synth.gml_text -> oracle gml_parse, all nodes "
                     "in use in GML order; oracle compute_shortest_paths mode 1",
           "nodes": n, "seed": seed, "gml_sha256": hashlib.sha256(text.encode()).hexdigest(),
           "table_sha256": h, "hash_of": "latency_ns u64[n*n] bytes || packet_loss f32[n*n] bytes, row-major",
           "min_latency_ns": int(elat.min()),
           "samples": [[int(i), int(j), int(elat[i, j]), int(eloss[i, j:j + 1].view(np.uint32)[0])]
                       for i, j in zip(ii, jj)]}
    with open(os.path.join(ROOT, "tests", "golden", "c1_table.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("table sha256", h)


if __name__ == "__main__":
    main()
