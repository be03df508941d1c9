"""GML ingest throughput at config scale:
the text of a complete n-node Shadow graph is written by tools/gml_gen.c into
one buffer (no Python formatting: 16k nodes is ~12 GB), then srt_gml_parse
reads it in place -- cold (first call of the process) and warm -- with the
chunk-parallel ingest on T threads; a 1k-node text is also parsed sequentially
and in parallel and the two CSRs compared.  Prints one JSON line.

usage: python tools/gml_scale.py [n_nodes] [threads]
"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from shadow_amd import _lib  # noqa: E402


def gen(n, seed=1):
    so = "/tmp/libgmlgen.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "gml_gen.c")], check=True)
    g = C.CDLL(so)
    g.gml_complete.restype = C.c_uint64
    g.gml_complete.argtypes = [C.c_uint32, C.c_uint64, C.c_void_p, C.c_uint64]
    cap = 64 + n * 110 + n * (n + 1) // 2 * 100
    buf = np.empty(cap, np.uint8)
    used = g.gml_complete(n, seed, buf.ctypes.data, cap)
    assert used, "buffer too small"
    return buf, int(used)


def parse(buf, used):
    L = _lib.lib()
    h = C.c_void_p()
    err = _lib.SrtErr()
    t0 = time.perf_counter()
    rc = L.srt_gml_parse(C.c_char_p(buf.ctypes.data), used, C.byref(h), C.byref(err))
    dt = time.perf_counter() - t0
    _lib.check(rc, err)
    csr = _lib.SrtCsr()
    L.srt_gml_csr(h, C.byref(csr))
    out = (csr.n_nodes, csr.n_adj)
    sig = None
    if csr.n_adj <= 1 << 24:
        as_np = np.ctypeslib.as_array
        sig = (as_np(csr.row_ptr, (csr.n_nodes + 1,)).copy(), as_np(csr.col, (csr.n_adj,)).copy(),
               as_np(csr.lat_ns, (csr.n_adj,)).copy(), as_np(csr.loss, (csr.n_adj,)).copy())
    L.srt_gml_free(h)
    return dt, out, sig


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    os.environ["SRT_GML_THREADS"] = str(threads)
    os.environ["SRT_GML_PAR_BYTES"] = "0"
    # correctness at 1k: parallel == sequential
    small, su = gen(1000, 7)
    _, _, a = parse(small, su)
    os.environ["SRT_GML_PAR_BYTES"] = str(1 << 50)
    _, _, b = parse(small, su)
    os.environ["SRT_GML_PAR_BYTES"] = "0"
    same = all(np.array_equal(x, y) for x, y in zip(a, b))
    t0 = time.perf_counter()
    buf, used = gen(n)
    gen_s = time.perf_counter() - t0
    cold, shape, _ = parse(buf, used)
    warm, _, _ = parse(buf, used)
    print(json.dumps({"nodes": n, "edges": n * (n + 1) // 2, "text_GB": round(used / 1e9, 3), "gen_s": round(gen_s, 1),
                      "threads": threads, "cold_s": round(cold, 3), "cold_GB_per_s": round(used / cold / 1e9, 3),
                      "warm_s": round(warm, 3), "warm_GB_per_s": round(used / warm / 1e9, 3),
                      "csr": {"n_nodes": shape[0], "n_adj": shape[1]}, "parallel_equals_sequential_1k": same}),
          flush=True)


if __name__ == "__main__":
    main()
