"""CPU tests of the chunk-parallel GML ingest (srt_gml.cpp):
forced onto small inputs (SRT_GML_PAR_BYTES=0), it must build the same
petgraph-shaped CSR as the sequential parser and the oracle, including strings
that contain '[' / ']' and every kind of top-level item, and it must report the
same error text as the sequential parser (which it falls back to)."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import _lib, synth
from shadow_amd.graph import NetworkGraph


def _parse(text, parallel, strict=False, threads=8):
    keys = ("SRT_GML_PAR_BYTES", "SRT_GML_THREADS", "SRT_GML_STRICT_PARALLEL")
    old = {k: os.environ.get(k) for k in keys}
    try:
        os.environ["SRT_GML_PAR_BYTES"] = "0" if parallel else str(1 << 40)
        os.environ["SRT_GML_THREADS"] = str(threads)
        if strict:
            os.environ["SRT_GML_STRICT_PARALLEL"] = "1"
        else:
            os.environ.pop("SRT_GML_STRICT_PARALLEL", None)
        return NetworkGraph.parse(text)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _tricky_gml(n, seed, directed):
    """Random graph with labels holding '[' ']' and spaces, extra top-level and
    block keys, jitter, CRLF line ends on some lines and odd spacing."""
    src, dst, lat, loss = synth.random_graph(n, seed, p_edge=0.2, directed=directed, lat_range_ns=(1, 9_000_000))
    rng = np.random.default_rng(seed)
    out = ["graph [", '  label "net [v2] ]["', f"  directed {1 if directed else 0}", "  weird_key 7"]
    for i in range(n):
        lab = f'"n]{i}[ x"'
        out.append(f"  node [\n    id {i}\n    label {lab}\n    host_bandwidth_up \"1 Gbit\"\n  ]")
    for k, (s, d, l, p) in enumerate(zip(src.tolist(), dst.tolist(), lat.tolist(), loss.tolist())):
        lat_s = f"{l // 1000} us" if l % 1000 == 0 else f"{l} ns"
        nl = "\r\n" if k % 7 == 0 else "\n"
        extra = f'    jitter "0 ms"{nl}' if k % 3 == 0 else ""
        out.append(f"  edge [{nl}    source {s}{nl}    target {d}{nl}    label \"e[{k}]\"{nl}"
                   f"    latency \"{lat_s}\"{nl}{extra}    packet_loss {p:.6f}{nl}  ]")
        if k == len(src) // 2:
            out.append('  middle_key "in [the] middle"')
    out.append("]")
    return "\n".join(out) + "\ntrailing [ junk \" ] after the graph\n"


def _same(a, b):
    assert a.directed == b.directed
    assert np.array_equal(a.node_ids, b.node_ids)
    assert np.array_equal(a.row_ptr, b.row_ptr)
    assert np.array_equal(a.col, b.col)
    assert np.array_equal(a.lat_ns, b.lat_ns)
    assert np.array_equal(a.loss.view(np.uint32), b.loss.view(np.uint32))


@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("threads", [2, 8])
def test_parallel_equals_sequential(directed, threads):
    text = _tricky_gml(120, 3 + threads, directed)
    seq = _parse(text, parallel=False)
    par = _parse(text, parallel=True, strict=True, threads=threads)
    _same(seq, par)
    og = O.gml_parse(text)  # and the oracle's own parse of the same text
    assert list(og.ids) == list(seq.node_ids) and bool(og.directed) == seq.directed


def test_parallel_complete_graph_matches_oracle():
    n = 150
    src, dst, lat, loss = synth.complete_graph(n, 1)
    text = synth.gml_text(n, src, dst, lat, loss)
    par = _parse(text, parallel=True, strict=True)
    seq = _parse(text, parallel=False)
    _same(seq, par)


BAD = [
    # syntax error inside an edge block in the middle
    lambda t: t.replace("    source 7\n", "    source 7 oops\n", 1),
    # unterminated string (fools the quote parity from there on)
    lambda t: t.replace('label "e[5]"', 'label "e[5]', 1),
    # validation: missing latency in a late edge
    lambda t: t[::-1].replace('"sm 1" ycnetal', "", 1)[::-1],
    # validation: unknown endpoint
    lambda t: t.replace("    target 3\n", "    target 999999\n", 1),
    # duplicate key inside a block
    lambda t: t.replace("    id 4\n", "    id 4\n    id 5\n", 1),
    # a second 'directed'
    lambda t: t.replace("  weird_key 7", "  weird_key 7\n  directed 1", 1),
    # packet_loss as an int literal ("not a float", parser.rs:214-224)
    lambda t: t.replace("packet_loss 0.", "packet_loss 0\n    x 0.", 1),
]


@pytest.mark.parametrize("k", range(len(BAD)))
def test_parallel_errors_match_sequential(k):
    n = 40
    src, dst, lat, loss = synth.random_graph(n, 9, p_edge=0.3, lat_range_ns=(1, 5))
    text = synth.gml_text(n, src, dst, lat * np.uint64(synth.MS), loss).replace(
        "graph [\n", "graph [\n  weird_key 7\n", 1)
    text = text.replace("  edge [\n    source", '  edge [\n    label "e[5]"\n    source', 1)
    bad = BAD[k](text)
    assert bad != text
    with pytest.raises(_lib.SrtError) as e1:
        _parse(bad, parallel=False)
    with pytest.raises(_lib.SrtError) as e2:
        _parse(bad, parallel=True)
    assert str(e1.value) == str(e2.value)


def test_float_fast_path_matches_strtof():
    """packet_loss tokens of 1..9 significant digits, leading zeros, '+', '.5',
    '1.' and exponent forms: the ingest's exact fast path (d / 10^k in f32)
    and its strtof fallback must equal the oracle's strtof bit for bit."""
    rng = np.random.default_rng(5)
    toks = ["0", "1", "1.", ".5", "+0.25", "0.0", "1.0", "0.000001", "0.9999999", "0.99999999", "1e-3",
            "2.5E-1", "0.1", "0.3", "0.7", "0.16777217", "0.16777216"]
    for _ in range(400):
        nd = int(rng.integers(1, 10))
        digits = "".join(str(int(x)) for x in rng.integers(0, 10, nd))
        lead = "0" * int(rng.integers(0, 4))
        toks.append("0." + lead + digits)
    lines = ["graph [", "  directed 1", "  node [", "    id 0", "  ]"]
    for t in toks:
        val = t if any(c in t for c in ".eE") else t + ".0"
        lines.append(f'  edge [\n    source 0\n    target 0\n    latency "1 ns"\n    packet_loss {val}\n  ]')
    text = "\n".join(lines) + "\n]\n"
    og = O.gml_parse(text)
    for par in (False, True):
        g = _parse(text, parallel=par)
        assert np.array_equal(np.sort(g.loss.view(np.uint32)), np.sort(og.loss.view(np.uint32)))
