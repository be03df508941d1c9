"""load_network_graph (mod.rs:479-509): plain / xz / inline / built-in graph
sources, parsed by the library's GML ingest (host code, no GPU)."""
import lzma

import numpy as np
import pytest

from shadow_amd import NetworkGraph, load_network_graph
from shadow_amd.graph import ONE_GBIT_SWITCH_GRAPH, GraphLoadError

GML = """graph [
  directed 0
  node [
    id 0
  ]
  node [
    id 1
  ]
  edge [
    source 0
    target 0
    latency "3 ms"
  ]
  edge [
    source 1
    target 1
    latency "5 ms"
  ]
  edge [
    source 0
    target 1
    latency "7 ms"
    packet_loss 0.25
  ]
]"""


def _same(a: NetworkGraph, b: NetworkGraph):
    assert a.n_nodes == b.n_nodes
    for x, y in zip((a.row_ptr, a.col, a.lat_ns, a.loss), (b.row_ptr, b.col, b.lat_ns, b.loss)):
        assert np.array_equal(np.asarray(x), np.asarray(y))


def test_plain_xz_inline_agree(tmp_path):
    plain = tmp_path / "g.gml"
    plain.write_text(GML)
    xz = tmp_path / "g.gml.xz"
    xz.write_bytes(lzma.compress(GML.encode(), format=lzma.FORMAT_XZ))
    t1 = load_network_graph({"type": "gml", "file": {"path": str(plain), "compression": None}})
    t2 = load_network_graph({"type": "gml", "file": {"path": str(xz), "compression": "xz"}})
    t3 = load_network_graph({"type": "gml", "inline": GML})
    assert t1 == t2 == t3 == GML
    _same(NetworkGraph.parse(t1), NetworkGraph.parse(t2))


def test_one_gbit_switch():
    text = load_network_graph({"type": "1_gbit_switch"})
    assert text == ONE_GBIT_SWITCH_GRAPH
    g = NetworkGraph.parse(text)
    assert g.n_nodes == 1
    assert int(np.asarray(g.lat_ns)[0]) == 1_000_000


def test_errors(tmp_path):
    with pytest.raises(GraphLoadError, match="Failed to read file"):
        load_network_graph({"type": "gml", "file": {"path": str(tmp_path / "missing.gml")}})
    with pytest.raises(GraphLoadError, match="Failed to open file"):
        load_network_graph({"type": "gml", "file": {"path": str(tmp_path / "missing.xz"), "compression": "xz"}})
    bad = tmp_path / "bad.xz"
    bad.write_bytes(b"not an xz stream")
    with pytest.raises(GraphLoadError, match="Failed to decompress file"):
        load_network_graph({"type": "gml", "file": {"path": str(bad), "compression": "xz"}})


def test_tilde_expansion(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", str(tmp_path))
    (tmp_path / "h.gml").write_text(GML)
    assert load_network_graph({"type": "gml", "file": {"path": "~/h.gml"}}) == GML
