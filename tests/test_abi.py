"""CPU tests of the drop-in boundary: libsrt.so loads, exports every symbol
include/srt.h declares, and its host-only pieces (GML ingest, validation
errors raised before any device work) behave like the reference."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import _lib, synth
from shadow_amd.graph import NetworkGraph

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    text = open(os.path.join(ROOT, "include", "srt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(srt_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_surface():
    names = _declared_functions()
    assert "srt_compute_shortest_paths" in names and "srt_packet_batch" in names
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with include/srt.h"


def test_library_exports_every_declared_symbol():
    L = C.CDLL(_lib.LIB_PATH)
    for name in _declared_functions():
        assert hasattr(L, name), name


def test_abi_version_and_struct_layout():
    L = _lib.lib()
    assert L.srt_abi_version() == 4
    assert C.sizeof(_lib.SrtPath) == 16  # #[repr(C)] PathProperties mirror
    assert C.sizeof(_lib.SrtTiming) == 88  # ABI 2: + edge_visits; ABI 4: + create_device_ms
    assert C.sizeof(_lib.SrtCsr) == 56
    assert C.sizeof(_lib.SrtErr) == 268


THREE = open(os.path.join(ROOT, "tests", "golden", "three_node.gml.in")).read() if os.path.exists(
    os.path.join(ROOT, "tests", "golden", "three_node.gml.in")) else None


def _same_graph(text):
    g = NetworkGraph.parse(text)
    o = O.gml_parse(text)
    assert g.directed == o.directed
    assert list(g.node_ids) == list(o.ids)
    # compare adjacency multisets per row
    for u in range(g.n_nodes):
        a = sorted(zip(g.col[g.row_ptr[u]:g.row_ptr[u + 1]].tolist(),
                       g.lat_ns[g.row_ptr[u]:g.row_ptr[u + 1]].tolist(),
                       g.loss[g.row_ptr[u]:g.row_ptr[u + 1]].view(np.uint32).tolist()))
        exp = []
        for s, d, l, p in zip(o.src.tolist(), o.dst.tolist(), o.lat.tolist(), o.loss.view(np.uint32).tolist()):
            if s == u:
                exp.append((d, l, p))
            elif not o.directed and d == u:
                exp.append((s, l, p))
        assert a == sorted(exp)
    return g


@pytest.mark.parametrize("directed", [False, True])
def test_gml_ingest_matches_oracle(directed):
    src, dst, lat, loss = synth.random_graph(12, 7, directed=directed, lat_range_ns=(1, 5_000_000))
    text = synth.gml_text(12, src, dst, lat, loss, directed=directed)
    _same_graph(text)


def test_gml_ingest_c1_slice():
    src, dst, lat, loss = synth.complete_graph(40, 1)
    _same_graph(synth.gml_text(40, src, dst, lat, loss))


@pytest.mark.parametrize("text", [
    "graph [\n]\n",
    "graph [\n  directed 1\n  label \"x y\"\n  node [\n    id 5\n    label \"n\"\n  ]\n]\ntrailing junk",
    "\n\n  graph [\n  node [\n    id 1\n  ]\n  node [\n    id 1\n  ]\n]",
])
def test_gml_ok_cases(text):
    _same_graph(text)


@pytest.mark.parametrize("text", [
    "graph [ node [\n id 1\n ]\n]",                      # '[' must be followed by a newline
    "graph [\n  directed 2\n]",
    "graph [\n  directed 1\n  directed 0\n]",
    "graph [\n  node [\n    label \"x\"\n  ]\n]",          # id missing
    "graph [\n  node [\n    id \"1\"\n  ]\n]",
    "graph [\n  node [\n    id 1\n    host_bandwidth_up \"1 Gbyte\"\n  ]\n]",
    "graph [\n  node [\n    id 1\n  ]\n  edge [\n    source 1\n    target 2\n    latency \"1 ms\"\n  ]\n]",
    "graph [\n  node [\n    id 1\n  ]\n  edge [\n    source 1\n    target 1\n    latency \"1 ms\"\n"
    "    packet_loss 1e\n  ]\n]",
    "graph [\n  a 1\n  a 2\n]",
    "graph [\n  node [\n    id 1\n    x \"\"\n  ]\n]",      # empty string is not a value
])
def test_gml_rejects_like_oracle(text):
    with pytest.raises(O.OracleError):
        O.gml_parse(text)
    with pytest.raises(_lib.SrtError):
        NetworkGraph.parse(text)


def test_selfloop_errors_before_device_work():
    # these fail during plan validation, so they need no GPU
    L = _lib.lib()
    g = NetworkGraph.from_edges(2, [0, 0], [1, 0], [5, 5], directed=True, node_ids=[10, 11])
    nodes = np.array([0, 1], np.uint32)
    plan = C.c_void_p()
    err = _lib.SrtErr()
    rc = L.srt_plan_create(C.byref(g.csr()), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), 2, None,
                           C.byref(plan), C.byref(err))
    assert rc == _lib.SRT_ERR_NO_EDGE
    assert err.msg.decode() == "No edge connecting node 11 to 11"
    g2 = NetworkGraph.from_edges(2, [0, 0, 1, 1], [1, 0, 1, 1], [5, 5, 5, 6], directed=True, node_ids=[10, 11])
    rc = L.srt_plan_create(C.byref(g2.csr()), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), 2, None,
                           C.byref(plan), C.byref(err))
    assert rc == _lib.SRT_ERR_MULTI_EDGE
    assert err.msg.decode() == "More than one edge connecting node 11 to 11"


def test_duplicate_in_use_nodes_rejected():
    L = _lib.lib()
    g = NetworkGraph.from_edges(2, [0, 1], [0, 1], [5, 5], directed=True)
    nodes = np.array([1, 1], np.uint32)
    plan = C.c_void_p()
    err = _lib.SrtErr()
    rc = L.srt_plan_create(C.byref(g.csr()), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), 2, None,
                           C.byref(plan), C.byref(err))
    assert rc == _lib.SRT_ERR_INVALID


def test_path_properties_algebra():
    from shadow_amd.graph import PathProperties
    p = PathProperties(23, 0.35) + PathProperties(11, 0.85)
    assert p.latency_ns == 34 and np.float32(p.packet_loss) == np.float32(0.90250003)
    assert PathProperties(1, 0.5) < PathProperties(2, 0.0) < PathProperties(2, 0.1)


def test_ip_assignment():
    from shadow_amd.graph import IpAssignment
    a = IpAssignment()
    ips = [str(a.assign(7)) for _ in range(3)]
    assert ips == ["11.0.0.1", "11.0.0.2", "11.0.0.3"]
    a.assign_ip(9, "11.0.0.4")
    assert str(a.assign(7)) == "11.0.0.5"
    with pytest.raises(ValueError):
        a.assign_ip(1, "11.0.0.4")
    b = IpAssignment()
    for _ in range(254):
        b.assign(0)
    assert str(b.assign(0)) == "11.0.1.1"  # skips .255 and .0
    assert a.get_nodes() == {7, 9} and a.get_node("11.0.0.4") == 9
