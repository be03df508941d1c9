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


# ---------------------------------------------------------------- the library's xz decoder
# (srt_xz.cpp, read_xz mod.rs:479-492 / lzma-rs 0.3.0): checked against
# Python's liblzma encoder output -- every check type, LZMA2 properties, dict
# sizes, incompressible (stored-chunk) data, concatenated streams, multi-block
# streams from the xz tool -- and corruption must fail loudly.
def _payloads():
    rng = np.random.default_rng(1)
    from shadow_amd import synth
    src, dst, lat, loss = synth.complete_graph(60, 1)
    gml = synth.gml_text(60, src, dst, lat, loss).encode()
    return {
        "empty": b"",
        "one": b"x",
        "gml": gml,
        "random": rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes(),  # stored LZMA2 chunks
        "runs": b"ab" * 200_000 + bytes(range(256)) * 300,  # long matches, rep distances
        "mixed": b"".join(rng.choice([b"edge [", b"node [", b" latency \"", b"ms\"", b"\n  "], 40_000).tolist()),
    }


@pytest.mark.parametrize("check", [lzma.CHECK_NONE, lzma.CHECK_CRC32, lzma.CHECK_CRC64, lzma.CHECK_SHA256])
@pytest.mark.parametrize("name", ["empty", "one", "gml", "random", "runs", "mixed"])
def test_xz_decoder_matches_liblzma(name, check):
    from shadow_amd.graph import xz_decompress
    data = _payloads()[name]
    assert xz_decompress(lzma.compress(data, format=lzma.FORMAT_XZ, check=check)) == data


@pytest.mark.parametrize("lc,lp,pb", [(0, 0, 0), (3, 0, 2), (1, 3, 4), (4, 0, 0), (0, 4, 1), (2, 2, 3)])
def test_xz_decoder_lzma2_properties(lc, lp, pb):
    from shadow_amd.graph import xz_decompress
    data = _payloads()["mixed"] + _payloads()["gml"]
    filt = [{"id": lzma.FILTER_LZMA2, "lc": lc, "lp": lp, "pb": pb, "dict_size": 1 << 16}]
    assert xz_decompress(lzma.compress(data, format=lzma.FORMAT_XZ, filters=filt)) == data


def test_xz_decoder_concatenated_streams_and_padding():
    from shadow_amd.graph import xz_decompress
    a, b = _payloads()["gml"], _payloads()["runs"]
    blob = lzma.compress(a, format=lzma.FORMAT_XZ) + b"\0" * 8 + lzma.compress(b, format=lzma.FORMAT_XZ)
    assert xz_decompress(blob) == a + b


def test_xz_decoder_multi_block_stream(tmp_path):
    import shutil
    import subprocess
    from shadow_amd.graph import xz_decompress
    if not shutil.which("xz"):
        pytest.skip("no xz tool to make a multi-block stream")
    data = _payloads()["mixed"] * 3 + _payloads()["random"]
    f = tmp_path / "m.bin"
    f.write_bytes(data)
    subprocess.run(["xz", "-k", "-6", "--block-size=65536", "-T1", str(f)], check=True)
    blob = (tmp_path / "m.bin.xz").read_bytes()
    assert xz_decompress(blob) == data


def test_xz_decoder_rejects_corruption():
    from shadow_amd import _lib
    from shadow_amd.graph import xz_decompress
    good = lzma.compress(_payloads()["gml"], format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64)
    rng = np.random.default_rng(5)
    for _ in range(40):
        b = bytearray(good)
        k = int(rng.integers(0, len(b)))
        b[k] ^= 1 << int(rng.integers(0, 8))
        with pytest.raises(_lib.SrtError, match="Failed to decompress file"):
            xz_decompress(bytes(b))
    for cut in (0, 5, 12, len(good) // 2, len(good) - 1):
        with pytest.raises(_lib.SrtError, match="Failed to decompress file"):
            xz_decompress(good[:cut])
    # other filters (BCJ, delta) are outside what lzma-rs decodes
    delta = lzma.compress(b"abc" * 100, format=lzma.FORMAT_XZ,
                          filters=[{"id": lzma.FILTER_DELTA, "dist": 1}, {"id": lzma.FILTER_LZMA2}])
    with pytest.raises(_lib.SrtError, match="unsupported filter"):
        xz_decompress(delta)


def test_parse_file_plain_and_xz(tmp_path):
    """srt_gml_parse_file: the whole source -> graph step in the library."""
    from shadow_amd import _lib
    plain = tmp_path / "g.gml"
    plain.write_text(GML)
    xzf = tmp_path / "g.gml.xz"
    xzf.write_bytes(lzma.compress(GML.encode(), format=lzma.FORMAT_XZ))
    ref = NetworkGraph.parse(GML)
    _same(NetworkGraph.parse_file(str(plain)), ref)
    _same(NetworkGraph.parse_file(str(xzf), xz=True), ref)
    with pytest.raises(_lib.SrtError, match="Failed to read file"):
        NetworkGraph.parse_file(str(tmp_path / "missing.gml"))
    with pytest.raises(_lib.SrtError, match='Failed to open file: "'):
        NetworkGraph.parse_file(str(tmp_path / "missing.xz"), xz=True)
    bad = tmp_path / "bad.xz"
    bad.write_bytes(lzma.compress(b"\xff\xfe not utf-8", format=lzma.FORMAT_XZ))
    with pytest.raises(_lib.SrtError, match="utf-8"):
        NetworkGraph.parse_file(str(bad), xz=True)
