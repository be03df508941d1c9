"""Host-side mirror of Shadow's network-graph API (src/main/network/graph/mod.rs)
over the gfx950 routing build in libsrt.so.

Names, argument meaning and error behaviour follow the reference:

  reference (mod.rs)                          here
  ------------------------------------------  ------------------------------------
  PathProperties {latency_ns, packet_loss}    PathProperties (+, ordering: 296-331)
  NetworkGraph::parse(text)        :134       NetworkGraph.parse(text)
  NetworkGraph::node_id_to_index   :126       NetworkGraph.node_id_to_index
  NetworkGraph::node_index_to_id   :130       NetworkGraph.node_index_to_id
  compute_shortest_paths(&[NodeIndex]) :183   NetworkGraph.compute_shortest_paths
  get_direct_paths(&[NodeIndex])   :230       NetworkGraph.get_direct_paths
  IpAssignment                     :352-420   IpAssignment
  RoutingInfo                      :428-477   RoutingInfo
  Err(Box<dyn Error>) / panic      :219       NetGraphError (code = srt_status)

The HashMap<(NodeIndex, NodeIndex), PathProperties> result becomes a dense
`PathTable` (row-major u64 latency + f32 loss over the caller's node list) that
also answers `table[(a, b)]` like the map did.
"""
from __future__ import annotations

import ctypes as C
import ipaddress
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import SrtError as NetGraphError


@dataclass(frozen=True)
class PathProperties:
    """mod.rs:296-340. Ordered by latency, then loss; `+` folds loss as
    1 - (1 - a)(1 - b) in f32."""

    latency_ns: int = 0
    packet_loss: float = 0.0

    def __add__(self, other: "PathProperties") -> "PathProperties":
        one = np.float32(1.0)
        a, b = np.float32(self.packet_loss), np.float32(other.packet_loss)
        loss = one - (one - a) * (one - b)
        return PathProperties((self.latency_ns + other.latency_ns) & (2**64 - 1), float(np.float32(loss)))

    def _key(self):
        return (self.latency_ns, self.packet_loss)

    def __lt__(self, o):
        return self._key() < o._key()

    def __le__(self, o):
        return self._key() <= o._key()


def _csr_from_edges(n_nodes: int, src, dst, lat_ns, loss, directed: bool):
    """petgraph adjacency (Graph::edges semantics) as CSR: directed -> outgoing;
    undirected -> every edge from both endpoints, self-loops once."""
    src = np.asarray(src, np.uint32)
    dst = np.asarray(dst, np.uint32)
    lat_ns = np.asarray(lat_ns, np.uint64)
    loss = np.asarray(loss, np.float32)
    if directed:
        rows, cols, lats, losses = src, dst, lat_ns, loss
    else:
        back = src != dst
        rows = np.concatenate([src, dst[back]])
        cols = np.concatenate([dst, src[back]])
        lats = np.concatenate([lat_ns, lat_ns[back]])
        losses = np.concatenate([loss, loss[back]])
    order = np.argsort(rows, kind="stable")
    counts = np.bincount(rows, minlength=n_nodes).astype(np.uint64)
    row_ptr = np.zeros(n_nodes + 1, np.uint64)
    np.cumsum(counts, out=row_ptr[1:])
    return (row_ptr, np.ascontiguousarray(cols[order], np.uint32), np.ascontiguousarray(lats[order], np.uint64),
            np.ascontiguousarray(losses[order], np.float32))


class PathTable:
    """Dense result of compute_shortest_paths / get_direct_paths over `nodes`
    (NodeIndex values): latency_ns[i, j], packet_loss[i, j] = nodes[i] -> nodes[j]."""

    def __init__(self, nodes: np.ndarray, latency_ns: np.ndarray, packet_loss: np.ndarray, min_latency_ns: int):
        self.nodes = nodes
        self.latency_ns = latency_ns
        self.packet_loss = packet_loss
        self.min_latency_ns = min_latency_ns
        self._pos = {int(v): i for i, v in enumerate(nodes)}

    def __len__(self):
        return len(self.nodes) ** 2

    def __getitem__(self, key: Tuple[int, int]) -> PathProperties:
        i, j = self._pos[int(key[0])], self._pos[int(key[1])]
        return PathProperties(int(self.latency_ns[i, j]), float(self.packet_loss[i, j]))

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def items(self):
        for i, a in enumerate(self.nodes):
            for j, b in enumerate(self.nodes):
                yield (int(a), int(b)), PathProperties(int(self.latency_ns[i, j]), float(self.packet_loss[i, j]))


class NetworkGraph:
    """A parsed network graph: petgraph adjacency in CSR plus the GML id map."""

    def __init__(self, n_nodes, node_ids, row_ptr, col, lat_ns, loss, directed, _owner=None):
        self.n_nodes = int(n_nodes)
        self.node_ids = np.ascontiguousarray(node_ids, np.uint32)
        self.row_ptr = np.ascontiguousarray(row_ptr, np.uint64)
        self.col = np.ascontiguousarray(col, np.uint32)
        self.lat_ns = np.ascontiguousarray(lat_ns, np.uint64)
        self.loss = np.ascontiguousarray(loss, np.float32)
        self.directed = bool(directed)
        self._owner = _owner
        # HashMap::insert semantics: a repeated GML id maps to the last node
        self._id_to_index: Dict[int, int] = {int(v): i for i, v in enumerate(self.node_ids)}

    # ---------------------------------------------------------------- build
    @classmethod
    def from_edges(cls, n_nodes: int, src, dst, lat_ns, loss=None, directed: bool = False,
                   node_ids: Optional[Sequence[int]] = None) -> "NetworkGraph":
        """Graph from a GML-order edge list with NodeIndex endpoints."""
        if loss is None:
            loss = np.zeros(len(src), np.float32)
        row_ptr, col, lat, los = _csr_from_edges(n_nodes, src, dst, lat_ns, loss, directed)
        ids = np.arange(n_nodes, dtype=np.uint32) if node_ids is None else node_ids
        return cls(n_nodes, ids, row_ptr, col, lat, los, directed)

    @classmethod
    def parse(cls, graph_text: str) -> "NetworkGraph":
        """NetworkGraph::parse (mod.rs:134-181) via the C++ GML ingest in libsrt."""
        L = _lib.lib()
        b = graph_text.encode()
        h = C.c_void_p()
        err = _lib.SrtErr()
        _lib.check(L.srt_gml_parse(b, len(b), C.byref(h), C.byref(err)), err)
        return cls._from_gml(h)

    @classmethod
    def parse_file(cls, path: str, xz: bool = False) -> "NetworkGraph":
        """load_network_graph's file source (mod.rs:494-509; read_xz :479-492 when
        xz) + parse, all in libsrt (srt_gml_parse_file: the library's xz decoder)."""
        import os
        L = _lib.lib()
        h = C.c_void_p()
        err = _lib.SrtErr()
        _lib.check(L.srt_gml_parse_file(os.path.expanduser(path).encode(), int(bool(xz)), C.byref(h),
                                        C.byref(err)), err)
        return cls._from_gml(h)

    @classmethod
    def _from_gml(cls, h) -> "NetworkGraph":
        L = _lib.lib()
        try:
            csr = _lib.SrtCsr()
            L.srt_gml_csr(h, C.byref(csr))
            n, m = csr.n_nodes, csr.n_adj
            as_np = np.ctypeslib.as_array
            row_ptr = as_np(csr.row_ptr, (n + 1,)).copy()
            col = as_np(csr.col, (m,)).copy() if m else np.zeros(0, np.uint32)
            lat = as_np(csr.lat_ns, (m,)).copy() if m else np.zeros(0, np.uint64)
            loss = as_np(csr.loss, (m,)).copy() if m else np.zeros(0, np.float32)
            ids = as_np(csr.node_ids, (n,)).copy() if n else np.zeros(0, np.uint32)
            return cls(n, ids, row_ptr, col, lat, loss, bool(csr.directed))
        finally:
            L.srt_gml_free(h)

    # ---------------------------------------------------------------- ids
    def node_id_to_index(self, gml_id: int) -> Optional[int]:
        return self._id_to_index.get(int(gml_id))

    def node_index_to_id(self, index: int) -> Optional[int]:
        return int(self.node_ids[index]) if 0 <= index < self.n_nodes else None

    # ---------------------------------------------------------------- ABI
    def csr(self) -> _lib.SrtCsr:
        c = _lib.SrtCsr()
        c.n_nodes = self.n_nodes
        c.directed = int(self.directed)
        c.n_adj = len(self.col)
        c.row_ptr = self.row_ptr.ctypes.data_as(C.POINTER(C.c_uint64))
        c.col = self.col.ctypes.data_as(C.POINTER(C.c_uint32))
        c.lat_ns = self.lat_ns.ctypes.data_as(C.POINTER(C.c_uint64))
        c.loss = self.loss.ctypes.data_as(C.POINTER(C.c_float))
        c.node_ids = self.node_ids.ctypes.data_as(C.POINTER(C.c_uint32))
        return c

    def _run(self, fn_name: str, nodes, algo: int, device: int, n_gpus: int = 1, same_device: bool = False) -> PathTable:
        L = _lib.lib()
        _lib.require_device()
        nodes = np.ascontiguousarray(np.asarray(list(nodes) if not isinstance(nodes, np.ndarray) else nodes),
                                     np.uint32)
        n = len(nodes)
        out = (_lib.SrtPath * max(n * n, 1))()
        mn = C.c_uint64()
        opts = _lib.SrtOpts(algo, device, _lib.SRT_OPT_SAME_DEVICE if same_device else 0, n_gpus)
        err = _lib.SrtErr()
        csr = self.csr()
        rc = getattr(L, fn_name)(C.byref(csr), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), n, out, C.byref(mn),
                                 C.byref(opts), C.byref(err))
        _lib.check(rc, err)
        raw = np.frombuffer(out, dtype=np.dtype([("lat", "<u8"), ("loss", "<f4"), ("pad", "<u4")]), count=n * n)
        return PathTable(nodes, raw["lat"].reshape(n, n).copy(), raw["loss"].reshape(n, n).copy(), mn.value)

    def compute_shortest_paths(self, nodes: Iterable[int], algo: int = _lib.SRT_ALGO_AUTO,
                               device: int = -1, n_gpus: int = 1, same_device: bool = False) -> PathTable:
        """mod.rs:183-228 on the GPU. Raises NetGraphError(code=NO_EDGE/MULTI_EDGE)
        for a missing/duplicate self-loop and code=DISCONNECTED where the
        reference panics on an unreachable pair.  n_gpus > 1: sharded over
        devices device .. device + n_gpus - 1 from this process (one library
        thread per device); same_device puts every rank on `device` (tests)."""
        return self._run("srt_compute_shortest_paths", nodes, algo, device, n_gpus, same_device)

    def get_direct_paths(self, nodes: Iterable[int], device: int = -1) -> PathTable:
        """mod.rs:230-252 on the GPU."""
        return self._run("srt_get_direct_paths", nodes, _lib.SRT_ALGO_AUTO, device)


def _ip_be(ip) -> int:
    """IPv4 (str / int / IPv4Address) -> u32 in network byte order."""
    return int.from_bytes(ipaddress.IPv4Address(ip).packed, "little")


def _ip_from_be(x: int) -> ipaddress.IPv4Address:
    return ipaddress.IPv4Address(int(x).to_bytes(4, "little"))


class IpAssignment:
    """IpAssignment<u32> (mod.rs:352-420) in libsrt (srt_ip_assignment_*):
    IP <-> node id; auto-assignment from 11.0.0.1 upward, skipping addresses
    ending in .0 or .255; assign_ip refuses a taken address."""

    def __init__(self):
        self._h = C.c_void_p()
        _lib.check(_lib.lib().srt_ip_assignment_create(C.byref(self._h)), _lib.SrtErr())

    def assign(self, node_id: int) -> ipaddress.IPv4Address:
        return _ip_from_be(_lib.lib().srt_ip_assignment_assign(self._h, int(node_id)))

    def assign_ip(self, node_id: int, ip) -> None:
        err = _lib.SrtErr()
        rc = _lib.lib().srt_ip_assignment_assign_ip(self._h, int(node_id), _ip_be(ip), C.byref(err))
        if rc != _lib.SRT_OK:
            raise ValueError(err.msg.decode())  # IpPreviouslyAssignedError (mod.rs:343-350)

    def get_node(self, ip) -> Optional[int]:
        v = C.c_uint32()
        return int(v.value) if _lib.lib().srt_ip_assignment_get_node(self._h, _ip_be(ip), C.byref(v)) else None

    def get_nodes(self) -> set:
        L = _lib.lib()
        k = L.srt_ip_assignment_get_nodes(self._h, None, 0)
        out = np.zeros(max(k, 1), np.uint32)
        L.srt_ip_assignment_get_nodes(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), k)
        return set(out[:k].tolist())

    def __len__(self) -> int:
        return int(_lib.lib().srt_ip_assignment_size(self._h))

    def resolver(self, row_ids) -> "IpResolver":
        """The assignment frozen against a table whose row i is GML node row_ids[i]."""
        return IpResolver(self, row_ids)

    def close(self):
        if self._h:
            _lib.lib().srt_ip_assignment_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class IpResolver:
    """srt_ip_resolver: IPv4 -> table row for the send path (the two get_node
    lookups + path() of WorkerShared::latency / reliability, worker.rs:539-553),
    on host threads (rows) or inside the device round (RoutingPlan.packet_batch_ip)."""

    def __init__(self, assignment: IpAssignment, row_ids):
        ids = np.ascontiguousarray(row_ids, np.uint32)
        self._h = C.c_void_p()
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_ip_resolver_create(assignment._h, ids.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                     len(ids), C.byref(self._h), C.byref(err)), err)

    def rows(self, ips_be: np.ndarray) -> np.ndarray:
        """int32 table rows of u32 network-byte-order addresses (-1: no row)."""
        ips = np.ascontiguousarray(ips_be, np.uint32)
        out = np.empty(len(ips), np.int32)
        _lib.check(_lib.lib().srt_ip_resolve_rows(self._h, ips.ctypes.data_as(C.POINTER(C.c_uint32)), len(ips),
                                                  out.ctypes.data_as(C.POINTER(C.c_int32))), _lib.SrtErr())
        return out

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            _lib.lib().srt_ip_resolver_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RoutingInfo:
    """RoutingInfo (mod.rs:428-477) over libsrt's dense srt_routing_info: the
    GPU-built table stays row-major over the in-use nodes, a GML id -> row map
    answers path(), and the packet counters are a dense array of atomics with
    the reference's saturating add (no RwLock<HashMap>)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def build(cls, graph: "NetworkGraph", nodes, use_shortest_paths: bool = True, algo: int = _lib.SRT_ALGO_AUTO,
              device: int = -1, n_gpus: int = 1, same_device: bool = False) -> "RoutingInfo":
        L = _lib.lib()
        _lib.require_device()
        nodes = np.ascontiguousarray(np.asarray(list(nodes) if not isinstance(nodes, np.ndarray) else nodes),
                                     np.uint32)
        h = C.c_void_p()
        err = _lib.SrtErr()
        opts = _lib.SrtOpts(algo, device, _lib.SRT_OPT_SAME_DEVICE if same_device else 0, n_gpus)
        csr = graph.csr()
        _lib.check(L.srt_routing_info_build(C.byref(csr), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), len(nodes),
                                            int(bool(use_shortest_paths)), C.byref(opts), C.byref(h), C.byref(err)),
                   err)
        return cls(h)

    @classmethod
    def from_plan(cls, plan) -> "RoutingInfo":
        h = C.c_void_p()
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_routing_info_from_plan(plan.handle, C.byref(h), C.byref(err)), err)
        return cls(h)

    def __len__(self) -> int:
        return int(_lib.lib().srt_routing_info_size(self._h))

    def path(self, start: int, end: int) -> Optional[PathProperties]:
        p = _lib.SrtPath()
        if _lib.lib().srt_routing_info_path(self._h, int(start), int(end), C.byref(p)) != _lib.SRT_OK:
            return None
        return PathProperties(int(p.latency_ns), float(np.float32(p.packet_loss)))

    def row_of(self, gml_id: int) -> Optional[int]:
        r = _lib.lib().srt_routing_info_row(self._h, int(gml_id))
        return None if r < 0 else int(r)

    def increment_packet_count(self, start: int, end: int) -> None:
        _lib.lib().srt_routing_info_increment_packet_count(self._h, int(start), int(end))

    def add_packet_counts(self, counts: np.ndarray) -> None:
        counts = np.ascontiguousarray(counts, np.uint64)
        assert counts.size == len(self) ** 2
        _lib.lib().srt_routing_info_add_packet_counts(self._h, counts.ctypes.data_as(C.POINTER(C.c_uint64)))

    def packet_count(self, start: int, end: int) -> int:
        return int(_lib.lib().srt_routing_info_packet_count(self._h, int(start), int(end)))

    def get_smallest_latency_ns(self) -> Optional[int]:
        v = C.c_uint64()
        return int(v.value) if _lib.lib().srt_routing_info_smallest_latency_ns(self._h, C.byref(v)) else None

    def record_bytes(self) -> int:
        """Bytes a pair of the stored table: 6 / 8 (compact records decoded by
        path()) or 16 (srt_path)."""
        return int(_lib.lib().srt_routing_info_record_bytes(self._h))

    def table(self):
        """(latency_ns u64[n,n], packet_loss f32[n,n]) copies of the dense table
        (srt_routing_info_copy_table: any storage)."""
        n = len(self)
        rec = np.empty(max(n * n, 1), np.dtype([("lat", "<u8"), ("loss", "<f4"), ("pad", "<u4")]))
        _lib.lib().srt_routing_info_copy_table(self._h, rec.ctypes.data_as(C.POINTER(_lib.SrtPath)))
        rec = rec[:n * n]
        return rec["lat"].reshape(n, n).copy(), rec["loss"].reshape(n, n).copy()

    def close(self):
        if self._h:
            _lib.lib().srt_routing_info_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# configuration.rs ONE_GBIT_SWITCH_GRAPH: one node, its self-loop at 1 ms
ONE_GBIT_SWITCH_GRAPH = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""


class GraphLoadError(RuntimeError):
    """load_network_graph failures (the reference's NetGraphError contexts)."""


def load_network_graph(options) -> str:
    """mod.rs:494-509 (load_network_graph) + :479-492 (read_xz): the GML text of
    a `network.graph` option, given as the configuration's mapping
    (configuration.rs:976-1004):
      {"type": "gml", "file": {"path": p, "compression": None | "xz"}}
      {"type": "gml", "inline": text}
      {"type": "1_gbit_switch"}
    Paths get tilde expansion; xz files are decompressed by libsrt's own
    .xz / LZMA2 decoder (the reference's lzma-rs step) and must be UTF-8."""
    import os

    kind = options.get("type")
    if kind == "1_gbit_switch":
        return ONE_GBIT_SWITCH_GRAPH
    if kind != "gml":
        raise GraphLoadError(f"unknown graph type: {kind!r}")
    if "inline" in options:
        return options["inline"]
    src = options.get("file") or {}
    path = os.path.expanduser(src["path"])
    comp = src.get("compression")
    if comp is None:
        try:
            with open(path, "r", encoding="utf-8") as f:
                return f.read()
        except (OSError, UnicodeDecodeError) as e:
            raise GraphLoadError(f"Failed to read file: {src['path']}") from e
    if comp != "xz":
        raise GraphLoadError(f"unknown compression: {comp!r}")
    try:
        f = open(path, "rb")
    except OSError as e:
        raise GraphLoadError(f"Failed to open file: {path!r}") from e
    with f:
        raw = f.read()
    try:
        data = xz_decompress(raw)
    except _lib.SrtError as e:
        raise GraphLoadError("Failed to decompress file") from e
    try:
        return data.decode("utf-8")
    except UnicodeDecodeError as e:
        raise GraphLoadError(f"invalid utf-8 in {path!r}") from e


def xz_decompress(raw: bytes) -> bytes:
    """read_xz's decompression (mod.rs:479-492) by libsrt's .xz / LZMA2 decoder
    (srt_xz_decompress); raises SrtError("Failed to decompress file: ...")."""
    L = _lib.lib()
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    err = _lib.SrtErr()
    _lib.check(L.srt_xz_decompress(raw, len(raw), C.byref(out), C.byref(n), C.byref(err)), err)
    try:
        return C.string_at(out, n.value)
    finally:
        L.srt_free(out)


def generate_routing_info(graph: NetworkGraph, node_ids: set, use_shortest_paths: bool = True) -> RoutingInfo:
    """sim_config.rs:424-461: GML ids of the in-use nodes -> NodeIndex list ->
    srt_routing_info_build (the table keyed by GML ids without re-keying every
    pair)."""
    nodes = np.array([graph.node_id_to_index(x) for x in node_ids], np.uint32)
    return RoutingInfo.build(graph, nodes, use_shortest_paths)
