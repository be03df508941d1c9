"""ctypes binding of liboracle.so -- the CPU restatement of Shadow's routing
build and send_packet decision.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker or the timed CPU baseline;
never by the product package (shadow_amd), which fails loudly without its HIP
library instead of falling back to anything here.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OK, NO_EDGE, MULTI_EDGE, DISCONNECTED, PARSE, ARG = range(6)
PDS_NONE, PDS_INET_SENT, PDS_INET_DROPPED = 0, 1 << 8, 1 << 9


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class _EdgeList(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("n_edges", C.c_uint32),
        ("src", C.POINTER(C.c_uint32)),
        ("dst", C.POINTER(C.c_uint32)),
        ("lat_ns", C.POINTER(C.c_uint64)),
        ("loss", C.POINTER(C.c_float)),
        ("directed", C.c_int),
    ]


class _Err(C.Structure):
    _fields_ = [("code", C.c_int), ("a_id", C.c_uint32), ("b_id", C.c_uint32), ("msg", C.c_char * 256)]


class Pkt(C.Structure):
    _fields_ = [
        ("src_host", C.c_uint32),
        ("src_row", C.c_uint32),
        ("dst_row", C.c_uint32),
        ("payload_size", C.c_uint32),
        ("t_ns", C.c_uint64),
    ]


PKT_DTYPE = np.dtype(
    [("src_host", "<u4"), ("src_row", "<u4"), ("dst_row", "<u4"), ("payload_size", "<u4"), ("t_ns", "<u8")]
)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u64p, u32p, f32p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_float)
        L.or_splitmix64_next.argtypes = [u64p]
        L.or_splitmix64_next.restype = C.c_uint64
        L.or_xoshiro_seed_from_u64.argtypes = [C.c_uint64, u64p]
        L.or_xoshiro_next.argtypes = [u64p]
        L.or_xoshiro_next.restype = C.c_uint64
        L.or_gen_f64.argtypes = [u64p]
        L.or_gen_f64.restype = C.c_double
        L.or_siphash13_str.argtypes = [C.c_char_p, C.c_size_t]
        L.or_siphash13_str.restype = C.c_uint64
        L.or_siphash_cd.argtypes = [C.c_char_p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
        L.or_siphash_cd.restype = C.c_uint64
        L.or_host_seed.argtypes = [C.c_uint32, C.c_char_p]
        L.or_host_seed.restype = C.c_uint64
        L.or_parse_time_ns.argtypes = [C.c_char_p, C.c_size_t, u64p, u64p, C.c_char_p, C.c_size_t]
        L.or_gml_parse.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.or_gml_parse.restype = C.c_void_p
        L.or_graph_free.argtypes = [C.c_void_p]
        L.or_graph_directed.argtypes = [C.c_void_p]
        L.or_graph_num_nodes.argtypes = [C.c_void_p]
        L.or_graph_num_nodes.restype = C.c_uint32
        L.or_graph_num_edges.argtypes = [C.c_void_p]
        L.or_graph_num_edges.restype = C.c_uint32
        L.or_graph_node_ids.argtypes = [C.c_void_p, u32p]
        L.or_graph_index_of.argtypes = [C.c_void_p, C.c_uint32]
        L.or_graph_index_of.restype = C.c_int64
        L.or_graph_edges.argtypes = [C.c_void_p, u32p, u32p, u64p, f32p]
        L.or_compute_shortest_paths.argtypes = [
            C.POINTER(_EdgeList), u32p, u32p, C.c_uint32, C.c_uint32, u64p, f32p, C.c_int, C.c_int,
            C.POINTER(_Err)]
        L.or_get_direct_paths.argtypes = [C.POINTER(_EdgeList), u32p, u32p, C.c_uint32, u64p, f32p,
                                          C.POINTER(_Err)]
        L.or_path_add.argtypes = [C.c_uint64, C.c_float, C.c_uint64, C.c_float, u64p, f32p]
        L.or_packet_batch.argtypes = [
            u64p, f32p, C.c_uint32, C.c_void_p, C.c_uint64, u64p, C.c_uint64, C.c_uint64, C.c_uint64,
            u32p, u64p, u64p, u64p, u64p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class OracleError(Exception):
    def __init__(self, code, msg, a_id=0, b_id=0):
        super().__init__(msg)
        self.code, self.a_id, self.b_id = code, a_id, b_id


# ------------------------------------------------------------ IpAssignment
class IpAssignment:
    """Restatement of IpAssignment<u32> (src/main/network/graph/mod.rs:352-420),
    addresses as host-order u32: a dict map, last_assigned_addr from 11.0.0.0
    (:366), assign loops increment_address (:406-420, skip *.0 / *.255) until a
    vacant entry (:371-381), assign_ip refuses an occupied one (:383-394)."""

    def __init__(self):
        self.map = {}
        self.last = 11 << 24

    def assign(self, node_id: int) -> int:
        while True:
            x = self.last
            while True:
                x += 1
                if x & 0xFF not in (0, 255):
                    break
            self.last = x
            if x not in self.map:
                self.map[x] = node_id
                return x

    def assign_ip(self, node_id: int, ip: int) -> bool:
        if ip in self.map:
            return False  # IpPreviouslyAssignedError
        self.map[ip] = node_id
        return True

    def get_node(self, ip: int):
        return self.map.get(ip)

    def get_nodes(self) -> set:
        return set(self.map.values())


# ---------------------------------------------------------------- RNG / units
def xoshiro_seed(seed: int) -> np.ndarray:
    s = np.zeros(4, np.uint64)
    lib().or_xoshiro_seed_from_u64(C.c_uint64(seed), _p(s, C.c_uint64))
    return s


def xoshiro_next(state: np.ndarray) -> int:
    return lib().or_xoshiro_next(_p(state, C.c_uint64))


def gen_f64(state: np.ndarray) -> float:
    return lib().or_gen_f64(_p(state, C.c_uint64))


def siphash13_str(s: str) -> int:
    b = s.encode()
    return lib().or_siphash13_str(b, len(b))


def siphash_cd(msg: bytes, k0: int, k1: int, c: int, d: int) -> int:
    return lib().or_siphash_cd(msg, len(msg), k0, k1, c, d)


def host_seed(general_seed: int, hostname: str) -> int:
    return lib().or_host_seed(general_seed, hostname.encode())


def parse_time_ns(s: str):
    b = s.encode()
    ns, v = C.c_uint64(), C.c_uint64()
    err = C.create_string_buffer(256)
    rc = lib().or_parse_time_ns(b, len(b), C.byref(ns), C.byref(v), err, 256)
    if rc:
        raise OracleError(rc, err.value.decode(errors="replace"))
    return ns.value, v.value


def path_add(la, pa, lb, pb):
    lo, po = C.c_uint64(), C.c_float()
    lib().or_path_add(la, pa, lb, pb, C.byref(lo), C.byref(po))
    return lo.value, po.value


# ---------------------------------------------------------------- graphs
class Graph:
    """Parsed GML graph (NetworkGraph::parse restated): node ids in GML order and
    the GML-order edge list with endpoints as node indices."""

    def __init__(self, directed, ids, src, dst, lat, loss):
        self.directed = bool(directed)
        self.ids = np.ascontiguousarray(ids, np.uint32)
        self.src = np.ascontiguousarray(src, np.uint32)
        self.dst = np.ascontiguousarray(dst, np.uint32)
        self.lat = np.ascontiguousarray(lat, np.uint64)
        self.loss = np.ascontiguousarray(loss, np.float32)

    @property
    def n_nodes(self):
        return len(self.ids)

    def index_of(self, gml_id):
        idx = np.nonzero(self.ids == gml_id)[0]
        return int(idx[-1]) if len(idx) else None

    def _el(self):
        el = _EdgeList()
        el.n_nodes = self.n_nodes
        el.n_edges = len(self.src)
        el.src = _p(self.src, C.c_uint32)
        el.dst = _p(self.dst, C.c_uint32)
        el.lat_ns = _p(self.lat, C.c_uint64)
        el.loss = _p(self.loss, C.c_float)
        el.directed = int(self.directed)
        return el


def gml_parse(text: str) -> Graph:
    b = text.encode()
    err = C.create_string_buffer(256)
    L = lib()
    h = L.or_gml_parse(b, len(b), err, 256)
    if not h:
        raise OracleError(PARSE, err.value.decode(errors="replace"))
    try:
        n, m = L.or_graph_num_nodes(h), L.or_graph_num_edges(h)
        ids = np.zeros(n, np.uint32)
        L.or_graph_node_ids(h, _p(ids, C.c_uint32))
        src, dst = np.zeros(m, np.uint32), np.zeros(m, np.uint32)
        lat, loss = np.zeros(m, np.uint64), np.zeros(m, np.float32)
        L.or_graph_edges(h, _p(src, C.c_uint32), _p(dst, C.c_uint32), _p(lat, C.c_uint64), _p(loss, C.c_float))
        return Graph(L.or_graph_directed(h), ids, src, dst, lat, loss)
    finally:
        L.or_graph_free(h)


def compute_shortest_paths(g: Graph, nodes, threads=0, mode=1, src_count=None):
    """Returns (lat[n,n] u64, loss[n,n] f32); raises OracleError like the reference."""
    nodes = np.ascontiguousarray(nodes, np.uint32)
    n = len(nodes)
    sc = n if src_count is None else int(src_count)
    lat = np.zeros((n, n), np.uint64)
    loss = np.zeros((n, n), np.float32)
    err = _Err()
    el = g._el()
    rc = lib().or_compute_shortest_paths(C.byref(el), _p(g.ids, C.c_uint32), _p(nodes, C.c_uint32), n, sc,
                                         _p(lat, C.c_uint64), _p(loss, C.c_float), threads, mode, C.byref(err))
    if rc:
        raise OracleError(rc, err.msg.decode(errors="replace"), err.a_id, err.b_id)
    return lat, loss


def get_direct_paths(g: Graph, nodes):
    nodes = np.ascontiguousarray(nodes, np.uint32)
    n = len(nodes)
    lat = np.zeros((n, n), np.uint64)
    loss = np.zeros((n, n), np.float32)
    err = _Err()
    el = g._el()
    rc = lib().or_get_direct_paths(C.byref(el), _p(g.ids, C.c_uint32), _p(nodes, C.c_uint32), n,
                                   _p(lat, C.c_uint64), _p(loss, C.c_float), C.byref(err))
    if rc:
        raise OracleError(rc, err.msg.decode(errors="replace"), err.a_id, err.b_id)
    return lat, loss


def packet_batch(lat, loss, pkts: np.ndarray, rng: np.ndarray, round_end, bootstrap_end, sim_end,
                 counters=None):
    """Sequential send_packet restatement. rng (n_hosts,4) u64 is updated in place.
    Returns (flags u32, deliver u64, min_latency, next_event)."""
    lat = np.ascontiguousarray(lat, np.uint64)
    loss = np.ascontiguousarray(loss, np.float32)
    pkts = np.ascontiguousarray(pkts, PKT_DTYPE)
    assert rng.dtype == np.uint64 and rng.flags.c_contiguous
    n = lat.shape[0]
    m = len(pkts)
    flags = np.zeros(m, np.uint32)
    deliver = np.zeros(m, np.uint64)
    mn, ne = C.c_uint64(), C.c_uint64()
    cp = _p(counters, C.c_uint64) if counters is not None else None
    lib().or_packet_batch(_p(lat, C.c_uint64), _p(loss, C.c_float), n, pkts.ctypes.data, m,
                          _p(rng, C.c_uint64), round_end, bootstrap_end, sim_end, _p(flags, C.c_uint32),
                          _p(deliver, C.c_uint64), cp, C.byref(mn), C.byref(ne))
    return flags, deliver, mn.value, ne.value


def packet_events(host_ptr, flags, deliver, dst_host, n_dst_hosts, event_base):
    """Restatement of Worker::push_packet_to_host (worker.rs:629-639) for a
    batch, in the reference's own terms: walk the packets in send order (hosts
    in HostId order), give every SENT packet Event::new_packet (event.rs:20-31)
    with the source host's next event id (host.rs:691-695), push it on its
    destination host's queue -- a binary heap ordered like Event (time, then
    PacketEventData: src_host_id, then src_host_event_id; event.rs:85-150) --
    and pop each queue empty.  event_base (per host, u64) is advanced in place.
    Returns (event_id u64 per packet, UINT64_MAX if not sent; order u32 of the
    sent packets by destination then pop order; dst_ptr u32[n_dst_hosts+1])."""
    import heapq

    host_ptr = np.asarray(host_ptr, np.int64)
    m = len(flags)
    event_id = np.full(m, np.iinfo(np.uint64).max, np.uint64)
    queues = [[] for _ in range(n_dst_hosts)]
    for h in range(len(host_ptr) - 1):
        for p in range(int(host_ptr[h]), int(host_ptr[h + 1])):
            if int(flags[p]) != PDS_INET_SENT:
                continue
            eid = int(event_base[h])
            event_base[h] = np.uint64(eid + 1)
            event_id[p] = eid
            heapq.heappush(queues[int(dst_host[p])], (int(deliver[p]), h, eid, p))
    order, dst_ptr = [], [0]
    for q in queues:
        while q:
            order.append(heapq.heappop(q)[3])
        dst_ptr.append(len(order))
    return event_id, np.array(order, np.uint32), np.array(dst_ptr, np.uint32)
