"""ctypes binding of libsrt.so (the C ABI declared in include/srt.h).

The product path has no CPU fallback: if libsrt.so is missing or no HIP device
is visible, every entry point raises instead of computing anything elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRT_LIB", os.path.join(_HERE, "libsrt.so"))  # SRT_LIB: A/B builds only

SRT_OK = 0
SRT_ERR_NO_EDGE = 1
SRT_ERR_MULTI_EDGE = 2
SRT_ERR_DISCONNECTED = 3
SRT_ERR_INVALID = 4
SRT_ERR_HIP = 5
SRT_ERR_OOM = 6
SRT_ERR_UNSUPPORTED = 7
SRT_ERR_COMM = 8

SRT_ALGO_AUTO, SRT_ALGO_FW, SRT_ALGO_SSSP, SRT_ALGO_LEVEL = 0, 1, 2, 3
SRT_OPT_SAME_DEVICE = 1  # srt_opts.flags: every n_gpus rank on `device` (tests)
PDS_NONE, PDS_INET_SENT, PDS_INET_DROPPED = 0, 1 << 8, 1 << 9


class SrtErr(C.Structure):
    _fields_ = [("code", C.c_int32), ("a_id", C.c_uint32), ("b_id", C.c_uint32), ("msg", C.c_char * 256)]


class SrtCsr(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("directed", C.c_uint32),
        ("n_adj", C.c_uint64),
        ("row_ptr", C.POINTER(C.c_uint64)),
        ("col", C.POINTER(C.c_uint32)),
        ("lat_ns", C.POINTER(C.c_uint64)),
        ("loss", C.POINTER(C.c_float)),
        ("node_ids", C.POINTER(C.c_uint32)),
    ]


class SrtPath(C.Structure):
    _fields_ = [("latency_ns", C.c_uint64), ("packet_loss", C.c_float), ("_pad", C.c_uint32)]


class SrtOpts(C.Structure):
    _fields_ = [("algo", C.c_uint32), ("device", C.c_int32), ("flags", C.c_uint32), ("n_gpus", C.c_uint32)]


class SrtTiming(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("dominant_ms", C.c_double), ("dominant_launches", C.c_uint64),
                ("dominant_work", C.c_double), ("loss_ms", C.c_double), ("tight_edges", C.c_uint64),
                ("sharded_tail", C.c_uint32), ("sparse_split", C.c_uint32),
                ("sparse_sweeps", C.c_uint64), ("loss_fold", C.c_uint32), ("reserved0", C.c_uint32),
                ("edge_visits", C.c_uint64), ("create_device_ms", C.c_double)]


class SrtRound(C.Structure):
    _fields_ = [("round_end_ns", C.c_uint64), ("bootstrap_end_ns", C.c_uint64), ("sim_end_ns", C.c_uint64)]


class SrtError(RuntimeError):
    """Error raised by the routing build; `code` is an srt_status."""

    def __init__(self, code: int, msg: str, a_id: int = 0, b_id: int = 0):
        super().__init__(msg)
        self.code, self.a_id, self.b_id = code, a_id, b_id


_lib = None

BCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64)

# name -> (restype, argtypes): the full exported surface of include/srt.h
_vp = C.c_void_p
_u64p, _u32p, _f32p = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_float)
_errp = C.POINTER(SrtErr)
SIGNATURES = {
    "srt_abi_version": (C.c_int, []),
    "srt_device_count": (C.c_int, []),
    "srt_compute_shortest_paths": (C.c_int, [C.POINTER(SrtCsr), _u32p, C.c_uint32, C.POINTER(SrtPath), _u64p,
                                             C.POINTER(SrtOpts), _errp]),
    "srt_get_direct_paths": (C.c_int, [C.POINTER(SrtCsr), _u32p, C.c_uint32, C.POINTER(SrtPath), _u64p,
                                       C.POINTER(SrtOpts), _errp]),
    "srt_plan_create": (C.c_int, [C.POINTER(SrtCsr), _u32p, C.c_uint32, C.POINTER(SrtOpts), C.POINTER(_vp), _errp]),
    "srt_plan_run": (C.c_int, [_vp, _errp]),
    "srt_plan_run_async": (C.c_int, [_vp, _errp]),
    "srt_plan_sync": (C.c_int, [_vp, _errp]),
    "srt_plan_fetch": (C.c_int, [_vp, C.POINTER(SrtPath), _u64p, _errp]),
    "srt_plan_table": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp), _u32p]),
    "srt_plan_describe": (C.c_char_p, [_vp]),
    "srt_plan_stream": (_vp, [_vp]),
    "srt_plan_kernel_tiles": (C.c_int, [_vp, _u64p]),
    "srt_plan_kernel_stats": (C.c_int, [_vp, C.POINTER(C.c_double), _u64p, C.POINTER(C.c_double),
                                        C.POINTER(C.c_double)]),
    "srt_plan_timing": (C.c_int, [_vp, C.POINTER(SrtTiming)]),
    "srt_plan_destroy": (None, [_vp]),
    "srt_comm_unique_id": (C.c_int, [C.c_void_p, _errp]),
    "srt_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(_vp), _errp]),
    "srt_comm_destroy": (None, [_vp]),
    "srt_comm_init_callbacks": (C.c_int, [C.c_int, C.c_int, _vp, _vp, _vp, C.POINTER(_vp), _errp]),
    "srt_comm_init_local": (C.c_int, [C.c_int, C.POINTER(C.c_int32), C.POINTER(_vp), _errp]),
    "srt_comm_abort": (None, [_vp]),
    "srt_plan_bind_comm": (C.c_int, [_vp, _vp, _errp]),
    "srt_plan_shard_rows": (C.c_int, [_vp, C.c_int, C.c_int, _errp]),
    "srt_packet_batch": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_uint64, _vp, C.POINTER(SrtRound), _vp, _vp, _vp,
                                   _vp, _errp]),
    "srt_packet_events_status": (C.c_int, [_vp, _errp]),
    "srt_packet_events": (C.c_int, [_vp, _vp, C.c_uint32, C.c_uint64, _vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp,
                                    _vp, _errp]),
    "srt_routing_info_build": (C.c_int, [C.POINTER(SrtCsr), _u32p, C.c_uint32, C.c_int, C.POINTER(SrtOpts),
                                         C.POINTER(_vp), _errp]),
    "srt_routing_info_from_plan": (C.c_int, [_vp, C.POINTER(_vp), _errp]),
    "srt_routing_info_path": (C.c_int, [_vp, C.c_uint32, C.c_uint32, C.POINTER(SrtPath)]),
    "srt_routing_info_increment_packet_count": (None, [_vp, C.c_uint32, C.c_uint32]),
    "srt_routing_info_add_packet_counts": (None, [_vp, _u64p]),
    "srt_routing_info_packet_count": (C.c_uint64, [_vp, C.c_uint32, C.c_uint32]),
    "srt_routing_info_smallest_latency_ns": (C.c_int, [_vp, _u64p]),
    "srt_routing_info_row": (C.c_int64, [_vp, C.c_uint32]),
    "srt_routing_info_size": (C.c_uint32, [_vp]),
    "srt_routing_info_table": (C.POINTER(SrtPath), [_vp]),
    "srt_routing_info_record_bytes": (C.c_int, [_vp]),
    "srt_routing_info_copy_table": (None, [_vp, C.POINTER(SrtPath)]),
    "srt_init": (C.c_int, [C.c_int, _errp]),
    "srt_init_async": (None, [C.c_int]),
    "srt_init_wait": (None, []),
    "srt_routing_info_destroy": (None, [_vp]),
    "srt_gml_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_vp), _errp]),
    "srt_gml_csr": (C.c_int, [_vp, C.POINTER(SrtCsr)]),
    "srt_gml_free": (None, [_vp]),
    "srt_gml_parse_file": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_vp), _errp]),
    "srt_xz_decompress": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t),
                                    _errp]),
    "srt_free": (None, [_vp]),
    "srt_ip_assignment_create": (C.c_int, [C.POINTER(_vp)]),
    "srt_ip_assignment_destroy": (None, [_vp]),
    "srt_ip_assignment_assign_ip": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _errp]),
    "srt_ip_assignment_assign": (C.c_uint32, [_vp, C.c_uint32]),
    "srt_ip_assignment_get_node": (C.c_int, [_vp, C.c_uint32, _u32p]),
    "srt_ip_assignment_get_nodes": (C.c_uint32, [_vp, _u32p, C.c_uint32]),
    "srt_ip_assignment_size": (C.c_uint32, [_vp]),
    "srt_ip_resolver_create": (C.c_int, [_vp, _u32p, C.c_uint32, C.POINTER(_vp), _errp]),
    "srt_ip_resolver_destroy": (None, [_vp]),
    "srt_ip_resolve_rows": (C.c_int, [_vp, _u32p, C.c_uint64, C.POINTER(C.c_int32)]),
    "srt_packet_batch_ip": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, C.c_uint64, _vp, C.POINTER(SrtRound), _vp,
                                      _vp, _vp, _vp, _errp]),
    "srt_packet_status": (C.c_int, [_vp, _errp]),
    "srt_xoshiro_seed_from_u64": (None, [C.c_uint64, _u64p]),
    "srt_xoshiro_next_u64": (None, [_u64p, C.c_uint64, _u64p]),
    "srt_host_node_seed": (C.c_uint64, [C.c_uint32, C.c_char_p, C.c_size_t]),
}


def lib():
    """Load libsrt.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If
        # libsrt.so were dlopen'd first, the system copy would load and torch
        # would later bring a second runtime that finds no GPU.  Importing torch
        # first makes libsrt bind to the already-loaded runtime (same SONAME).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise SrtError(SRT_ERR_UNSUPPORTED,
                           f"{LIB_PATH} not built: run __graft_entry__.build() (make -C shadow_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.srt_abi_version() != 4:
            raise SrtError(SRT_ERR_UNSUPPORTED, "libsrt ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, err: SrtErr):
    if rc != SRT_OK:
        raise SrtError(rc, err.msg.decode(errors="replace"), err.a_id, err.b_id)


def init(device: int = -1) -> None:
    """srt_init: HIP runtime, kernel code objects and pinned staging, ahead of
    the first build (the cold-start work of generate_routing_info)."""
    err = SrtErr()
    check(lib().srt_init(int(device), C.byref(err)), err)


_exit_wait = []


def init_async(device: int = -1) -> None:
    """srt_init_async: the same on a library thread; the next build waits for it.

    Exit mid-init is safe in the library itself (the calling thread's exit
    joins the init thread before any static destructor runs); the package
    also waits (srt_init_wait: no device work) before the interpreter's
    finalisation, so the join never overlaps it."""
    if not _exit_wait:
        import atexit

        def _wait():
            lib().srt_init_wait()

        atexit.register(_wait)
        _exit_wait.append(_wait)
    lib().srt_init_async(int(device))


def require_device():
    n = lib().srt_device_count()
    if n <= 0:
        raise SrtError(SRT_ERR_HIP, "no HIP device visible: the routing build runs only on MI355X (gfx950)")
    return n
