"""Device-resident routing plan (srt_plan_* in include/srt.h) and the batched
packet stage (srt_packet_batch).

Used by bench.py (inputs resident in HBM before the timed region), the
multi-GPU driver and the per-round packet decision.  Device buffers for the
packet stage are torch tensors on the plan's device: torch is only the HBM
allocator here, every kernel is in libsrt.so.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from .graph import NetworkGraph, PathTable


class RoutingPlan:
    def __init__(self, graph: NetworkGraph, nodes, algo: int = _lib.SRT_ALGO_AUTO, device: int = -1):
        L = _lib.lib()
        _lib.require_device()
        self.graph = graph
        self.nodes = np.ascontiguousarray(nodes, np.uint32)
        self.n = len(self.nodes)
        self._h = C.c_void_p()
        err = _lib.SrtErr()
        opts = _lib.SrtOpts(algo, device, 0, 0)
        csr = graph.csr()
        _lib.check(L.srt_plan_create(C.byref(csr), self.nodes.ctypes.data_as(C.POINTER(C.c_uint32)), self.n,
                                     C.byref(opts), C.byref(self._h), C.byref(err)), err)

    # ---------------------------------------------------------------- build
    def run(self):
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_plan_run(self._h, C.byref(err)), err)
        return self

    def run_async(self):
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_plan_run_async(self._h, C.byref(err)), err)
        return self

    def sync(self):
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_plan_sync(self._h, C.byref(err)), err)

    def fetch(self, table: bool = True) -> Optional[PathTable]:
        n = self.n
        err = _lib.SrtErr()
        mn = C.c_uint64()
        out = (_lib.SrtPath * max(n * n, 1))() if table else None
        _lib.check(_lib.lib().srt_plan_fetch(self._h, out, C.byref(mn), C.byref(err)), err)
        self.min_latency_ns = mn.value
        if not table:
            return None
        raw = np.frombuffer(out, dtype=np.dtype([("lat", "<u8"), ("loss", "<f4"), ("pad", "<u4")]), count=n * n)
        return PathTable(self.nodes, raw["lat"].reshape(n, n).copy(), raw["loss"].reshape(n, n).copy(), mn.value)

    def describe(self) -> str:
        return _lib.lib().srt_plan_describe(self._h).decode()

    def kernel_stats(self):
        """(dominant-kernel ms summed over its launches, launches, relaxations they
        performed, whole-build device ms) of the last run."""
        a, b, w, c = C.c_double(), C.c_uint64(), C.c_double(), C.c_double()
        _lib.lib().srt_plan_kernel_stats(self._h, C.byref(a), C.byref(b), C.byref(w), C.byref(c))
        return a.value, b.value, w.value, c.value

    def timing(self) -> dict:
        """Phase breakdown of the last run (srt_plan_timing)."""
        t = _lib.SrtTiming()
        _lib.check(_lib.lib().srt_plan_timing(self._h, C.byref(t)), _lib.SrtErr())
        return {k: getattr(t, k) for k, _ in _lib.SrtTiming._fields_}

    def kernel_tiles(self) -> int:
        """C tiles the last run's dominant (FW rest) launches loaded and stored."""
        t = C.c_uint64()
        _lib.lib().srt_plan_kernel_tiles(self._h, C.byref(t))
        return t.value

    def stream_ptr(self) -> int:
        """hipStream_t the plan launches on (for HIP events on that stream)."""
        return _lib.lib().srt_plan_stream(self._h)

    def table_ptrs(self):
        lat, loss, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
        _lib.lib().srt_plan_table(self._h, C.byref(lat), C.byref(loss), C.byref(n))
        return lat.value, loss.value, n.value

    def shard_rows(self, nranks: int, rank: int):
        """srt_plan_shard_rows: this plan builds only table rows
        [rank*n/nranks, (rank+1)*n/nranks), no exchange (LEVEL / SSSP plans)."""
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_plan_shard_rows(self._h, int(nranks), int(rank), C.byref(err)), err)
        return self

    def bind_comm(self, comm):
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_plan_bind_comm(self._h, comm, C.byref(err)), err)

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            _lib.lib().srt_plan_destroy(self._h)
            self._h = C.c_void_p()
        comm = getattr(self, "_comm", None)
        if comm is not None:  # the plan referenced it: destroy after the plan
            comm.close()
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- packets
    def packet_events(self, host_ptr, flags, deliver, dst_host, n_dst_hosts: int, event_base, event_id, order,
                      dst_ptr, check: bool = True):
        """srt_packet_events (worker.rs:629-639 + event.rs:85-150) on torch CUDA
        tensors of this plan's device: host_ptr int32 [n_hosts+1], flags int32,
        deliver int64, dst_host int32 [n_pkts], event_base int64 [n_hosts]
        (advanced in place); outputs event_id int64 [n_pkts], order int32
        [n_pkts] (first dst_ptr[-1] meaningful), dst_ptr int32 [n_dst_hosts+1]."""
        import torch

        ps = torch.cuda.ExternalStream(self.stream_ptr(), device=flags.device)
        cur = torch.cuda.current_stream(flags.device)
        ps.wait_stream(cur)
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_packet_events(
            self._h, host_ptr.data_ptr(), host_ptr.numel() - 1, flags.numel(), flags.data_ptr(), deliver.data_ptr(),
            dst_host.data_ptr(), n_dst_hosts, event_base.data_ptr(), event_id.data_ptr(), order.data_ptr(),
            dst_ptr.data_ptr(), C.byref(err)), err)
        cur.wait_stream(ps)  # torch-side consumers see the outputs (device-side ordering)
        if check:  # the asynchronous call's destination check (synchronises the plan's stream)
            self.packet_events_status()

    def packet_events_status(self):
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_packet_events_status(self._h, C.byref(err)), err)

    def packet_batch(self, pkts, host_ptr, rng, round_end_ns: int, bootstrap_end_ns: int, sim_end_ns: int,
                     flags, deliver, counters=None, stats=None, sync: bool = True):
        """All array arguments are torch CUDA tensors on this plan's device:
        pkts (uint8 view of srt_pkt records), host_ptr int32/uint32 [n_hosts+1],
        rng int64 [n_hosts, 4] (xoshiro256++ state, advanced in place),
        flags int32 [n_pkts], deliver int64 [n_pkts], counters int64 [n*n] or
        None, stats int64 [2] (min-combined; initialise to -1 == UINT64_MAX)."""
        import torch

        n_hosts = host_ptr.numel() - 1
        n_pkts = flags.numel()
        # the plan's stream waits for the producer of the inputs (torch's
        # current stream) on the device: no host round trip per batch
        torch.cuda.ExternalStream(self.stream_ptr(), device=flags.device).wait_stream(
            torch.cuda.current_stream(flags.device))
        r = _lib.SrtRound(round_end_ns, bootstrap_end_ns, sim_end_ns)
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_packet_batch(
            self._h, pkts.data_ptr(), host_ptr.data_ptr(), n_hosts, n_pkts, rng.data_ptr(), C.byref(r),
            flags.data_ptr(), deliver.data_ptr(), counters.data_ptr() if counters is not None else None,
            stats.data_ptr() if stats is not None else None, C.byref(err)), err)
        if sync:
            self.sync()

    def packet_batch_ip(self, resolver, pkts, host_ptr, rng, round_end_ns: int, bootstrap_end_ns: int,
                        sim_end_ns: int, flags, deliver, counters=None, stats=None, sync: bool = True):
        """srt_packet_batch_ip: as packet_batch, with pkts a uint8 view of
        srt_pkt_ip records (source / destination IPv4 in network byte order,
        resolved on the device through `resolver`, an IpResolver over this
        plan's table rows).  sync=True also checks srt_packet_status (an
        address without a row raises, as the reference's unwrap panics)."""
        import torch

        n_hosts = host_ptr.numel() - 1
        n_pkts = flags.numel()
        torch.cuda.ExternalStream(self.stream_ptr(), device=flags.device).wait_stream(
            torch.cuda.current_stream(flags.device))
        r = _lib.SrtRound(round_end_ns, bootstrap_end_ns, sim_end_ns)
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_packet_batch_ip(
            self._h, resolver.handle, pkts.data_ptr(), host_ptr.data_ptr(), n_hosts, n_pkts, rng.data_ptr(),
            C.byref(r), flags.data_ptr(), deliver.data_ptr(),
            counters.data_ptr() if counters is not None else None,
            stats.data_ptr() if stats is not None else None, C.byref(err)), err)
        if sync:
            self.packet_status()

    def packet_status(self):
        """srt_packet_status: synchronises; raises if a batch met an address without a row."""
        err = _lib.SrtErr()
        _lib.check(_lib.lib().srt_packet_status(self._h, C.byref(err)), err)
