"""Multi-GPU routing build: one process per GPU, source block-rows sharded over
ranks (include/srt.h: srt_comm_*, srt_plan_bind_comm).

The reference parallelises compute_shortest_paths only over a rayon thread
pool (src/main/network/graph/mod.rs:190-208); it has no collective.  Here the
closure's two exchange steps -- the per-round pivot block-row broadcast and the
final all-gather of path keys -- run either

  * natively over RCCL/xGMI from inside libsrt (transport="rccl", default;
    the 128-byte ncclUniqueId is shipped with torch.distributed), or
  * through host callbacks into torch.distributed (transport="torch"; with the
    gloo backend this runs the exact same sharded schedule on CPU collectives,
    which is how the N>1 path is tested without a multi-GPU box).
"""
from __future__ import annotations

import ctypes as C

from . import _lib


class _CudaBuf:
    """Zero-copy torch view of a device pointer (__cuda_array_interface__)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2}


class Comm:
    def __init__(self, handle, keepalive=()):
        self.handle = handle
        self._keep = keepalive

    def close(self):
        if self.handle:
            _lib.lib().srt_comm_destroy(self.handle)
            self.handle = C.c_void_p()


def rccl_comm(rank: int, world: int, device: int) -> Comm:
    import torch
    import torch.distributed as dist

    L = _lib.lib()
    err = _lib.SrtErr()
    uid = (C.c_uint8 * 128)()
    if rank == 0:
        _lib.check(L.srt_comm_unique_id(uid, C.byref(err)), err)
    on_cuda = dist.get_backend() == "nccl"
    t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=f"cuda:{device}" if on_cuda else "cpu")
    dist.broadcast(t, src=0)
    data = bytes(t.cpu().tolist())
    uid = (C.c_uint8 * 128).from_buffer_copy(data)
    h = C.c_void_p()
    _lib.check(L.srt_comm_init(uid, world, rank, device, C.byref(h), C.byref(err)), err)
    return Comm(h)


def bcast_tensor(t, root: int, on_cuda: bool):
    """Broadcast a uint8 tensor in place from `root` (the bcast callback body)."""
    import torch.distributed as dist

    if on_cuda:
        dist.broadcast(t, src=root)
    else:
        h = t.cpu() if t.is_cuda else t
        dist.broadcast(h, src=root)
        if h is not t:
            t.copy_(h)


def allgather_tensor(t, nbytes_per_rank: int, rank: int, world: int, on_cuda: bool):
    """In-place all-gather: rank r's bytes live at t[r*n:(r+1)*n] (the allgather
    callback body)."""
    import torch
    import torch.distributed as dist

    if on_cuda:
        mine = t[rank * nbytes_per_rank:(rank + 1) * nbytes_per_rank].clone()
        dist.all_gather_into_tensor(t, mine)
    else:
        h = t.cpu() if t.is_cuda else t
        parts = [torch.empty(nbytes_per_rank, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, h[rank * nbytes_per_rank:(rank + 1) * nbytes_per_rank].clone())
        t.copy_(torch.cat(parts))


def block_rows(n_nodes: int, world: int, block: int = 128):
    """Row partition used by srt_plan_bind_comm: the node range is padded to a
    multiple of block*world and every rank owns the same number of block-rows.
    Returns [(row_begin, row_end)] per rank and the padded size."""
    unit = block * world
    vp = max(((n_nodes + unit - 1) // unit) * unit, unit)
    per = vp // block // world
    return [(r * per * block, (r + 1) * per * block) for r in range(world)], vp


def torch_comm(rank: int, world: int, device: int) -> Comm:
    """Callback transport over the default torch.distributed process group."""
    import torch
    import torch.distributed as dist

    on_cuda = dist.get_backend() == "nccl"
    dev = torch.device("cuda", device)

    def _view(ptr, nbytes):
        return torch.as_tensor(_CudaBuf(ptr, nbytes), device=dev)

    def bcast(user, ptr, nbytes, root):
        try:
            bcast_tensor(_view(ptr, nbytes), root, on_cuda)
            torch.cuda.synchronize(dev)
            return 0
        except Exception as e:  # never let an exception cross the C ABI
            print(f"[rank {rank}] bcast callback failed: {e!r}", flush=True)
            return 1

    def allgather(user, ptr, nbytes_per_rank):
        try:
            allgather_tensor(_view(ptr, nbytes_per_rank * world), nbytes_per_rank, rank, world, on_cuda)
            torch.cuda.synchronize(dev)
            return 0
        except Exception as e:
            print(f"[rank {rank}] allgather callback failed: {e!r}", flush=True)
            return 1

    cb1 = _lib.BCAST_FN(bcast)
    cb2 = _lib.ALLGATHER_FN(allgather)
    h = C.c_void_p()
    err = _lib.SrtErr()
    _lib.check(_lib.lib().srt_comm_init_callbacks(world, rank, C.cast(cb1, C.c_void_p), C.cast(cb2, C.c_void_p),
                                                  None, C.byref(h), C.byref(err)), err)
    return Comm(h, keepalive=(cb1, cb2))


def bind(plan, rank: int, world: int, device: int, transport: str = "rccl") -> Comm:
    """Create the communicator and bind `plan` (a RoutingPlan) to it.  The
    returned Comm must be kept alive as long as the plan runs."""
    comm = rccl_comm(rank, world, device) if transport == "rccl" else torch_comm(rank, world, device)
    plan.bind_comm(comm.handle)
    plan._comm = comm
    return comm


def local_comms(devices) -> list:
    """srt_comm_init_local: one communicator per rank of THIS process (rank r
    on devices[r]; a device may repeat).  Each rank's plan must be driven by
    its own thread (see local_build)."""
    L = _lib.lib()
    n = len(devices)
    devs = (C.c_int32 * n)(*devices)
    hs = (_lib._vp * n)()
    err = _lib.SrtErr()
    _lib.check(L.srt_comm_init_local(n, devs, hs, C.byref(err)), err)
    return [Comm(C.c_void_p(hs[r])) for r in range(n)]


class LocalPlans:
    """Every rank's plan of an in-process sharded build, kept on the device
    (local_build(..., keep=True)): the caller inspects the device tables, then
    close() destroys the plans before their communicators."""

    def __init__(self, plans, comms):
        self.plans = plans
        self._comms = comms

    def close(self):
        for p in self.plans:
            if p is not None:
                p.close()
        for c in self._comms:
            c.close()
        self.plans, self._comms = [], []


def local_build(graph, nodes, devices, algo: int = _lib.SRT_ALGO_AUTO, keep: bool = False):
    """The in-process sharded build (what srt_opts.n_gpus does inside the
    library), from Python so tests can inspect every rank's plan: one plan and
    one thread per rank, collectives over srt_comm_init_local.  Returns rank
    0's table and every rank's plan description and timing -- or, keep=True,
    a LocalPlans holding every rank's plan with its table still on the device
    (nothing fetched)."""
    import threading

    from .plan import RoutingPlan

    comms = local_comms(devices)
    plans = [None] * len(devices)
    errors = [None] * len(devices)

    def rank(r):
        try:
            p = RoutingPlan(graph, nodes, algo=algo, device=devices[r])
            plans[r] = p
            p.bind_comm(comms[r].handle)
            p.run()
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errors[r] = e
            _lib.lib().srt_comm_abort(comms[r].handle)

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(len(devices))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    kept = LocalPlans(plans, comms)
    try:
        for e in errors:
            if e is not None and not (isinstance(e, _lib.SrtError) and e.code == _lib.SRT_ERR_COMM):
                raise e
        for e in errors:
            if e is not None:
                raise e
        if keep:
            kept, out = None, kept
            return out
        table = plans[0].fetch()
        return table, [p.describe() for p in plans], [p.timing() for p in plans]
    finally:
        if kept is not None:
            kept.close()
