"""CPU (gloo, world_size 2 and 3) tests of the multi-GPU exchange layer: the
broadcast / in-place all-gather bodies the callback transport runs every round,
and the block-row partition srt_plan_bind_comm uses."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shadow_amd import dist as sdist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        # pivot-row broadcast: every round a different root
        for root in range(world):
            t = torch.full((1000,), rank, dtype=torch.uint8)
            sdist.bcast_tensor(t, root, on_cuda=False)
            assert bool((t == root).all())
        # final in-place all-gather of row shards
        n = 777
        buf = torch.zeros(n * world, dtype=torch.uint8)
        buf[rank * n:(rank + 1) * n] = rank + 1
        sdist.allgather_tensor(buf, n, rank, world, on_cuda=False)
        for r in range(world):
            assert bool((buf[r * n:(r + 1) * n] == r + 1).all())
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


@pytest.mark.parametrize("n,world", [(16384, 8), (16384, 2), (1000, 8), (300, 3), (1, 4)])
def test_block_row_partition(n, world):
    rows, vp = sdist.block_rows(n, world)
    assert vp >= n and vp % (128 * world) == 0
    assert rows[0][0] == 0 and rows[-1][1] == vp
    sizes = {e - b for b, e in rows}
    assert len(sizes) == 1  # equal all-gather chunks
    for (b0, e0), (b1, e1) in zip(rows, rows[1:]):
        assert e0 == b1
