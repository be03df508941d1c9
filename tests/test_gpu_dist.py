"""GPU test of the row-sharded multi-GPU build: 2 and 3 ranks on the one GPU of
the box, collectives through torch.distributed/gloo (callback transport), the
same per-round schedule the RCCL transport runs on a multi-GPU node."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,n,seed,algo,wide,group", [
    (2, 300, 1, "fw", False, None), (3, 520, 2, "fw", False, None),
    (2, 301, 3, "sssp", False, None), (3, 200, 4, "sssp", False, None),
    # the driver's 8-rank layout: 16 block-rows, the pivot owner changes every 2 rounds
    (8, 1100, 5, "fw", False, None), (8, 700, 6, "sssp", False, None),
    # grouped sharded rounds: 4 block-rows per rank in groups of 4, and groups of 2 (the default)
    (2, 1000, 8, "fw", False, "4:2"), (3, 1300, 9, "fw", False, "4:3"), (8, 1100, 10, "fw", False, "2:8"),
    (2, 1000, 11, "fw", False, "2:4"),
    # u64 keys: replicated loss pass after the key all-gather
    (3, 400, 7, "fw", True, None),
    # symmetric graphs: triangle tiles dealt by (i + j) mod N, a row all-gather per 2 rounds
    # (the default; 300 nodes = 3 block-rows: one round a group), and per round ("s1:...")
    (2, 300, 12, "fw", "undirected", None), (3, 520, 13, "fw", "undirected", None),
    (8, 1100, 14, "fw", "undirected", None), (3, 200, 15, "sssp", "undirected", None),
    (2, 1000, 20, "fw", "undirected", "s1:8"), (8, 1100, 21, "fw", "undirected", "s1:16"),
    # ... in groups of g rounds, one row all-gather per group ("s<g>:<rest launches>"; a sharded
    # plan pads to whole block-rows a rank: 8 ranks 16 block-rows, the last group of 3 ragged)
    (2, 1000, 16, "fw", "undirected", "s2:4"), (3, 1300, 17, "fw", "undirected", "s4:3"),
    (8, 1100, 18, "fw", "undirected", "s2:8"), (8, 1500, 19, "fw", "undirected", "s3:6"),
    # the level solve: rows by node-index ranges, 6-byte staged rows all-gathered
    (2, 600, 22, "level", "undirected", None), (3, 500, 23, "level", False, None),
    (8, 1100, 24, "level", "undirected", None)])
def test_sharded_build_matches_oracle(world, n, seed, algo, wide, group):
    """Dense builds assert the sharded tail ran (or, "wide", the replicated
    fallback) and, for undirected graphs, the symmetric schedule; every rank's
    table equals the oracle's bit for bit."""
    port = _port()
    env = dict(os.environ)
    if group and group.startswith("s"):  # symmetric schedule, "s<g>:<rest launches>"
        env["SRT_FW_SYM_GROUP"], env["SRT_TEST_EXPECT_RESTS"] = group[1:].split(":")
    elif group:  # "g:rest launches"
        env["SRT_FW_SHARD_GROUP"], env["SRT_TEST_EXPECT_RESTS"] = group.split(":")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               str(n), str(seed), "torch", algo] +
                              (["undirected"] if wide == "undirected" else ["wide"] if wide else []), env=env,
                              stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=110)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]


def test_symmetric_sharded_full_tile_chain():
    """The symmetric schedule's chain with full-tile cross / p2row launches
    (SRT_FW_SYM_SMALL=0; the default at >= 4096 own tiles a rank, i.e. 2 ranks
    at 16k) -- small graphs otherwise take the packed quarter-tile chain; one
    round per all-gather (SRT_FW_SYM_GROUP=1: the grouped schedule always runs
    the quarter-tile chain)."""
    port = _port()
    env = dict(os.environ, SRT_FW_SYM_SMALL="0", SRT_FW_SYM_GROUP="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), "2", str(port), "400",
                               "16", "torch", "fw", "undirected"], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=110)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]


@pytest.mark.parametrize("algo_name", ["fw", "sssp"])
def test_rccl_transport_single_rank(algo_name):
    """Native RCCL communicator (1 rank on the box): runs the sharded schedule
    (owner phase 2 row launch, ncclBroadcast of each pivot block-row, column
    launch, ncclAllGather) and must reproduce the unsharded table exactly."""
    import ctypes as C

    import numpy as np

    from shadow_amd import NetworkGraph, _lib, synth
    from shadow_amd.plan import RoutingPlan

    n = 333
    src, dst, lat, loss = synth.random_graph(n, 4, p_edge=0.05, directed=False, lat_range_ns=(1, 9))
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    algo = _lib.SRT_ALGO_FW if algo_name == "fw" else _lib.SRT_ALGO_SSSP
    ref = RoutingPlan(g, nodes, algo=algo, device=0).run().fetch()
    L = _lib.lib()
    err = _lib.SrtErr()
    uid = (C.c_uint8 * 128)()
    _lib.check(L.srt_comm_unique_id(uid, C.byref(err)), err)
    h = C.c_void_p()
    _lib.check(L.srt_comm_init(uid, 1, 0, 0, C.byref(h), C.byref(err)), err)
    plan = RoutingPlan(g, nodes, algo=algo, device=0)
    plan.bind_comm(h)
    t = plan.run().fetch()
    assert "ranks=1" in plan.describe()
    assert plan.timing()["sharded_tail"] == (1 if algo_name == "fw" else 0)
    plan.close()
    L.srt_comm_destroy(h)
    assert np.array_equal(t.latency_ns, ref.latency_ns)
    assert np.array_equal(t.packet_loss.view(np.uint32), ref.packet_loss.view(np.uint32))
