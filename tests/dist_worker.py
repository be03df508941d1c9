"""One rank of the sharded routing build (spawned by tests/test_gpu_dist.py).

usage: dist_worker.py RANK WORLD PORT N SEED TRANSPORT [ALGO [wide|undirected]]
("wide": latencies << 34 plus 1, past the u32 key range -- the dense build takes the
replicated loss pass, key all-gather included; "undirected": a symmetric graph,
so the dense build runs the symmetric sharded schedule -- triangle tiles dealt
by (i + j) mod N, one row all-gather a round)
All ranks share cuda:0 (the box has one GPU); collectives go through
torch.distributed/gloo via the callback transport, which exercises exactly the
same per-round schedule as the RCCL transport.  Exit code 0 = table matches
the oracle (rank 0 checks; every rank checks its own table equals rank 0's
via a checksum).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, n, seed = (int(x) for x in sys.argv[1:6])
    transport = sys.argv[6]
    algo_name = sys.argv[7] if len(sys.argv) > 7 else "auto"
    wide = len(sys.argv) > 8 and sys.argv[8] == "wide"
    undirected = len(sys.argv) > 8 and sys.argv[8] == "undirected"
    import numpy as np
    import torch
    import torch.distributed as dist

    from shadow_amd import NetworkGraph, _lib, synth
    from shadow_amd import dist as sdist
    from shadow_amd.plan import RoutingPlan

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    src, dst, lat, loss = synth.random_graph(n, seed, p_edge=0.08, directed=not undirected, lat_range_ns=(1, 9),
                                             loss_max=0.05)
    if wide:
        lat = (np.asarray(lat, dtype=np.uint64) << np.uint64(34)) + np.uint64(1)  # gcd 1: no unit rescale
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=not undirected)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    algo = {"auto": _lib.SRT_ALGO_AUTO, "fw": _lib.SRT_ALGO_FW, "sssp": _lib.SRT_ALGO_SSSP,
            "level": _lib.SRT_ALGO_LEVEL}[algo_name]
    plan = RoutingPlan(g, nodes, algo=algo, device=0)
    sdist.bind(plan, rank, world, 0, transport=transport)
    plan.run()
    t = plan.fetch()
    tm = plan.timing()
    tail = tm["sharded_tail"]
    # grouped sharded rounds: one rest launch per group (SRT_TEST_EXPECT_RESTS)
    want_rests = os.environ.get("SRT_TEST_EXPECT_RESTS")
    ck = torch.tensor([int(np.bitwise_xor.reduce(t.latency_ns.reshape(-1) * np.uint64(2654435761))),
                       int(np.bitwise_xor.reduce(t.packet_loss.view(np.uint32).reshape(-1)))], dtype=torch.int64)
    all_ck = [torch.zeros_like(ck) for _ in range(world)]
    dist.all_gather(all_ck, ck)
    ok = all(bool((c == all_ck[0]).all()) for c in all_ck)
    if rank == 0:
        from oracle import oracle as O
        elat, eloss = O.compute_shortest_paths(O.Graph(not undirected, np.arange(n), src, dst, lat, loss), nodes)
        ok = ok and np.array_equal(t.latency_ns, elat)
        # both kernel families fold loss exactly like the reference
        ok = ok and np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))
        # dense builds: the loss pass ran on the rank's own closure rows
        ok = ok and (algo_name != "fw" or tail == (0 if wide else 1))
        # level solve: rows staged as 6-byte records and all-gathered chunk by chunk
        ok = ok and (algo_name != "level" or (plan.describe().startswith("level:") and tail == 1))
        ok = ok and (want_rests is None or tm["dominant_launches"] == int(want_rests))
        # a symmetric dense graph runs the triangle schedule, a directed one never
        ok = ok and (algo_name != "fw" or ("sym=triangle" in plan.describe()) == undirected)
        print(f"rank0: {plan.describe()} sharded_tail={tail} rests={tm['dominant_launches']} ok={ok}", flush=True)
    plan.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
