"""GPU tests of the in-process multi-GPU build (srt_comm_init_local,
srt_opts.n_gpus): N host threads, one plan each, collectives stream-ordered on
the device (events + one peer-read kernel a collective).  On the one-GPU box
every rank shares device 0 -- the same schedules, the same exchange code; on a
multi-GPU node the ranks sit on distinct devices and read each other over
xGMI.  Bar: every table bit-exact against the oracle."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, RoutingInfo, _lib, synth
from shadow_amd import dist as sdist

pytestmark = pytest.mark.gpu


def _graph(n, seed, undirected, wide=False):
    src, dst, lat, loss = synth.random_graph(n, seed, p_edge=0.08, directed=not undirected, lat_range_ns=(1, 9),
                                             loss_max=0.05)
    if wide:
        lat = (np.asarray(lat, dtype=np.uint64) << np.uint64(34)) + np.uint64(1)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss, directed=not undirected)
    nodes = np.random.default_rng(seed).permutation(n).astype(np.uint32)
    return g, nodes, O.Graph(not undirected, np.arange(n), src, dst, lat, loss)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("world,n,seed,algo,undirected,wide", [
    (2, 300, 1, "fw", False, False), (3, 520, 2, "fw", False, False), (8, 1100, 5, "fw", False, False),
    (2, 300, 12, "fw", True, False), (3, 520, 13, "fw", True, False), (8, 1100, 14, "fw", True, False),
    (8, 1500, 19, "fw", True, False),
    (3, 400, 7, "fw", False, True),
    (2, 301, 3, "sssp", False, False), (3, 200, 15, "sssp", True, False), (8, 700, 6, "sssp", False, False),
    (8, 1300, 16, "sssp", True, False)])
def test_local_build_matches_oracle(world, n, seed, algo, undirected, wide):
    """Every rank on device 0, threads of this process: rank 0's table equals
    the oracle bit for bit; the dense builds ran the sharded tail (or, wide
    keys, the replicated fallback) and, on undirected graphs, the symmetric
    triangle schedule."""
    g, nodes, og = _graph(n, seed, undirected, wide)
    a = {"fw": _lib.SRT_ALGO_FW, "sssp": _lib.SRT_ALGO_SSSP}[algo]
    t, descs, timings = sdist.local_build(g, nodes, [0] * world, algo=a)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(_bits(t.packet_loss), _bits(eloss))
    assert t.min_latency_ns == int(elat.min())
    for r, d in enumerate(descs):
        assert f"ranks={world}" in d, d
        if algo == "fw":
            assert ("sym=triangle" in d) == undirected, d
            assert timings[r]["sharded_tail"] == (0 if wide else 1)


@pytest.mark.parametrize("world,algo", [(2, _lib.SRT_ALGO_FW), (3, _lib.SRT_ALGO_SSSP), (8, _lib.SRT_ALGO_AUTO)])
def test_compute_shortest_paths_n_gpus(world, algo):
    """The drop-in entry point with srt_opts.n_gpus (the ranks on one device
    here: SRT_OPT_SAME_DEVICE) returns the single-GPU bits."""
    g, nodes, og = _graph(640, 30 + world, True)
    t = g.compute_shortest_paths(nodes, algo=algo, device=0, n_gpus=world, same_device=True)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(_bits(t.packet_loss), _bits(eloss))


def test_routing_info_n_gpus():
    """generate_routing_info over 4 in-process ranks: every path() equals the
    one-GPU RoutingInfo's."""
    src, dst, lat, loss = synth.complete_graph(300, 9)
    g = NetworkGraph.from_edges(300, src, dst, lat, loss)
    nodes = np.arange(0, 300, 2, dtype=np.uint32)
    one = RoutingInfo.build(g, nodes, device=0)
    four = RoutingInfo.build(g, nodes, device=0, n_gpus=4, same_device=True)
    rng = np.random.default_rng(1)
    for _ in range(200):
        a, b = (int(x) for x in rng.choice(nodes, 2))
        assert one.path(a, b) == four.path(a, b)
    assert one.get_smallest_latency_ns() == four.get_smallest_latency_ns()


def test_n_gpus_errors():
    """Graph errors surface with the reference's text from the multi-GPU
    build (every rank finds them; the first rank's is reported), and asking
    for more devices than the node has is refused."""
    g = NetworkGraph.from_edges(3, [0, 1, 0], [0, 1, 1], [5, 5, 5], directed=False, node_ids=[4, 8, 9])
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1, 2], device=0, n_gpus=3, same_device=True)
    assert e.value.code == _lib.SRT_ERR_NO_EDGE and str(e.value) == "No edge connecting node 9 to 9"
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1], device=0, n_gpus=17, same_device=True)
    assert e.value.code == _lib.SRT_ERR_INVALID
    n_dev = _lib.lib().srt_device_count()
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths([0, 1], device=0, n_gpus=n_dev + 1)
    assert e.value.code == _lib.SRT_ERR_INVALID


def test_level_peer_copies_checked(monkeypatch):
    """The in-process level build copies the class CSRs to every other device
    and checks each copy against rank 0's checksum before a row is solved
    (SRT_MULTI_FORCE_COPY=1 makes ranks sharing the one GPU take that copy
    path): a clean copy gives the oracle's table, a corrupted one
    (SRT_TEST_CORRUPT_PEER=2) is refused with SRT_ERR_COMM."""
    n = 700
    src, dst, lat, loss = synth.complete_graph(n, 17, lat_ms=(1, 30))
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.random.default_rng(17).permutation(n).astype(np.uint32)
    og = O.Graph(False, np.arange(n), src, dst, lat, loss)
    monkeypatch.setenv("SRT_MULTI_FORCE_COPY", "1")
    t = g.compute_shortest_paths(nodes, n_gpus=3, same_device=True)
    elat, eloss = O.compute_shortest_paths(og, nodes)
    assert np.array_equal(t.latency_ns, elat)
    assert np.array_equal(t.packet_loss.view(np.uint32), eloss.view(np.uint32))
    monkeypatch.setenv("SRT_TEST_CORRUPT_PEER", "2")
    with pytest.raises(_lib.SrtError) as e:
        g.compute_shortest_paths(nodes, n_gpus=3, same_device=True)
    assert e.value.code == _lib.SRT_ERR_COMM and "checksum" in str(e.value)


@pytest.mark.parametrize("algo", [_lib.SRT_ALGO_LEVEL])
def test_local_collective_corruption_detected(monkeypatch, algo):
    """Every in-process collective is checked: senders checksum their slots,
    receivers what arrived; a flipped value bit on rank 1
    (SRT_TEST_CORRUPT_PEER=1) surfaces as SRT_ERR_COMM instead of a wrong
    table.  (The level build's collectives carry values only -- staged rows
    and stats -- so the damaged copy cannot steer the build; the FW schedule's
    also carry sizes that pick the next collective, which a damaged copy
    could desynchronise before the check reports it.)"""
    n = 500
    src, dst, lat, loss = synth.random_graph(n, 23, p_edge=0.08, directed=False, lat_range_ns=(1, 9))
    lat = np.asarray(lat, np.uint64) * np.uint64(synth.MS)
    g = NetworkGraph.from_edges(n, src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    monkeypatch.setenv("SRT_TEST_CORRUPT_PEER", "1")
    with pytest.raises(_lib.SrtError) as e:
        sdist.local_build(g, nodes, [0, 0, 0], algo=algo)
    assert e.value.code == _lib.SRT_ERR_COMM, str(e.value)
