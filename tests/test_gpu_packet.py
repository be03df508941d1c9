"""GPU parity of the batched send_packet decision (srt_packet_batch) against
the sequential oracle restatement of worker.rs:326-410, end to end: the GPU
builds its routing table (dense closure + exact-loss pass) and decides the
round; the oracle builds ITS OWN table (petgraph-faithful Dijkstra) and
decides the same round on it.  Bar: tables, flags, deliver times, RNG states
after the round, per-path counters, min latency and next event time all
bit-exact."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import NetworkGraph, synth
from shadow_amd.plan import RoutingPlan

pytestmark = pytest.mark.gpu


def _run(n_nodes, n_hosts, n_pkts, seed, bootstrap_end, sim_end, loss_max=0.25):
    import torch

    src, dst, lat, loss = synth.complete_graph(n_nodes, seed, loss_max=loss_max)
    g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss)
    plan = RoutingPlan(g, np.arange(n_nodes, dtype=np.uint32)).run()
    table = plan.fetch()
    # the oracle's own table (not the GPU's): drop decisions read its loss bits
    o_lat, o_loss = O.compute_shortest_paths(O.Graph(False, np.arange(n_nodes), src, dst, lat, loss),
                                             np.arange(n_nodes, dtype=np.uint32))
    assert np.array_equal(table.latency_ns, o_lat)
    assert np.array_equal(table.packet_loss.view(np.uint32), o_loss.view(np.uint32))
    r0, r1 = 1_000_000_000, 1_000_000_000 + 5 * synth.MS
    pk, host_ptr, _ = synth.packet_round(n_hosts, n_nodes, n_pkts, seed, r0, r1)
    rng = synth.host_rng_states(n_hosts, general_seed=1)
    rng_o = rng.copy()
    cnt_o = np.zeros((n_nodes, n_nodes), np.uint64)
    f_o, d_o, mn_o, ne_o = O.packet_batch(o_lat, o_loss, pk.view(O.PKT_DTYPE), rng_o,
                                          r1, bootstrap_end, sim_end, counters=cnt_o)
    dev = torch.device("cuda:0")
    t_pk = torch.from_numpy(pk.view(np.uint8).copy()).to(dev)
    t_hp = torch.from_numpy(host_ptr.view(np.int32).copy()).to(dev)
    t_rng = torch.from_numpy(rng.view(np.int64).copy()).to(dev)
    t_f = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
    t_d = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
    t_c = torch.zeros(n_nodes * n_nodes, dtype=torch.int64, device=dev)
    t_s = torch.full((2,), -1, dtype=torch.int64, device=dev)
    plan.packet_batch(t_pk, t_hp, t_rng, r1, bootstrap_end, sim_end, t_f, t_d, t_c, t_s)
    f = t_f.cpu().numpy().view(np.uint32)
    d = t_d.cpu().numpy().view(np.uint64)
    assert np.array_equal(f, f_o)
    assert np.array_equal(d, d_o)
    assert np.array_equal(t_rng.cpu().numpy().view(np.uint64), rng_o)
    assert np.array_equal(t_c.cpu().numpy().view(np.uint64).reshape(n_nodes, n_nodes), cnt_o)
    s = t_s.cpu().numpy().view(np.uint64)
    assert int(s[0]) == mn_o and int(s[1]) == ne_o
    return f


@pytest.mark.parametrize("seed", [5, 6])
def test_packet_round_parity(seed):
    f = _run(n_nodes=100, n_hosts=1000, n_pkts=100_000, seed=seed, bootstrap_end=0, sim_end=2**62)
    assert (f == O.PDS_INET_DROPPED).sum() > 1000  # loss U[0,0.25]: drops are frequent


def test_packet_bootstrapping_never_drops():
    f = _run(n_nodes=64, n_hosts=300, n_pkts=20_000, seed=7, bootstrap_end=2**62, sim_end=2**63)
    assert not (f == O.PDS_INET_DROPPED).any()


def test_packet_sim_end_mid_round():
    # packets at or after sim_end are completed: no flag and no RNG draw
    r0 = 1_000_000_000
    f = _run(n_nodes=50, n_hosts=200, n_pkts=30_000, seed=8, bootstrap_end=0, sim_end=r0 + 2 * synth.MS)
    assert (f == O.PDS_NONE).sum() > 0


def test_empty_round():
    _run(n_nodes=8, n_hosts=4, n_pkts=1, seed=9, bootstrap_end=0, sim_end=2**62)
