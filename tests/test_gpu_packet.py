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


def _ip_packets(pk, host_row, n_hosts, seed, scattered):
    """The same round by address: every host gets an IPv4 from an IpAssignment
    (auto-assigned, or a configured scattered one -- the resolver's hash form),
    a packet carries its hosts' addresses (network byte order)."""
    from shadow_amd.graph import IpAssignment
    rng = np.random.default_rng(seed)
    ia = IpAssignment()
    host_ip = np.zeros(n_hosts, np.uint32)
    used = set()
    for h in range(n_hosts):
        if scattered:
            while True:
                ip = int(rng.integers(1 << 24, 1 << 31))
                if ip not in used:
                    break
            used.add(ip)
            ia.assign_ip(int(host_row[h]), ip)
        else:
            ip = int(ia.assign(int(host_row[h])))
        host_ip[h] = int.from_bytes(ip.to_bytes(4, "big"), "little")
    # destination host of a packet: any host on its dst_row (hosts are
    # round-robin over the rows, so host dst_row itself is one)
    pki = np.zeros(len(pk), synth.PKT_IP_DTYPE)
    pki["src_host"] = pk["src_host"]
    pki["src_ip"] = host_ip[pk["src_host"]]
    pki["dst_ip"] = host_ip[pk["dst_row"]]
    pki["payload_size"] = pk["payload_size"]
    pki["t_ns"] = pk["t_ns"]
    return ia, pki


def _run(n_nodes, n_hosts, n_pkts, seed, bootstrap_end, sim_end, loss_max=0.25, ip=None):
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
    pk, host_ptr, host_row = synth.packet_round(n_hosts, n_nodes, n_pkts, seed, r0, r1)
    rng = synth.host_rng_states(n_hosts, general_seed=1)
    rng_o = rng.copy()
    cnt_o = np.zeros((n_nodes, n_nodes), np.uint64)
    f_o, d_o, mn_o, ne_o = O.packet_batch(o_lat, o_loss, pk.view(O.PKT_DTYPE), rng_o,
                                          r1, bootstrap_end, sim_end, counters=cnt_o)
    dev = torch.device("cuda:0")
    if ip is not None:
        ia, pki = _ip_packets(pk, host_row, n_hosts, seed, scattered=(ip == "scattered"))
        res = ia.resolver(np.arange(n_nodes, dtype=np.uint32))  # table row i = GML node i
        t_pk = torch.from_numpy(pki.view(np.uint8).copy()).to(dev)
    else:
        t_pk = torch.from_numpy(pk.view(np.uint8).copy()).to(dev)
    t_hp = torch.from_numpy(host_ptr.view(np.int32).copy()).to(dev)
    t_rng = torch.from_numpy(rng.view(np.int64).copy()).to(dev)
    t_f = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
    t_d = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
    t_c = torch.zeros(n_nodes * n_nodes, dtype=torch.int64, device=dev)
    t_s = torch.full((2,), -1, dtype=torch.int64, device=dev)
    if ip is not None:
        plan.packet_batch_ip(res, t_pk, t_hp, t_rng, r1, bootstrap_end, sim_end, t_f, t_d, t_c, t_s)
    else:
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


@pytest.mark.parametrize("ip", ["assigned", "scattered"])
def test_packet_round_by_address(ip):
    """srt_packet_batch_ip: the addresses resolve on the device through the
    frozen IpAssignment (direct table / hash) to the same bits."""
    f = _run(n_nodes=100, n_hosts=1000, n_pkts=100_000, seed=5, bootstrap_end=0, sim_end=2**62, ip=ip)
    assert (f == O.PDS_INET_DROPPED).sum() > 1000


def test_packet_unassigned_address_is_an_error():
    import torch

    from shadow_amd import _lib
    from shadow_amd.graph import IpAssignment
    n = 16
    src, dst, lat, loss = synth.complete_graph(n, 3)
    plan = RoutingPlan(NetworkGraph.from_edges(n, src, dst, lat, loss), np.arange(n, dtype=np.uint32)).run()
    ia = IpAssignment()
    ips = [int(ia.assign(i)) for i in range(n)]
    res = ia.resolver(np.arange(n, dtype=np.uint32))
    pki = np.zeros(4, synth.PKT_IP_DTYPE)
    be = lambda x: int.from_bytes(int(x).to_bytes(4, "big"), "little")  # noqa: E731
    pki["src_ip"] = [be(ips[0])] * 4
    pki["dst_ip"] = [be(ips[1]), be(ips[2]), be((10 << 24) + 1), be(ips[3])]  # 10.0.0.1: not assigned
    pki["payload_size"] = 100
    pki["t_ns"] = 5
    dev = torch.device("cuda:0")
    t_pk = torch.from_numpy(pki.view(np.uint8).copy()).to(dev)
    t_hp = torch.tensor([0, 4], dtype=torch.int32, device=dev)
    t_rng = torch.from_numpy(synth.host_rng_states(1).view(np.int64).copy()).to(dev)
    t_f = torch.zeros(4, dtype=torch.int32, device=dev)
    t_d = torch.zeros(4, dtype=torch.int64, device=dev)
    with pytest.raises(_lib.SrtError, match="no node in the routing table"):
        plan.packet_batch_ip(res, t_pk, t_hp, t_rng, 10, 0, 2**62, t_f, t_d)
    # a completed packet (t >= sim_end) is not looked up (worker.rs:336-339): no error
    plan.packet_batch_ip(res, t_pk, t_hp, t_rng, 10, 0, 5, t_f, t_d)
    plan.close()


def test_packet_block_overflows_lds():
    """A workgroup's hosts with more packets than its LDS holds keep their
    draws in the global scratch: same bits."""
    _run(n_nodes=40, n_hosts=24, n_pkts=60_000, seed=10, bootstrap_end=0, sim_end=2**62)


def test_packet_two_gather_table(monkeypatch):
    """Tables over 1 GiB skip the packed 16-B records (two gathers a packet)."""
    monkeypatch.setenv("SRT_PKT_TAB16", "0")
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import tests.test_gpu_packet as T; "
            "T._run(n_nodes=100, n_hosts=1000, n_pkts=50_000, seed=6, bootstrap_end=0, sim_end=2**62)")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code % root], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
