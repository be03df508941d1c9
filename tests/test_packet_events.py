"""Batched packet-event push (srt_packet_events; worker.rs:629-639,
event.rs:20-31/85-150, host.rs:691-695).

CPU: the oracle's restatement -- per-destination binary heaps of Event keys,
popped empty -- agrees with an independent statement of the same order
(a lexicographic sort by (destination, time, source host, event id)).
GPU: srt_packet_events on the flags/deliver times of a real srt_packet_batch
round equals the oracle bit for bit (event ids, order, offsets)."""
import numpy as np
import pytest

from oracle import oracle as O


def _random_batch(seed, n_hosts=40, n_pkts=3000, n_dst=25, tie_range=7):
    rng = np.random.default_rng(seed)
    counts = rng.multinomial(n_pkts, np.ones(n_hosts) / n_hosts)
    host_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    flags = rng.choice([O.PDS_INET_SENT, O.PDS_INET_DROPPED, O.PDS_NONE], size=n_pkts, p=[0.7, 0.2, 0.1])
    # few distinct deliver times: many equal-time events per destination
    deliver = (1_000_000 + rng.integers(0, tie_range, size=n_pkts)).astype(np.uint64)
    dst = rng.integers(0, n_dst, size=n_pkts).astype(np.uint32)
    base = rng.integers(0, 1000, size=n_hosts).astype(np.uint64)
    return host_ptr, flags.astype(np.uint32), deliver, dst, n_dst, base


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_heap_order_is_lexicographic(seed):
    host_ptr, flags, deliver, dst, n_dst, base = _random_batch(seed)
    b0 = base.copy()
    eid, order, dst_ptr = O.packet_events(host_ptr, flags, deliver, dst, n_dst, base)
    sent = np.nonzero(flags == O.PDS_INET_SENT)[0]
    host_of = np.repeat(np.arange(len(host_ptr) - 1), np.diff(host_ptr.astype(np.int64)))
    # event ids: per host, consecutive from its base in send order
    for h in range(len(host_ptr) - 1):
        ps = [p for p in range(host_ptr[h], host_ptr[h + 1]) if flags[p] == O.PDS_INET_SENT]
        assert [int(eid[p]) for p in ps] == list(range(int(b0[h]), int(b0[h]) + len(ps)))
        assert int(base[h]) == int(b0[h]) + len(ps)
    assert (eid[flags != O.PDS_INET_SENT] == np.iinfo(np.uint64).max).all()
    lex = sent[np.lexsort((eid[sent], host_of[sent], deliver[sent], dst[sent]))]
    assert np.array_equal(order, lex.astype(np.uint32))
    assert np.array_equal(dst_ptr, np.searchsorted(dst[lex], np.arange(n_dst + 1)).astype(np.uint32))


gpu = pytest.mark.gpu


def _gpu_events(plan, host_ptr, flags, deliver, dst, n_dst, base):
    import torch

    dev = torch.device("cuda:0")
    n = len(flags)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)  # noqa: E731
    t_base = t(base, np.int64)
    t_eid = torch.zeros(n, dtype=torch.int64, device=dev)
    t_ord = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    t_ptr = torch.zeros(n_dst + 1, dtype=torch.int32, device=dev)
    plan.packet_events(t(host_ptr, np.int32), t(flags, np.int32), t(deliver, np.int64), t(dst, np.int32), n_dst,
                       t_base, t_eid, t_ord, t_ptr)
    ptr = t_ptr.cpu().numpy().view(np.uint32)
    return (t_eid.cpu().numpy().view(np.uint64), t_ord.cpu().numpy().view(np.uint32)[:ptr[-1]], ptr,
            t_base.cpu().numpy().view(np.uint64))


def _plan():
    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan

    src, dst, lat, loss = synth.complete_graph(16, 1)
    return RoutingPlan(NetworkGraph.from_edges(16, src, dst, lat, loss), np.arange(16, dtype=np.uint32)).run()


@gpu
@pytest.mark.parametrize("seed,n_dst", [(1, 200), (2, 200), (3, 20_000)])
def test_gpu_events_random_batch(seed, n_dst):
    """200 destinations: the chunked LDS count / scatter; 20,000 (more than
    its LDS histogram holds): the global-atomic count / scatter."""
    host_ptr, flags, deliver, dst, n_dst, base = _random_batch(seed, n_hosts=300, n_pkts=50_000, n_dst=n_dst)
    plan = _plan()
    ob = base.copy()
    eid_o, ord_o, ptr_o = O.packet_events(host_ptr, flags, deliver, dst, n_dst, ob)
    eid, order, ptr, nb = _gpu_events(plan, host_ptr, flags, deliver, dst, n_dst, base)
    assert np.array_equal(eid, eid_o)
    assert np.array_equal(order, ord_o)
    assert np.array_equal(ptr, ptr_o)
    assert np.array_equal(nb, ob)


@gpu
def test_gpu_events_after_packet_round():
    """flags/deliver from a real srt_packet_batch round (C5-shaped, smaller)."""
    import torch

    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan

    n_nodes, n_hosts, n_pkts = 100, 1000, 100_000
    src, dst, lat, loss = synth.complete_graph(n_nodes, 5, loss_max=0.25)
    plan = RoutingPlan(NetworkGraph.from_edges(n_nodes, src, dst, lat, loss), np.arange(n_nodes, dtype=np.uint32)).run()
    r0, r1 = 1_000_000_000, 1_000_000_000 + 5 * synth.MS
    pk, host_ptr, _ = synth.packet_round(n_hosts, n_nodes, n_pkts, 5, r0, r1)
    dev = torch.device("cuda:0")
    t_f = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
    t_d = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
    plan.packet_batch(torch.from_numpy(pk.view(np.uint8).copy()).to(dev),
                      torch.from_numpy(host_ptr.view(np.int32).copy()).to(dev),
                      torch.from_numpy(synth.host_rng_states(n_hosts, 1).view(np.int64).copy()).to(dev),
                      r1, 0, 2**62, t_f, t_d)
    flags = t_f.cpu().numpy().view(np.uint32)
    deliver = t_d.cpu().numpy().view(np.uint64)
    # destination host: hosts sit round-robin on the nodes; pick any host of dst_row
    dst_host = (pk.view(O.PKT_DTYPE)["dst_row"].astype(np.uint32) + n_nodes * (np.arange(n_pkts) % 10)).astype(
        np.uint32) % n_hosts
    base = np.zeros(n_hosts, np.uint64)
    ob = base.copy()
    eid_o, ord_o, ptr_o = O.packet_events(host_ptr, flags, deliver, dst_host, n_hosts, ob)
    eid, order, ptr, nb = _gpu_events(plan, host_ptr, flags, deliver, dst_host, n_hosts, base)
    assert (flags == O.PDS_INET_SENT).sum() == ptr[-1] > 0
    assert np.array_equal(eid, eid_o) and np.array_equal(order, ord_o) and np.array_equal(ptr, ptr_o)
    assert np.array_equal(nb, ob)


@gpu
def test_gpu_events_edge_cases():
    from shadow_amd import _lib

    plan = _plan()
    # nothing sent
    host_ptr = np.array([0, 3, 5], np.uint32)
    flags = np.array([O.PDS_INET_DROPPED, O.PDS_NONE, O.PDS_INET_DROPPED, O.PDS_NONE, O.PDS_NONE], np.uint32)
    deliver = np.zeros(5, np.uint64)
    dst = np.array([0, 1, 2, 0, 1], np.uint32)
    base = np.array([7, 9], np.uint64)
    eid, order, ptr, nb = _gpu_events(plan, host_ptr, flags, deliver, dst, 3, base)
    assert len(order) == 0 and (ptr == 0).all() and np.array_equal(nb, [7, 9])
    assert (eid == np.iinfo(np.uint64).max).all()
    # a destination out of range is an error
    flags[0] = O.PDS_INET_SENT
    dst[0] = 3
    with pytest.raises(_lib.SrtError, match="out of range"):
        _gpu_events(plan, host_ptr, flags, deliver, dst, 3, base)


@gpu
def test_gpu_events_big_group():
    """one destination receives far more than the on-chip group sort holds
    (1024 events): the call flags it and the status check redoes the batch
    with the exact two-sort path; the small groups beside it stay exact."""
    host_ptr, flags, deliver, dst, n_dst, base = _random_batch(5, n_hosts=60, n_pkts=12_000, n_dst=30)
    dst = dst.copy()
    dst[::2] = 7  # ~4,200 sent events to destination 7
    plan = _plan()
    ob = base.copy()
    eid_o, ord_o, ptr_o = O.packet_events(host_ptr, flags, deliver, dst, n_dst, ob)
    eid, order, ptr, nb = _gpu_events(plan, host_ptr, flags, deliver, dst, n_dst, base)
    assert ptr_o[8] - ptr_o[7] > 1024
    assert np.array_equal(eid, eid_o) and np.array_equal(order, ord_o) and np.array_equal(ptr, ptr_o)
    assert np.array_equal(nb, ob)


@gpu
def test_gpu_events_wide_time_span():
    """deliver times spanning ~2^60 ns: the group sort compares full 64-bit
    deliver times (no time-field width)."""
    host_ptr, flags, deliver, dst, n_dst, base = _random_batch(4, n_hosts=50, n_pkts=20_000, n_dst=40)
    rng = np.random.default_rng(4)
    deliver = (rng.integers(0, 8, size=len(deliver)).astype(np.uint64) << np.uint64(57)) + deliver
    plan = _plan()
    ob = base.copy()
    eid_o, ord_o, ptr_o = O.packet_events(host_ptr, flags, deliver, dst, n_dst, ob)
    eid, order, ptr, nb = _gpu_events(plan, host_ptr, flags, deliver, dst, n_dst, base)
    assert np.array_equal(eid, eid_o) and np.array_equal(order, ord_o) and np.array_equal(ptr, ptr_o)
    assert np.array_equal(nb, ob)


@gpu
def test_gpu_events_unchecked_big_group_is_reported():
    """A batch with a group over the on-chip sort's 1024 events, then another
    batch before any status check: the first batch can no longer be redone, so
    the status check reports it instead of returning OK (the second batch's own
    bits are still exact)."""
    from shadow_amd import _lib

    host_ptr, flags, deliver, dst, n_dst, base = _random_batch(5, n_hosts=60, n_pkts=12_000, n_dst=30)
    big = dst.copy()
    big[::2] = 7
    plan = _plan()
    import torch

    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)  # noqa: E731
    n = len(flags)
    outs = lambda: (torch.zeros(n, dtype=torch.int64, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),  # noqa
                    torch.zeros(n_dst + 1, dtype=torch.int32, device=dev))
    e1, o1, p1 = outs()
    plan.packet_events(t(host_ptr, np.int32), t(flags, np.int32), t(deliver, np.int64), t(big, np.int32), n_dst,
                       t(base, np.int64), e1, o1, p1, check=False)
    e2, o2, p2 = outs()
    plan.packet_events(t(host_ptr, np.int32), t(flags, np.int32), t(deliver, np.int64), t(dst, np.int32), n_dst,
                       t(base, np.int64), e2, o2, p2, check=False)
    with pytest.raises(_lib.SrtError, match="not checked"):
        plan.packet_events_status()
    plan.packet_events_status()  # the flags were cleared with the report
    ob = base.copy()
    _, ord_o, ptr_o = O.packet_events(host_ptr, flags, deliver, dst, n_dst, ob)
    ptr = p2.cpu().numpy().view(np.uint32)
    assert np.array_equal(ptr, ptr_o)
    assert np.array_equal(o2.cpu().numpy().view(np.uint32)[:ptr[-1]], ord_o)
