"""CPU tests of the packet stage's host-side pieces behind the C ABI:
IpAssignment (mod.rs:352-420) and the frozen IP -> table-row resolver
(worker.rs:539-553 lookups) against the oracle's restatement, and the host RNG
helpers (host.rs:233, sim_config.rs:47-53 / 222-244) against the oracle and
rand_xoshiro's published vector.  No device work."""
import ctypes as C
import ipaddress
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import _lib
from shadow_amd.graph import IpAssignment

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def be(ip: int) -> int:
    return int.from_bytes(ip.to_bytes(4, "big"), "little")


def test_assign_sequence_like_reference():
    a = IpAssignment()
    assert [str(a.assign(7)) for _ in range(3)] == ["11.0.0.1", "11.0.0.2", "11.0.0.3"]
    a.assign_ip(9, "11.0.0.4")
    assert str(a.assign(7)) == "11.0.0.5"  # skips the address assign_ip took
    with pytest.raises(ValueError, match="IP address has already been assigned"):
        a.assign_ip(1, "11.0.0.4")
    b = IpAssignment()
    for _ in range(254):
        b.assign(0)
    assert str(b.assign(0)) == "11.0.1.1"  # skips .255 and .0
    assert a.get_nodes() == {7, 9} and a.get_node("11.0.0.4") == 9 and a.get_node("10.0.0.1") is None
    assert len(a) == 5


def test_assign_interleaved_matches_oracle():
    """sim_config.rs:399-420: configured addresses first, then assign() for the
    rest -- random interleavings, including configured addresses that the
    auto-assignment later has to skip."""
    rng = np.random.default_rng(11)
    for trial in range(20):
        a, o = IpAssignment(), O.IpAssignment()
        for _ in range(400):
            node = int(rng.integers(0, 50))
            if rng.random() < 0.3:
                ip = (11 << 24) + int(rng.integers(0, 600))
                ok = o.assign_ip(node, ip)
                if ok:
                    a.assign_ip(node, ipaddress.IPv4Address(ip))
                else:
                    with pytest.raises(ValueError):
                        a.assign_ip(node, ipaddress.IPv4Address(ip))
            else:
                assert int(a.assign(node)) == o.assign(node)
        assert a.get_nodes() == o.get_nodes()
        for ip, node in o.map.items():
            assert a.get_node(ipaddress.IPv4Address(ip)) == node


@pytest.mark.parametrize("sparse", [False, True])
def test_resolver_rows_match_oracle(sparse):
    """IP -> node (get_node) -> table row (the RoutingInfo's rows), -1 where
    the reference's get_node or path() gives None; dense address spans use the
    direct table, scattered ones the hash."""
    rng = np.random.default_rng(3)
    a, o = IpAssignment(), O.IpAssignment()
    n_nodes = 300
    for h in range(5000):
        node = int(rng.integers(0, n_nodes))
        if sparse:
            ip = int(rng.integers(1 << 24, 1 << 31))
            if o.assign_ip(node, ip):
                a.assign_ip(node, ipaddress.IPv4Address(ip))
        else:
            assert int(a.assign(node)) == o.assign(node)
    # table rows: a subset of the nodes in a shuffled order
    in_use = rng.permutation(n_nodes)[:250].astype(np.uint32)
    row_of = {int(x): i for i, x in enumerate(in_use)}
    res = a.resolver(in_use)
    ips = list(o.map.keys())
    probe = np.array(ips + [int(rng.integers(0, 1 << 32)) for _ in range(2000)] + [0, 0xFFFFFFFF], np.uint64)
    got = res.rows(np.array([be(int(x)) for x in probe], np.uint32))
    exp = np.array([row_of.get(o.get_node(int(x)), -1) if o.get_node(int(x)) is not None else -1 for x in probe],
                   np.int32)
    assert np.array_equal(got, exp)
    # a big batch takes the threaded path
    big = np.repeat(probe, 200)[:300_000]
    gb = res.rows(np.array([be(int(x)) for x in big[:1000]], np.uint32))
    assert np.array_equal(gb, np.repeat(exp, 200)[:1000])
    res.close()


def test_resolver_rejects_duplicate_rows():
    a = IpAssignment()
    a.assign(1)
    with pytest.raises(_lib.SrtError):
        a.resolver(np.array([1, 1], np.uint32))


def test_host_rng_helpers_match_oracle_and_published_vector():
    L = _lib.lib()
    # rand_xoshiro's published xoshiro256++ vector from state [1, 2, 3, 4]
    vec = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
    st = np.array([1, 2, 3, 4], np.uint64)
    out = np.zeros(10, np.uint64)
    L.srt_xoshiro_next_u64(st.ctypes.data_as(C.POINTER(C.c_uint64)), 10, out.ctypes.data_as(C.POINTER(C.c_uint64)))
    kat = [int(x) for x in vec["xoshiro256pp_from_1234"]["values"]]
    assert out.tolist() == kat
    for seed in (0, 1, 12345, 2**63 + 5):
        s = np.zeros(4, np.uint64)
        L.srt_xoshiro_seed_from_u64(seed, s.ctypes.data_as(C.POINTER(C.c_uint64)))
        assert np.array_equal(s, O.xoshiro_seed(seed))
    s = np.zeros(4, np.uint64)
    L.srt_xoshiro_seed_from_u64(0, s.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert int(s[0]) == int(vec["splitmix64_state0_first"], 16)  # SplitMix64(0)'s first output
    for gs, name in ((1, "host0"), (1, "host9999"), (7, "a-much-longer-hostname-than-eight-bytes"), (0, "")):
        b = name.encode()
        assert L.srt_host_node_seed(gs, b, len(b)) == O.host_seed(gs, name)


def test_rng_handoff_continues_the_stream():
    """The hand-off of INTEGRATION.md section 4: a host's state goes out, N
    draws happen elsewhere (the device round), and the state that comes back
    continues the same stream the host's own draws (syscalls) would see."""
    L = _lib.lib()
    seed = L.srt_host_node_seed(1, b"host42", 6)
    s = np.zeros(4, np.uint64)
    L.srt_xoshiro_seed_from_u64(seed, s.ctypes.data_as(C.POINTER(C.c_uint64)))
    ref = s.copy()
    seq = [O.xoshiro_next(ref) for _ in range(37)]
    first = np.zeros(30, np.uint64)
    L.srt_xoshiro_next_u64(s.ctypes.data_as(C.POINTER(C.c_uint64)), 30, first.ctypes.data_as(C.POINTER(C.c_uint64)))
    rest = np.zeros(7, np.uint64)
    L.srt_xoshiro_next_u64(s.ctypes.data_as(C.POINTER(C.c_uint64)), 7, rest.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert first.tolist() + rest.tolist() == seq
    assert np.array_equal(s, ref)
