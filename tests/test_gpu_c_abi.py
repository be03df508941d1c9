"""The drop-in boundary called from plain C (tests/c_abi/srt_c_smoke.c, built
by tests/c_abi/Makefile against the in-tree libsrt.so): the reference's own
3-node golden latencies through both kernel families, and its error text."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "c_abi", "srt_c_smoke")


def test_c_abi_binary_is_built():
    assert os.path.exists(EXE), "run __graft_entry__.build() (make -C tests/c_abi)"


@pytest.mark.gpu
def test_c_consumer_on_gpu():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c abi ok" in r.stdout


EXIT_EXE = os.path.join(HERE, "c_abi", "srt_init_exit")


@pytest.mark.gpu
@pytest.mark.parametrize("delay_us", [0, 3000, 30000, 150000, 600000])
@pytest.mark.parametrize("how", ["return", "exit"])
def test_c_exit_during_async_init(delay_us, how):
    """A C process that calls srt_init_async and leaves main (or calls exit)
    before any build, at several points of the init thread's work, ends with
    its own status -- no signal, no hang (the library makes exit safe without
    the caller's help)."""
    r = subprocess.run([EXIT_EXE, str(delay_us), how], capture_output=True, text=True, timeout=100)
    assert r.returncode == 3, (r.returncode, r.stdout + r.stderr)
