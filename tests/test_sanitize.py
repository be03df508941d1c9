"""The GPU-free host code of libsrt -- GML ingest, the CSR scan, the .xz
decoder, IpAssignment and its resolver, RoutingInfo's concurrent path() and
counters -- and the oracle, built for the CPU under AddressSanitizer and
UndefinedBehaviorSanitizer (tests/asan/Makefile: every -fsanitize= after
-Xarch_host) and driven by tests/asan/host_check.cpp with generated, truncated
and corrupted inputs; the threaded parts also under ThreadSanitizer.  Any
sanitizer report fails the run."""
import lzma
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan(tmp_path):
    d = os.path.join(ROOT, "tests", "asan")
    b = subprocess.run(["make", "-s", "-j8", "-C", d], capture_output=True, text=True, timeout=900)
    if b.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + b.stderr[-3000:])
    rng = np.random.default_rng(7)
    blobs = []
    for k, (data, check) in enumerate([
            (b"graph [ node [ id 1 ] ]\n" * 400, lzma.CHECK_CRC64),
            (rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes(), lzma.CHECK_CRC32),
            (b"ab" * 30_000 + bytes(range(256)) * 40, lzma.CHECK_SHA256),
            (b"", lzma.CHECK_NONE)]):
        f = tmp_path / f"b{k}.xz"
        f.write_bytes(lzma.compress(data, format=lzma.FORMAT_XZ, check=check))
        blobs.append(str(f))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(d, "host_check")] + blobs, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "host_check: clean" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    # the threaded parts again under ThreadSanitizer
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(d, "host_check_tsan")] + blobs, capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0 and "host_check: clean" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
