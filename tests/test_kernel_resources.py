"""Build-time guard on the gfx950 kernels (CPU: hipcc cross-compiles).

The hot kernels are register-tiled and sized for a fixed occupancy: an extra
kernel argument or a pointer into the argument struct can silently push them
into scratch (private memory) spills, which costs far more than any change it
came with.  This compiles the HIP sources for gfx950 and checks, from the
compiler's own resource report, that no kernel uses scratch and that the dense
tile kernels keep their two-workgroups-per-CU register budget.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "shadow_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _resources(src):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only", "-c",
           os.path.join(CSRC, src), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=CSRC)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
        if m and cur:
            kernels[cur][m.group(1).strip()] = int(m.group(2))
    return kernels


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", ["srt_fw.hip", "srt_sssp.hip", "srt_frontier.hip", "srt_packet.hip", "srt_direct.hip", "srt_loss.hip"])
def test_no_scratch_spills(src):
    ks = _resources(src)
    assert ks, "no kernels reported"
    spills = {k: v.get("ScratchSize [bytes/lane]") for k, v in ks.items() if v.get("ScratchSize [bytes/lane]", 0)}
    # the frontier sweeps are held at 8 waves/SIMD (<= 64 VGPRs) on purpose:
    # a few bytes of spill there measured faster than the unspilled 5-7 waves
    # (C4 1.03 -> 0.79 s) -- allowed, and capped
    allowed = {k: n for k, n in spills.items() if ("fr_lat_sweep_kernel" in k or "fr_loss_sweep_kernel" in k) and n <= 32}
    spills = {k: n for k, n in spills.items() if k not in allowed}
    assert not spills, f"kernels using scratch: {spills}"


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="hipcc not available")
def test_dense_tile_kernels_keep_two_workgroups_per_cu():
    ks = _resources("srt_fw.hip")
    tiles = {k: v for k, v in ks.items() if "minplus_glds_kernel" in k or "minplus_tile_kernel" in k}
    assert tiles
    for k, v in tiles.items():
        # 256 threads = one wave per SIMD per workgroup; 2 workgroups per CU
        # need <= 256 VGPRs per lane (512-entry VGPR file per SIMD lane)
        assert v.get("VGPRs", 999) + v.get("AGPRs", 0) <= 256, (k, v)
        assert v.get("Occupancy [waves/SIMD]", 0) >= 2, (k, v)
