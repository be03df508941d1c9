#!/bin/bash
# Banded tile order for grouped rest launches: parity, then C3 A/B (band on / off) on the same box.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fw_pair.py tests/test_gpu_apsp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/band_pytest.txt 2>&1 && tail -2 gpurun_out/band_pytest.txt &&
for v in "SRT_FW_BAND=1" "SRT_FW_BAND=0" "SRT_FW_BAND=1"; do
  env $v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bandab.txt 2>&1 || exit 1
  echo "[$v] $(python -c "import json;d=json.loads(open('gpurun_out/bandab.txt').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), round(d['roofline']['frac'],3))")"
done
