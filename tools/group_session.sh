#!/bin/bash
# Grouped-round FW: parity tests, then C3 A/B (g=4 default, g=2, single round) on the same box.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fw_pair.py tests/test_gpu_apsp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/grp_pytest.txt 2>&1 && tail -3 gpurun_out/grp_pytest.txt &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grp_c3_g4.txt 2>&1 && tail -1 gpurun_out/grp_c3_g4.txt | cut -c 1-900 &&
SRT_FW_GROUP=2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grp_c3_g2.txt 2>&1 && tail -1 gpurun_out/grp_c3_g2.txt | cut -c 1-900 &&
SRT_FW_NO_PAIR=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grp_c3_g1.txt 2>&1 && tail -1 gpurun_out/grp_c3_g1.txt | cut -c 1-900
