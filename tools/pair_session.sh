#!/bin/bash
# Paired-round FW: parity tests, then C3 A/B (paired vs SRT_FW_NO_PAIR) on the same box.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fw_pair.py tests/test_gpu_apsp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pair_pytest.txt 2>&1 && tail -3 gpurun_out/pair_pytest.txt &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pair_c3.txt 2>&1 && tail -1 gpurun_out/pair_c3.txt &&
SRT_FW_NO_PAIR=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pair_c3_nopair.txt 2>&1 && tail -1 gpurun_out/pair_c3_nopair.txt
