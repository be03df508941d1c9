#!/bin/bash
# Tail-sweep target activation (SRT_SSSP_ACT: 0 off, 1 auto, k from sweep k): sparse parity tests, C4 build.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sssp.py tests/test_gpu_dist.py -x -q --timeout 150 --timeout-method thread > gpurun_out/act_tests.txt 2>&1 || { tail -30 gpurun_out/act_tests.txt; exit 1; }
tail -1 gpurun_out/act_tests.txt
SRT_SSSP_ACT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_sssp.py -x -q --timeout 150 --timeout-method thread > gpurun_out/act_tests2.txt 2>&1 || { tail -30 gpurun_out/act_tests2.txt; exit 1; }
tail -1 gpurun_out/act_tests2.txt
for a in 0 1 24 1 0; do
  SRT_SSSP_ACT=$a timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/act_$a.txt 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/act_$a.txt').read().strip().splitlines()[-1]);print('act=$a c4 ms', round(d['ms_per_step'],1))"
done
