#!/bin/bash
# Phase-1 shape A/B (SRT_FW_P1_ROWS = rows per thread: 8 -> 256 threads, 4 -> 512, 2 -> 1024):
# C2 build time and the phase-1 kernel's average duration under rocprofv3.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
for r in 8 4 2; do
  cd $R && SRT_FW_P1_ROWS=$r timeout -k 10 120 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p1_$r.txt 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/p1_$r.txt').read().strip().splitlines()[-1]);print('rows=$r c2 ms', round(d['ms_per_step'],3))"
  cd /tmp && SRT_FW_P1_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p1prof$r -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/p1prof$r.log 2>&1 || exit 1
  grep phase1 $R/gpurun_out/p1prof$r/run_kernel_stats.csv | cut -d, -f2-7
done
