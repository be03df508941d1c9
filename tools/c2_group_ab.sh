#!/bin/bash
# C2 (4k, chain-bound) A/B: default single-round vs forced round groups g=2, 4.
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "" "SRT_FW_PAIR=1 SRT_FW_GROUP=2" "SRT_FW_PAIR=1 SRT_FW_GROUP=4" "SRT_FW_PAIR=1 SRT_FW_GROUP=4 SRT_FW_NO_SMALL_CHAIN=1"; do
  env $v timeout -k 10 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c2ab.txt 2>&1 || exit 1
  echo "[$v] $(python -c "import json;d=json.loads(open('gpurun_out/c2ab.txt').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), round(d['roofline']['frac'],3))")"
done
