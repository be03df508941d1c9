#!/bin/bash
# Where grouping starts to pay: 8k and 12k complete graphs, single-round vs g=2 vs g=4.
export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 8192 12288; do
for v in "SRT_FW_NO_PAIR=1" "SRT_FW_GROUP=2" "SRT_FW_GROUP=4"; do
  env $v timeout -k 10 200 python -u bench.py --nodes $n --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/gateab.txt 2>&1 || exit 1
  echo "[$n $v] $(python -c "import json;d=json.loads(open('gpurun_out/gateab.txt').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), round(d['roofline']['frac'],3))")"
done; done
