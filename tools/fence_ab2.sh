#!/bin/bash
# Sync-event fence x timing-event A/B on the real schedule (C2 and emulated 8 ranks).
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
for v in "0 1" "1 1" "0 1000" "1 1000"; do
  set -- $v
  if [ $1 = 1 ]; then export SRT_FW_SYNC_FENCE=dev; else unset SRT_FW_SYNC_FENCE; fi
  export SRT_FW_EVENT_EVERY=$2
  timeout -k 10 120 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/f2.txt 2>&1 || exit 1
  a=$(python3 -c "import json;d=json.loads(open('gpurun_out/f2.txt').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3))")
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks 8 > gpurun_out/f8.txt 2>&1 || exit 1
  b=$(python3 -c "import json;d=json.loads(open('gpurun_out/f8.txt').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3))")
  echo "nofence=$1 event_every=$2: c2 $a ms, emu8 $b ms"
done
done
