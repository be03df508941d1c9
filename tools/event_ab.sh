#!/bin/bash
# Cost of the per-round timing events: SRT_FW_EVENT_EVERY=1 (every rest launch
# bracketed) vs 1000 (one launch), 1 GPU C3 and emulated 8 / 4 ranks.
export TMPDIR=/tmp; mkdir -p gpurun_out
for ev in 1 1000 1 1000; do
  for n in 8 4; do
    SRT_FW_EVENT_EVERY=$ev timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $n > gpurun_out/ev_$ev_$n.txt 2>&1 || exit 1
    echo "ev=$ev emu=$n $(tail -1 gpurun_out/ev_$ev_$n.txt)"
  done
  SRT_FW_EVENT_EVERY=$ev timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_$ev_1.txt 2>&1 || exit 1
  echo "ev=$ev 1gpu $(tail -1 gpurun_out/ev_$ev_1.txt | cut -c1-220)"
done
